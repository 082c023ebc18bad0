// Host event tracer (reference: paddle/phi/api/profiler/host_tracer.cc + host_event_recorder.h —
// per-thread lock-free event buffers merged at collection; chrome_tracing_logger.cc export).
//
// Each thread appends to its own buffer guarded by its own mutex — uncontended on the hot path (only a
// collection takes it from another thread); names are interned once.  RecordEvent in Python maps to
// push/pop; collection walks every thread's buffer.  (The first version appended lock-free and let a
// concurrent collection copy a vector the owner was reallocating: found by the TSan/ASan stress build,
// csrc/runtime/stress/runtime_stress.cpp.)
#include <atomic>
#include <chrono>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "runtime.h"

namespace pdrt {
namespace {

struct ThreadBuf {
  uint64_t tid;
  std::mutex mu;                 // owner appends, collectors copy / clear
  std::vector<HostEvent> done;
  std::vector<HostEvent> stack;  // owner-only
};

std::mutex g_mu;                       // guards the registry and the name table
std::vector<std::shared_ptr<ThreadBuf>> g_bufs;
std::unordered_map<std::string, uint32_t> g_name_ids;
std::vector<std::string> g_names;
std::atomic<bool> g_on{false};

ThreadBuf& tbuf() {
  thread_local std::shared_ptr<ThreadBuf> b;
  if (!b) {
    b = std::make_shared<ThreadBuf>();
    b->tid = std::hash<std::thread::id>()(std::this_thread::get_id()) & 0xffffffffull;
    std::lock_guard<std::mutex> g(g_mu);
    g_bufs.push_back(b);
  }
  return *b;
}

uint32_t intern(const std::string& n) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_name_ids.find(n);
  if (it != g_name_ids.end()) return it->second;
  uint32_t id = (uint32_t)g_names.size();
  g_names.push_back(n);
  g_name_ids.emplace(n, id);
  return id;
}

void json_escape(std::ostringstream& o, const std::string& s) {
  for (char c : s) {
    if (c == '"' || c == '\\') o << '\\' << c;
    else if ((unsigned char)c < 0x20) o << ' ';
    else o << c;
  }
}

}  // namespace

uint64_t tracer_now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void tracer_enable(bool on) { g_on = on; }
bool tracer_enabled() { return g_on; }

void tracer_push(const std::string& name, uint32_t type) {
  if (!g_on) return;
  auto& b = tbuf();
  b.stack.push_back({intern(name), type, b.tid, tracer_now_ns(), 0});
}

void tracer_pop() {
  auto& b = tbuf();
  if (b.stack.empty()) return;
  HostEvent e = b.stack.back();
  b.stack.pop_back();
  if (!g_on) return;
  e.end_ns = tracer_now_ns();
  std::lock_guard<std::mutex> g(b.mu);
  b.done.push_back(e);
}

void tracer_instant(const std::string& name, uint32_t type, uint64_t s, uint64_t e) {
  if (!g_on) return;
  auto& b = tbuf();
  const uint32_t id = intern(name);
  std::lock_guard<std::mutex> g(b.mu);
  b.done.push_back({id, type, b.tid, s, e});
}

void tracer_clear() {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> gb(b->mu);
    b->done.clear();
  }
}

std::vector<HostEvent> tracer_events() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<HostEvent> out;
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> gb(b->mu);
    out.insert(out.end(), b->done.begin(), b->done.end());
  }
  return out;
}

std::string tracer_name(uint32_t id) {
  std::lock_guard<std::mutex> g(g_mu);
  return id < g_names.size() ? g_names[id] : std::string("?");
}

std::string tracer_chrome_json(int pid) {
  static const char* kCat[] = {"UserDefined", "Operator", "Communication", "Dataloader", "Optimization"};
  auto evs = tracer_events();
  std::ostringstream o;
  o << "{\"traceEvents\":[";
  bool first = true;
  for (auto& e : evs) {
    if (!first) o << ',';
    first = false;
    o << "{\"name\":\"";
    json_escape(o, tracer_name(e.name_id));
    o << "\",\"cat\":\"" << kCat[e.type < 5 ? e.type : 0] << "\",\"ph\":\"X\",\"pid\":" << pid
      << ",\"tid\":" << e.tid << ",\"ts\":" << (double)e.start_ns / 1000.0
      << ",\"dur\":" << (double)(e.end_ns - e.start_ns) / 1000.0 << '}';
  }
  o << "],\"displayTimeUnit\":\"ms\"}";
  return o.str();
}

}  // namespace pdrt
