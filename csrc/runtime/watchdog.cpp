// Communication watchdog (reference: paddle/phi/core/distributed/comm_task_manager.cc — a
// background thread that scans in-flight comm tasks and reports/aborts the ones past their
// timeout, plus the dynamic checks of the NCCL process group).
//
// Collectives register (description, deadline) on launch and deregister when their completion
// is observed; a native thread polls the table and, for any task past its deadline, logs the
// hang with the op description to stderr and optionally aborts the process so the launcher can
// tear the job down instead of letting every rank wait forever.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <thread>

#include "runtime.h"

namespace pdrt {
namespace {

struct Task {
  std::string desc;
  std::chrono::steady_clock::time_point deadline;
  bool reported = false;
  void* event = nullptr;  // hipEvent_t recorded after the collective's launch (nullptr: host task)
};

// hipEventQuery resolved lazily from the already-loaded HIP runtime (the module itself links no
// HIP so it also loads on CPU-only hosts); returns 0 (hipSuccess) once the event has completed.
typedef int (*EventQueryFn)(void*);
EventQueryFn event_query() {
  static EventQueryFn fn = [] {
    void* h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_NOLOAD);
    return h ? (EventQueryFn)dlsym(h, "hipEventQuery") : (EventQueryFn) nullptr;
  }();
  return fn;
}
std::vector<int64_t> w_finished;

std::mutex w_mu;
std::map<int64_t, Task> w_tasks;
std::vector<std::string> w_timed_out;
std::atomic<int64_t> w_next{1};
std::thread w_thread;
std::atomic<bool> w_run{false};  // also read by the poller between condition-variable waits
bool w_abort = false;
std::atomic<double> w_poll{1.0};

// Sleep in <= 5 ms slices between scans (no condition variable: stop latency is one slice, and the loop
// stays analysable by the sanitizer build, whose runtime does not model libstdc++'s clockwait waits).
bool nap(double seconds) {
  const auto until = std::chrono::steady_clock::now() + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                                            std::chrono::duration<double>(seconds));
  while (w_run.load()) {
    const auto now = std::chrono::steady_clock::now();
    if (now >= until) return true;
    std::this_thread::sleep_for(std::min<std::chrono::steady_clock::duration>(until - now, std::chrono::milliseconds(5)));
  }
  return false;
}

void loop() {
  while (nap(w_poll)) {
    std::lock_guard<std::mutex> lk(w_mu);
    auto now = std::chrono::steady_clock::now();
    EventQueryFn q = event_query();
    for (auto it = w_tasks.begin(); it != w_tasks.end();) {
      if (it->second.event && q && q(it->second.event) == 0) {
        w_finished.push_back(it->first);
        it = w_tasks.erase(it);
      } else {
        ++it;
      }
    }
    for (auto& kv : w_tasks) {
      Task& t = kv.second;
      if (!t.reported && now > t.deadline) {
        t.reported = true;
        w_timed_out.push_back(t.desc);
        std::fprintf(stderr, "[paddle2_amd watchdog] collective timed out: %s\n", t.desc.c_str());
        std::fflush(stderr);
        if (w_abort) std::abort();
      }
    }
  }
}

}  // namespace

void watchdog_start(double poll_s, bool abort_on_timeout) {
  std::lock_guard<std::mutex> g(w_mu);
  w_poll = poll_s;
  w_abort = abort_on_timeout;
  if (w_run) return;
  w_run = true;
  w_thread = std::thread(loop);
}

void watchdog_stop() {
  {
    std::lock_guard<std::mutex> g(w_mu);
    if (!w_run) return;
    w_run = false;
  }
  if (w_thread.joinable()) w_thread.join();
}

int64_t watchdog_begin(const std::string& desc, double timeout_s, uintptr_t event) {
  int64_t id = w_next.fetch_add(1);
  std::lock_guard<std::mutex> g(w_mu);
  Task t;
  t.desc = desc;
  t.deadline = std::chrono::steady_clock::now() + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                                       std::chrono::duration<double>(timeout_s));
  t.event = reinterpret_cast<void*>(event);
  w_tasks[id] = t;
  return id;
}

std::vector<int64_t> watchdog_take_finished() {
  std::lock_guard<std::mutex> g(w_mu);
  std::vector<int64_t> out;
  out.swap(w_finished);
  return out;
}

void watchdog_end(int64_t id) {
  std::lock_guard<std::mutex> g(w_mu);
  w_tasks.erase(id);
}

std::vector<std::string> watchdog_timed_out() {
  std::lock_guard<std::mutex> g(w_mu);
  return w_timed_out;
}

namespace {
// stop and join the poller before the statics it uses are destroyed (a joinable std::thread at
// static destruction would call std::terminate)
struct StopAtExit {
  ~StopAtExit() { watchdog_stop(); }
} g_stop_at_exit;
}  // namespace

int64_t watchdog_inflight() {
  std::lock_guard<std::mutex> g(w_mu);
  return (int64_t)w_tasks.size();
}

}  // namespace pdrt
