// Static-graph interpreter core: instruction dependency graph, stream/event plan, garbage-collection plan and a
// dependency-counting ready queue for asynchronous execution.
//
// Reference behaviour: paddle/fluid/framework/new_executor/interpreter/dependency_builder.cc (RAW / WAR / WAW
// edges between instructions, ShrinkDownstreamMap's transitive reduction), stream_analyzer.cc (events only on
// cross-stream edges), pir_interpreter.cc:804 (BuildInstructionDependences), :1077 / :1458 (RunInstruction /
// RunNextInstructions: dependency counters decremented as instructions finish, ready ones pushed to the async
// work queue) and interpreter_util's garbage collection (a variable is released once its last reader ran).
//
// Not a translation: one compact plan object built from per-op read / write variable ids, a stream class per op
// and a "barrier" flag for ops with hidden side effects (backward, optimizer step), consumed by the Python
// executor (static/executor.py) either as a deterministic issue order for device work (kernels are async on
// their streams; only cross-stream edges get events) or through the thread-safe ReadyQueue by N host worker
// threads (independent CPU ops of a Program run concurrently; torch ops release the GIL while they compute).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <queue>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

#include "runtime.h"

namespace pdrt {

namespace {

// dense bitset over instruction ids (transitive reduction)
struct Bits {
  std::vector<uint64_t> w;
  explicit Bits(int n = 0) : w((n + 63) / 64, 0) {}
  bool test(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  void set(int i) { w[i >> 6] |= 1ull << (i & 63); }
  void merge(const Bits& o) {
    for (size_t k = 0; k < w.size(); ++k) w[k] |= o.w[k];
  }
};

constexpr int kReduceLimit = 8192;  // above this many instructions the edge set is kept unreduced (memory)

}  // namespace

InterpPlan build_interp_plan(const std::vector<std::vector<int64_t>>& reads,
                             const std::vector<std::vector<int64_t>>& writes, const std::vector<int>& stream,
                             const std::vector<int>& barrier, const std::vector<int64_t>& keep) {
  const int n = (int)reads.size();
  if ((int)writes.size() != n || (int)stream.size() != n || (int)barrier.size() != n)
    throw std::invalid_argument("build_interp_plan: per-op vectors differ in length");
  InterpPlan P;
  P.n = n;

  // ---- edges (always from a lower to a higher instruction id: the recorded order is a valid schedule)
  std::vector<std::vector<int>> succ(n);
  auto edge = [&](int a, int b) {
    if (a >= 0 && a != b) succ[a].push_back(b);
  };
  std::unordered_map<int64_t, int> last_writer;
  std::unordered_map<int64_t, std::vector<int>> readers;  // since the last write
  int last_barrier = -1;
  std::vector<int> since_barrier;
  for (int i = 0; i < n; ++i) {
    if (barrier[i]) {
      // hidden side effects (autograd engine, optimizer state): after everything before, before everything after
      for (int j : since_barrier) edge(j, i);
      edge(last_barrier, i);
      since_barrier.clear();
    } else {
      edge(last_barrier, i);
    }
    for (int64_t v : reads[i]) {
      auto it = last_writer.find(v);
      if (it != last_writer.end()) edge(it->second, i);  // RAW
      readers[v].push_back(i);
    }
    for (int64_t v : writes[i]) {
      auto rit = readers.find(v);
      if (rit != readers.end()) {
        for (int r : rit->second) edge(r, i);  // WAR
        rit->second.clear();
      }
      auto it = last_writer.find(v);
      if (it != last_writer.end()) edge(it->second, i);  // WAW
      last_writer[v] = i;
    }
    if (barrier[i]) last_barrier = i;
    else since_barrier.push_back(i);
  }
  for (auto& s : succ) {
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
  }
  for (auto& s : succ) P.num_edges_raw += (int64_t)s.size();

  // ---- transitive reduction (ShrinkDownstreamMap): drop a -> c when c is reachable through another successor
  if (n <= kReduceLimit) {
    std::vector<Bits> reach(n, Bits(n));
    for (int i = n - 1; i >= 0; --i) {
      Bits covered(n);
      std::vector<int> kept;
      for (int s : succ[i]) {  // ascending: a successor can only be reached through smaller ones
        if (covered.test(s)) continue;
        kept.push_back(s);
        covered.merge(reach[s]);
      }
      succ[i].swap(kept);
      reach[i] = covered;
      reach[i].set(i);
    }
  }
  P.downstream = succ;
  P.dep_count.assign(n, 0);
  for (int i = 0; i < n; ++i)
    for (int s : succ[i]) ++P.dep_count[s];

  // ---- issue order: Kahn's algorithm, side-stream (communication / copy) instructions first among the ready
  // ones so their streams start as early as the data allows, then by recorded position
  {
    std::vector<int> cnt = P.dep_count;
    auto cmp = [&](int a, int b) {  // priority_queue: "a after b"
      const int pa = stream[a] != 0 ? 0 : 1, pb = stream[b] != 0 ? 0 : 1;
      return pa != pb ? pa > pb : a > b;
    };
    std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
    for (int i = 0; i < n; ++i)
      if (cnt[i] == 0) ready.push(i);
    while (!ready.empty()) {
      const int i = ready.top();
      ready.pop();
      P.order.push_back(i);
      for (int s : succ[i])
        if (--cnt[s] == 0) ready.push(s);
    }
    if ((int)P.order.size() != n) throw std::logic_error("build_interp_plan: dependency cycle");
  }

  // ---- events: a cross-stream edge p -> i makes i's stream wait on an event p records after it
  P.waits.assign(n, {});
  P.record.assign(n, 0);
  for (int p = 0; p < n; ++p)
    for (int i : succ[p])
      if (stream[p] != stream[i]) {
        P.waits[i].push_back(p);
        P.record[p] = 1;
      }

  // ---- garbage collection: per variable the number of instructions reading it (the async queue frees it when
  // the count drains) and, for the sequential issue order, the instruction after which it is dead
  std::unordered_map<int64_t, int> keepset;
  for (int64_t v : keep) keepset[v] = 1;
  std::unordered_map<int64_t, int> last_pos;  // position in `order` of the last reader
  std::vector<int> pos(n);
  for (int k = 0; k < n; ++k) pos[P.order[k]] = k;
  for (int i = 0; i < n; ++i)
    for (int64_t v : reads[i]) {
      if (keepset.count(v)) continue;
      auto it = last_pos.find(v);
      if (it == last_pos.end() || it->second < pos[i]) last_pos[v] = pos[i];
    }
  P.free_after.assign(n, {});
  for (auto& kv : last_pos) P.free_after[P.order[kv.second]].push_back(kv.first);
  for (auto& f : P.free_after) std::sort(f.begin(), f.end());
  P.reader_count.clear();
  for (int i = 0; i < n; ++i) {
    std::vector<int64_t> uniq = reads[i];
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    for (int64_t v : uniq)
      if (!keepset.count(v)) P.reader_count[v] += 1;
  }
  P.reads = reads;
  for (auto& r : P.reads) {
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
  }
  return P;
}

// ------------------------------------------------------------------ ReadyQueue
struct ReadyQueue::Impl {
  const InterpPlan* plan = nullptr;
  InterpPlan owned;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<int> ready;
  std::vector<int> cnt;
  std::unordered_map<int64_t, int> readers_left;
  int finished = 0, running = 0;
  bool failed = false, started = false;
};

ReadyQueue::ReadyQueue(const InterpPlan& plan) : impl_(new Impl) {
  impl_->owned = plan;
  impl_->plan = &impl_->owned;
}
ReadyQueue::~ReadyQueue() = default;

void ReadyQueue::start() {
  std::lock_guard<std::mutex> g(impl_->mu);
  const InterpPlan& P = *impl_->plan;
  impl_->cnt = P.dep_count;
  impl_->readers_left = P.reader_count;
  impl_->ready.clear();
  for (int i : P.order)
    if (impl_->cnt[i] == 0) impl_->ready.push_back(i);
  impl_->finished = impl_->running = 0;
  impl_->failed = false;
  impl_->started = true;
}

int ReadyQueue::pop(double timeout_s) {
  std::unique_lock<std::mutex> lk(impl_->mu);
  const int n = impl_->plan->n;
  auto pred = [&] { return impl_->failed || !impl_->ready.empty() || impl_->finished == n; };
  if (timeout_s < 0) impl_->cv.wait(lk, pred);
  else if (!impl_->cv.wait_for(lk, std::chrono::duration<double>(timeout_s), pred)) return -2;  // timed out
  if (impl_->failed || impl_->ready.empty()) return -1;  // aborted or everything finished
  const int i = impl_->ready.front();
  impl_->ready.pop_front();
  ++impl_->running;
  return i;
}

std::vector<int64_t> ReadyQueue::done(int i) {
  std::vector<int64_t> dead;
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    const InterpPlan& P = *impl_->plan;
    if (i < 0 || i >= P.n) throw std::out_of_range("ReadyQueue.done: bad instruction id");
    for (int s : P.downstream[i])
      if (--impl_->cnt[s] == 0) impl_->ready.push_back(s);
    for (int64_t v : P.reads[i]) {
      auto it = impl_->readers_left.find(v);
      if (it != impl_->readers_left.end() && --it->second == 0) dead.push_back(v);
    }
    --impl_->running;
    ++impl_->finished;
  }
  impl_->cv.notify_all();
  return dead;
}

void ReadyQueue::fail() {
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    impl_->failed = true;
  }
  impl_->cv.notify_all();
}

bool ReadyQueue::finished() {
  std::lock_guard<std::mutex> g(impl_->mu);
  return impl_->finished == impl_->plan->n;
}

}  // namespace pdrt
