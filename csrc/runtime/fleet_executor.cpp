// FleetExecutor: actor-model task runtime for pipelined / multi-stage execution
// (reference: paddle/fluid/distributed/fleet_executor/ — carrier.cc, interceptor.cc, compute_interceptor.cc,
//  amplifier_interceptor.cc, source_interceptor.cc, sink_interceptor.cc, message_bus.cc, task_loop*.cc).
//
// A Carrier owns this rank's interceptors (one per task node) and a few loop threads; each interceptor is bound
// to one loop, so its state is only touched by that thread and messages to it are serialized through the
// loop's queue.  Control flow is credit-based, as in the reference:
//   * an edge up -> down has a buffer size B: `down` counts ready micro-steps per upstream, `up` counts how
//     many of its B buffers `down` still holds; DATA_IS_READY moves a credit downstream, DATA_IS_USELESS
//     returns it;
//   * a Compute interceptor runs step s when every upstream has a ready step and every downstream has a free
//     buffer; an Amplifier runs its callback only on steps with s % run_per_steps == run_at_offset (e.g. the
//     optimizer once per mini-batch) but forwards every step; a Source feeds max_run_times steps; a Sink counts
//     them and finishes the run.
// Interceptors on other ranks are reached through the MessageBus: one TCP listener per carrier, lazily opened
// connections, fixed 32-byte frames.  The compute callback is user code (Python through the binding); an
// exception stops the carrier and is re-raised by wait().
// Runs are epochs: start() bumps the carrier's run id and every frame carries the run it belongs to.  A frame of a
// newer run that reaches a node before that run's kStart (a faster rank's next run may reach us while this node
// still finishes the current one, or before our start()) is stashed on the node and replayed, in arrival order,
// right after the node resets its counters for that run on its own loop thread; frames of older runs (the last
// DATA_IS_USELESS of the previous run, still in flight) are dropped.  No counter is touched by two runs or two
// threads, and no step of the current run is lost to an early frame of the next (resetting on that frame dropped
// the node's last steps of the current run).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <stdexcept>
#include <thread>

#include "runtime.h"

namespace pdrt {

namespace {

enum MsgType : int64_t { kReady = 0, kUseless = 1, kStart = 2, kStop = 3 };

struct Msg {
  int64_t src, dst, type, step, run;
};

bool send_frame(int fd, const Msg& m) {
  const char* p = reinterpret_cast<const char*>(&m);
  size_t n = sizeof(Msg);
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w <= 0) return false;
    p += w;
    n -= size_t(w);
  }
  return true;
}

bool recv_frame(int fd, Msg* m) {
  char* p = reinterpret_cast<char*>(m);
  size_t n = sizeof(Msg);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) return false;
    p += r;
    n -= size_t(r);
  }
  return true;
}

}  // namespace

struct FleetCarrier::Impl {
  struct Node {
    FleetTask spec;
    int loop = 0;
    std::map<int64_t, int64_t> ready;     // upstream id -> ready steps not yet consumed
    std::map<int64_t, int64_t> used;      // downstream id -> buffers held by it
    std::map<int64_t, int64_t> cap;       // downstream id -> buffer size
    int64_t step = 0;                     // steps run (compute / amplifier / source) or received (sink)
    bool started = false;
    int64_t run = 0;                      // run (epoch) the counters belong to; touched by the loop thread only
    int64_t finished_run = 0;             // last run this node completed (guarded by done_mu)
    bool counted = false;                 // sink, or a task with max_run_times > 0: wait() waits for it
    std::deque<Msg> stash;                // frames of a newer run that arrived before its kStart (loop thread only)
  };

  struct Loop {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Msg> q;
    std::thread th;
  };

  int rank;
  std::map<int64_t, Node> nodes;          // local task id -> node
  std::map<int64_t, int> task_rank;       // every task id -> rank
  std::vector<std::unique_ptr<Loop>> loops;
  FleetCarrier::ComputeFn compute;
  std::atomic<bool> running{false};
  std::mutex done_mu;
  std::condition_variable done_cv;
  std::atomic<int64_t> epoch{0};          // current run id of this carrier (bumped by start())
  std::string error;                      // guarded by done_mu
  std::atomic<bool> failed{false};        // lock-free view of !error.empty() for the loop threads
  std::vector<std::array<int64_t, 3>> trace;  // (task, step, sequence) of compute callbacks
  std::mutex trace_mu;
  std::atomic<int64_t> seq{0};
  // message bus
  int listen_fd = -1;
  int port = 0;
  std::thread acceptor;
  std::vector<std::thread> readers;
  std::vector<int> reader_fds;
  std::map<int, std::pair<std::string, int>> peers;  // rank -> address
  std::map<int, int> out_fd;
  std::mutex out_mu;
  std::atomic<bool> bus_up{false};

  void post(const Msg& m) {
    auto it = nodes.find(m.dst);
    if (it == nodes.end()) {
      send_remote(m);
      return;
    }
    Loop& L = *loops[it->second.loop];
    {
      std::lock_guard<std::mutex> lk(L.mu);
      L.q.push_back(m);
    }
    L.cv.notify_one();
  }

  void send_remote(const Msg& m) {
    auto tr = task_rank.find(m.dst);
    if (tr == task_rank.end()) {
      fail("message to unknown task " + std::to_string(m.dst));
      return;
    }
    std::lock_guard<std::mutex> lk(out_mu);
    int fd;
    auto f = out_fd.find(tr->second);
    if (f == out_fd.end()) {
      auto pr = peers.find(tr->second);
      if (pr == peers.end()) {
        fail("no address for rank " + std::to_string(tr->second));
        return;
      }
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons(uint16_t(pr->second.second));
      ::inet_pton(AF_INET, pr->second.first.c_str(), &a.sin_addr);
      bool ok = false;
      for (int tries = 0; tries < 200 && !ok; ++tries) {
        ok = ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0;
        if (!ok) std::this_thread::sleep_for(std::chrono::milliseconds(25));
      }
      if (!ok) {
        ::close(fd);
        fail("cannot connect to rank " + std::to_string(tr->second));
        return;
      }
      int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      out_fd[tr->second] = fd;
    } else {
      fd = f->second;
    }
    if (!send_frame(fd, m)) fail("send to rank " + std::to_string(tr->second) + " failed");
  }

  void fail(const std::string& why) {
    {
      std::lock_guard<std::mutex> lk(done_mu);
      if (error.empty()) error = why;
      failed = true;
    }
    done_cv.notify_all();
  }

  void finish_one(Node& n) {
    std::lock_guard<std::mutex> lk(done_mu);
    n.finished_run = n.run;
    done_cv.notify_all();
  }

  // every counted node has completed run r (caller holds done_mu)
  bool all_finished(int64_t r) {
    for (auto& kv : nodes)
      if (kv.second.counted && kv.second.finished_run < r) return false;
    return true;
  }

  // fresh counters for run r, on the node's loop thread
  static void reset(Node& n, int64_t r) {
    n.run = r;
    n.step = 0;
    n.started = false;
    for (auto& kv : n.ready) kv.second = 0;
    for (auto& kv : n.used) kv.second = 0;
  }

  bool can_run(Node& n) {
    if (n.step >= n.spec.max_run_times) return false;
    for (auto& kv : n.ready)
      if (kv.second <= 0) return false;
    for (auto& kv : n.used)
      if (kv.second >= n.cap[kv.first]) return false;
    return true;
  }

  void run_compute(Node& n) {
    int64_t s = n.step;
    bool call = n.spec.role == FleetTask::kCompute ||
                (n.spec.role == FleetTask::kAmplifier && n.spec.run_per_steps > 0 &&
                 s % n.spec.run_per_steps == n.spec.run_at_offset);
    if (call && compute) {
      {
        std::lock_guard<std::mutex> lk(trace_mu);
        trace.push_back({n.spec.id, s, seq++});
      }
      try {
        compute(n.spec.id, s);
      } catch (const std::exception& e) {
        fail(std::string("task ") + std::to_string(n.spec.id) + " step " + std::to_string(s) + ": " + e.what());
        return;
      }
    }
    n.step++;
    for (auto& kv : n.ready) {
      kv.second--;
      post({n.spec.id, kv.first, kUseless, s, n.run});
    }
    for (auto& kv : n.used) {
      kv.second++;
      post({n.spec.id, kv.first, kReady, s, n.run});
    }
    if (n.step == n.spec.max_run_times) finish_one(n);
  }

  void handle(Node& n, const Msg& m) {
    if (failed.load()) return;
    if (m.run < n.run) return;          // a frame of a finished run
    if (m.run > n.run) {
      if (m.type != kStart) {           // a newer run's frame before its start reached this node: keep it
        n.stash.push_back(m);
        return;
      }
      reset(n, m.run);
      dispatch(n, m);
      std::deque<Msg> st;
      st.swap(n.stash);
      for (const Msg& f : st) {
        if (f.run == n.run) dispatch(n, f);
        else if (f.run > n.run) n.stash.push_back(f);
      }
      return;
    }
    dispatch(n, m);
  }

  // a frame of the node's current run
  void dispatch(Node& n, const Msg& m) {
    if (failed.load()) return;
    switch (m.type) {
      case kStart:
        // roots (sources, and nodes without upstream such as an lr Amplifier) start on their own
        n.started = n.spec.role == FleetTask::kSource || n.spec.upstream.empty();
        if (!n.started) return;
        break;
      case kReady:
        if (n.spec.role == FleetTask::kSink) {
          n.step++;
          post({n.spec.id, m.src, kUseless, m.step, n.run});
          if (n.step == n.spec.max_run_times) finish_one(n);
          return;
        }
        n.ready[m.src]++;
        break;
      case kUseless:
        n.used[m.src]--;
        break;
      case kStop:
        return;
    }
    if (n.spec.role == FleetTask::kSource) {
      if (!n.started) return;
      while (n.step < n.spec.max_run_times) {
        bool room = true;
        for (auto& kv : n.used)
          if (kv.second >= n.cap[kv.first]) room = false;
        if (!room) break;
        int64_t s = n.step++;
        for (auto& kv : n.used) {
          kv.second++;
          post({n.spec.id, kv.first, kReady, s, n.run});
        }
        if (n.step == n.spec.max_run_times) finish_one(n);
      }
      return;
    }
    while (!failed.load() && can_run(n)) run_compute(n);
  }

  void loop_main(Loop* L) {
    for (;;) {
      Msg m;
      {
        std::unique_lock<std::mutex> lk(L->mu);
        L->cv.wait(lk, [&] { return !L->q.empty() || !running.load(); });
        if (L->q.empty()) return;
        m = L->q.front();
        L->q.pop_front();
      }
      auto it = nodes.find(m.dst);
      if (it != nodes.end()) handle(it->second, m);
    }
  }

  void accept_main() {
    while (bus_up.load()) {
      sockaddr_in a{};
      socklen_t len = sizeof(a);
      int fd = ::accept(listen_fd, reinterpret_cast<sockaddr*>(&a), &len);
      if (fd < 0) {
        if (!bus_up.load()) return;
        continue;
      }
      std::lock_guard<std::mutex> lk(out_mu);
      reader_fds.push_back(fd);
      readers.emplace_back([this, fd] {
        Msg m;
        while (recv_frame(fd, &m)) post(m);
      });
    }
  }
};

FleetCarrier::FleetCarrier(int rank, int num_threads) : impl_(new Impl) {
  impl_->rank = rank;
  int n = num_threads > 0 ? num_threads : 1;
  for (int i = 0; i < n; ++i) impl_->loops.emplace_back(new Impl::Loop);
}

FleetCarrier::~FleetCarrier() { shutdown(); }

void FleetCarrier::add_task(const FleetTask& t) {
  impl_->task_rank[t.id] = t.rank;
  if (t.rank != impl_->rank) return;
  Impl::Node n;
  n.spec = t;
  n.loop = int(impl_->nodes.size() % impl_->loops.size());
  n.counted = t.role == FleetTask::kSink || t.max_run_times > 0;
  for (auto& u : t.upstream) n.ready[u.first] = 0;
  for (auto& d : t.downstream) {
    n.used[d.first] = 0;
    n.cap[d.first] = d.second > 0 ? d.second : (int64_t(1) << 40);
  }
  impl_->nodes.emplace(t.id, std::move(n));
}

void FleetCarrier::add_remote_task(int64_t id, int rank) { impl_->task_rank[id] = rank; }

void FleetCarrier::set_compute(ComputeFn fn) { impl_->compute = std::move(fn); }

int FleetCarrier::listen(const std::string& host) {
  Impl& I = *impl_;
  I.listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  ::setsockopt(I.listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = 0;
  ::inet_pton(AF_INET, host.c_str(), &a.sin_addr);
  if (::bind(I.listen_fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(I.listen_fd, 64) != 0)
    throw std::runtime_error("FleetCarrier: cannot listen on " + host);
  socklen_t len = sizeof(a);
  ::getsockname(I.listen_fd, reinterpret_cast<sockaddr*>(&a), &len);
  I.port = ntohs(a.sin_port);
  I.bus_up = true;
  I.acceptor = std::thread([&I] { I.accept_main(); });
  return I.port;
}

void FleetCarrier::set_peer(int rank, const std::string& host, int port) { impl_->peers[rank] = {host, port}; }

void FleetCarrier::start() {
  Impl& I = *impl_;
  {
    std::lock_guard<std::mutex> lk(I.done_mu);
    I.error.clear();
    I.failed = false;
  }
  // a new run: every node learns it from its kStart (or from an earlier frame of the run) on its loop thread
  const int64_t r = ++I.epoch;
  I.running = true;
  for (auto& L : I.loops)
    if (!L->th.joinable()) L->th = std::thread([&I, Lp = L.get()] { I.loop_main(Lp); });
  for (auto& kv : I.nodes) I.post({-1, kv.first, kStart, 0, r});
}

bool FleetCarrier::wait(double timeout_s) {
  Impl& I = *impl_;
  std::unique_lock<std::mutex> lk(I.done_mu);
  const int64_t r = I.epoch.load();
  auto pred = [&] { return !I.error.empty() || I.all_finished(r); };
  // system_clock deadline: wait_until maps to pthread_cond_timedwait (steady-clock waits use
  // pthread_cond_clockwait, which GCC 11's TSan runtime does not intercept)
  bool ok = true;
  if (timeout_s < 0) {
    I.done_cv.wait(lk, pred);
  } else {
    auto deadline = std::chrono::system_clock::now() +
                    std::chrono::duration_cast<std::chrono::system_clock::duration>(
                        std::chrono::duration<double>(timeout_s));
    ok = I.done_cv.wait_until(lk, deadline, pred);
  }
  if (!I.error.empty()) throw std::runtime_error("FleetExecutor: " + I.error);
  return ok;
}

std::vector<std::array<int64_t, 3>> FleetCarrier::trace() {
  std::lock_guard<std::mutex> lk(impl_->trace_mu);
  return impl_->trace;
}

void FleetCarrier::clear_trace() {
  std::lock_guard<std::mutex> lk(impl_->trace_mu);
  impl_->trace.clear();
}

void FleetCarrier::shutdown() {
  if (!impl_) return;
  Impl& I = *impl_;
  I.running = false;
  for (auto& L : I.loops) {
    L->cv.notify_all();
    if (L->th.joinable()) L->th.join();
  }
  if (I.bus_up.exchange(false)) {
    ::shutdown(I.listen_fd, SHUT_RDWR);
    ::close(I.listen_fd);
    if (I.acceptor.joinable()) I.acceptor.join();
  }
  {
    std::lock_guard<std::mutex> lk(I.out_mu);
    for (auto& kv : I.out_fd) ::close(kv.second);
    I.out_fd.clear();
    for (int fd : I.reader_fds) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : I.readers)
    if (t.joinable()) t.join();
  I.readers.clear();
  for (int fd : I.reader_fds) ::close(fd);
  I.reader_fds.clear();
}

}  // namespace pdrt
