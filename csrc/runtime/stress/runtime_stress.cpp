// Concurrency stress driver for the host runtime (tcp_store.cpp, watchdog.cpp, tracer.cpp,
// fleet_executor.cpp), built with
// -fsanitize=thread (data races) or -fsanitize=address,undefined (memory errors / UB) by
// paddle2_amd/_build.py build_sanitized(); tests/test_sanitizers.py runs both.  Reference role: SURVEY §5.2
// (race detection / sanitizer builds of the native runtime).  CPU only: watchdog entries carry no HIP event,
// so their completion is driven by watchdog_end from the worker threads.
#include <atomic>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../runtime.h"

using namespace pdrt;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main() {
  constexpr int kThreads = 8, kIters = 200;
  TCPStoreServer server("127.0.0.1", 0);
  const int port = server.port();
  std::atomic<int> errors{0};

  // ---- store: concurrent add / set / get / compare_set from independent clients
  std::vector<std::thread> ts;
  for (int t = 0; t < kThreads; ++t) {
    ts.emplace_back([&, t] {
      TCPStoreClient c("127.0.0.1", port, 30.0);
      for (int i = 0; i < kIters; ++i) {
        c.add("counter", 1);
        const std::string k = "k" + std::to_string(t) + "_" + std::to_string(i);
        c.set(k, std::to_string(i));
        if (c.get(k) != std::to_string(i)) errors++;
        c.compare_set("cas", "", "t" + std::to_string(t));
      }
      c.wait({"k0_" + std::to_string(kIters - 1)});
    });
  }
  // ---- tracer: concurrent push / pop / instant while another thread snapshots
  tracer_enable(true);
  std::atomic<bool> stop{false};
  std::thread snap([&] {
    while (!stop.load()) (void)tracer_events().size();
  });
  for (int t = 0; t < kThreads; ++t) {
    ts.emplace_back([&, t] {
      for (int i = 0; i < kIters; ++i) {
        tracer_push("range" + std::to_string(t), 0);
        tracer_instant("inst", 1, tracer_now_ns(), tracer_now_ns());
        tracer_pop();
      }
    });
  }
  // ---- watchdog: begin / end from many threads while the poller runs
  watchdog_start(0.001, false);
  for (int t = 0; t < kThreads; ++t) {
    ts.emplace_back([&] {
      for (int i = 0; i < kIters; ++i) {
        const int64_t id = watchdog_begin("allreduce", 60.0);
        watchdog_end(id);
      }
    });
  }
  for (auto& th : ts) th.join();
  stop = true;
  snap.join();
  (void)watchdog_take_finished();
  watchdog_stop();
  tracer_enable(false);

  // ---- FleetExecutor: a 3-stage pipeline split over two carriers (message bus over TCP), 4 loop threads
  // each, 200 micro-steps; every stage must see every step exactly once and in order
  {
    constexpr int64_t kSteps = 200;
    FleetCarrier c0(0, 4), c1(1, 4);
    std::vector<FleetTask> tasks(5);
    int64_t ids[5] = {1, 2, 3, 4, 5};
    int ranks[5] = {0, 0, 1, 1, 1};
    int roles[5] = {FleetTask::kSource, FleetTask::kCompute, FleetTask::kCompute, FleetTask::kCompute,
                    FleetTask::kSink};
    for (int i = 0; i < 5; ++i) {
      tasks[i].id = ids[i];
      tasks[i].rank = ranks[i];
      tasks[i].role = roles[i];
      tasks[i].max_run_times = kSteps;
      if (i > 0) tasks[i].upstream = {{ids[i - 1], 2}};
      if (i < 4) tasks[i].downstream = {{ids[i + 1], 2}};
    }
    std::atomic<int64_t> next[6];
    for (auto& n : next) n = 0;
    std::atomic<int> order_errors{0};
    auto fn = [&](int64_t task, int64_t step) {
      if (next[task].fetch_add(1) != step) order_errors++;
    };
    for (auto& t : tasks) {
      c0.add_task(t);
      c1.add_task(t);
    }
    c0.set_compute(fn);
    c1.set_compute(fn);
    int p0 = c0.listen("127.0.0.1"), p1 = c1.listen("127.0.0.1");
    c0.set_peer(1, "127.0.0.1", p1);
    c1.set_peer(0, "127.0.0.1", p0);
    c1.start();
    c0.start();
    if (!c0.wait(60.0) || !c1.wait(60.0)) return fail("fleet executor timed out");
    if (order_errors.load()) return fail("fleet executor step order");
    for (int t = 2; t <= 4; ++t)
      if (next[t].load() != kSteps) return fail("fleet executor lost steps");
    if (c0.trace().size() + c1.trace().size() != 3 * kSteps) return fail("fleet executor trace");
    c0.shutdown();
    c1.shutdown();
  }

  TCPStoreClient c("127.0.0.1", port, 30.0);
  if (c.add("counter", 0) != kThreads * kIters) return fail("store counter");
  if (errors.load()) return fail("store get/set mismatch");
  if (watchdog_inflight() != 0) return fail("watchdog leaked entries");
  if (tracer_events().size() < (size_t)kThreads * kIters * 2) return fail("tracer lost events");
  server.shutdown();
  std::printf("runtime_stress OK\n");
  return 0;
}
