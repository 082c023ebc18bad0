// Concurrency stress driver for the host runtime (tcp_store.cpp, watchdog.cpp, tracer.cpp), built with
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

  TCPStoreClient c("127.0.0.1", port, 30.0);
  if (c.add("counter", 0) != kThreads * kIters) return fail("store counter");
  if (errors.load()) return fail("store get/set mismatch");
  if (watchdog_inflight() != 0) return fail("watchdog leaked entries");
  if (tracer_events().size() < (size_t)kThreads * kIters * 2) return fail("tracer lost events");
  server.shutdown();
  std::printf("runtime_stress OK\n");
  return 0;
}
