// Multi-threaded stress driver for the native allocator's bookkeeping (built against the fake HIP header in
// fake_hip/, run under ASan+UBSan and TSan by tests/test_native_allocator.py).  Each thread owns a "stream",
// allocates log-uniform sizes, fills every allocation with its own tag, verifies the tag before freeing
// (overlapping live blocks would corrupt it), and hands some blocks to other threads' streams so the
// cross-stream fence path runs.  Exits non-zero on any corruption or accounting mismatch.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

typedef struct FakeStream* hipStream_t;
extern "C" {
void* pd_alloc_malloc(size_t size, int device, hipStream_t stream);
void pd_alloc_free(void* ptr, size_t size, int device, hipStream_t stream);
void pd_alloc_record_stream(void* ptr, hipStream_t stream);
void pd_alloc_configure(uint64_t chunk_bytes, uint64_t limit_bytes);
void pd_alloc_set_headroom(uint64_t bytes);
void pd_alloc_stats(int device, uint64_t* out);
uint64_t pd_alloc_empty_cache(int device);
}

struct Live {
  unsigned char* p;
  size_t n;
  unsigned char tag;
  hipStream_t s;
};

static std::mutex g_handoff_mu;
static std::vector<Live> g_handoff;
static std::atomic<int> g_errors{0};

static bool check(const Live& l) {
  for (size_t i = 0; i < l.n; i += 97) {
    if (l.p[i] != l.tag) return false;
  }
  return l.p[l.n - 1] == l.tag;
}

static void worker(int tid, int iters) {
  std::mt19937_64 rng(1234 + tid);
  hipStream_t stream = reinterpret_cast<hipStream_t>(uintptr_t(0x1000 + tid * 0x10));
  std::vector<Live> live;
  std::uniform_real_distribution<double> logsz(0.0, 20.0);  // 1 B .. 1 MiB
  for (int it = 0; it < iters; ++it) {
    int op = int(rng() % 10);
    if (op < 5 || live.empty()) {
      size_t n = size_t(std::pow(2.0, logsz(rng))) + 1;
      auto* p = static_cast<unsigned char*>(pd_alloc_malloc(n, 0, stream));
      if (!p) { g_errors++; std::fprintf(stderr, "alloc failed\n"); return; }
      if (reinterpret_cast<uintptr_t>(p) % 256 != 0) { g_errors++; std::fprintf(stderr, "misaligned\n"); }
      unsigned char tag = static_cast<unsigned char>(1 + rng() % 250);
      std::memset(p, tag, n);
      if (rng() % 8 == 0)  // also "used" on another thread's stream: its free is deferred behind that stream
        pd_alloc_record_stream(p, reinterpret_cast<hipStream_t>(uintptr_t(0x1000 + ((tid + 1) % 4) * 0x10)));
      live.push_back({p, n, tag, stream});
    } else if (op < 9) {
      size_t k = rng() % live.size();
      Live l = live[k];
      live[k] = live.back();
      live.pop_back();
      if (!check(l)) { g_errors++; std::fprintf(stderr, "corruption tid %d\n", tid); }
      pd_alloc_free(l.p, l.n, 0, l.s);
    } else {
      // hand a block to another thread: it is freed on the allocating stream by whoever pops it
      size_t k = rng() % live.size();
      std::lock_guard<std::mutex> lk(g_handoff_mu);
      g_handoff.push_back(live[k]);
      live[k] = live.back();
      live.pop_back();
      if (g_handoff.size() > 8) {
        Live l = g_handoff.front();
        g_handoff.erase(g_handoff.begin());
        if (!check(l)) { g_errors++; std::fprintf(stderr, "corruption (handoff)\n"); }
        pd_alloc_free(l.p, l.n, 0, l.s);
      }
    }
  }
  for (auto& l : live) {
    if (!check(l)) { g_errors++; std::fprintf(stderr, "corruption at exit\n"); }
    pd_alloc_free(l.p, l.n, 0, l.s);
  }
}

#include <cmath>

int main(int argc, char** argv) {
  int threads = argc > 1 ? std::atoi(argv[1]) : 4;
  int iters = argc > 2 ? std::atoi(argv[2]) : 20000;
  pd_alloc_configure(uint64_t(8) << 20, 0);
  // headroom: the fake device holds 4 GiB; with 3 GiB kept free a 512 MiB request fits, a second 768 MiB one
  // (which would leave < 3 GiB) must be refused instead of eating the runtime's share
  {
    pd_alloc_set_headroom(uint64_t(3) << 30);
    hipStream_t s0 = reinterpret_cast<hipStream_t>(uintptr_t(0x999));
    void* a = pd_alloc_malloc(size_t(512) << 20, 0, s0);
    void* b = a ? pd_alloc_malloc(size_t(768) << 20, 0, s0) : nullptr;
    if (!a || b) {
      std::fprintf(stderr, "headroom: a=%p b=%p (want a != null, b == null)\n", a, b);
      g_errors++;
    }
    if (a) pd_alloc_free(a, size_t(512) << 20, 0, s0);
    if (b) pd_alloc_free(b, size_t(768) << 20, 0, s0);
    pd_alloc_empty_cache(0);
    pd_alloc_set_headroom(uint64_t(64) << 20);
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(worker, t, iters);
  for (auto& t : ts) t.join();
  for (auto& l : g_handoff) {
    if (!check(l)) g_errors++;
    pd_alloc_free(l.p, l.n, 0, l.s);
  }
  uint64_t st[13];
  pd_alloc_stats(0, st);
  if (st[0] != 0) { std::fprintf(stderr, "leaked %llu bytes\n", (unsigned long long)st[0]); g_errors++; }
  if (st[4] != st[5]) { std::fprintf(stderr, "allocs %llu != frees %llu\n", (unsigned long long)st[4],
                                     (unsigned long long)st[5]); g_errors++; }
  uint64_t released = pd_alloc_empty_cache(0);
  pd_alloc_stats(0, st);
  if (st[1] != 0 || released == 0) { std::fprintf(stderr, "empty_cache left %llu reserved\n",
                                                  (unsigned long long)st[1]); g_errors++; }
  std::printf("allocs=%llu chunks_peak_reserved=%llu cross_stream_reuse=%llu record_stream=%llu deferred=%llu errors=%d\n",
              (unsigned long long)st[4], (unsigned long long)st[3], (unsigned long long)st[9],
              (unsigned long long)st[10], (unsigned long long)st[11], g_errors.load());
  return g_errors.load() ? 1 : 0;
}
