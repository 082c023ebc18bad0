// CPU multi-rank test of the ProcessGroupRCCL core (csrc/comm/rccl_core.h) against the threaded fake RCCL / HIP
// (csrc/comm/test/fake/): 4 ranks = 4 threads, each with its own RcclGroup, calc stream and buffers, run every
// operation the torch process group issues and check each rank's result against the closed form:
//   all-reduce sum / avg / premul / max / min / prod (f32, f64, bf16, f16, i32; in place and out of place),
//   reduce-scatter (sum, avg), all-gather, broadcast, reduce, all-to-all, all-to-all-v, send / recv on the
//   lo->hi pair communicators (the `1 - c->rank` mapping), coalesced p2p over several pair communicators in one
//   group, use_calc_stream, calc -> comm and comm -> calc fences against work that is still queued on the calc
//   stream, barrier, and a collective that only one rank issues (timeout -> abort -> error on that rank, async
//   error on the others).  Built by paddle2_amd._build.build_rccl_stress under TSan and ASan+UBSan
//   (tests/test_rccl_group_cpu.py).  Exit code 0 = every check passed.
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../rccl_core.h"

using pdrccl::RcclGroup;
using pdrccl::TaskPtr;

namespace {

constexpr int kRanks = 4;
std::atomic<int> g_fail{0};
std::atomic<int> g_phase[kRanks];   // progress marker per rank (printed by the watchdog on a hang)
#define PHASE(n) g_phase[rank] = (n)

#define CHECK(cond, ...)                                           \
  do {                                                             \
    if (!(cond)) {                                                 \
      std::fprintf(stderr, "[rank %d] CHECK failed %s:%d: ", rank, __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                           \
      std::fprintf(stderr, "\n");                                  \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

class MemStore : public pdrccl::Store {
 public:
  void set(const std::string& k, const std::string& v) override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      kv_[k] = v;
    }
    cv_.notify_all();
  }
  std::string get(const std::string& k) override {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return kv_.count(k) > 0; });
    return kv_[k];
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
};

// dtype codes of rccl_core.h
enum { F32 = 0, F16 = 1, BF16 = 2, F64 = 3, I32 = 4 };
enum { SUM = 0, PROD = 1, MAX = 2, MIN = 3, AVG = 4, PREMUL = 5 };

uintptr_t P(const void* p) { return (uintptr_t)p; }

// the host waits for a task (Task::synchronize), then the calc stream is drained so host reads see the data
void done(const TaskPtr& t, hipStream_t calc) {
  if (t) t->synchronize();
  hipStreamSynchronize(calc);
}

void run_rank(int rank, std::shared_ptr<pdrccl::Store> store) {
  hipStream_t calc;
  hipStreamCreate(&calc);
  const uintptr_t cs = P(calc);
  {
    RcclGroup g(store, "t", rank, kRanks, 0, 20000);
    const int n = 1000;

    PHASE(1);
    // ---- all-reduce, every op, f32, out of place and in place; repeated so events / slots get reused
    for (int it = 0; it < 6; ++it) {
      std::vector<float> in(n), out(n, -1.f);
      for (int i = 0; i < n; ++i) in[i] = (float)(rank + 1) * (i % 7 + 1) + it;
      const int ops[] = {SUM, AVG, MAX, MIN, PREMUL, PROD};
      const int op = ops[it];
      done(g.all_reduce(P(in.data()), P(out.data()), n, F32, op, 0.5, cs, false), calc);
      for (int i = 0; i < n; i += 37) {
        double exp = 0, mx = -1e30, mn = 1e30, pr = 1;
        for (int r = 0; r < kRanks; ++r) {
          const double v = (double)(r + 1) * (i % 7 + 1) + it;
          exp += v;
          mx = std::max(mx, v);
          mn = std::min(mn, v);
          pr *= v;
        }
        const double want = op == SUM ? exp : op == AVG ? exp / kRanks : op == MAX ? mx : op == MIN ? mn
                          : op == PREMUL ? 0.5 * exp : pr;
        CHECK(std::fabs(out[i] - want) <= 1e-5 * std::fabs(want) + 1e-5, "all_reduce op %d i %d: %f vs %f", op, i,
              out[i], want);
      }
      // in place
      done(g.all_reduce(P(in.data()), P(in.data()), n, F32, SUM, 0.0, cs, false), calc);
      double s0 = 0;
      for (int r = 0; r < kRanks; ++r) s0 += (double)(r + 1) * 1 + it;
      CHECK(std::fabs(in[0] - s0) < 1e-4, "in-place all_reduce: %f vs %f", in[0], s0);
    }
    PHASE(2);
    // ---- other dtypes
    {
      std::vector<double> d(64, rank + 0.25);
      done(g.all_reduce(P(d.data()), P(d.data()), 64, F64, SUM, 0.0, cs, false), calc);
      CHECK(d[63] == 0 + 1 + 2 + 3 + 4 * 0.25, "f64 sum %f", d[63]);
      std::vector<int32_t> iv(64, rank * 3);
      done(g.all_reduce(P(iv.data()), P(iv.data()), 64, I32, MAX, 0.0, cs, false), calc);
      CHECK(iv[5] == 9, "i32 max %d", iv[5]);
      std::vector<uint16_t> bf(64, fakenccl::f_to_bf16(1.0f + rank)), hf(64, fakenccl::f_to_h(0.5f * (rank + 1)));
      done(g.all_reduce(P(bf.data()), P(bf.data()), 64, BF16, SUM, 0.0, cs, false), calc);
      CHECK(fakenccl::bf16_to_f(bf[7]) == 10.f, "bf16 sum %f", fakenccl::bf16_to_f(bf[7]));
      done(g.all_reduce(P(hf.data()), P(hf.data()), 64, F16, AVG, 0.0, cs, false), calc);
      CHECK(fakenccl::h_to_f(hf[3]) == 1.25f, "f16 avg %f", fakenccl::h_to_f(hf[3]));
      std::vector<uint16_t> bp(64, fakenccl::f_to_bf16(2.0f));
      done(g.all_reduce(P(bp.data()), P(bp.data()), 64, BF16, PREMUL, 0.25, cs, false), calc);
      CHECK(fakenccl::bf16_to_f(bp[0]) == 2.0f, "bf16 premul %f", fakenccl::bf16_to_f(bp[0]));
    }
    PHASE(3);
    // ---- reduce-scatter (sum, avg) and all-gather
    {
      const int c = 16;
      std::vector<float> in(c * kRanks), out(c);
      for (int i = 0; i < c * kRanks; ++i) in[i] = (float)(i + 100 * rank);
      done(g.reduce_scatter(P(in.data()), P(out.data()), c, F32, SUM, 0.0, cs, false), calc);
      for (int i = 0; i < c; ++i) {
        const float want = kRanks * (float)(rank * c + i) + 100.f * (0 + 1 + 2 + 3);
        CHECK(out[i] == want, "reduce_scatter %d: %f vs %f", i, out[i], want);
      }
      done(g.reduce_scatter(P(in.data()), P(out.data()), c, F32, AVG, 0.0, cs, false), calc);
      CHECK(out[0] == (float)(rank * c) + 150.f, "reduce_scatter avg %f", out[0]);
      std::vector<float> mine(c, (float)rank), all(c * kRanks, -1.f);
      done(g.all_gather(P(mine.data()), P(all.data()), c, F32, cs, false), calc);
      for (int r = 0; r < kRanks; ++r) CHECK(all[r * c + 3] == (float)r, "all_gather block %d", r);
    }
    PHASE(4);
    // ---- broadcast (root 2) and reduce (root 1)
    {
      std::vector<float> b(32, (float)rank * 10.f), o(32, -1.f);
      done(g.broadcast(P(b.data()), P(o.data()), 32, F32, 2, cs, false), calc);
      CHECK(o[31] == 20.f, "broadcast %f", o[31]);
      std::vector<float> ro(32, -7.f);
      done(g.reduce(P(b.data()), P(ro.data()), 32, F32, SUM, 0.0, 1, cs, false), calc);
      if (rank == 1) CHECK(ro[0] == 60.f, "reduce root %f", ro[0]);
      else CHECK(ro[0] == -7.f, "reduce non-root touched %f", ro[0]);
    }
    PHASE(5);
    // ---- all-to-all (equal) and all-to-all-v
    {
      const int c = 8;
      std::vector<float> in(c * kRanks), out(c * kRanks);
      for (int j = 0; j < kRanks; ++j)
        for (int i = 0; i < c; ++i) in[j * c + i] = (float)(rank * 100 + j * 10 + i);
      done(g.all_to_all(P(in.data()), P(out.data()), c, F32, cs, false), calc);
      for (int j = 0; j < kRanks; ++j) CHECK(out[j * c + 2] == (float)(j * 100 + rank * 10 + 2), "all_to_all %d", j);
      // rank r sends (r + j + 1) elements to rank j, all of value 1000 r + j
      std::vector<size_t> sc(kRanks), sd(kRanks), rc(kRanks), rd(kRanks);
      size_t so = 0, ro = 0;
      for (int j = 0; j < kRanks; ++j) {
        sc[j] = rank + j + 1;
        sd[j] = so;
        so += sc[j];
        rc[j] = j + rank + 1;
        rd[j] = ro;
        ro += rc[j];
      }
      std::vector<float> vin(so), vout(ro, -1.f);
      for (int j = 0; j < kRanks; ++j)
        for (size_t i = 0; i < sc[j]; ++i) vin[sd[j] + i] = (float)(1000 * rank + j);
      done(g.all_to_all_v(P(vin.data()), P(vout.data()), sc, sd, rc, rd, F32, cs, false), calc);
      for (int j = 0; j < kRanks; ++j)
        for (size_t i = 0; i < rc[j]; ++i)
          CHECK(vout[rd[j] + i] == (float)(1000 * j + rank), "all_to_all_v from %d elem %zu: %f", j, i,
                vout[rd[j] + i]);
    }
    PHASE(6);
    // ---- p2p on pair communicators: even ranks send to the odd neighbour first, then a coalesced ring
    {
      std::vector<float> s(50, (float)rank + 0.5f), r(50, -1.f);
      const int peer = rank ^ 1;   // pairs (0,1), (2,3): lo sends, hi receives, then back
      if (rank < peer) {
        done(g.send(P(s.data()), 50, F32, peer, cs, false), calc);
        done(g.recv(P(r.data()), 50, F32, peer, cs, false), calc);
      } else {
        done(g.recv(P(r.data()), 50, F32, peer, cs, false), calc);
        done(g.send(P(s.data()), 50, F32, peer, cs, false), calc);
      }
      CHECK(r[49] == (float)peer + 0.5f, "pair p2p %f", r[49]);
      CHECK(g.num_comms() >= 2, "a pair communicator was created");
      // ring: send right, receive left; every pair communicator must exist before a group (issue one op each)
      const int right = (rank + 1) % kRanks, left = (rank + kRanks - 1) % kRanks;
      for (int it = 0; it < 3; ++it) {
        std::vector<float> a(40, (float)(rank * 7 + it)), b(40, -1.f);
        if (it == 0) {   // create the (rank, right) / (left, rank) communicators outside a group
          if (rank % 2 == 0) {
            done(g.send(P(a.data()), 40, F32, right, cs, false), calc);
            done(g.recv(P(b.data()), 40, F32, left, cs, false), calc);
          } else {
            done(g.recv(P(b.data()), 40, F32, left, cs, false), calc);
            done(g.send(P(a.data()), 40, F32, right, cs, false), calc);
          }
        } else {
          g.group_start(cs);
          g.recv(P(b.data()), 40, F32, left, cs, false);   // recv queued before send on this rank's streams
          g.send(P(a.data()), 40, F32, right, cs, false);
          TaskPtr t = g.group_end();
          CHECK(t != nullptr, "group_end returns one task");
          done(t, calc);
        }
        CHECK(b[39] == (float)(left * 7 + it), "ring it %d: %f", it, b[39]);
      }
    }
    PHASE(7);
    // ---- use_calc_stream: enqueued on the caller's stream, no task
    {
      std::vector<float> v(10, 1.f);
      TaskPtr t = g.all_reduce(P(v.data()), P(v.data()), 10, F32, SUM, 0.0, cs, true);
      CHECK(t == nullptr, "use_calc returns no task");
      hipStreamSynchronize(calc);
      CHECK(v[9] == 4.f, "use_calc all_reduce %f", v[9]);
    }
    PHASE(8);
    // ---- fences: the input is produced by calc-stream work still queued when the collective is issued, and the
    // output is consumed by calc-stream work ordered only by Task::wait (no host block in between)
    for (int it = 0; it < 20; ++it) {
      std::vector<float> buf(256, -100.f), seen(1, 0.f);
      float* bp = buf.data();
      float* sp = seen.data();
      const int rr = rank;
      calc->push([bp, rr, it] {
        std::this_thread::sleep_for(std::chrono::microseconds(50 * ((rr + it) % 3)));
        for (int i = 0; i < 256; ++i) bp[i] = (float)(rr + it);
      });
      TaskPtr t = g.all_reduce(P(bp), P(bp), 256, F32, SUM, 0.0, cs, false);
      t->wait(cs);
      calc->push([bp, sp] { sp[0] = bp[255]; });
      hipStreamSynchronize(calc);
      const float want = (float)(0 + 1 + 2 + 3 + 4 * it);
      CHECK(seen[0] == want, "fenced all_reduce it %d: saw %f want %f", it, seen[0], want);
      done(t, calc);   // the task's end event has completed; its destructor returns the event to the pool
    }
    PHASE(9);
    // ---- barrier
    {
      std::vector<int32_t> scratch(1, 0);
      g.barrier(P(scratch.data()), cs);
    }
    hipStreamSynchronize(calc);
  }

  PHASE(10);
  // ---- a collective only rank 0 issues: its synchronize times out and aborts; the others see the abort as an
  // asynchronous error on their next query of the same communicator
  {
    RcclGroup h(store, "timeout", rank, kRanks, 0, 300);
    std::vector<float> v(8, 1.f);
    done(h.all_reduce(P(v.data()), P(v.data()), 8, F32, SUM, 0.0, cs, false), calc);   // creates the comm
    if (rank == 0) {
      TaskPtr t = h.all_reduce(P(v.data()), P(v.data()), 8, F32, SUM, 0.0, cs, false);
      bool threw = false;
      try {
        t->synchronize();
      } catch (const std::exception& e) {
        threw = std::string(e.what()).find("timed out") != std::string::npos;
      }
      CHECK(threw, "rank 0 collective timed out and aborted");
    } else {
      std::this_thread::sleep_for(std::chrono::milliseconds(900));   // rank 0 aborts meanwhile
      TaskPtr t = h.all_reduce(P(v.data()), P(v.data()), 8, F32, SUM, 0.0, cs, false);
      bool threw = false;
      try {
        t->synchronize();
      } catch (const std::exception& e) {
        threw = true;
      }
      CHECK(threw, "peers see the aborted communicator");
    }
    hipDeviceSynchronize();
  }
  hipStreamDestroy(calc);
}

}  // namespace

int main() {
  auto store = std::make_shared<MemStore>();
  std::vector<std::thread> ts;
  std::atomic<bool> finished{false};
  std::thread dog([&] {   // a hang prints every rank's phase and fails the run instead of blocking the suite
    for (int i = 0; i < 1200 && !finished; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    if (finished) return;
    for (int r = 0; r < kRanks; ++r) std::fprintf(stderr, "HANG: rank %d in phase %d\n", r, g_phase[r].load());
    std::fflush(stderr);
    std::_Exit(3);
  });
  for (int r = 0; r < kRanks; ++r) ts.emplace_back(run_rank, r, store);
  for (auto& t : ts) t.join();
  finished = true;
  dog.join();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail.load());
    return 1;
  }
  std::printf("rccl_stress: all checks passed (%d ranks)\n", kRanks);
  return 0;
}
