// Host-only stand-in for the RCCL API subset csrc/comm/rccl_core.h uses, for the CPU stress test
// (csrc/comm/test/rccl_stress.cpp): ranks are threads of one process, communicators rendezvous through an
// in-process registry keyed by the unique id, and every collective runs on the caller's fake stream (a worker
// thread, fake/hip/hip_runtime.h) the way RCCL kernels run on a HIP stream:
//  * collectives: each rank posts its buffers under the communicator's next sequence number, waits for all
//    ranks, computes ITS OWN output from every rank's input into a private buffer, waits again (so no rank
//    overwrites an input — in-place ops — while a peer still reads it), then writes its output;
//  * send: copies the bytes into the (src -> dst) mailbox of the communicator and returns; recv: blocks until
//    the next message from src is there, checks its size;
//  * ncclGroupStart / End: operations issued inside a group are held per thread and handed to their streams at
//    ncclGroupEnd, sends first (a same-stream recv-before-send pair of two ranks would otherwise deadlock, which
//    real RCCL avoids by launching a group as one fused kernel);
//  * ncclCommAbort marks the communicator's world aborted: every rank blocked in it gives up and reports
//    ncclRemoteError through ncclCommGetAsyncError (the timeout / abort path of Task::synchronize).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <cstdlib>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7
} ncclResult_t;
typedef enum {
  ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
  ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9, ncclFloat8e4m3 = 10, ncclFloat8e5m2 = 11
} ncclDataType_t;
typedef int ncclRedOp_t;
enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3, ncclAvg = 4 };
typedef enum { ncclScalarDevice = 0, ncclScalarHostImmediate = 1 } ncclScalarResidence_t;
typedef struct {
  char internal[128];
} ncclUniqueId;

namespace fakenccl {

struct Slot {   // one collective call, all ranks
  std::vector<const void*> in;
  int arrived = 0, computed = 0, left = 0;
};

struct World {
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int joined = 0;
  bool aborted = false;
  std::map<uint64_t, Slot> slots;
  std::map<std::pair<int, int>, std::deque<std::vector<char>>> mail;   // (src, dst) -> messages
  explicit World(int n_) : n(n_) {}
};

inline std::mutex& reg_mu() {
  static std::mutex m;
  return m;
}
inline std::map<std::string, std::shared_ptr<World>>& registry() {
  static std::map<std::string, std::shared_ptr<World>> r;
  return r;
}
inline std::atomic<uint64_t>& id_counter() {
  static std::atomic<uint64_t> c{0};
  return c;
}

inline size_t esize(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}
inline float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
inline float h_to_f(uint16_t h) {
  const uint32_t s = (h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {   // subnormal
      int ee = -1;
      uint32_t mm = m;
      do { ++ee; mm <<= 1; } while (!(mm & 0x400));
      u = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e - 15 + 127) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_h(float f) {   // round to nearest even, no NaN payloads needed here
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const int exp = (int)((x >> 23) & 0xff) - 127 + 15;
  uint32_t man = x & 0x7fffffu;
  if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return (uint16_t)sign;
    man |= 0x800000u;
    const int shift = 14 - exp;
    uint32_t h = man >> shift;
    const uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)exp << 10) | (man >> 13);
  const uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
  return (uint16_t)(sign | h);
}

// element i of a typed buffer as double, and back
inline double load(const void* p, size_t i, ncclDataType_t t) {
  switch (t) {
    case ncclInt8: return ((const int8_t*)p)[i];
    case ncclUint8: return ((const uint8_t*)p)[i];
    case ncclInt32: return ((const int32_t*)p)[i];
    case ncclUint32: return ((const uint32_t*)p)[i];
    case ncclInt64: return (double)((const int64_t*)p)[i];
    case ncclUint64: return (double)((const uint64_t*)p)[i];
    case ncclFloat16: return h_to_f(((const uint16_t*)p)[i]);
    case ncclBfloat16: return bf16_to_f(((const uint16_t*)p)[i]);
    case ncclFloat32: return ((const float*)p)[i];
    default: return ((const double*)p)[i];
  }
}
inline void store(void* p, size_t i, ncclDataType_t t, double v) {
  switch (t) {
    case ncclInt8: ((int8_t*)p)[i] = (int8_t)v; break;
    case ncclUint8: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case ncclInt32: ((int32_t*)p)[i] = (int32_t)v; break;
    case ncclUint32: ((uint32_t*)p)[i] = (uint32_t)v; break;
    case ncclInt64: ((int64_t*)p)[i] = (int64_t)v; break;
    case ncclUint64: ((uint64_t*)p)[i] = (uint64_t)v; break;
    case ncclFloat16: ((uint16_t*)p)[i] = f_to_h((float)v); break;
    case ncclBfloat16: ((uint16_t*)p)[i] = f_to_bf16((float)v); break;
    case ncclFloat32: ((float*)p)[i] = (float)v; break;
    default: ((double*)p)[i] = v; break;
  }
}

}  // namespace fakenccl

struct ncclComm {
  std::atomic<int> refs{1};                       // the handle + every queued operation on it
  std::shared_ptr<fakenccl::World> w;
  int rank = 0;
  uint64_t seq = 0;                               // collectives issued (stream order == issue order here)
  std::atomic<int> async_err{ncclSuccess};
  std::mutex op_mu;
  std::map<int, double> premul;                   // PreMulSum ops: id -> scalar
  int next_op = 100;
};
typedef ncclComm* ncclComm_t;

namespace fakenccl {

// live communicator handles: using one after ncclCommDestroy / ncclCommAbort (both free it, as in RCCL) is a
// fatal error here, so a double abort or a query of an aborted communicator fails the test deterministically
inline std::mutex& live_mu() {
  static std::mutex m;
  return m;
}
inline std::set<ncclComm*>& live() {
  static std::set<ncclComm*> s;
  return s;
}
inline void require_live(ncclComm* c, const char* fn) {
  std::lock_guard<std::mutex> lk(live_mu());
  if (!live().count(c)) {
    std::fprintf(stderr, "fake rccl: %s on a destroyed / aborted communicator %p\n", fn, (void*)c);
    std::abort();
  }
}
inline void unref(ncclComm* c) {
  if (--c->refs == 0) delete c;
}
inline ncclComm* ref(ncclComm* c) {
  ++c->refs;
  return c;
}

struct Pending {
  hipStream_t s;
  bool is_send;
  std::function<void()> f;
};
inline thread_local int group_depth = 0;
inline thread_local std::vector<Pending> group_ops;

inline void submit(hipStream_t s, bool is_send, std::function<void()> f) {
  if (group_depth > 0) {
    group_ops.push_back({s, is_send, std::move(f)});
  } else {
    s->push(std::move(f));
  }
}

// rendezvous of collective `seq` on world w: post `in`, run `compute(inputs)` once everyone posted (returns the
// bytes of this rank's output), barrier, `write(bytes)`.  Gives up (async error) if the world is aborted.
inline void collective(ncclComm* c, uint64_t seq, const void* in,
                       const std::function<std::vector<char>(const std::vector<const void*>&)>& compute,
                       const std::function<void(const std::vector<char>&)>& write) {
  World& w = *c->w;
  std::unique_lock<std::mutex> lk(w.mu);
  Slot& sl = w.slots[seq];
  if (sl.in.empty()) sl.in.assign(w.n, nullptr);
  sl.in[c->rank] = in;
  ++sl.arrived;
  w.cv.notify_all();
  w.cv.wait(lk, [&] { return w.aborted || sl.arrived == w.n; });
  if (w.aborted) {
    c->async_err = ncclRemoteError;
    return;
  }
  const std::vector<const void*> ins = sl.in;
  lk.unlock();
  std::vector<char> out = compute(ins);
  lk.lock();
  ++sl.computed;
  w.cv.notify_all();
  w.cv.wait(lk, [&] { return w.aborted || sl.computed == w.n; });
  if (w.aborted) {
    c->async_err = ncclRemoteError;
    return;
  }
  if (++sl.left == w.n) w.slots.erase(seq);
  lk.unlock();
  write(out);
}

inline double reduce2(double a, double b, int op) {
  switch (op) {
    case ncclProd: return a * b;
    case ncclMax: return a > b ? a : b;
    case ncclMin: return a < b ? a : b;
    default: return a + b;   // sum, avg (divided later), premul (pre-scaled)
  }
}

// reduce element range [off, off + count) of every rank's input into a typed byte buffer
inline std::vector<char> reduce_block(ncclComm* c, const std::vector<const void*>& ins, size_t off, size_t count,
                                      ncclDataType_t t, int op) {
  const size_t es = esize(t);
  std::vector<char> out(count * es);
  double scale = 1.0;
  int rop = op;
  if (op >= 100) {
    std::lock_guard<std::mutex> lk(c->op_mu);
    scale = c->premul.at(op);
    rop = ncclSum;
  }
  const int n = (int)ins.size();
  for (size_t i = 0; i < count; ++i) {
    double acc = scale * load(ins[0], off + i, t);
    for (int r = 1; r < n; ++r) acc = reduce2(acc, scale * load(ins[r], off + i, t), rop);
    if (rop == ncclAvg) acc /= n;
    store(out.data(), i, t, acc);
  }
  return out;
}

}  // namespace fakenccl

inline const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInvalidArgument: return "invalid argument";
    case ncclInvalidUsage: return "invalid usage";
    default: return "fake rccl error";
  }
}
inline ncclResult_t ncclGetVersion(int* v) {
  *v = 99999;
  return ncclSuccess;
}
inline ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id, 0, sizeof(*id));
  std::snprintf(id->internal, sizeof(id->internal), "fake-%llu",
                (unsigned long long)fakenccl::id_counter().fetch_add(1));
  return ncclSuccess;
}
// blocks until all nranks joined (as the real one does)
inline ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  std::shared_ptr<fakenccl::World> w;
  {
    std::lock_guard<std::mutex> lk(fakenccl::reg_mu());
    auto& slot = fakenccl::registry()[std::string(id.internal)];
    if (!slot) slot = std::make_shared<fakenccl::World>(nranks);
    w = slot;
  }
  if (w->n != nranks) return ncclInvalidUsage;
  auto* c = new ncclComm();
  c->w = w;
  c->rank = rank;
  std::unique_lock<std::mutex> lk(w->mu);
  ++w->joined;
  w->cv.notify_all();
  w->cv.wait(lk, [&] { return w->joined >= w->n; });
  *comm = c;
  std::lock_guard<std::mutex> lk2(fakenccl::live_mu());
  fakenccl::live().insert(c);
  return ncclSuccess;
}
inline ncclResult_t ncclCommDestroy(ncclComm_t c) {
  fakenccl::require_live(c, "ncclCommDestroy");
  {
    std::lock_guard<std::mutex> lk(fakenccl::live_mu());
    fakenccl::live().erase(c);
  }
  fakenccl::unref(c);
  return ncclSuccess;
}
// aborts the whole world (every rank blocked in it gives up) and frees this rank's handle
inline ncclResult_t ncclCommAbort(ncclComm_t c) {
  fakenccl::require_live(c, "ncclCommAbort");
  {
    std::lock_guard<std::mutex> lk(c->w->mu);
    c->w->aborted = true;
  }
  c->w->cv.notify_all();
  {
    std::lock_guard<std::mutex> lk(fakenccl::live_mu());
    fakenccl::live().erase(c);
  }
  fakenccl::unref(c);
  return ncclSuccess;
}
inline ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* e) {
  fakenccl::require_live(c, "ncclCommGetAsyncError");
  *e = (ncclResult_t)c->async_err.load();
  return ncclSuccess;
}
inline ncclResult_t ncclGroupStart() {
  ++fakenccl::group_depth;
  return ncclSuccess;
}
inline ncclResult_t ncclGroupEnd() {
  if (fakenccl::group_depth <= 0) return ncclInvalidUsage;
  if (--fakenccl::group_depth > 0) return ncclSuccess;
  std::vector<fakenccl::Pending> ops;
  ops.swap(fakenccl::group_ops);
  for (auto& p : ops)
    if (p.is_send) p.s->push(std::move(p.f));
  for (auto& p : ops)
    if (!p.is_send) p.s->push(std::move(p.f));
  return ncclSuccess;
}
inline ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t t,
                                             ncclScalarResidence_t res, ncclComm_t c) {
  fakenccl::require_live(c, "ncclRedOpCreatePreMulSum");
  if (res != ncclScalarHostImmediate) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->op_mu);
  *op = c->next_op++;
  c->premul[*op] = fakenccl::load(scalar, 0, t);
  return ncclSuccess;
}
// the op may be destroyed right after the enqueue: keep its scalar until the queued reductions used it (the
// fake never recycles ids, so the entry just stays)
inline ncclResult_t ncclRedOpDestroy(ncclRedOp_t, ncclComm_t) { return ncclSuccess; }

inline ncclResult_t ncclAllReduce(const void* in, void* out, size_t count, ncclDataType_t t, ncclRedOp_t op,
                                  ncclComm_t c, hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in, [&](const std::vector<const void*>& ins) { return fakenccl::reduce_block(c, ins, 0, count, t, op); },
        [&](const std::vector<char>& b) { std::memcpy(out, b.data(), b.size()); });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclReduce(const void* in, void* out, size_t count, ncclDataType_t t, ncclRedOp_t op, int root,
                               ncclComm_t c, hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in,
        [&](const std::vector<const void*>& ins) {
          return c->rank == root ? fakenccl::reduce_block(c, ins, 0, count, t, op) : std::vector<char>();
        },
        [&](const std::vector<char>& b) {
          if (c->rank == root) std::memcpy(out, b.data(), b.size());
        });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclBroadcast(const void* in, void* out, size_t count, ncclDataType_t t, int root, ncclComm_t c,
                                  hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in,
        [&](const std::vector<const void*>& ins) {
          const size_t n = count * fakenccl::esize(t);
          std::vector<char> b(n);
          std::memcpy(b.data(), ins[root], n);
          return b;
        },
        [&](const std::vector<char>& b) { std::memcpy(out, b.data(), b.size()); });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclAllGather(const void* in, void* out, size_t count, ncclDataType_t t, ncclComm_t c,
                                  hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in,
        [&](const std::vector<const void*>& ins) {
          const size_t n = count * fakenccl::esize(t);
          std::vector<char> b(n * ins.size());
          for (size_t r = 0; r < ins.size(); ++r) std::memcpy(b.data() + r * n, ins[r], n);
          return b;
        },
        [&](const std::vector<char>& b) { std::memcpy(out, b.data(), b.size()); });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclReduceScatter(const void* in, void* out, size_t count, ncclDataType_t t, ncclRedOp_t op,
                                      ncclComm_t c, hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in,
        [&](const std::vector<const void*>& ins) {
          return fakenccl::reduce_block(c, ins, (size_t)c->rank * count, count, t, op);
        },
        [&](const std::vector<char>& b) { std::memcpy(out, b.data(), b.size()); });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclAllToAll(const void* in, void* out, size_t count, ncclDataType_t t, ncclComm_t c,
                                 hipStream_t s) {
  fakenccl::require_live(c, "collective");
  const uint64_t seq = c->seq++;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    fakenccl::collective(
        c, seq, in,
        [&](const std::vector<const void*>& ins) {
          const size_t n = count * fakenccl::esize(t);
          std::vector<char> b(n * ins.size());
          for (size_t r = 0; r < ins.size(); ++r)
            std::memcpy(b.data() + r * n, (const char*)ins[r] + (size_t)c->rank * n, n);
          return b;
        },
        [&](const std::vector<char>& b) { std::memcpy(out, b.data(), b.size()); });
  });
  return ncclSuccess;
}
inline ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  fakenccl::require_live(c, "ncclSend");
  if (peer < 0 || peer >= c->w->n) return ncclInvalidArgument;
  fakenccl::ref(c);
  fakenccl::submit(s, true, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    const size_t n = count * fakenccl::esize(t);
    std::vector<char> msg((const char*)buf, (const char*)buf + n);
    {
      std::lock_guard<std::mutex> lk(c->w->mu);
      c->w->mail[{c->rank, peer}].push_back(std::move(msg));
    }
    c->w->cv.notify_all();
  });
  return ncclSuccess;
}
inline ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  fakenccl::require_live(c, "ncclRecv");
  if (peer < 0 || peer >= c->w->n) return ncclInvalidArgument;
  fakenccl::ref(c);
  fakenccl::submit(s, false, [=] {
    struct Unref { ncclComm* c; ~Unref() { fakenccl::unref(c); } } u{c};
    const size_t n = count * fakenccl::esize(t);
    fakenccl::World& w = *c->w;
    std::unique_lock<std::mutex> lk(w.mu);
    auto& q = w.mail[{peer, c->rank}];
    w.cv.wait(lk, [&] { return w.aborted || !q.empty(); });
    if (w.aborted) {
      c->async_err = ncclRemoteError;
      return;
    }
    std::vector<char> msg = std::move(q.front());
    q.pop_front();
    lk.unlock();
    if (msg.size() != n) {
      c->async_err = ncclInvalidUsage;   // size mismatch between the paired send and recv
      return;
    }
    std::memcpy(buf, msg.data(), n);
  });
  return ncclSuccess;
}
