// ProcessGroupRCCL core: RCCL communicators, comm streams, event fences and tasks.  Python-free: the pybind module
// paddle2_amd._rccl (rccl_group.cpp) wraps it, and csrc/comm/test/rccl_stress.cpp drives it against a threaded fake
// RCCL / HIP (csrc/comm/test/fake/) on the CPU.  The torch-facing process group is paddle2_amd/distributed/rccl_pg.py.
//
// Reference roles: paddle/fluid/distributed/collective/process_group_nccl.cc — per-device comm stream with
// calc->comm / comm->calc event sync (:840-847), the generic Collective path (:902), dedicated lo->hi p2p
// communicators (:1023-1028), group start/end coalescing (:999-1037); paddle/phi/core/distributed/
// nccl_comm_context.cc:79-248 (native ncclAvg / PreMulSum); comm_context_manager.cc:61-122 (rank 0 creates the
// unique id, publishes it through the TCPStore, every rank ncclCommInitRank's).
//
// MI355X design:
//  * one high-priority HIP stream per communicator: collectives overlap the compute stream, and p2p on its
//    own lo->hi communicator + stream never queues behind a large reduce-scatter of the data-parallel group
//    (xGMI links are point-to-point; independent streams keep several links busy at once);
//  * every operation: record an event on the caller's (calc) stream, make the comm stream wait on it, enqueue
//    the RCCL call, record the end event on the comm stream -> Task.  Task.wait(stream) makes the caller's
//    stream wait on the end event (no host block); Task.synchronize() blocks the host with async-error polling
//    and a timeout that aborts the communicator instead of hanging; use_calc_stream enqueues straight on the
//    caller's stream (no events);
//  * coalescing: group_start() opens ncclGroupStart; operations inside fence each communicator they touch once
//    and return no task; group_end() closes the group and returns ONE task over every touched communicator;
//  * AVG is ncclAvg and PreMulSum a ncclRedOpCreatePreMulSum op (host scalar), destroyed right after enqueue;
//  * events come from a per-group pool; communicators are created lazily through the caller's store object
//    (anything with set(key, bytes) / get(key) -> bytes: the native TCPStore or a c10d store).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pdrccl {

class Task;
using TaskPtr = std::shared_ptr<Task>;

inline namespace detail {

// set by shutdown() (Python atexit / destroy_process_group): later destructors must not touch the HIP runtime or
// RCCL, which may already be torn down when the interpreter finalises the last Python references
inline std::atomic<bool> g_shutdown{false};

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("[rccl_group] ") + what + ": " + hipGetErrorString(e));
}
inline void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("[rccl_group] ") + what + ": " + ncclGetErrorString(r));
}

// dtype codes shared with rccl_pg.py
inline ncclDataType_t nccl_dtype(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclFloat16;
    case 2: return ncclBfloat16;
    case 3: return ncclFloat64;
    case 4: return ncclInt32;
    case 5: return ncclInt64;
    case 6: return ncclInt8;
    case 7: return ncclUint8;
    case 8: return ncclFloat8e4m3;
    case 9: return ncclFloat8e5m2;
    default: throw std::invalid_argument("[rccl_group] unsupported dtype code " + std::to_string(code));
  }
}
inline size_t dtype_size(int code) {
  static const size_t s[] = {4, 2, 2, 8, 4, 8, 1, 1, 1, 1};
  if (code < 0 || code > 9) throw std::invalid_argument("[rccl_group] unsupported dtype code");
  return s[code];
}
// op codes: 0 sum, 1 prod, 2 max, 3 min, 4 avg, 5 premul-sum (scalar argument)
inline ncclRedOp_t nccl_op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: throw std::invalid_argument("[rccl_group] unsupported reduce op " + std::to_string(code));
  }
}

struct Comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int device = 0, rank = 0, nranks = 1;
  bool aborted = false;
  void release() {
    if (comm && !aborted) ncclCommDestroy(comm);
    if (stream) hipStreamDestroy(stream);
    comm = nullptr;
    stream = nullptr;
  }
  ~Comm() {
    if (!g_shutdown) release();
  }
};

// Events are never destroyed (or handed out again) while a stream may still signal them: a finished task's end
// event and a fence event go to `pending_` and return to the free list only once hipEventQuery reports them
// complete (swept on every get()).  Destroying a still-pending end event — the Task of an async collective is
// dropped as soon as the caller's stream has been told to wait for it, long before the GPU passed the event —
// raced with the stream's later signal on the 7B stage-3 comm path (illegal memory access without a per-step sync).
class EventPool {
 public:
  hipEvent_t get() {
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.empty()) sweep();
    if (!free_.empty()) {
      hipEvent_t e = free_.back();
      free_.pop_back();
      return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  // an event that may still be pending on a stream: reusable once it has completed
  void retire(hipEvent_t e) {
    std::lock_guard<std::mutex> lk(mu_);
    pending_.push_back(e);
    if (pending_.size() > 256) sweep();
  }
  void put(hipEvent_t e) { retire(e); }
  void release() {
    std::lock_guard<std::mutex> lk(mu_);
    for (hipEvent_t e : free_) hipEventDestroy(e);
    free_.clear();
    for (hipEvent_t e : pending_) hipEventDestroy(e);   // shutdown: the device work is over
    pending_.clear();
  }
  ~EventPool() {
    if (!g_shutdown) release();
  }

 private:
  // move completed pending events to the free list (caller holds mu_)
  void sweep() {
    size_t keep = 0;
    for (size_t i = 0; i < pending_.size(); ++i) {
      if (hipEventQuery(pending_[i]) == hipSuccess) free_.push_back(pending_[i]);
      else pending_[keep++] = pending_[i];
    }
    pending_.resize(keep);
  }
  std::mutex mu_;
  std::vector<hipEvent_t> free_;
  std::vector<hipEvent_t> pending_;
};

// IEEE binary16 from binary32, round to nearest even (the PreMulSum scalar of an fp16 reduction)
inline uint16_t f32_to_f16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const int exp = (int)((x >> 23) & 0xff) - 127 + 15;
  uint32_t man = x & 0x7fffffu;
  if (((x >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (man ? 0x200u : 0));
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

}  // namespace

// The rendezvous store the communicators' unique ids go through (the pybind layer adapts the native TCPStore /
// a c10d store; the CPU stress test uses an in-memory one).  get() blocks until the key exists.
class Store {
 public:
  virtual ~Store() = default;
  virtual void set(const std::string& key, const std::string& value) = 0;
  virtual std::string get(const std::string& key) = 0;
};

class Task {
 public:
  Task(std::vector<std::shared_ptr<Comm>> comms, std::vector<hipEvent_t> ends, std::shared_ptr<EventPool> pool,
       int timeout_ms)
      : comms_(std::move(comms)), ends_(std::move(ends)), pool_(std::move(pool)), timeout_ms_(timeout_ms) {}
  ~Task() {
    if (g_shutdown) return;
    // an end event may still be pending on the comm stream (the caller's stream only WAITS for it): the pool
    // recycles it after it completes — never destroyed while the GPU may still signal it
    for (hipEvent_t e : ends_) pool_->retire(e);
  }
  // the caller's stream waits for the communication (no host block)
  void wait(uintptr_t stream) {
    for (hipEvent_t e : ends_) hip_check(hipStreamWaitEvent((hipStream_t)stream, e, 0), "hipStreamWaitEvent");
  }
  bool is_completed() {
    check_async();
    for (hipEvent_t e : ends_) {
      const hipError_t r = hipEventQuery(e);
      if (r == hipErrorNotReady) return false;
      hip_check(r, "hipEventQuery");
    }
    return true;
  }
  // host blocks until done; a communicator error or the timeout aborts the communicators and raises
  void synchronize() {
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
      bool done = true;
      for (hipEvent_t e : ends_) {
        const hipError_t r = hipEventQuery(e);
        if (r == hipErrorNotReady) {
          done = false;
          break;
        }
        hip_check(r, "hipEventQuery");
      }
      // a finished end event does not mean a good result: a communicator that failed (a peer aborted) may have
      // completed its kernels with garbage, so the async error is checked on completion too
      check_async();
      if (done) return;
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
      if (timeout_ms_ > 0 && ms.count() > timeout_ms_) {
        for (auto& c : comms_) {
          if (c->aborted) continue;   // ncclCommAbort frees the communicator: never twice
          ncclCommAbort(c->comm);
          c->aborted = true;
        }
        throw std::runtime_error("[rccl_group] collective timed out after " + std::to_string(timeout_ms_) +
                                 " ms; communicator aborted");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

 private:
  void check_async() {
    for (auto& c : comms_) {
      if (c->aborted) throw std::runtime_error("[rccl_group] communicator was aborted");
      ncclResult_t ae = ncclSuccess;
      nccl_check(ncclCommGetAsyncError(c->comm, &ae), "ncclCommGetAsyncError");
      if (ae != ncclSuccess && ae != ncclInProgress) {
        ncclCommAbort(c->comm);
        c->aborted = true;
        throw std::runtime_error(std::string("[rccl_group] asynchronous communicator error: ") +
                                 ncclGetErrorString(ae));
      }
    }
  }
  std::vector<std::shared_ptr<Comm>> comms_;
  std::vector<hipEvent_t> ends_;
  std::shared_ptr<EventPool> pool_;
  int timeout_ms_;
};

class RcclGroup {
 public:
  RcclGroup(std::shared_ptr<Store> store, std::string prefix, int rank, int nranks, int device, int timeout_ms)
      : store_(std::move(store)), prefix_(std::move(prefix)), rank_(rank), nranks_(nranks), device_(device),
        timeout_ms_(timeout_ms), pool_(std::make_shared<EventPool>()) {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("[rccl_group] bad rank / size");
  }

  int rank() const { return rank_; }
  // host-wait bound of the tasks created from now on (0 = unbounded)
  int timeout_ms() const { return timeout_ms_; }
  void set_timeout_ms(int ms) { timeout_ms_ = ms; }
  int size() const { return nranks_; }

  // the main communicator's stream (callers record tensors on it for allocator lifetime fencing)
  uintptr_t comm_stream() { return (uintptr_t)main()->stream; }
  uintptr_t p2p_stream(int peer) { return (uintptr_t)p2p(peer)->stream; }
  // number of communicators created so far (main + p2p pairs)
  int num_comms() const { return (int)comms_.size(); }

  TaskPtr all_reduce(uintptr_t in, uintptr_t out, size_t count, int dtype, int op, double scalar, uintptr_t calc,
                        bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      ncclRedOp_t rop;
      const bool premul = op == 5;
      if (premul) rop = make_premul(c, dtype, scalar);
      else rop = nccl_op(op);
      nccl_check(ncclAllReduce((const void*)in, (void*)out, count, nccl_dtype(dtype), rop, c->comm, s),
                 "ncclAllReduce");
      if (premul) ncclRedOpDestroy(rop, c->comm);
    });
  }

  TaskPtr broadcast(uintptr_t in, uintptr_t out, size_t count, int dtype, int root, uintptr_t calc, bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclBroadcast((const void*)in, (void*)out, count, nccl_dtype(dtype), root, c->comm, s),
                 "ncclBroadcast");
    });
  }

  TaskPtr reduce(uintptr_t in, uintptr_t out, size_t count, int dtype, int op, double scalar, int root,
                    uintptr_t calc, bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      const bool premul = op == 5;
      ncclRedOp_t rop = premul ? make_premul(c, dtype, scalar) : nccl_op(op);
      nccl_check(ncclReduce((const void*)in, (void*)out, count, nccl_dtype(dtype), rop, root, c->comm, s),
                 "ncclReduce");
      if (premul) ncclRedOpDestroy(rop, c->comm);
    });
  }

  // out = concat over ranks of `count` elements each
  TaskPtr all_gather(uintptr_t in, uintptr_t out, size_t count, int dtype, uintptr_t calc, bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclAllGather((const void*)in, (void*)out, count, nccl_dtype(dtype), c->comm, s), "ncclAllGather");
    });
  }

  // in = nranks x `count` elements; out (count) = reduced block `rank`
  TaskPtr reduce_scatter(uintptr_t in, uintptr_t out, size_t count, int dtype, int op, double scalar,
                            uintptr_t calc, bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      const bool premul = op == 5;
      ncclRedOp_t rop = premul ? make_premul(c, dtype, scalar) : nccl_op(op);
      nccl_check(ncclReduceScatter((const void*)in, (void*)out, count, nccl_dtype(dtype), rop, c->comm, s),
                 "ncclReduceScatter");
      if (premul) ncclRedOpDestroy(rop, c->comm);
    });
  }

  // equal splits: `count` elements to / from every rank
  TaskPtr all_to_all(uintptr_t in, uintptr_t out, size_t count, int dtype, uintptr_t calc, bool use_calc) {
    auto c = main();
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclAllToAll((const void*)in, (void*)out, count, nccl_dtype(dtype), c->comm, s), "ncclAllToAll");
    });
  }

  // unequal splits (element counts / offsets per rank), one grouped send/recv round on the main communicator
  TaskPtr all_to_all_v(uintptr_t in, uintptr_t out, std::vector<size_t> scounts, std::vector<size_t> sdispls,
                          std::vector<size_t> rcounts, std::vector<size_t> rdispls, int dtype, uintptr_t calc,
                          bool use_calc) {
    if ((int)scounts.size() != nranks_ || (int)rcounts.size() != nranks_ || (int)sdispls.size() != nranks_ ||
        (int)rdispls.size() != nranks_)
      throw std::invalid_argument("[rccl_group] all_to_all_v: one count / displacement per rank");
    auto c = main();
    const size_t es = dtype_size(dtype);
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclGroupStart(), "ncclGroupStart");
      for (int r = 0; r < nranks_; ++r) {
        if (scounts[r])
          nccl_check(ncclSend((const char*)in + sdispls[r] * es, scounts[r], nccl_dtype(dtype), r, c->comm, s),
                     "ncclSend");
        if (rcounts[r])
          nccl_check(ncclRecv((char*)out + rdispls[r] * es, rcounts[r], nccl_dtype(dtype), r, c->comm, s),
                     "ncclRecv");
      }
      nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    });
  }

  // point-to-point on the dedicated (lo, hi) communicator of this pair
  TaskPtr send(uintptr_t ptr, size_t count, int dtype, int peer, uintptr_t calc, bool use_calc) {
    auto c = p2p(peer);
    const int pr = peer == rank_ ? c->rank : 1 - c->rank;
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclSend((const void*)ptr, count, nccl_dtype(dtype), pr, c->comm, s), "ncclSend");
    });
  }
  TaskPtr recv(uintptr_t ptr, size_t count, int dtype, int peer, uintptr_t calc, bool use_calc) {
    auto c = p2p(peer);
    const int pr = peer == rank_ ? c->rank : 1 - c->rank;
    return run({c}, calc, use_calc, [&](hipStream_t s) {
      nccl_check(ncclRecv((void*)ptr, count, nccl_dtype(dtype), pr, c->comm, s), "ncclRecv");
    });
  }

  void group_start(uintptr_t calc) {
    if (coalescing_) throw std::runtime_error("[rccl_group] group_start inside an open group");
    coalescing_ = true;
    co_calc_ = calc;
    co_comms_.clear();
    nccl_check(ncclGroupStart(), "ncclGroupStart");
  }
  TaskPtr group_end() {
    if (!coalescing_) throw std::runtime_error("[rccl_group] group_end without group_start");
    coalescing_ = false;
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    if (co_comms_.empty()) return nullptr;
    std::vector<hipEvent_t> ends;
    for (auto& c : co_comms_) {
      hipEvent_t e = pool_->get();
      hip_check(hipEventRecord(e, c->stream), "hipEventRecord");
      ends.push_back(e);
    }
    auto t = std::make_shared<Task>(co_comms_, std::move(ends), pool_, timeout_ms_);
    co_comms_.clear();
    return t;
  }

  // interpreter exit: finish outstanding work, then leave communicators / streams / events to process teardown.
  // Tensors freed later in finalisation may still carry record_stream marks on a comm stream (the allocator
  // fences their reuse with events on it), so the streams must stay valid; destructors become no-ops.
  void shutdown() {
    if (g_shutdown) return;
    hipDeviceSynchronize();
    g_shutdown = true;
  }

  void abort() {
    for (auto& kv : comms_) {
      if (!kv.second->aborted) {
        ncclCommAbort(kv.second->comm);
        kv.second->aborted = true;
      }
    }
  }

  // a device-side barrier: a 1-element all-reduce, host-synchronised
  void barrier(uintptr_t scratch, uintptr_t calc) {
    TaskPtr t = all_reduce(scratch, scratch, 1, 4, 0, 0.0, calc, false);
    t->synchronize();
  }

 private:
  template <typename F>
  TaskPtr run(std::vector<std::shared_ptr<Comm>> cs, uintptr_t calc, bool use_calc, F&& enqueue) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hipStream_t cstream = (hipStream_t)calc;
    if (use_calc) {   // on the caller's stream: ordered by construction, nothing to fence or track
      enqueue(cstream);
      return nullptr;
    }
    auto& c = cs[0];
    bool fenced = false;
    if (coalescing_) {
      for (auto& x : co_comms_) fenced |= x.get() == c.get();
    }
    if (!fenced) {   // calc -> comm: the comm stream waits for everything queued on the caller's stream so far
      hipEvent_t pre = pool_->get();
      hip_check(hipEventRecord(pre, coalescing_ ? (hipStream_t)co_calc_ : cstream), "hipEventRecord");
      hip_check(hipStreamWaitEvent(c->stream, pre, 0), "hipStreamWaitEvent");
      pool_->retire(pre);   // reused only after the calc stream passed it
      if (coalescing_) co_comms_.push_back(c);
    }
    enqueue(c->stream);
    if (coalescing_) return nullptr;
    hipEvent_t end = pool_->get();
    hip_check(hipEventRecord(end, c->stream), "hipEventRecord");
    return std::make_shared<Task>(cs, std::vector<hipEvent_t>{end}, pool_, timeout_ms_);
  }

  ncclRedOp_t make_premul(const std::shared_ptr<Comm>& c, int dtype, double scalar) {
    ncclRedOp_t op;
    union {
      float f;
      double d;
      uint16_t h;
    } v;
    std::memset(&v, 0, sizeof(v));
    switch (dtype) {
      case 0: v.f = (float)scalar; break;
      case 3: v.d = scalar; break;
      case 1: v.h = f32_to_f16((float)scalar); break;
      case 2: {
        float f = (float)scalar;
        uint32_t u;
        std::memcpy(&u, &f, 4);
        v.h = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);   // round to nearest even
        break;
      }
      default: throw std::invalid_argument("[rccl_group] PreMulSum needs a floating dtype");
    }
    nccl_check(ncclRedOpCreatePreMulSum(&op, &v, nccl_dtype(dtype), ncclScalarHostImmediate, c->comm),
               "ncclRedOpCreatePreMulSum");
    return op;
  }

  std::shared_ptr<Comm> main() {
    if (!main_) main_ = create("main", rank_, nranks_, rank_ == 0);
    return main_;
  }
  std::shared_ptr<Comm> p2p(int peer) {
    if (peer < 0 || peer >= nranks_) throw std::invalid_argument("[rccl_group] p2p peer out of range");
    const int lo = std::min(rank_, peer), hi = std::max(rank_, peer);
    const std::string key = "p2p_" + std::to_string(lo) + "_" + std::to_string(hi);
    auto it = comms_.find(key);
    if (it != comms_.end()) return it->second;
    if (lo == hi) return main();   // to self: any communicator containing this rank works
    return create(key, rank_ == lo ? 0 : 1, 2, rank_ == lo);
  }

  std::shared_ptr<Comm> create(const std::string& key, int sub_rank, int sub_n, bool make_id) {
    auto it = comms_.find(key);
    if (it != comms_.end()) return it->second;
    if (coalescing_)
      throw std::runtime_error("[rccl_group] communicator '" + key +
                               "' would be created inside a group; issue one op on it first");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ncclUniqueId id;
    const std::string skey = prefix_ + "/rccl_uid/" + key + "/" + std::to_string(generation_);
    if (sub_n == 1) {
      nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    } else if (make_id) {
      nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
      store_->set(skey, std::string(reinterpret_cast<const char*>(&id), sizeof(id)));
    } else {
      const std::string s = store_->get(skey);
      if (s.size() != sizeof(id)) throw std::runtime_error("[rccl_group] bad unique id in the store");
      std::memcpy(&id, s.data(), sizeof(id));
    }
    auto c = std::make_shared<Comm>();
    c->device = device_;
    c->rank = sub_rank;
    c->nranks = sub_n;
    int lo_pri = 0, hi_pri = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_pri), "hipStreamCreateWithPriority");
    nccl_check(ncclCommInitRank(&c->comm, sub_n, id, sub_rank), "ncclCommInitRank");
    comms_[key] = c;
    return c;
  }

  std::shared_ptr<Store> store_;
  std::string prefix_;
  int rank_, nranks_, device_, timeout_ms_;
  int generation_ = 0;
  std::shared_ptr<EventPool> pool_;
  std::shared_ptr<Comm> main_;
  std::map<std::string, std::shared_ptr<Comm>> comms_;
  bool coalescing_ = false;
  uintptr_t co_calc_ = 0;
  std::vector<std::shared_ptr<Comm>> co_comms_;
};

}  // namespace pdrccl
