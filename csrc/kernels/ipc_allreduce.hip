// All-reduce over IPC-mapped peer buffers (xGMI point-to-point), for latency-bound messages.
//
// Reference role: SURVEY §5.8 item 2 / process_group_nccl.cc:267 — the reference always goes through
// NCCL; on an 8 x MI355X node every GPU has a direct xGMI link to every other GPU, so a message small
// enough to be latency bound is reduced faster by letting each GPU READ its peers' buffers directly than by
// an RCCL ring (2(N-1) link hops, each with its own launch/handshake latency).
//
//  * one-shot: every rank copies its input into its own IPC data buffer; after a flag barrier each rank reads
//    the N inputs (N-1 over xGMI, all links in parallel) and sums them in rank order 0..N-1, so every rank
//    produces bit-identical results;
//  * two-shot (larger messages): rank r reduces slice r of the message from all peers into the second half
//    of its IPC buffer (reduce-scatter), barrier, then gathers every peer's reduced slice (all-gather) —
//    each byte crosses a link twice instead of N-1 times;
//  * barriers are per workgroup: block b of every rank owns the same element range in every phase, so
//    block b only waits for block b of its peers (flags [phase][block][rank] in each rank's signal area);
//  * flag stores / loads are system-scope release / acquire atomics through the vector memory path; the
//    data and signal buffers are allocated uncached (hipDeviceMallocUncached) so peers always read HBM;
//  * every wait is bounded (~`timeout_ms` of the 100 MHz realtime counter): a peer that never arrives sets
//    *err and the kernel finishes instead of spinning forever.
#include <cstring>

#include "common.h"

namespace pd {
namespace ar {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kPhases = 3;
// signal area per rank: [kPhases][kMaxBlocks][kMaxRanks] unsigned
constexpr long kSigBytes = (long)kPhases * kMaxBlocks * kMaxRanks * 4;

struct Peers {
  char* data[kMaxRanks];       // rank p's data buffer (p == rank: our own)
  unsigned* sig[kMaxRanks];    // rank p's signal area
};

__device__ __forceinline__ unsigned* flag(unsigned* sig, int phase, int blk, int src) {
  return sig + ((long)phase * kMaxBlocks + blk) * kMaxRanks + src;
}

// Block barrier across ranks for phase `ph`: thread p < nranks signals peer p and waits for peer p's signal.
// The release store of lane p covers only lane p's own writes, so first EVERY thread retires its memory
// operations system-wide (its data stores visible to peers, its peer reads complete) and the block meets:
// only then may a peer read what this block wrote, or overwrite what it was reading.
__device__ __forceinline__ void xbarrier(const Peers& P, int rank, int nranks, int ph, unsigned epoch, unsigned* err,
                                         long long budget) {
  __threadfence_system();
  __syncthreads();
  const int p = threadIdx.x;
  if (p < nranks) {
    __hip_atomic_store(flag(P.sig[p], ph, blockIdx.x, rank), epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* mine = flag(P.sig[rank], ph, blockIdx.x, p);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (wall_clock64() - t0 > budget) {
        __hip_atomic_fetch_or(err, 1u << p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ void load8(const char* p, float (&v)[16 / sizeof(T)]) {
  load_vec<T, 16 / sizeof(T)>(reinterpret_cast<const T*>(p), v);
}

// element range [lo, hi) (in 16-B vectors) owned by block b within a range of nv vectors
__device__ __forceinline__ void block_range(long nv, long& lo, long& hi) {
  const long per = (nv + gridDim.x - 1) / gridDim.x;
  lo = min(nv, per * blockIdx.x);
  hi = min(nv, lo + per);
}

// one-shot: out[i] = sum_r data_r[i] (rank order), nv = number of 16-B vectors
template <typename T>
__global__ __launch_bounds__(256) void oneshot_kernel(Peers P, int rank, int nranks, char* out, long out_stride,
                                                      long nv, unsigned epoch, unsigned* err, long long budget) {
  constexpr int E = 16 / sizeof(T);
  if (rank < 0) {  // in-process simulation: blockIdx.y plays rank y (all ranks' blocks co-resident in one grid)
    rank = blockIdx.y;
    out += rank * out_stride;
  }
  xbarrier(P, rank, nranks, 0, epoch, err, budget);
  long lo, hi;
  block_range(nv, lo, hi);
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float acc[E], v[E];
    load8<T>(P.data[0] + i * 16, acc);
    for (int r = 1; r < nranks; ++r) {
      load8<T>(P.data[r] + i * 16, v);
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += v[e];
    }
    store_vec<T, E>(reinterpret_cast<T*>(out + i * 16), acc);
  }
  // nobody may overwrite its data buffer (next call) before every peer finished reading this block's range
  xbarrier(P, rank, nranks, 1, epoch, err, budget);
}

// two-shot: slice s = [s*nv/N, (s+1)*nv/N); rank r reduces slice r into data_r[red_off + ...], then gathers
template <typename T>
__global__ __launch_bounds__(256) void twoshot_kernel(Peers P, int rank, int nranks, char* out, long out_stride,
                                                      long nv, long red_off, unsigned epoch, unsigned* err,
                                                      long long budget) {
  constexpr int E = 16 / sizeof(T);
  if (rank < 0) {
    rank = blockIdx.y;
    out += rank * out_stride;
  }
  const long sl = (nv + nranks - 1) / nranks;
  xbarrier(P, rank, nranks, 0, epoch, err, budget);
  {
    const long s0 = min(nv, sl * rank), s1 = min(nv, s0 + sl);
    long lo, hi;
    block_range(s1 - s0, lo, hi);
    for (long i = s0 + lo + threadIdx.x; i < s0 + hi; i += blockDim.x) {
      float acc[E], v[E];
      load8<T>(P.data[0] + i * 16, acc);
      for (int r = 1; r < nranks; ++r) {
        load8<T>(P.data[r] + i * 16, v);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += v[e];
      }
      store_vec<T, E>(reinterpret_cast<T*>(P.data[rank] + red_off + i * 16), acc);
      store_vec<T, E>(reinterpret_cast<T*>(out + i * 16), acc);
    }
  }
  xbarrier(P, rank, nranks, 1, epoch, err, budget);
  for (int r = 0; r < nranks; ++r) {
    if (r == rank) continue;
    const long s0 = min(nv, sl * r), s1 = min(nv, s0 + sl);
    long lo, hi;
    block_range(s1 - s0, lo, hi);
    for (long i = s0 + lo + threadIdx.x; i < s0 + hi; i += blockDim.x) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(P.data[r] + red_off + i * 16);
      *reinterpret_cast<u16x8*>(out + i * 16) = v;
    }
  }
  xbarrier(P, rank, nranks, 2, epoch, err, budget);
}

}  // namespace ar
}  // namespace pd

using namespace pd;

extern "C" long pd_ar_sig_bytes() { return ar::kSigBytes; }

// Uncached device allocation (peers read it over xGMI; no stale lines in any L2).  Falls back to a plain
// allocation if the uncached flag is refused.  Returns 0 on success.
extern "C" int pd_ar_alloc(long bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipMalloc(ptr, (size_t)bytes);
  }
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

extern "C" int pd_ar_free(void* p) { return (int)hipFree(p); }

extern "C" int pd_memcpy_d2d(void* dst, const void* src, long bytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
}

// 64-byte IPC handle of an allocation made by pd_ar_alloc
extern "C" int pd_ar_get_handle(void* p, void* handle64) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle64), p);
}

extern "C" int pd_ar_open_handle(const void* handle64, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int pd_ar_close_handle(void* p) { return (int)hipIpcCloseMemHandle(p); }

// mode 0 one-shot, 1 two-shot.  data[r] / sig[r]: the N ranks' buffers as mapped in THIS process (ours at
// data[rank]); the input must already be in data[rank][0, bytes).  two-shot also uses data[r][red_off, +bytes).
// dt: kF32 / kBF16 / kF16; bytes % 16 == 0.  rank = -1: one launch simulates all N ranks (grid.y = N, rank y
// writes out + y * out_stride) — the single-GPU test of the protocol.
extern "C" int pd_ar_allreduce(int mode, int dt, const void* const* data, const void* const* sig, int rank, int nranks,
                               void* out, long out_stride, long bytes, long red_off, unsigned epoch, unsigned* err,
                               int blocks, int timeout_ms, void* stream) {
  if (nranks < 1 || nranks > ar::kMaxRanks || rank < -1 || rank >= nranks || bytes % 16 || bytes <= 0) return -1;
  if (blocks < 1) blocks = 1;
  if (blocks > ar::kMaxBlocks) blocks = ar::kMaxBlocks;
  ar::Peers P;
  for (int r = 0; r < ar::kMaxRanks; ++r) {
    P.data[r] = r < nranks ? (char*)data[r] : nullptr;
    P.sig[r] = r < nranks ? (unsigned*)sig[r] : nullptr;
  }
  const long nv = bytes / 16;
  const long long budget = (long long)timeout_ms * 100000;  // 100 MHz realtime counter
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(blocks, rank < 0 ? nranks : 1);
#define PD_AR(T)                                                                                                   \
  if (mode == 0)                                                                                                   \
    ar::oneshot_kernel<T><<<grid, 256, 0, st>>>(P, rank, nranks, (char*)out, out_stride, nv, epoch, err, budget);  \
  else                                                                                                             \
    ar::twoshot_kernel<T><<<grid, 256, 0, st>>>(P, rank, nranks, (char*)out, out_stride, nv, red_off, epoch, err,  \
                                                budget);
  if (dt == kF32) { PD_AR(float) }
  else if (dt == kBF16) { PD_AR(bf16) }
  else if (dt == kF16) { PD_AR(half16) }
  else return -2;
#undef PD_AR
  return (int)hipGetLastError();
}
