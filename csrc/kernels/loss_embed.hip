// Softmax cross-entropy (single-rank and vocab-parallel stats) and (vocab-parallel) embedding.
//
// Reference behaviour: phi/kernels/gpu/cross_entropy_kernel.cu (hard-label softmax CE),
// fluid/operators/collective/c_softmax_with_cross_entropy_op.cu (MaskLabelByIndex/CaculateLoss:
// local max -> AR(max) -> target logit -> AR(sum) -> sum exp -> AR(sum)), and
// gpu/c_embedding_kernel.cu (rows outside [start, start+V_local) give 0).
//
// MI355X design: CE is an HBM stream over [N, V] logits (V = 32000 for Llama-2 → 62.5 KB bf16
// per row).  One 256-thread block per row computes (max, sum exp) in ONE pass with an online
// rescale per lane, so logits are read once in forward and once in backward; the vocab-parallel
// variant emits the same per-row stats, and the tiny [N]-sized cross-rank combine happens in the
// caller with 1 all-reduce of packed stats instead of the reference's three.
#include "common.h"

namespace pd {

constexpr int kCEBlock = 256;

// stats: mx[N], se[N] (sum exp(x - mx)), tgt[N] (logit at label-start or 0 if not local),
// has[N] (1 if label is local on this rank)
template <typename T, bool VEC>
__global__ __launch_bounds__(kCEBlock) void ce_stats_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                            float* __restrict__ mx, float* __restrict__ se,
                                                            float* __restrict__ tgt, long V, long start) {
  __shared__ float sm[2 * (kCEBlock / 64)];
  const long row = blockIdx.x;
  const T* x = logits + row * V;
  float m = -INFINITY, s = 0.f;
  if (VEC) {
    constexpr int W = 16 / sizeof(T);
    for (long i = threadIdx.x * W; i < V; i += kCEBlock * W) {
      float v[W];
      load_vec<T, W>(x + i, v);
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < W; ++j) lm = fmaxf(lm, v[j]);
      const float nm = fmaxf(m, lm);
      float acc = s * __expf(m - nm);
#pragma unroll
      for (int j = 0; j < W; ++j) acc += __expf(v[j] - nm);
      m = nm; s = acc;
    }
  } else {
    for (long i = threadIdx.x; i < V; i += kCEBlock) {
      const float v = Elt<T>::ld(x + i);
      const float nm = fmaxf(m, v);
      s = s * __expf(m - nm) + __expf(v - nm);
      m = nm;
    }
  }
  // wave combine of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; sm[kCEBlock / 64 + wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = -INFINITY;
    for (int i = 0; i < kCEBlock / 64; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < kCEBlock / 64; ++i) S += sm[kCEBlock / 64 + i] * __expf(sm[i] - M);
    mx[row] = M;
    se[row] = S;
    const long lab = labels[row] - start;
    tgt[row] = (lab >= 0 && lab < V) ? Elt<T>::ld(x + lab) : 0.f;
  }
}

// dx = (exp(x - lse) - onehot(label - start)) * dloss ; rows with ignore_index get 0
template <typename T, bool VEC>
__global__ __launch_bounds__(kCEBlock) void ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                          const float* __restrict__ lse, const float* __restrict__ dloss,
                                                          T* __restrict__ dx, long V, long start, long ignore_index,
                                                          int dloss_scalar) {
  const long row = blockIdx.x;
  const long lab_raw = labels[row];
  const bool ign = lab_raw == ignore_index;
  const long lab = lab_raw - start;
  const float l = lse[row];
  const float g = ign ? 0.f : (dloss_scalar ? dloss[0] : dloss[row]);
  const T* x = logits + row * V;
  T* d = dx + row * V;
  if (VEC) {
    constexpr int W = 16 / sizeof(T);
    for (long i = threadIdx.x * W; i < V; i += kCEBlock * W) {
      float v[W];
      load_vec<T, W>(x + i, v);
#pragma unroll
      for (int j = 0; j < W; ++j) v[j] = (__expf(v[j] - l) - (i + j == lab ? 1.f : 0.f)) * g;
      store_vec<T, W>(d + i, v);
    }
  } else {
    for (long i = threadIdx.x; i < V; i += kCEBlock) {
      const float v = Elt<T>::ld(x + i);
      Elt<T>::st(d + i, (__expf(v - l) - (i == lab ? 1.f : 0.f)) * g);
    }
  }
}

// ------------------------------------------------------------------------- embedding
// out[i, :] = (start <= ids[i] < start+Vl) ? W[ids[i]-start, :] : 0 ; one wave per token
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const T* __restrict__ w,
                                                        T* __restrict__ out, long Ntok, int H, long start, long Vl) {
  constexpr int W = 16 / sizeof(T);
  const long tok = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (tok >= Ntok) return;
  const int lane = threadIdx.x & 63;
  const long id = ids[tok] - start;
  const bool ok = id >= 0 && id < Vl;
  const u16x8* src = reinterpret_cast<const u16x8*>(w + (ok ? id : 0) * (long)H);
  u16x8* dst = reinterpret_cast<u16x8*>(out + tok * (long)H);
  const int nv = H / W;
  for (int i = lane; i < nv; i += 64) {
    u16x8 v = ok ? src[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    dst[i] = v;
  }
}

// dW32[ids[i]-start, :] += dout[i, :] ; f32 accumulation buffer, one wave per token,
// each wave-instruction adds 256 contiguous bytes (full-rate atomic shape, Guideline 12).
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ ids, const T* __restrict__ dout,
                                                        float* __restrict__ dw, long Ntok, int H, long start, long Vl,
                                                        long padding_idx) {
  const long tok = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (tok >= Ntok) return;
  const int lane = threadIdx.x & 63;
  const long raw = ids[tok];
  if (raw == padding_idx) return;
  const long id = raw - start;
  if (id < 0 || id >= Vl) return;
  const T* g = dout + tok * (long)H;
  float* d = dw + id * (long)H;
  for (int i = lane; i < H; i += 64) atomicAdd(d + i, Elt<T>::ld(g + i));
}

template <typename T>
__global__ __launch_bounds__(256) void cast_f32_kernel(const float* __restrict__ src, T* __restrict__ dst, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) Elt<T>::st(dst + i, src[i]);
}

}  // namespace pd

using namespace pd;

extern "C" int pd_ce_stats(int dt, const void* logits, const int64_t* labels, float* mx, float* se, float* tgt, long N,
                           long V, long start, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (V % (dt == kF32 ? 4 : 8)) == 0;
  PD_DISPATCH_FLOAT(dt, T,
                    if (vec) ce_stats_kernel<T, true><<<N, kCEBlock, 0, st>>>((const T*)logits, labels, mx, se, tgt, V, start);
                    else ce_stats_kernel<T, false><<<N, kCEBlock, 0, st>>>((const T*)logits, labels, mx, se, tgt, V, start));
  return (int)hipGetLastError();
}

extern "C" int pd_ce_bwd(int dt, const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                         void* dx, long N, long V, long start, long ignore_index, int dloss_scalar, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (V % (dt == kF32 ? 4 : 8)) == 0;
  PD_DISPATCH_FLOAT(dt, T,
                    if (vec) ce_bwd_kernel<T, true><<<N, kCEBlock, 0, st>>>((const T*)logits, labels, lse, dloss, (T*)dx, V,
                                                                            start, ignore_index, dloss_scalar);
                    else ce_bwd_kernel<T, false><<<N, kCEBlock, 0, st>>>((const T*)logits, labels, lse, dloss, (T*)dx, V,
                                                                          start, ignore_index, dloss_scalar));
  return (int)hipGetLastError();
}

extern "C" int pd_embed_fwd(int dt, const int64_t* ids, const void* w, void* out, long Ntok, int H, long start, long Vl,
                            void* stream) {
  if ((H * (dt == kF32 ? 4 : 2)) % 16) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int g = (int)((Ntok + 3) / 4);
  PD_DISPATCH_FLOAT(dt, T, embed_fwd_kernel<T><<<g, 256, 0, st>>>(ids, (const T*)w, (T*)out, Ntok, H, start, Vl));
  return (int)hipGetLastError();
}

extern "C" int pd_embed_bwd(int dt, const int64_t* ids, const void* dout, float* dw32, long Ntok, int H, long start,
                            long Vl, long padding_idx, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = (int)((Ntok + 3) / 4);
  PD_DISPATCH_FLOAT(dt, T, embed_bwd_kernel<T><<<g, 256, 0, st>>>(ids, (const T*)dout, dw32, Ntok, H, start, Vl, padding_idx));
  return (int)hipGetLastError();
}

extern "C" int pd_cast_from_f32(int dt, const float* src, void* dst, long n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  PD_DISPATCH_FLOAT(dt, T, cast_f32_kernel<T><<<(int)g, 256, 0, st>>>(src, (T*)dst, n));
  return (int)hipGetLastError();
}
