// Fused bias + activation and fused dropout + residual add (gfx950), forward and backward.
//
// Reference: phi/kernels/fusion/gpu/fused_bias_act_kernel.cu (bias add + act / gated act in one pass) and
// phi/kernels/fusion/gpu/fused_dropout_add_kernel.cu (dropout(x) + y, mask from Philox seed/offset,
// regenerated in the backward).  Both are HBM-bound elementwise passes: one 16-B vector (8 bf16/f16 or 4 f32)
// per lane per load, a grid-stride loop over rows x 8-column chunks, fp32 math in registers.
//  * bias_act: out[r, c] = act(x[r, c] + b[c]); gated (swiglu / geglu): x = [a | g] halves of width H,
//    out[r, c] = act(a + ba) * (g + bg), c < H.  Backward returns dx (and the host sums it for dbias).
//  * dropout_add: out = x * keep * 1/(1-p) + y with keep = hash(seed, element) >= p * 2^32 — a counter-based
//    mask (the flash-attention dropout hash), so the backward regenerates it instead of storing a mask.
#include "common.h"

namespace pd {
namespace fa2 {

enum Act : int { kIdentity = 0, kRelu = 1, kGelu = 2, kGeluTanh = 3, kSilu = 4, kSigmoid = 5 };

__device__ __forceinline__ float act_f(int act, float v) {
  switch (act) {
    case kRelu: return v > 0.f ? v : 0.f;
    case kGelu: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    case kGeluTanh: {
      const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      return 0.5f * v * (1.f + tanhf(u));
    }
    case kSilu: return v * __builtin_amdgcn_rcpf(1.f + __expf(-v));
    case kSigmoid: return __builtin_amdgcn_rcpf(1.f + __expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ float act_grad(int act, float v) {
  switch (act) {
    case kRelu: return v > 0.f ? 1.f : 0.f;
    case kGelu: {
      const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * v * v);
      return cdf + v * pdf;
    }
    case kGeluTanh: {
      const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      const float t = tanhf(u);
      const float du = 0.7978845608028654f * (1.f + 3.f * 0.044715f * v * v);
      return 0.5f * (1.f + t) + 0.5f * v * (1.f - t * t) * du;
    }
    case kSilu: {
      const float s = __builtin_amdgcn_rcpf(1.f + __expf(-v));
      return s * (1.f + v * (1.f - s));
    }
    case kSigmoid: {
      const float s = __builtin_amdgcn_rcpf(1.f + __expf(-v));
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[16 / sizeof(T)]) {
  load_vec<T, 16 / sizeof(T)>(p, v);
}

// rows x N (non-gated) or rows x 2H -> rows x H (gated); E elements per lane-vector
template <typename T, bool GATED>
__global__ __launch_bounds__(256) void bias_act_fwd(const T* __restrict__ x, const T* __restrict__ b,
                                                    T* __restrict__ out, long rows, int H, long sx, long so, int act) {
  constexpr int E = 16 / sizeof(T);
  const int cv = H / E;
  for (long r = blockIdx.y; r < rows; r += gridDim.y)
  for (int vi = blockIdx.x * 256 + threadIdx.x; vi < cv; vi += gridDim.x * 256) {
    const int c = vi * E;
    float a[E];
    ld8<T>(x + r * sx + c, a);
    if (b) {
      float bb[E];
      ld8<T>(b + c, bb);
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] += bb[e];
    }
    if constexpr (GATED) {
      float g[E];
      ld8<T>(x + r * sx + H + c, g);
      if (b) {
        float bg[E];
        ld8<T>(b + H + c, bg);
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] += bg[e];
      }
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = act_f(act, a[e]) * g[e];
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = act_f(act, a[e]);
    }
    store_vec<T, E>(out + r * so + c, a);
  }
}

// dx from dout: non-gated dx = dout * act'(x + b); gated dxa = dout * g * act'(a), dxg = dout * act(a)
template <typename T, bool GATED>
__global__ __launch_bounds__(256) void bias_act_bwd(const T* __restrict__ x, const T* __restrict__ b,
                                                    const T* __restrict__ dout, T* __restrict__ dx, long rows, int H,
                                                    long sx, long sd, int act) {
  constexpr int E = 16 / sizeof(T);
  const int cv = H / E;
  for (long r = blockIdx.y; r < rows; r += gridDim.y)
  for (int vi = blockIdx.x * 256 + threadIdx.x; vi < cv; vi += gridDim.x * 256) {
    const int c = vi * E;
    float a[E], d[E];
    ld8<T>(x + r * sx + c, a);
    ld8<T>(dout + r * sd + c, d);
    if (b) {
      float bb[E];
      ld8<T>(b + c, bb);
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] += bb[e];
    }
    if constexpr (GATED) {
      float g[E], da[E], dg[E];
      ld8<T>(x + r * sx + H + c, g);
      if (b) {
        float bg[E];
        ld8<T>(b + H + c, bg);
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] += bg[e];
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        da[e] = d[e] * g[e] * act_grad(act, a[e]);
        dg[e] = d[e] * act_f(act, a[e]);
      }
      store_vec<T, E>(dx + r * sx + c, da);
      store_vec<T, E>(dx + r * sx + H + c, dg);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = d[e] * act_grad(act, a[e]);
      store_vec<T, E>(dx + r * sx + c, a);
    }
  }
}

// counter-based keep mask over the flat element index (64-bit), same hash family as flash-attention dropout
__device__ __forceinline__ bool keep_at(unsigned seed, unsigned long long idx, unsigned thresh) {
  unsigned x = seed ^ (unsigned)(idx >> 32) * 0x27D4EB2Du;
  x += (unsigned)idx * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  x *= 0x27D4EB2Fu;
  x ^= x >> 16;
  return x >= thresh;
}

// out = x * keep * scale + y (BWD: dx = dout * keep * scale, written to out; y unused)
template <typename T, bool BWD>
__global__ __launch_bounds__(256) void dropout_add_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                          T* __restrict__ out, long n, unsigned seed, unsigned thresh,
                                                          float scale) {
  constexpr int E = 16 / sizeof(T);
  const long nv = n / E;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float a[E];
    ld8<T>(x + i * E, a);
    float c[E];
    if constexpr (!BWD) ld8<T>(y + i * E, c);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float k = keep_at(seed, (unsigned long long)(i * E + e), thresh) ? scale : 0.f;
      a[e] = BWD ? a[e] * k : a[e] * k + c[e];
    }
    store_vec<T, E>(out + i * E, a);
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace fa2
}  // namespace pd

using namespace pd;

// gated: 0 plain (x [rows, H]), 1 gated (x [rows, 2H] -> out [rows, H]); H % (16/sizeof(T)) == 0
extern "C" int pd_bias_act(int dt, int gated, int act, const void* x, const void* b, void* out, long rows, int H,
                           long sx, long so, void* stream) {
  const int E = dt == kF32 ? 4 : 8;
  if (H % E || sx % E || so % E) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g = rowcol_grid(rows, H / E);
#define PD_BA(T)                                                                                                     \
  if (gated) fa2::bias_act_fwd<T, true><<<g, 256, 0, st>>>((const T*)x, (const T*)b, (T*)out, rows, H, sx, so, act); \
  else fa2::bias_act_fwd<T, false><<<g, 256, 0, st>>>((const T*)x, (const T*)b, (T*)out, rows, H, sx, so, act);
  if (dt == kBF16) { PD_BA(bf16) } else if (dt == kF16) { PD_BA(half16) } else if (dt == kF32) { PD_BA(float) }
  else return -2;
#undef PD_BA
  return (int)hipGetLastError();
}

extern "C" int pd_bias_act_bwd(int dt, int gated, int act, const void* x, const void* b, const void* dout, void* dx,
                               long rows, int H, long sx, long sd, void* stream) {
  const int E = dt == kF32 ? 4 : 8;
  if (H % E || sx % E || sd % E) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g = rowcol_grid(rows, H / E);
#define PD_BAB(T)                                                                                                  \
  if (gated)                                                                                                       \
    fa2::bias_act_bwd<T, true><<<g, 256, 0, st>>>((const T*)x, (const T*)b, (const T*)dout, (T*)dx, rows, H, sx, \
                                                  sd, act);                                                        \
  else                                                                                                             \
    fa2::bias_act_bwd<T, false><<<g, 256, 0, st>>>((const T*)x, (const T*)b, (const T*)dout, (T*)dx, rows, H,    \
                                                   sx, sd, act);
  if (dt == kBF16) { PD_BAB(bf16) } else if (dt == kF16) { PD_BAB(half16) } else if (dt == kF32) { PD_BAB(float) }
  else return -2;
#undef PD_BAB
  return (int)hipGetLastError();
}

// bwd = 0: out = dropout(x) + y; bwd = 1: out = dout * keep * scale (x = dout).  n % (16 / sizeof(T)) == 0.
extern "C" int pd_dropout_add(int dt, int bwd, const void* x, const void* y, void* out, long n, unsigned seed,
                              float p, void* stream) {
  const int E = dt == kF32 ? 4 : 8;
  if (n % E || !(p >= 0.f && p < 1.f)) return -1;
  const unsigned thresh = (unsigned)fminf(p * 4294967296.f, 4294967040.f);
  const float scale = 1.f / (1.f - p);
  hipStream_t st = (hipStream_t)stream;
  const int g = fa2::grid_for(n / E);
#define PD_DA(T)                                                                                                  \
  if (bwd) fa2::dropout_add_kernel<T, true><<<g, 256, 0, st>>>((const T*)x, nullptr, (T*)out, n, seed, thresh,  \
                                                               scale);                                           \
  else fa2::dropout_add_kernel<T, false><<<g, 256, 0, st>>>((const T*)x, (const T*)y, (T*)out, n, seed, thresh, \
                                                            scale);
  if (dt == kBF16) { PD_DA(bf16) } else if (dt == kF16) { PD_DA(half16) } else if (dt == kF32) { PD_DA(float) }
  else return -2;
#undef PD_DA
  return (int)hipGetLastError();
}
