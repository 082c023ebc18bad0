// Multi-tensor optimizer / AMP kernels for gfx950.
//
// Reference behaviour: phi/kernels/gpu/adamw_kernel.cu (per-parameter AdamW with lr_ratio,
// coeff, with_decay, multi_precision master weights, skip_update) and
// phi/kernels/gpu/fused_adam_kernel.cu (multi-tensor apply), gpu/amp_kernel.cu
// (check_finite_and_unscale), gpu/squared_l2_norm_kernel.cu.
//
// MI355X design: the reference launches ONE kernel PER PARAMETER (adamw.py:495).  Here a
// single persistent launch walks a device-resident tensor table: block b takes global chunks
// b, b+G, ... and binary-searches the chunk prefix to find its tensor.  The table is uploaded
// once per parameter set, per-step scalars travel as kernel args, so the whole optimizer step
// is 1 launch per dtype group (graph-capturable: no host sync, no per-step allocation).
// found_inf / inv_scale are device pointers so AMP unscale + skip fuse into the same pass.
#include "common.h"

namespace pd {

struct TensorMeta {
  void* p;          // param (PT)
  const void* g;    // grad (GT)
  float* m;         // moment1 (f32)
  float* v;         // moment2 (f32)
  float* master;    // f32 master weights or nullptr
  long n;
  float lr_ratio;
  float decay;      // weight-decay coeff for this tensor (0 = no decay)
};

constexpr int kOptBlock = 256;
constexpr int kChunk = kOptBlock * 8 * 4;  // elements per chunk

__device__ __forceinline__ int find_tensor(const long* __restrict__ prefix, int T, long c) {
  int lo = 0, hi = T;  // prefix[0]=0 ... prefix[T]=total; find t with prefix[t] <= c < prefix[t+1]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (prefix[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

template <typename GT>
__device__ __forceinline__ float ldg_(const void* g, long i) { return Elt<GT>::ld((const GT*)g + i); }

// 4 consecutive elements per lane per step (16 B of f32 state, 8 B of bf16 param/grad);
// every tensor pointer is 16-B aligned (checked on the host) and the <4 tail is scalar.
template <typename T>
__device__ __forceinline__ void ld4(const void* p, long i, float (&o)[4]) {
  if constexpr (sizeof(T) == 4) {
    float4 v = *reinterpret_cast<const float4*>((const float*)p + i);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    ushort4 v = *reinterpret_cast<const ushort4*>((const unsigned short*)p + i);
    o[0] = Elt<T>::ld((const T*)&v.x); o[1] = Elt<T>::ld((const T*)&v.y);
    o[2] = Elt<T>::ld((const T*)&v.z); o[3] = Elt<T>::ld((const T*)&v.w);
  }
}

template <typename T>
__device__ __forceinline__ void st4(void* p, long i, const float (&o)[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>((float*)p + i) = make_float4(o[0], o[1], o[2], o[3]);
  } else {
    T a, b, c, d;
    Elt<T>::st(&a, o[0]); Elt<T>::st(&b, o[1]); Elt<T>::st(&c, o[2]); Elt<T>::st(&d, o[3]);
    *reinterpret_cast<ushort4*>((unsigned short*)p + i) = make_ushort4(a.x, b.x, c.x, d.x);
  }
}

template <typename PT, typename GT, bool MASTER>
__global__ __launch_bounds__(kOptBlock) void adamw_mt_kernel(const TensorMeta* __restrict__ meta,
                                                             const long* __restrict__ prefix, int T,
                                                             float lr, float beta1, float beta2, float eps,
                                                             float bc1, float bc2, const float* __restrict__ found_inf,
                                                             const float* __restrict__ inv_scale, int amsgrad_unused) {
  if (found_inf && *found_inf != 0.f) return;  // skip_update (AMP found inf/nan)
  const float iscale = inv_scale ? *inv_scale : 1.f;
  const long total = prefix[T];
  const float sbc2 = sqrtf(bc2);
  for (long c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(prefix, T, c);
    const TensorMeta mt = meta[t];
    const long base = (c - prefix[t]) * (long)kChunk;
    const float lr_t = lr * mt.lr_ratio;
    const float step = lr_t / bc1;
    const float wd = 1.f - lr_t * mt.decay;
#pragma unroll 2
    for (int it = 0; it < kChunk / (kOptBlock * 4); ++it) {
      const long i = base + ((long)it * kOptBlock + threadIdx.x) * 4;
      if (i >= mt.n) break;
      if (i + 4 <= mt.n) {
        float g[4], p[4], m[4], v[4];
        ld4<GT>(mt.g, i, g);
        if (MASTER) ld4<float>(mt.master, i, p); else ld4<PT>(mt.p, i, p);
        ld4<float>(mt.m, i, m);
        ld4<float>(mt.v, i, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gj = g[j] * iscale;
          m[j] = beta1 * m[j] + (1.f - beta1) * gj;
          v[j] = beta2 * v[j] + (1.f - beta2) * gj * gj;
          p[j] = p[j] * wd - step * m[j] / (sqrtf(v[j]) / sbc2 + eps);
        }
        st4<float>(mt.m, i, m);
        st4<float>(mt.v, i, v);
        if (MASTER) st4<float>(mt.master, i, p);
        st4<PT>(mt.p, i, p);
      } else {
        for (long k = i; k < mt.n; ++k) {
          const float g = ldg_<GT>(mt.g, k) * iscale;
          float p = MASTER ? mt.master[k] : Elt<PT>::ld((const PT*)mt.p + k);
          float m = beta1 * mt.m[k] + (1.f - beta1) * g;
          float v = beta2 * mt.v[k] + (1.f - beta2) * g * g;
          p = p * wd - step * m / (sqrtf(v) / sbc2 + eps);
          mt.m[k] = m; mt.v[k] = v;
          if (MASTER) mt.master[k] = p;
          Elt<PT>::st((PT*)mt.p + k, p);
        }
      }
    }
  }
}

// ---- check_finite_and_unscale: g *= inv_scale in place; found_inf |= !isfinite(g)
template <typename GT>
__global__ __launch_bounds__(kOptBlock) void unscale_mt_kernel(const TensorMeta* __restrict__ meta,
                                                               const long* __restrict__ prefix, int T,
                                                               const float* __restrict__ scale,
                                                               float* __restrict__ found_inf) {
  const long total = prefix[T];
  const float iscale = 1.f / *scale;
  bool bad = false;
  for (long c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(prefix, T, c);
    const TensorMeta mt = meta[t];
    const long base = (c - prefix[t]) * (long)kChunk;
    GT* g = (GT*)mt.g;
    for (int it = 0; it < kChunk / kOptBlock; ++it) {
      const long i = base + it * kOptBlock + threadIdx.x;
      if (i >= mt.n) break;
      const float v = Elt<GT>::ld(g + i) * iscale;
      bad |= !isfinite(v);
      Elt<GT>::st(g + i, v);
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicExch(found_inf, 1.f);
}

// ---- sum of squares over all tensors' grads -> out (f32, accumulated with one atomic per wave)
template <typename GT>
__global__ __launch_bounds__(kOptBlock) void sqnorm_mt_kernel(const TensorMeta* __restrict__ meta,
                                                              const long* __restrict__ prefix, int T,
                                                              float* __restrict__ out) {
  const long total = prefix[T];
  float acc = 0.f;
  for (long c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(prefix, T, c);
    const TensorMeta mt = meta[t];
    const long base = (c - prefix[t]) * (long)kChunk;
#pragma unroll 2
    for (int it = 0; it < kChunk / (kOptBlock * 4); ++it) {
      const long i = base + ((long)it * kOptBlock + threadIdx.x) * 4;
      if (i >= mt.n) break;
      if (i + 4 <= mt.n) {
        float v[4];
        ld4<GT>(mt.g, i, v);
        acc += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      } else {
        for (long k = i; k < mt.n; ++k) { const float v = ldg_<GT>(mt.g, k); acc += v * v; }
      }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

// ---- g *= coef (clip-by-global-norm apply); coef from device pointer (no host sync)
template <typename GT>
__global__ __launch_bounds__(kOptBlock) void scale_mt_kernel(const TensorMeta* __restrict__ meta,
                                                             const long* __restrict__ prefix, int T,
                                                             const float* __restrict__ coef) {
  const long total = prefix[T];
  const float s = *coef;
  for (long c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(prefix, T, c);
    const TensorMeta mt = meta[t];
    const long base = (c - prefix[t]) * (long)kChunk;
    GT* g = (GT*)mt.g;
    for (int it = 0; it < kChunk / kOptBlock; ++it) {
      const long i = base + it * kOptBlock + threadIdx.x;
      if (i >= mt.n) break;
      Elt<GT>::st(g + i, Elt<GT>::ld(g + i) * s);
    }
  }
}

// ---- dynamic loss scaling update (reference: gpu/amp_kernel.cu GpuUpdateLossScaling)
__global__ void update_loss_scaling_kernel(const float* found_inf, float* scale, int* good, int* bad,
                                           int incr_every_n, int decr_every_n_nan_or_inf, float incr_ratio,
                                           float decr_ratio) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (*found_inf != 0.f) {
    *good = 0;
    *bad += 1;
    if (*bad == decr_every_n_nan_or_inf) {
      float ns = *scale * decr_ratio;
      *scale = ns < 1.f ? 1.f : ns;
      *bad = 0;
    }
  } else {
    *bad = 0;
    *good += 1;
    if (*good == incr_every_n) {
      float ns = *scale * incr_ratio;
      if (isfinite(ns)) *scale = ns;
      *good = 0;
    }
  }
}

}  // namespace pd

using namespace pd;

static int opt_grid(long chunks) {
  long g = chunks < 2048 ? chunks : 2048;  // 256 CUs x 8 resident blocks
  return (int)(g < 1 ? 1 : g);
}

extern "C" int pd_opt_chunk_size() { return kChunk; }
extern "C" int pd_opt_meta_bytes() { return (int)sizeof(TensorMeta); }

extern "C" int pd_adamw_mt(int pdt, int gdt, int master, const void* meta, const long* prefix, int T, long chunks,
                           float lr, float beta1, float beta2, float eps, float bc1, float bc2,
                           const float* found_inf, const float* inv_scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = opt_grid(chunks);
  const TensorMeta* m = (const TensorMeta*)meta;
#define PD_ADAM(PT, GT, MA) adamw_mt_kernel<PT, GT, MA><<<g, kOptBlock, 0, st>>>(m, prefix, T, lr, beta1, beta2, eps, bc1, bc2, found_inf, inv_scale, 0)
  if (pdt == kF32 && gdt == kF32) PD_ADAM(float, float, false);
  else if (pdt == kBF16 && gdt == kBF16) { if (master) PD_ADAM(bf16, bf16, true); else PD_ADAM(bf16, bf16, false); }
  else if (pdt == kBF16 && gdt == kF32) { if (master) PD_ADAM(bf16, float, true); else PD_ADAM(bf16, float, false); }
  else if (pdt == kF16 && gdt == kF16) { if (master) PD_ADAM(half16, half16, true); else PD_ADAM(half16, half16, false); }
  else if (pdt == kF16 && gdt == kF32) { if (master) PD_ADAM(half16, float, true); else PD_ADAM(half16, float, false); }
  else if (pdt == kF32 && gdt == kBF16) PD_ADAM(float, bf16, false);
  else return -1;
#undef PD_ADAM
  return (int)hipGetLastError();
}

extern "C" int pd_unscale_mt(int gdt, const void* meta, const long* prefix, int T, long chunks, const float* scale,
                             float* found_inf, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = opt_grid(chunks);
  PD_DISPATCH_FLOAT(gdt, GT, unscale_mt_kernel<GT><<<g, kOptBlock, 0, st>>>((const TensorMeta*)meta, prefix, T, scale, found_inf));
  return (int)hipGetLastError();
}

extern "C" int pd_sqnorm_mt(int gdt, const void* meta, const long* prefix, int T, long chunks, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = opt_grid(chunks);
  PD_DISPATCH_FLOAT(gdt, GT, sqnorm_mt_kernel<GT><<<g, kOptBlock, 0, st>>>((const TensorMeta*)meta, prefix, T, out));
  return (int)hipGetLastError();
}

extern "C" int pd_scale_mt(int gdt, const void* meta, const long* prefix, int T, long chunks, const float* coef,
                           void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = opt_grid(chunks);
  PD_DISPATCH_FLOAT(gdt, GT, scale_mt_kernel<GT><<<g, kOptBlock, 0, st>>>((const TensorMeta*)meta, prefix, T, coef));
  return (int)hipGetLastError();
}

extern "C" int pd_update_loss_scaling(const float* found_inf, float* scale, int* good, int* bad, int incr_every_n,
                                      int decr_every_n, float incr_ratio, float decr_ratio, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  update_loss_scaling_kernel<<<1, 64, 0, st>>>(found_inf, scale, good, bad, incr_every_n, decr_every_n, incr_ratio,
                                                decr_ratio);
  return (int)hipGetLastError();
}
