// Shared device helpers for the paddle2_amd CDNA4 (gfx950) kernels.
//
// Conventions (see /opt/skills/guides/cdna_hip_programming.md):
//  * wave = 64 lanes; block sizes are multiples of 64;
//  * bf16/f16 are moved 16 bytes per lane (8 elements) — hipcc does not vectorise scalar
//    16-bit loads (Guideline 13);
//  * f32 -> bf16 uses the native __bf16 conversion (v_cvt_pk_bf16_f32, NaN-preserving).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pd {

typedef unsigned short bf16_raw;
typedef _Float16 f16;

using u16x8 = __attribute__((ext_vector_type(8))) unsigned short;
using f32x4 = __attribute__((ext_vector_type(4))) float;

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float(((unsigned)v) << 16); }

__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

__device__ __forceinline__ float h2f(unsigned short v) { return (float)__builtin_bit_cast(f16, v); }
__device__ __forceinline__ unsigned short f2h(float f) { return __builtin_bit_cast(unsigned short, (f16)f); }

// Element traits: T is the storage type in memory.
template <typename T> struct Elt;
template <> struct Elt<float> {
  static constexpr int kVec = 4;  // 16 bytes
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
struct bf16 { unsigned short x; };
struct half16 { unsigned short x; };
template <> struct Elt<bf16> {
  static constexpr int kVec = 8;
  __device__ __forceinline__ static float ld(const bf16* p) { return bf2f(p->x); }
  __device__ __forceinline__ static void st(bf16* p, float v) { p->x = f2bf(v); }
};
template <> struct Elt<half16> {
  static constexpr int kVec = 8;
  __device__ __forceinline__ static float ld(const half16* p) { return h2f(p->x); }
  __device__ __forceinline__ static void st(half16* p, float v) { p->x = f2h(v); }
};

// Load/store 16 bytes worth of T as floats (N = 16 / sizeof(T)).
template <typename T, int N>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&out)[N]) {
  static_assert(N * sizeof(T) == 16, "16-byte vectors");
  if constexpr (sizeof(T) == 4) {
    float4 v = *reinterpret_cast<const float4*>(p);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  } else {
    u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (std::is_same<T, bf16>::value) out[i] = bf2f(v[i]);
      else out[i] = h2f(v[i]);
    }
  }
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float (&in)[N]) {
  static_assert(N * sizeof(T) == 16, "16-byte vectors");
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  } else {
    u16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (std::is_same<T, bf16>::value) v[i] = f2bf(in[i]);
      else v[i] = f2h(in[i]);
    }
    *reinterpret_cast<u16x8*>(p) = v;
  }
}

// Round a float to storage type T and back (models the store/load of an intermediate).
template <typename T>
__device__ __forceinline__ float round_to(float v) {
  if constexpr (sizeof(T) == 4) return v;
  else if constexpr (std::is_same<T, bf16>::value) return bf2f(f2bf(v));
  else return h2f(f2h(v));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `smem` needs blockDim.x/64 floats. Result broadcast to all threads.
template <int BLOCK>
__device__ __forceinline__ float block_sum(float v, float* smem) {
  constexpr int W = BLOCK / 64;
  v = wave_sum(v);
  if constexpr (W == 1) return v;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < W; ++i) r += smem[i];
  return r;
}

template <int BLOCK>
__device__ __forceinline__ float block_max(float v, float* smem) {
  constexpr int W = BLOCK / 64;
  v = wave_max(v);
  if constexpr (W == 1) return v;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < W; ++i) r = fmaxf(r, smem[i]);
  return r;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }


// 2-D launch for row-wise elementwise kernels: x = blocks of 256 column vectors, y = row groups (rows strided by
// gridDim.y).  Replaces the flat grid-stride loop whose per-element 64-bit `i / vectors_per_row` division cost more
// VALU than the op itself (swiglu ran at ~5.2 TB/s).
static inline dim3 rowcol_grid(long rows, long nvec) {
  long gx = (nvec + 255) / 256;
  if (gx < 1) gx = 1;
  if (gx > 64) gx = 64;
  long gy = 8192 / gx;
  if (gy > rows) gy = rows;
  if (gy < 1) gy = 1;
  if (gy > 65535) gy = 65535;
  return dim3((unsigned)gx, (unsigned)gy);
}
}  // namespace pd

#define PD_DISPATCH_FLOAT(dt, T, ...)                 \
  switch (dt) {                                       \
    case pd::kF32: { using T = float; __VA_ARGS__; break; }     \
    case pd::kBF16: { using T = pd::bf16; __VA_ARGS__; break; } \
    case pd::kF16: { using T = pd::half16; __VA_ARGS__; break; }\
    default: break;                                   \
  }
