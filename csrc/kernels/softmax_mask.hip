// Fused masked softmax for attention scores: softmax_mask_fuse (additive mask broadcast over heads) and
// softmax_mask_fuse_upper_triangle (causal), forward and backward.
//
// Reference behaviour: phi/kernels/fusion/gpu/fused_softmax_mask_kernel.cu (y = softmax(x + mask), mask
// [B, 1, Sq, Sk] shared by all heads, key length <= 8192) and
// fused_softmax_mask_upper_triangle_kernel.cu (column c > row r is masked, masked outputs are exactly 0);
// the grads are dx = y * (dy - sum(dy * y)) per row.
//
// MI355X design: a row of at most 8192 scores is 16 KB in bf16, so ONE wave64 owns one row and keeps it in
// VGPRs (W-element vector chunks, C chunks per lane): a single HBM read of x (and mask) and a single write
// of y, with the max and sum reductions done by DPP-style xor shuffles inside the wave — no LDS, no block
// barriers.  Four waves per 256-thread block handle four independent rows, so [B*H*Sq] rows give
// thousands of workgroups for the 256 CUs.  Backward reads y and dy once each and writes dx once.
#include "common.h"

namespace pd {

constexpr int kSMBlock = 256;
constexpr int kSMRows = kSMBlock / 64;

// MODE 0: additive mask [B, 1, Sq, Sk]; MODE 1: causal (col > row-in-sequence masked).
template <typename T, int W, int C, int MODE>
__global__ __launch_bounds__(kSMBlock) void softmax_mask_fwd_kernel(const T* __restrict__ x, const T* __restrict__ mask,
                                                                    T* __restrict__ y, long rows, int H, int Sq,
                                                                    int Sk) {
  const long row = (long)blockIdx.x * kSMRows + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole wave exits together
  const int lane = threadIdx.x & 63;
  const int r = (int)(row % Sq);
  const T* xr = x + row * Sk;
  const T* mr = nullptr;
  if constexpr (MODE == 0) mr = mask + ((row / ((long)H * Sq)) * Sq + r) * (long)Sk;
  float v[C][W];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int c0 = (k * 64 + lane) * W;
    if (c0 < Sk) {
      if constexpr (W > 1) {
        load_vec<T, W>(xr + c0, v[k]);
        if constexpr (MODE == 0) {
          float mv[W];
          load_vec<T, W>(mr + c0, mv);
#pragma unroll
          for (int j = 0; j < W; ++j) v[k][j] += mv[j];
        }
      } else {
        v[k][0] = Elt<T>::ld(xr + c0);
        if constexpr (MODE == 0) v[k][0] += Elt<T>::ld(mr + c0);
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (MODE == 1 && c0 + j > r) v[k][j] = -INFINITY;
        m = fmaxf(m, v[k][j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < W; ++j) v[k][j] = -INFINITY;
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < C; ++k)
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const float e = v[k][j] == -INFINITY ? 0.f : __expf(v[k][j] - m);
      v[k][j] = e;
      s += e;
    }
  const float inv = 1.f / wave_sum(s);
  T* yr = y + row * Sk;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int c0 = (k * 64 + lane) * W;
    if (c0 < Sk) {
#pragma unroll
      for (int j = 0; j < W; ++j) v[k][j] *= inv;
      if constexpr (W > 1) store_vec<T, W>(yr + c0, v[k]);
      else Elt<T>::st(yr + c0, v[k][0]);
    }
  }
}

template <typename T, int W, int C>
__global__ __launch_bounds__(kSMBlock) void softmax_mask_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                                    T* __restrict__ dx, long rows, int Sk) {
  const long row = (long)blockIdx.x * kSMRows + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const T* yr = y + row * Sk;
  const T* gr = dy + row * Sk;
  float yv[C][W], gv[C][W];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int c0 = (k * 64 + lane) * W;
    if (c0 < Sk) {
      if constexpr (W > 1) {
        load_vec<T, W>(yr + c0, yv[k]);
        load_vec<T, W>(gr + c0, gv[k]);
      } else {
        yv[k][0] = Elt<T>::ld(yr + c0);
        gv[k][0] = Elt<T>::ld(gr + c0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < W; ++j) { yv[k][j] = 0.f; gv[k][j] = 0.f; }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) dot += yv[k][j] * gv[k][j];
  }
  dot = wave_sum(dot);
  T* dr = dx + row * Sk;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int c0 = (k * 64 + lane) * W;
    if (c0 < Sk) {
#pragma unroll
      for (int j = 0; j < W; ++j) yv[k][j] = yv[k][j] * (gv[k][j] - dot);
      if constexpr (W > 1) store_vec<T, W>(dr + c0, yv[k]);
      else Elt<T>::st(dr + c0, yv[k][0]);
    }
  }
}

// Calls F.template operator()<W, C>() for the smallest power-of-two chunk count that covers Sk.
template <int W, int CMAX, typename F>
bool sm_dispatch_chunks(int Sk, const F& f) {
  const int need = (Sk + 64 * W - 1) / (64 * W);
  if (need <= 1) { f.template operator()<W, 1>(); return true; }
  if (need <= 2) { f.template operator()<W, 2>(); return true; }
  if (need <= 4) { f.template operator()<W, 4>(); return true; }
  if (need <= 8) { f.template operator()<W, 8>(); return true; }
  if constexpr (CMAX >= 16) if (need <= 16) { f.template operator()<W, 16>(); return true; }
  if constexpr (CMAX >= 32) if (need <= 32) { f.template operator()<W, 32>(); return true; }
  if constexpr (CMAX >= 64) if (need <= 64) { f.template operator()<W, 64>(); return true; }
  if constexpr (CMAX >= 128) if (need <= 128) { f.template operator()<W, 128>(); return true; }
  return false;
}

template <typename T, typename F>
bool sm_dispatch(int Sk, const F& f) {
  constexpr int VW = 16 / sizeof(T);
  if (Sk % VW == 0) return sm_dispatch_chunks<VW, 8192 / (64 * VW)>(Sk, f);
  return sm_dispatch_chunks<1, 128>(Sk, f);
}

template <typename T>
struct SMFwdLaunch {
  int causal; const T* x; const T* mask; T* y; long rows; int H, Sq, Sk; unsigned grid; hipStream_t st;
  template <int W, int C> void operator()() const {
    if (causal) softmax_mask_fwd_kernel<T, W, C, 1><<<grid, kSMBlock, 0, st>>>(x, nullptr, y, rows, H, Sq, Sk);
    else softmax_mask_fwd_kernel<T, W, C, 0><<<grid, kSMBlock, 0, st>>>(x, mask, y, rows, H, Sq, Sk);
  }
};

template <typename T>
struct SMBwdLaunch {
  const T* y; const T* dy; T* dx; long rows; int Sk; unsigned grid; hipStream_t st;
  template <int W, int C> void operator()() const {
    softmax_mask_bwd_kernel<T, W, C><<<grid, kSMBlock, 0, st>>>(y, dy, dx, rows, Sk);
  }
};

}  // namespace pd

using namespace pd;

extern "C" int pd_softmax_mask_fwd(int dt, int causal, const void* x, const void* mask, void* y, long rows, int H,
                                   int Sq, int Sk, void* stream) {
  if (Sk <= 0 || Sk > 8192 || rows <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((rows + kSMRows - 1) / kSMRows);
  bool ok = false;
  PD_DISPATCH_FLOAT(dt, T, ok = sm_dispatch<T>(Sk, SMFwdLaunch<T>{causal, (const T*)x, (const T*)mask, (T*)y, rows, H, Sq, Sk,
                                                                  grid, st}));
  if (!ok) return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

extern "C" int pd_softmax_mask_bwd(int dt, const void* y, const void* dy, void* dx, long rows, int Sk, void* stream) {
  if (Sk <= 0 || Sk > 8192 || rows <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((rows + kSMRows - 1) / kSMRows);
  bool ok = false;
  PD_DISPATCH_FLOAT(dt, T, ok = sm_dispatch<T>(Sk, SMBwdLaunch<T>{(const T*)y, (const T*)dy, (T*)dx, rows, Sk, grid, st}));
  if (!ok) return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
