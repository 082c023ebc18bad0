// SwiGLU and rotary position embedding (fwd + bwd) for gfx950.
//
// Reference behaviour: phi/kernels/gpu/swiglu_kernel.cu (out = silu(x) * y; y optional ->
// split x in halves) and fusion/gpu/fused_rope_kernel.cu / fused_rope_utils.h (rotate-half and
// rotate-every-two styles, sin/cos tables, optional position_ids).
// MI355X design: memory-bound, so every lane moves 16 B per access, grid is capped at
// 256 CUs x 8 blocks and grid-strides (Guideline 11); RoPE reads cos/sin once per (s, d) tile
// and rotates all heads of q and k in the same block so the table stays in L1.
#include "common.h"

namespace pd {

__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// ------------------------------------------------------------------------------ SwiGLU
// x, y: [rows, H] with row strides sx, sy (elements) — for the packed form y = x + H.
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                         T* __restrict__ out, long rows, int H, long sx, long sy) {
  constexpr int V = 16 / sizeof(T);
  const int hv = H / V;
  // two rows per iteration: four independent 16-B loads in flight per lane before the first use
  for (long r = 2L * blockIdx.y; r < rows; r += 2L * gridDim.y) {
    const bool two = r + 1 < rows;
    for (int vi = blockIdx.x * 256 + threadIdx.x; vi < hv; vi += gridDim.x * 256) {
      const int c = vi * V;
      float a[V], b[V], a2[V], b2[V], o[V];
      load_vec<T, V>(x + r * sx + c, a);
      load_vec<T, V>(y + r * sy + c, b);
      if (two) {
        load_vec<T, V>(x + (r + 1) * sx + c, a2);
        load_vec<T, V>(y + (r + 1) * sy + c, b2);
      }
#pragma unroll
      for (int j = 0; j < V; ++j) o[j] = a[j] * sigmoidf_(a[j]) * b[j];
      store_vec<T, V>(out + r * H + c, o);
      if (two) {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = a2[j] * sigmoidf_(a2[j]) * b2[j];
        store_vec<T, V>(out + (r + 1) * H + c, o);
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                         const T* __restrict__ dout, T* __restrict__ dx,
                                                         T* __restrict__ dy, long rows, int H, long sx, long sy,
                                                         long sdx, long sdy) {
  constexpr int V = 16 / sizeof(T);
  const int hv = H / V;
  // two rows per iteration: six independent 16-B loads in flight per lane before the first use
  for (long r0 = 2L * blockIdx.y; r0 < rows; r0 += 2L * gridDim.y) {
    const int nr = r0 + 1 < rows ? 2 : 1;
    for (int vi = blockIdx.x * 256 + threadIdx.x; vi < hv; vi += gridDim.x * 256) {
      const int c = vi * V;
      float a[2][V], b[2][V], g[2][V];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k < nr) {
          const long r = r0 + k;
          load_vec<T, V>(x + r * sx + c, a[k]);
          load_vec<T, V>(y + r * sy + c, b[k]);
          load_vec<T, V>(dout + r * H + c, g[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k < nr) {
          const long r = r0 + k;
          float da[V], db[V];
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float s = sigmoidf_(a[k][j]);
            const float silu = a[k][j] * s;
            db[j] = g[k][j] * silu;
            da[j] = g[k][j] * b[k][j] * s * (1.f + a[k][j] * (1.f - s));
          }
          store_vec<T, V>(dx + r * sdx + c, da);
          store_vec<T, V>(dy + r * sdy + c, db);
        }
      }
    }
  }
}

static inline int ew_grid(long work) {
  long g = (work + 255) / 256;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

// ------------------------------------------------------------------------------ RoPE
// x: [B, S, Hn, D] (or time-major [S, B, Hn, D]); cos/sin: [S, D] fp32 (already expanded per
// style); pos: optional [B, S] int64 position ids. One thread handles one (token, head) x 8
// rotation pairs with 16-byte loads (D % 16 == 0 fast path; scalar path otherwise).
// STYLE 0 = rotate-half (front/back halves), 1 = rotate-every-two (adjacent pairs).
// BWD applies the transposed rotation (R^T = rotation by -theta with partner sines swapped).
__device__ __forceinline__ void rot8(const float (&xa)[8], const float (&xb)[8], const float (&ca)[8],
                                     const float (&cb)[8], const float (&sa)[8], const float (&sb)[8],
                                     float (&oa)[8], float (&ob)[8], bool bwd) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (!bwd) { oa[k] = xa[k] * ca[k] - xb[k] * sa[k]; ob[k] = xb[k] * cb[k] + xa[k] * sb[k]; }
    else { oa[k] = xa[k] * ca[k] + xb[k] * sb[k]; ob[k] = xb[k] * cb[k] - xa[k] * sa[k]; }
  }
}

__device__ __forceinline__ void ld8f(const float* p, float (&o)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&o)[8]) {
  if constexpr (sizeof(T) == 4) ld8f((const float*)p, o);
  else load_vec<T, 8>(p, o);
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&o)[8]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>((float*)p + 4) = make_float4(o[4], o[5], o[6], o[7]);
  } else store_vec<T, 8>(p, o);
}

template <typename T, int STYLE, bool BWD, bool VEC>
__global__ __launch_bounds__(256) void rope_kernel(const T* __restrict__ x, T* __restrict__ out,
                                                   const float* __restrict__ cosv, const float* __restrict__ sinv,
                                                   const int64_t* __restrict__ pos, int B, int S, int Hn, int D,
                                                   int time_major, long sx, long so) {
  // sx / so: elements between consecutive tokens of x / out (heads are D apart), so q/k can be
  // read straight out of a fused QKV projection and gradients written straight into dQKV.
  // one workgroup per token (grid-strided): threads cover its (head, 8-pair chunk) items, so the only integer
  // divisions are one 32-bit token split per token and one small head / chunk split per item (the flat 64-bit
  // `i % chunks`, `/ Hn`, `/ S` chain cost more VALU than the rotation itself)
  const int half = D / 2;
  const int chunks = (half + 7) / 8;
  const int per_tok = Hn * chunks;
  const unsigned ntok = (unsigned)B * (unsigned)S;
  for (unsigned tt = blockIdx.x; tt < ntok; tt += gridDim.x)
  for (int j = threadIdx.x; j < per_tok; j += 256) {
    const int h = j / chunks, ch = j - h * chunks;
    const long t = tt;  // token index in storage order
    int b, s;
    if (time_major) { s = (int)(tt / (unsigned)B); b = (int)(tt - (unsigned)s * (unsigned)B); }
    else { b = (int)(tt / (unsigned)S); s = (int)(tt - (unsigned)b * (unsigned)S); }
    const int p = pos ? (int)pos[(long)b * S + s] : s;
    const T* xr = x + t * sx + (long)h * D;
    T* orow = out + t * so + (long)h * D;
    const float* cr = cosv + (long)p * D;
    const float* sr = sinv + (long)p * D;
    if constexpr (VEC) {
      const int q0 = ch * 8;
      float xa[8], xb[8], ca[8], cb[8], sa[8], sb[8], oa[8], ob[8];
      if constexpr (STYLE == 0) {
        ld8<T>(xr + q0, xa); ld8<T>(xr + q0 + half, xb);
        ld8f(cr + q0, ca); ld8f(cr + q0 + half, cb); ld8f(sr + q0, sa); ld8f(sr + q0 + half, sb);
        rot8(xa, xb, ca, cb, sa, sb, oa, ob, BWD);
        st8<T>(orow + q0, oa); st8<T>(orow + q0 + half, ob);
      } else {
        float e0[8], e1[8], c0[8], c1[8], s0[8], s1[8];
        ld8<T>(xr + 2 * q0, e0); ld8<T>(xr + 2 * q0 + 8, e1);
        ld8f(cr + 2 * q0, c0); ld8f(cr + 2 * q0 + 8, c1); ld8f(sr + 2 * q0, s0); ld8f(sr + 2 * q0 + 8, s1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xa[k] = e0[2 * k]; xb[k] = e0[2 * k + 1]; xa[k + 4] = e1[2 * k]; xb[k + 4] = e1[2 * k + 1];
          ca[k] = c0[2 * k]; cb[k] = c0[2 * k + 1]; ca[k + 4] = c1[2 * k]; cb[k + 4] = c1[2 * k + 1];
          sa[k] = s0[2 * k]; sb[k] = s0[2 * k + 1]; sa[k + 4] = s1[2 * k]; sb[k + 4] = s1[2 * k + 1];
        }
        rot8(xa, xb, ca, cb, sa, sb, oa, ob, BWD);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          e0[2 * k] = oa[k]; e0[2 * k + 1] = ob[k]; e1[2 * k] = oa[k + 4]; e1[2 * k + 1] = ob[k + 4];
        }
        st8<T>(orow + 2 * q0, e0); st8<T>(orow + 2 * q0 + 8, e1);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = ch * 8 + k;
        if (q >= half) break;
        int ia, ib;
        if (STYLE == 0) { ia = q; ib = q + half; }
        else { ia = 2 * q; ib = 2 * q + 1; }
        const float xa = Elt<T>::ld(xr + ia), xb = Elt<T>::ld(xr + ib);
        const float ca = cr[ia], cb = cr[ib], sa = sr[ia], sb = sr[ib];
        float oa, ob;
        if (!BWD) { oa = xa * ca - xb * sa; ob = xb * cb + xa * sb; }
        else { oa = xa * ca + xb * sb; ob = xb * cb - xa * sa; }
        Elt<T>::st(orow + ia, oa);
        Elt<T>::st(orow + ib, ob);
      }
    }
  }
}


// ------------------------------------------------------------------------------ SwiGLU bwd + transposed dXY
// Packed gate|up input x [M, 2H] (row stride sx), upstream g [M, H] -> dxy [M, 2H] and dxyT [2H, M] (the
// weight-gradient GEMM of the gate_up projection wants dY with tokens contiguous: writing it here costs one
// extra 2-byte store per element instead of a separate read+write transpose pass).  One workgroup = a tile of
// 64 tokens x 64 features of both halves; the transposed tiles go through XOR-swizzled LDS images so the
// column gathers stay conflict-free and every wave-instruction stores whole 128-B runs of dxyT.
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const bf16* __restrict__ x, const bf16* __restrict__ g,
                                                           bf16* __restrict__ dxy, bf16* __restrict__ dxyT, long M,
                                                           int H, long sx, long tiles_h, long ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned short tl[2][64][64];  // [gate|up][token][feature]
  const int tid = threadIdx.x;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long r0 = (t / tiles_h) * 64;
    const int c0 = (int)(t % tiles_h) * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ch = tid + 256 * i;
      const int r = ch >> 3, c8 = ch & 7;
      const long row = r0 + r;
      const int col = c0 + c8 * 8;
      u16x8 og = u16x8{0, 0, 0, 0, 0, 0, 0, 0}, ou = og;
      if (row < M) {
        float a[8], b[8], gg[8], da[8], db[8];
        load_vec<bf16, 8>(x + row * sx + col, a);
        load_vec<bf16, 8>(x + row * sx + H + col, b);
        load_vec<bf16, 8>(g + row * H + col, gg);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sg = sigmoidf_(a[j]);
          db[j] = gg[j] * a[j] * sg;
          da[j] = gg[j] * b[j] * sg * (1.f + a[j] * (1.f - sg));
        }
        store_vec<bf16, 8>(dxy + row * 2 * H + col, da);
        store_vec<bf16, 8>(dxy + row * 2 * H + H + col, db);
#pragma unroll
        for (int j = 0; j < 8; ++j) { og[j] = f2bf(da[j]); ou[j] = f2bf(db[j]); }
      }
      const int sw = (c8 ^ ((r >> 3) & 7)) * 8;
      *reinterpret_cast<u16x8*>(&tl[0][r][sw]) = og;
      *reinterpret_cast<u16x8*>(&tl[1][r][sw]) = ou;
    }
    __syncthreads();
    // transposed: per half 64 feature rows x 8 chunks of 8 tokens; a wave stores 8 rows x 128 B
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = tid + 256 * i;
      const int half = ch >> 9, f = (ch >> 3) & 63, gq = ch & 7;  // feature f, tokens 8gq..8gq+8
      const int colsw = (((f >> 3) ^ gq) << 3) | (f & 7);
      u16x8 w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = tl[half][8 * gq + j][colsw];
      const long orow = (long)half * H + c0 + f, ocol = r0 + 8 * gq;
      if (ocol + 8 <= M) {
        *reinterpret_cast<u16x8*>(dxyT + orow * M + ocol) = w;
      } else {
        for (int j = 0; j < 8; ++j)
          if (ocol + j < M) reinterpret_cast<unsigned short*>(dxyT)[orow * M + ocol + j] = w[j];
      }
    }
    __syncthreads();
  }
}

}  // namespace pd

using namespace pd;

extern "C" int pd_swiglu_fwd(int dt, const void* x, const void* y, void* out, long rows, int H, long sx, long sy,
                             void* stream) {
  const int V = dt == kF32 ? 4 : 8;
  if (H % V) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g = rowcol_grid(rows, H / V);
  PD_DISPATCH_FLOAT(dt, T, swiglu_fwd_kernel<T><<<g, 256, 0, st>>>((const T*)x, (const T*)y, (T*)out, rows, H, sx, sy));
  return (int)hipGetLastError();
}

extern "C" int pd_swiglu_bwd(int dt, const void* x, const void* y, const void* dout, void* dx, void* dy, long rows,
                             int H, long sx, long sy, long sdx, long sdy, void* stream) {
  const int V = dt == kF32 ? 4 : 8;
  if (H % V) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g = rowcol_grid(rows, H / V);
  PD_DISPATCH_FLOAT(dt, T, swiglu_bwd_kernel<T><<<g, 256, 0, st>>>((const T*)x, (const T*)y, (const T*)dout, (T*)dx,
                                                                    (T*)dy, rows, H, sx, sy, sdx, sdy));
  return (int)hipGetLastError();
}

extern "C" int pd_swiglu_bwd_t(const void* x, const void* g, void* dxy, void* dxyT, long M, int H, long sx,
                               void* stream) {
  if (H % 64 || sx % 8) return -1;
  const long tiles_h = H / 64, ntiles = ((M + 63) / 64) * tiles_h;
  const long grid = ntiles < 256L * 16 ? ntiles : 256L * 16;
  swiglu_bwd_t_kernel<<<(int)grid, 256, 0, (hipStream_t)stream>>>((const bf16*)x, (const bf16*)g, (bf16*)dxy,
                                                                   (bf16*)dxyT, M, H, sx, tiles_h, ntiles);
  return (int)hipGetLastError();
}

extern "C" int pd_rope(int dt, int style, int bwd, const void* x, void* out, const float* cosv, const float* sinv,
                       const int64_t* pos, int B, int S, int Hn, int D, int time_major, long sx, long so,
                       void* stream) {
  if (D % 2) return -1;
  hipStream_t st = (hipStream_t)stream;
  const long ntok = (long)B * S;
  if (ntok >= (1L << 32)) return -1;
  const int g = (int)(ntok < 65536 ? (ntok < 1 ? 1 : ntok) : 65536);
  const int es = dt == kF32 ? 4 : 2;
  const bool vec = (D % 16) == 0 && ((sx * es) % 16) == 0 && ((so * es) % 16) == 0;
#define PD_ROPE1(T, SY, BW, VE) rope_kernel<T, SY, BW, VE><<<g, 256, 0, st>>>((const T*)x, (T*)out, cosv, sinv, pos, B, S, Hn, D, time_major, sx, so)
#define PD_ROPE(T)                                                                                    \
  if (vec) {                                                                                          \
    if (style == 0) { if (bwd) PD_ROPE1(T, 0, true, true); else PD_ROPE1(T, 0, false, true); }        \
    else { if (bwd) PD_ROPE1(T, 1, true, true); else PD_ROPE1(T, 1, false, true); }                   \
  } else {                                                                                            \
    if (style == 0) { if (bwd) PD_ROPE1(T, 0, true, false); else PD_ROPE1(T, 0, false, false); }      \
    else { if (bwd) PD_ROPE1(T, 1, true, false); else PD_ROPE1(T, 1, false, false); }                 \
  }
  PD_DISPATCH_FLOAT(dt, T, PD_ROPE(T));
#undef PD_ROPE
#undef PD_ROPE1
  return (int)hipGetLastError();
}
