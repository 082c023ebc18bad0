// RMSNorm / LayerNorm forward + backward for gfx950.
//
// Reference behaviour: phi/kernels/gpu/rms_norm_kernel.cu (RmsNormBlockSMemImpl, residual
// fusion) and funcs/layer_norm_impl.cu.h.  Design here is MI355X-first:
//  * one 64-lane wave per row (no __syncthreads in the row reduction), 4 rows per 256-thread
//    block, row cached in VGPRs (MAXV x 16 B per lane) so x is read from HBM exactly once;
//  * 16-byte vector loads/stores for bf16/f16/f32;
//  * backward is a persistent grid-stride over rows (one 256-thread block per row); each block
//    keeps its dW/dB partials in registers across rows and writes one fp32 partial row at the
//    end; a second tiny kernel reduces the partials (no float atomics: deterministic and not
//    bound by the chip-wide float-atomic rate).
#include "common.h"

namespace pd {

constexpr int kNormBlock = 256;            // 4 waves
constexpr int kRowsPerBlock = kNormBlock / 64;

// ------------------------------------------------------------------------------------ fwd
template <typename T, typename WT, int MAXV, bool LAYERNORM, bool HAS_RES, bool HAS_BIAS>
__global__ __launch_bounds__(kNormBlock) void norm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const WT* __restrict__ w, const WT* __restrict__ b,
    T* __restrict__ y, T* __restrict__ res_out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int M, int N, float eps) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = N / V;
  const long off = (long)row * N;
  float buf[MAXV][V];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + k * 64;
    if (vi < nv) {
      load_vec<T, V>(x + off + vi * V, buf[k]);
      if constexpr (HAS_RES) {
        float r[V];
        load_vec<T, V>(res + off + vi * V, r);
#pragma unroll
        for (int j = 0; j < V; ++j) buf[k][j] += r[j];
        store_vec<T, V>(res_out + off + vi * V, buf[k]);
        // normalise the *rounded* h so forward and backward (which re-reads h) agree
#pragma unroll
        for (int j = 0; j < V; ++j) buf[k][j] = round_to<T>(buf[k][j]);
      }
#pragma unroll
      for (int j = 0; j < V; ++j) s += LAYERNORM ? buf[k][j] : buf[k][j] * buf[k][j];
    }
  }
  float mu = 0.f, rstd;
  if constexpr (LAYERNORM) {
    mu = wave_sum(s) / N;
    float v2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = lane + k * 64;
      if (vi < nv) {
#pragma unroll
        for (int j = 0; j < V; ++j) { float d = buf[k][j] - mu; v2 += d * d; }
      }
    }
    rstd = rsqrtf(wave_sum(v2) / N + eps);
  } else {
    rstd = rsqrtf(wave_sum(s) / N + eps);
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + k * 64;
    if (vi < nv) {
      constexpr int WV = 16 / sizeof(WT);
      float wv[V], bv[V];
      if constexpr (WV == V) {
        load_vec<WT, V>(w + vi * V, wv);
        if constexpr (HAS_BIAS) load_vec<WT, V>(b + vi * V, bv);
      } else {  // fp32 weight with 16-bit activations: two 16 B loads
        float t0[4], t1[4];
        load_vec<WT, 4>(w + vi * V, t0); load_vec<WT, 4>(w + vi * V + 4, t1);
#pragma unroll
        for (int j = 0; j < 4; ++j) { wv[j] = t0[j]; wv[j + 4] = t1[j]; }
        if constexpr (HAS_BIAS) {
          load_vec<WT, 4>(b + vi * V, t0); load_vec<WT, 4>(b + vi * V + 4, t1);
#pragma unroll
          for (int j = 0; j < 4; ++j) { bv[j] = t0[j]; bv[j + 4] = t1[j]; }
        }
      }
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        o[j] = (buf[k][j] - mu) * rstd * wv[j];
        if constexpr (HAS_BIAS) o[j] += bv[j];
      }
      store_vec<T, V>(y + off + vi * V, o);
    }
  }
  if (lane == 0) {
    rstd_out[row] = rstd;
    if constexpr (LAYERNORM) mean_out[row] = mu;
  }
}

// ------------------------------------------------------------------------------------ bwd
// dx = rstd * (g - xhat*mean(g*xhat) [- mean(g) for LN]),  g = dy*w
// One 256-thread block per row (persistent over rows): per-thread register footprint stays
// at ~4 x MAXV x V floats, so N=4096 bf16 needs MAXV=2 (no spills at any N <= 16K).
template <typename T, typename WT, int MAXV, bool LAYERNORM, bool HAS_DRES>
__global__ __launch_bounds__(kNormBlock) void norm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const WT* __restrict__ w,
    const float* __restrict__ mean, const float* __restrict__ rstd, const T* __restrict__ dres,
    T* __restrict__ dx, float* __restrict__ dw_part, float* __restrict__ db_part, int M, int N) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float red[2 * kRowsPerBlock];
  const int tid = threadIdx.x;
  const int nv = N / V;
  float wreg[MAXV][V];
  float dwacc[MAXV][V];
  float dbacc[MAXV][V];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = tid + k * kNormBlock;
#pragma unroll
    for (int j = 0; j < V; ++j) { dwacc[k][j] = 0.f; dbacc[k][j] = 0.f; wreg[k][j] = 0.f; }
    if (vi < nv) {
      constexpr int WV = 16 / sizeof(WT);
      if constexpr (WV == V) load_vec<WT, V>(w + vi * V, wreg[k]);
      else {
        float t0[4], t1[4];
        load_vec<WT, 4>(w + vi * V, t0); load_vec<WT, 4>(w + vi * V + 4, t1);
#pragma unroll
        for (int j = 0; j < 4; ++j) { wreg[k][j] = t0[j]; wreg[k][j + 4] = t1[j]; }
      }
    }
  }
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const long off = (long)row * N;
    const float r = rstd[row];
    const float mu = LAYERNORM ? mean[row] : 0.f;
    float xh[MAXV][V], g[MAXV][V];
    float dr[HAS_DRES ? MAXV : 1][V];   // the residual-branch gradient, loaded with dy / x (not after the reduction)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = tid + k * kNormBlock;
      if (vi < nv) {
        float dyv[V];
        load_vec<T, V>(dy + off + vi * V, dyv);
        load_vec<T, V>(x + off + vi * V, xh[k]);
        if constexpr (HAS_DRES) load_vec<T, V>(dres + off + vi * V, dr[k]);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          xh[k][j] = (xh[k][j] - mu) * r;
          g[k][j] = dyv[j] * wreg[k][j];
          s1 += g[k][j] * xh[k][j];
          dwacc[k][j] += dyv[j] * xh[k][j];
          if constexpr (LAYERNORM) { s2 += g[k][j]; dbacc[k][j] += dyv[j]; }
        }
      }
    }
    // block reduction of (s1, s2) in one LDS round trip
    s1 = wave_sum(s1);
    if constexpr (LAYERNORM) s2 = wave_sum(s2);
    __syncthreads();
    if ((tid & 63) == 0) { red[tid >> 6] = s1; red[kRowsPerBlock + (tid >> 6)] = s2; }
    __syncthreads();
    s1 = 0.f; s2 = 0.f;
#pragma unroll
    for (int i = 0; i < kRowsPerBlock; ++i) { s1 += red[i]; s2 += red[kRowsPerBlock + i]; }
    s1 /= N; s2 /= N;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = tid + k * kNormBlock;
      if (vi < nv) {
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = r * (g[k][j] - xh[k][j] * s1 - (LAYERNORM ? s2 : 0.f));
        if constexpr (HAS_DRES) {
#pragma unroll
          for (int j = 0; j < V; ++j) o[j] += dr[k][j];
        }
        store_vec<T, V>(dx + off + vi * V, o);
      }
    }
  }
  // one fp32 partial row per block
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = tid + k * kNormBlock;
    if (vi < nv) {
      float* dst = dw_part + (long)blockIdx.x * N + vi * V;
#pragma unroll
      for (int j = 0; j < V; j += 4)
        *reinterpret_cast<float4*>(dst + j) = make_float4(dwacc[k][j], dwacc[k][j + 1], dwacc[k][j + 2], dwacc[k][j + 3]);
      if constexpr (LAYERNORM) {
        float* dsb = db_part + (long)blockIdx.x * N + vi * V;
#pragma unroll
        for (int j = 0; j < V; j += 4)
          *reinterpret_cast<float4*>(dsb + j) = make_float4(dbacc[k][j], dbacc[k][j + 1], dbacc[k][j + 2], dbacc[k][j + 3]);
      }
    }
  }
}

// Reduce P partial rows [P, N] (fp32) into out [N] (type WT). Block = 16 column-quads (64 columns)
// x 16 row lanes; each lane streams P/16 rows with 16-B loads, then one LDS reduction. Deterministic
// (fixed summation order) and ~P/16 loads in flight per lane instead of a serial P-long chain.
template <typename WT>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, WT* __restrict__ out, int P, int N,
                                                     int accumulate) {
  __shared__ float4 red[16][16];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = (blockIdx.x * 16 + cq) * 4;
  float4 acc = make_float4(0, 0, 0, 0);
  if (c < N) {
#pragma unroll 8
    for (int p = rl; p < P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)p * N + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[rl][cq] = acc;
  __syncthreads();
  if (rl == 0 && c < N) {
    float4 s = red[0][cq];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      const float4 v = red[i][cq];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (accumulate) {   // out += sum: a gradient accumulated into its fp32 main-grad slot
      s.x += Elt<WT>::ld(out + c); s.y += Elt<WT>::ld(out + c + 1);
      s.z += Elt<WT>::ld(out + c + 2); s.w += Elt<WT>::ld(out + c + 3);
    }
    Elt<WT>::st(out + c, s.x); Elt<WT>::st(out + c + 1, s.y);
    Elt<WT>::st(out + c + 2, s.z); Elt<WT>::st(out + c + 3, s.w);
  }
}

// Few rows (the serving decode step, M <= 64): one workgroup per row, its 4 waves splitting the row (vector vi of
// thread tid: tid + 256 k) with an LDS sum across the waves.  The one-wave-per-row kernel above leaves a single wave
// walking 8 dependent-issue vectors per lane at M = 1 (9 us per call in the b1 decode trace).
__device__ __forceinline__ float block_sum4(float v, float* sm) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  const float t = sm[0] + sm[1] + sm[2] + sm[3];
  __syncthreads();
  return t;
}

// PART (decode, bf16): x is not a tensor but the S fp32 split-K partials [S, M, N] of the decode GEMM that produced it
// (pd_dec_gemm noreduce): summed here in split order and rounded to T — exactly wo_reduce_kernel's bf16 output, so the
// reduce launch between the projection and its residual-add + norm disappears
template <typename T, typename WT, int MAXV, bool LAYERNORM, bool HAS_RES, bool HAS_BIAS, bool PART = false>
__global__ __launch_bounds__(kNormBlock) void norm_fwd_row_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const WT* __restrict__ w, const WT* __restrict__ b,
    T* __restrict__ y, T* __restrict__ res_out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int M, int N, float eps, const float* __restrict__ part = nullptr, int S = 0) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float sm[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int nv = N / V;
  const long off = (long)row * N;
  float buf[MAXV][V];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = tid + k * kNormBlock;
    if (vi < nv) {
      if constexpr (PART) {
        static_assert(V == 8, "PART: 16-bit rows");
        const float* p0 = part + off + vi * V;
        float4 a0 = *reinterpret_cast<const float4*>(p0), a1 = *reinterpret_cast<const float4*>(p0 + 4);
#pragma unroll 8
        for (int sp = 1; sp < S; ++sp) {
          const float* ps = p0 + (long)sp * M * N;
          const float4 b0 = *reinterpret_cast<const float4*>(ps), b1 = *reinterpret_cast<const float4*>(ps + 4);
          a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
          a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
        }
        const float t[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) buf[k][j] = round_to<T>(t[j]);
      } else {
        load_vec<T, V>(x + off + vi * V, buf[k]);
      }
      if constexpr (HAS_RES) {
        float r[V];
        load_vec<T, V>(res + off + vi * V, r);
#pragma unroll
        for (int j = 0; j < V; ++j) buf[k][j] += r[j];
        store_vec<T, V>(res_out + off + vi * V, buf[k]);
#pragma unroll
        for (int j = 0; j < V; ++j) buf[k][j] = round_to<T>(buf[k][j]);
      }
#pragma unroll
      for (int j = 0; j < V; ++j) s += LAYERNORM ? buf[k][j] : buf[k][j] * buf[k][j];
    }
  }
  float mu = 0.f, rstd;
  if constexpr (LAYERNORM) {
    mu = block_sum4(s, sm) / N;
    float v2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      if (tid + k * kNormBlock < nv) {
#pragma unroll
        for (int j = 0; j < V; ++j) { const float d = buf[k][j] - mu; v2 += d * d; }
      }
    }
    rstd = rsqrtf(block_sum4(v2, sm) / N + eps);
  } else {
    rstd = rsqrtf(block_sum4(s, sm) / N + eps);
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = tid + k * kNormBlock;
    if (vi < nv) {
      constexpr int WV = 16 / sizeof(WT);
      float wv[V], bv[V];
      if constexpr (WV == V) {
        load_vec<WT, V>(w + vi * V, wv);
        if constexpr (HAS_BIAS) load_vec<WT, V>(b + vi * V, bv);
      } else {
        float t0[4], t1[4];
        load_vec<WT, 4>(w + vi * V, t0); load_vec<WT, 4>(w + vi * V + 4, t1);
#pragma unroll
        for (int j = 0; j < 4; ++j) { wv[j] = t0[j]; wv[j + 4] = t1[j]; }
        if constexpr (HAS_BIAS) {
          load_vec<WT, 4>(b + vi * V, t0); load_vec<WT, 4>(b + vi * V + 4, t1);
#pragma unroll
          for (int j = 0; j < 4; ++j) { bv[j] = t0[j]; bv[j + 4] = t1[j]; }
        }
      }
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        o[j] = (buf[k][j] - mu) * rstd * wv[j];
        if constexpr (HAS_BIAS) o[j] += bv[j];
      }
      store_vec<T, V>(y + off + vi * V, o);
    }
  }
  if (tid == 0) {
    if (mean_out) mean_out[row] = mu;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// ------------------------------------------------------------------------------------ host
template <typename T, typename WT, bool LN>
static void fwd_launch(const void* x, const void* res, const void* w, const void* b, void* y, void* res_out,
                       float* mean, float* rstd, int M, int N, float eps, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const int nv = N / V;
  const int maxv = (nv + 63) / 64;
  dim3 grid(ceil_div(M, kRowsPerBlock)), block(kNormBlock);
#define PD_NORM_FWD(MV)                                                                                      \
  if (res) {                                                                                                 \
    if (b) norm_fwd_kernel<T, WT, MV, LN, true, true><<<grid, block, 0, st>>>((const T*)x, (const T*)res,   \
             (const WT*)w, (const WT*)b, (T*)y, (T*)res_out, mean, rstd, M, N, eps);                         \
    else norm_fwd_kernel<T, WT, MV, LN, true, false><<<grid, block, 0, st>>>((const T*)x, (const T*)res,    \
             (const WT*)w, (const WT*)b, (T*)y, (T*)res_out, mean, rstd, M, N, eps);                         \
  } else {                                                                                                   \
    if (b) norm_fwd_kernel<T, WT, MV, LN, false, true><<<grid, block, 0, st>>>((const T*)x, nullptr,        \
             (const WT*)w, (const WT*)b, (T*)y, nullptr, mean, rstd, M, N, eps);                             \
    else norm_fwd_kernel<T, WT, MV, LN, false, false><<<grid, block, 0, st>>>((const T*)x, nullptr,         \
             (const WT*)w, (const WT*)b, (T*)y, nullptr, mean, rstd, M, N, eps);                             \
  }
  const int maxr = (nv + kNormBlock - 1) / kNormBlock;
  // few rows: a workgroup per row (PADDLE2_AMD_NORM_ROW_MAXM, default 64; 0 = off)
  static const int row_maxm = getenv("PADDLE2_AMD_NORM_ROW_MAXM") ? atoi(getenv("PADDLE2_AMD_NORM_ROW_MAXM")) : 64;
  if (M <= row_maxm && maxr <= 4) {
    dim3 grow(M);
#define PD_NORM_FWD_ROW(MV)                                                                                  \
    if (res) {                                                                                               \
      if (b) norm_fwd_row_kernel<T, WT, MV, LN, true, true><<<grow, block, 0, st>>>((const T*)x,            \
               (const T*)res, (const WT*)w, (const WT*)b, (T*)y, (T*)res_out, mean, rstd, M, N, eps);        \
      else norm_fwd_row_kernel<T, WT, MV, LN, true, false><<<grow, block, 0, st>>>((const T*)x,             \
               (const T*)res, (const WT*)w, (const WT*)b, (T*)y, (T*)res_out, mean, rstd, M, N, eps);        \
    } else {                                                                                                 \
      if (b) norm_fwd_row_kernel<T, WT, MV, LN, false, true><<<grow, block, 0, st>>>((const T*)x, nullptr,  \
               (const WT*)w, (const WT*)b, (T*)y, nullptr, mean, rstd, M, N, eps);                           \
      else norm_fwd_row_kernel<T, WT, MV, LN, false, false><<<grow, block, 0, st>>>((const T*)x, nullptr,   \
               (const WT*)w, (const WT*)b, (T*)y, nullptr, mean, rstd, M, N, eps);                           \
    }
    if (maxr <= 1) { PD_NORM_FWD_ROW(1) }
    else if (maxr <= 2) { PD_NORM_FWD_ROW(2) }
    else { PD_NORM_FWD_ROW(4) }
#undef PD_NORM_FWD_ROW
  } else if (maxv <= 1) { PD_NORM_FWD(1) }
  else if (maxv <= 2) { PD_NORM_FWD(2) }
  else if (maxv <= 4) { PD_NORM_FWD(4) }
  else if (maxv <= 8) { PD_NORM_FWD(8) }
  else { PD_NORM_FWD(16) }
#undef PD_NORM_FWD
}

// colsum_kernel with the output dtype chosen at run time (a parameter's own dtype, or fp32 for its main-grad slot)
static void colsum_to(int odt, const float* part, void* out, int P, int N, int acc, hipStream_t st) {
  dim3 g2(ceil_div(N, 64));
  if (odt == kBF16) colsum_kernel<bf16><<<g2, 256, 0, st>>>(part, (bf16*)out, P, N, acc);
  else if (odt == kF16) colsum_kernel<half16><<<g2, 256, 0, st>>>(part, (half16*)out, P, N, acc);
  else colsum_kernel<float><<<g2, 256, 0, st>>>(part, (float*)out, P, N, acc);
}

template <typename T, typename WT, bool LN>
static void bwd_launch(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                       const void* dres, void* dx, float* dw_part, float* db_part, void* dw, void* db,
                       int M, int N, int nblocks, int odt, int acc_w, int acc_b, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const int nv = N / V;
  const int maxv = (nv + kNormBlock - 1) / kNormBlock;
  dim3 grid(nblocks), block(kNormBlock);
#define PD_NORM_BWD(MV)                                                                                     \
  if (dres) norm_bwd_kernel<T, WT, MV, LN, true><<<grid, block, 0, st>>>((const T*)dy, (const T*)x,        \
        (const WT*)w, mean, rstd, (const T*)dres, (T*)dx, dw_part, db_part, M, N);                          \
  else norm_bwd_kernel<T, WT, MV, LN, false><<<grid, block, 0, st>>>((const T*)dy, (const T*)x,            \
        (const WT*)w, mean, rstd, nullptr, (T*)dx, dw_part, db_part, M, N);
  if (maxv <= 1) { PD_NORM_BWD(1) }
  else if (maxv <= 2) { PD_NORM_BWD(2) }
  else if (maxv <= 4) { PD_NORM_BWD(4) }
  else { PD_NORM_BWD(4) }
#undef PD_NORM_BWD
  colsum_to(odt, dw_part, dw, nblocks, N, acc_w, st);
  if (db_part) colsum_to(odt, db_part, db, nblocks, N, acc_b, st);
}

// Bias gradient db[n] = sum_m dy[m, n] (reference: the bias-grad reduction of fused_gemm_epilogue_grad /
// matmul_with_bias backward).  Pass 1: workgroup (column block of 512, row chunk) — each wave streams every 4th
// row of the chunk with one 16-B load per lane (a wave reads 1 KiB of a row: full cachelines), fp32 sums, one LDS
// reduction over the 4 waves, fp32 partial row [chunk, N].  Pass 2: colsum_kernel over the chunks (fixed order:
// deterministic).  Grid = ceil(N/512) x chunks with chunks sized so the launch is >= 1024 workgroups.
template <typename T>
__global__ __launch_bounds__(256) void bias_grad_part_kernel(const T* __restrict__ dy, float* __restrict__ part, int M,
                                                             int N, int rows_per_chunk) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < N) {
    for (int r = r0 + w; r < r1; r += 4) {
      float v[8];
      if constexpr (sizeof(T) == 4) {
        float a[4], b[4];
        load_vec<T, 4>(dy + (long)r * N + c0, a);
        load_vec<T, 4>(dy + (long)r * N + c0 + 4, b);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
      } else {
        load_vec<T, 8>(dy + (long)r * N + c0, v);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.x * 512 + i;
    if (c < N) part[(long)blockIdx.y * N + c] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

}  // namespace pd

// db [N] (dtype odt) = column sums of dy [M, N] (dtype dt); part: fp32 workspace of pd_bias_grad_chunks(M, N) * N.
extern "C" int pd_bias_grad_chunks(int M, int N) {
  const int cb = (N + 511) / 512;
  int chunks = (1024 + cb - 1) / cb;
  chunks = chunks < 1 ? 1 : chunks;
  const int min_rows = 64;  // keep >= 16 rows per wave
  if (chunks * min_rows > M) chunks = (M + min_rows - 1) / min_rows;
  return chunks < 1 ? 1 : chunks;
}

// db[n] = sum_p part[p, n] (fixed order) -> odt: the second pass of the bias gradient on partial row sums some
// other kernel produced (the fp8 dY cast's per-64-row-block column sums).
// acc: db += sum (accumulate into an existing fp32 main-grad slot) instead of db = sum.
extern "C" int pd_colsum(int odt, const float* part, void* db, int P, int N, int acc, void* stream) {
  using namespace pd;
  if (N % 4 != 0 || P <= 0) return -1;
  colsum_to(odt, part, db, P, N, acc, (hipStream_t)stream);
  return (int)hipGetLastError();
}

extern "C" int pd_bias_grad(int dt, int odt, const void* dy, float* part, void* db, int M, int N, int acc,
                            void* stream) {
  using namespace pd;
  if (N % 8 != 0 || M <= 0) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int chunks = pd_bias_grad_chunks(M, N);
  const int rpc = (M + chunks - 1) / chunks;
  dim3 g1((N + 511) / 512, chunks);
  if (dt == kBF16) bias_grad_part_kernel<bf16><<<g1, 256, 0, st>>>((const bf16*)dy, part, M, N, rpc);
  else if (dt == kF16) bias_grad_part_kernel<half16><<<g1, 256, 0, st>>>((const half16*)dy, part, M, N, rpc);
  else if (dt == kF32) bias_grad_part_kernel<float><<<g1, 256, 0, st>>>((const float*)dy, part, M, N, rpc);
  else return -2;
  colsum_to(odt, part, db, chunks, N, acc, st);
  return (int)hipGetLastError();
}

// C ABI entry points (bound in bindings.cpp). dtype codes: 0 f32, 1 bf16, 2 f16.
// Weight dtype may be the activation dtype or f32.
// RMSNorm with residual of a few decode rows whose input is a decode GEMM's split-K partials (see PART above):
// res_out = round(sum of the partials) + res, y = norm(res_out) * w.  bf16 rows, bf16 or fp32 weight, M <= 64.
extern "C" int pd_norm_fwd_part(int wdt, const float* part, int S, const void* res, const void* w, void* y,
                                void* res_out, int M, int N, float eps, void* stream) {
  using namespace pd;
  hipStream_t st = (hipStream_t)stream;
  constexpr int V = 8;
  const int nv = N / V;
  const int maxr = (nv + kNormBlock - 1) / kNormBlock;
  if (N % V || maxr > 4 || M < 1 || M > 64 || S < 1 || !res || !res_out) return -1;
  if (wdt != kBF16 && wdt != kF32) return -2;
  dim3 grow(M), block(kNormBlock);
#define PD_NORM_PART(WT_, MV)                                                                                     \
  norm_fwd_row_kernel<bf16, WT_, MV, false, true, false, true><<<grow, block, 0, st>>>(                          \
      nullptr, (const bf16*)res, (const WT_*)w, nullptr, (bf16*)y, (bf16*)res_out, nullptr, nullptr, M, N, eps, part, S);
#define PD_NORM_PART_W(WT_)                                                                                       \
  if (maxr <= 1) { PD_NORM_PART(WT_, 1) } else if (maxr <= 2) { PD_NORM_PART(WT_, 2) } else { PD_NORM_PART(WT_, 4) }
  if (wdt == kBF16) { PD_NORM_PART_W(bf16) } else { PD_NORM_PART_W(float) }
#undef PD_NORM_PART_W
#undef PD_NORM_PART
  return (int)hipGetLastError();
}

extern "C" int pd_norm_fwd(int layernorm, int dt, int wdt, const void* x, const void* res, const void* w,
                           const void* b, void* y, void* res_out, float* mean, float* rstd, int M, int N,
                           float eps, void* stream) {
  using namespace pd;
  hipStream_t st = (hipStream_t)stream;
  const int V = dt == kF32 ? 4 : 8;
  if (N % V != 0 || N / V > 64 * 16) return -1;
  if (wdt != dt && wdt != kF32) return -2;
#define PD_FWD_CASE(T)                                                                                   \
  if (wdt == kF32 && dt != kF32) {                                                                       \
    if (layernorm) fwd_launch<T, float, true>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st);       \
    else fwd_launch<T, float, false>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st);                \
  } else {                                                                                               \
    if (layernorm) fwd_launch<T, T, true>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st);           \
    else fwd_launch<T, T, false>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st);                    \
  }
  if (dt == kF32) { using T = float; if (layernorm) fwd_launch<T, T, true>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st);
                    else fwd_launch<T, T, false>(x, res, w, b, y, res_out, mean, rstd, M, N, eps, st); }
  else if (dt == kBF16) { PD_FWD_CASE(bf16) }
  else { PD_FWD_CASE(half16) }
#undef PD_FWD_CASE
  return (int)hipGetLastError();
}

// Number of blocks the backward uses; caller allocates partials of nblocks x N floats.  Each block keeps ONE row in
// flight (load -> block reduction -> store), so the rows in flight per CU set the bandwidth: 1024 blocks (4 per CU)
// instead of 512 (the Llama-2-7B step's [32768, 4096] backward ran latency-bound at 4.7 TB/s with 2 per CU).
extern "C" int pd_norm_bwd_blocks(int M) { return M < 1024 ? M : 1024; }

extern "C" int pd_norm_bwd(int layernorm, int dt, int wdt, const void* dy, const void* x, const void* w,
                           const float* mean, const float* rstd, const void* dres, void* dx, float* dw_part,
                           float* db_part, void* dw, void* db, int M, int N, int nblocks, int odt, int acc_w,
                           int acc_b, void* stream) {
  using namespace pd;
  hipStream_t st = (hipStream_t)stream;
  // dw / db dtype: the weight's compute dtype by default (odt < 0), or fp32 main-grad slots written in place
  if (odt < 0) odt = (wdt == kF32 || dt == kF32) ? kF32 : dt;
  const int V = dt == kF32 ? 4 : 8;
  if (N % V != 0 || N / V > kNormBlock * 4 || N % 4 != 0) return -1;
#define PD_BWD_CASE(T)                                                                                           \
  if (wdt == kF32 && dt != kF32) {                                                                               \
    if (layernorm) bwd_launch<T, float, true>(dy, x, w, mean, rstd, dres, dx, dw_part, db_part, dw, db, M, N, nblocks, odt, acc_w, acc_b, st); \
    else bwd_launch<T, float, false>(dy, x, w, mean, rstd, dres, dx, dw_part, nullptr, dw, nullptr, M, N, nblocks, odt, acc_w, acc_b, st);   \
  } else {                                                                                                       \
    if (layernorm) bwd_launch<T, T, true>(dy, x, w, mean, rstd, dres, dx, dw_part, db_part, dw, db, M, N, nblocks, odt, acc_w, acc_b, st);     \
    else bwd_launch<T, T, false>(dy, x, w, mean, rstd, dres, dx, dw_part, nullptr, dw, nullptr, M, N, nblocks, odt, acc_w, acc_b, st);       \
  }
  if (dt == kF32) {
    using T = float;
    if (layernorm) bwd_launch<T, T, true>(dy, x, w, mean, rstd, dres, dx, dw_part, db_part, dw, db, M, N, nblocks, odt, acc_w, acc_b, st);
    else bwd_launch<T, T, false>(dy, x, w, mean, rstd, dres, dx, dw_part, nullptr, dw, nullptr, M, N, nblocks, odt, acc_w, acc_b, st);
  } else if (dt == kBF16) { PD_BWD_CASE(bf16) }
  else { PD_BWD_CASE(half16) }
#undef PD_BWD_CASE
  return (int)hipGetLastError();
}
