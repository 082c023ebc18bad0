// Channels-last (NHWC) BatchNorm for gfx950 with the activation and the residual add fused in.
//
// Reference behaviour: phi/kernels/gpu/batch_norm_kernel.cu / batch_norm_grad_kernel.cu (training
// statistics, running-stat update with the unbiased variance, saved mean / inv-std) and
// fluid/operators/fused/fused_bn_add_activation_op.cu (y = act(bn(x) + z)).  MIOpen's NHWC BN +
// separate add/ReLU kernels cost ~60% of a ResNet50 step on the MI355X (profiles/
// r1_resnet50_b256_nhwc_kernel_stats.md); here a BN layer is two memory passes each way:
//
//   fwd:  stats  (read x)                 -> per-block partial sums
//         final  (per channel)            -> mean, inv-std, running stats, scale/shift
//         apply  (read x [, z], write y)  y = relu?(x*scale + shift [+ z])
//   bwd:  reduce (read dy, x [, y])       -> partial sum(g), sum(g*(x-mean)),  g = dy*(y>0)
//         final  (per channel)            -> dgamma, dbeta, dx = A*g + B*x + C coefficients
//         dx     (read dy, x [, y], write dx [, dz = g])
//
// Layout of every pass: a 512-thread block is TPR lanes across channels (16-byte vectors, V
// channels per lane) x RPB = 512/TPR rows; each lane keeps its V channels' per-channel constants
// in registers for the whole grid-stride over rows.  The block grid is (channel tiles, row
// groups) sized to ~768 blocks (3 x 8 waves per CU) so the 256 CUs stay saturated down to 7x7
// feature maps, with 2-4 rows of loads in flight per lane; the per-block partials are combined
// by 16 channels x 16 slices per final block (the final pass is latency-, not bandwidth-bound).
// Statistics are accumulated shifted by the running mean (forward) / the batch mean (backward) in
// fp32 per lane and combined across blocks in fp64, which keeps E[x^2]-E[x]^2 well conditioned.
#include "common.h"

namespace pd {

constexpr int kBnBlock = 512;          // 8 waves
constexpr int kBnTargetBlocks = 768;   // 3 blocks per CU
constexpr int kFinCh = 16, kFinSl = 16;  // final reduction: 16 channels x 16 partial slices per block

template <typename T>
__device__ __forceinline__ void ld_f32v(const float* __restrict__ p, float (&o)[16 / sizeof(T)]) {
  constexpr int V = 16 / sizeof(T);
#pragma unroll
  for (int j = 0; j < V; j += 4) {
    float4 t = *reinterpret_cast<const float4*>(p + j);
    o[j] = t.x; o[j + 1] = t.y; o[j + 2] = t.z; o[j + 3] = t.w;
  }
}

// Block-level column reduction of two per-lane [V] accumulators into part[blockIdx.y][2][C]:
// xor-shuffles fold the 64/TPR rows a wave holds, LDS folds the 8 waves.
template <typename T, int TPR>
__device__ __forceinline__ void bn_block_reduce(float (&a)[16 / sizeof(T)], float (&b)[16 / sizeof(T)],
                                                float* __restrict__ part, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int CT = TPR * V;
  constexpr int W = kBnBlock / 64;
#pragma unroll
  for (int o = TPR; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      a[j] += __shfl_xor(a[j], o, 64);
      b[j] += __shfl_xor(b[j], o, 64);
    }
  }
  __shared__ float sh[2][W][CT];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < TPR) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sh[0][wid][lane * V + j] = a[j];
      sh[1][wid][lane * V + j] = b[j];
    }
  }
  __syncthreads();
  const int cbase = blockIdx.x * CT;
  float* out = part + (long)blockIdx.y * 2 * C;
  for (int col = threadIdx.x; col < 2 * CT; col += kBnBlock) {
    const int k = col / CT, cc = col % CT;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) acc += sh[k][w][cc];
    if (cbase + cc < C) out[k * C + cbase + cc] = acc;
  }
}

// Cross-block combine of part[gy][2][C] for channel c: 16 slices per channel in parallel, fp64.
__device__ __forceinline__ bool bn_combine(const float* __restrict__ part, int gy, int C, double& s, double& q) {
  __shared__ double red[2][kFinSl][kFinCh];
  const int ci = threadIdx.x % kFinCh, sl = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + ci;
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int i = sl; i < gy; i += kFinSl) {
      a += part[(long)i * 2 * C + c];
      b += part[(long)i * 2 * C + C + c];
    }
  }
  red[0][sl][ci] = a;
  red[1][sl][ci] = b;
  __syncthreads();
  if (sl != 0 || c >= C) return false;
  s = 0.0; q = 0.0;
#pragma unroll
  for (int k = 0; k < kFinSl; ++k) { s += red[0][k][ci]; q += red[1][k][ci]; }
  return true;
}

// --------------------------------------------------------------------------- forward statistics
template <typename T, int TPR>
__global__ __launch_bounds__(kBnBlock) void bn_stats_kernel(const T* __restrict__ x, const float* __restrict__ shift,
                                                            float* __restrict__ part, long M, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int RPB = kBnBlock / TPR;
  const int tc = threadIdx.x % TPR, tr = threadIdx.x / TPR;
  const int c0 = blockIdx.x * TPR * V + tc * V;
  const bool cok = c0 < C;
  float k[V], s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { k[j] = 0.f; s[j] = 0.f; q[j] = 0.f; }
  if (cok) ld_f32v<T>(shift + c0, k);
  const long stride = (long)gridDim.y * RPB;
  long r = (long)blockIdx.y * RPB + tr;
  if (cok) {
    // four rows in flight per iteration
    for (; r + 3 * stride < M; r += 4 * stride) {
      float v[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_vec<T, V>(x + (r + u * stride) * C + c0, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float d = v[u][j] - k[j];
          s[j] += d;
          q[j] = fmaf(d, d, q[j]);
        }
      }
    }
    for (; r < M; r += stride) {
      float v0[V];
      load_vec<T, V>(x + r * C + c0, v0);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d0 = v0[j] - k[j];
        s[j] += d0;
        q[j] = fmaf(d0, d0, q[j]);
      }
    }
  }
  bn_block_reduce<T, TPR>(s, q, part, C);
}

// Per channel: combine partials, update running stats, emit scale/shift for the apply pass.
__global__ __launch_bounds__(kFinCh * kFinSl) void bn_stats_final_kernel(
    const float* __restrict__ part, int gy, long M, int C, float* __restrict__ run_mean, float* __restrict__ run_var,
    const float* __restrict__ gamma, const float* __restrict__ beta, float momentum, float eps,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, float* __restrict__ scale,
    float* __restrict__ shift_out, int update_running) {
  double s, q;
  if (!bn_combine(part, gy, C, s, q)) return;
  const int c = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  const double k = run_mean[c];
  const double m1 = s / (double)M;
  double var = q / (double)M - m1 * m1;
  var = var > 0.0 ? var : 0.0;
  const float mean = (float)(k + m1);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  if (update_running) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = momentum * run_mean[c] + (1.f - momentum) * mean;
    run_var[c] = momentum * run_var[c] + (1.f - momentum) * (float)unbiased;
  }
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * invstd;
  shift_out[c] = b - mean * g * invstd;
}

// --------------------------------------------------------------------------- forward apply
template <typename T, int TPR, bool RELU, bool RES>
__global__ __launch_bounds__(kBnBlock) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ z,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ y,
                                                            long M, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int RPB = kBnBlock / TPR;
  const int tc = threadIdx.x % TPR, tr = threadIdx.x / TPR;
  const int c0 = blockIdx.x * TPR * V + tc * V;
  if (c0 >= C) return;
  float a[V], b[V];
  ld_f32v<T>(scale + c0, a);
  ld_f32v<T>(shift + c0, b);
  const long stride = (long)gridDim.y * RPB;
  for (long r = (long)blockIdx.y * RPB + tr; r < M; r += stride) {
    float v[V];
    load_vec<T, V>(x + r * C + c0, v);
    if constexpr (RES) {
      float w[V];
      load_vec<T, V>(z + r * C + c0, w);
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = fmaf(v[j], a[j], b[j]) + w[j];
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = fmaf(v[j], a[j], b[j]);
    }
    if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    store_vec<T, V>(y + r * C + c0, v);
  }
}

// --------------------------------------------------------------------------- backward
template <typename T, int TPR, bool RELU>
__global__ __launch_bounds__(kBnBlock) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                 const T* __restrict__ y,
                                                                 const float* __restrict__ mean,
                                                                 float* __restrict__ part, long M, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int RPB = kBnBlock / TPR;
  const int tc = threadIdx.x % TPR, tr = threadIdx.x / TPR;
  const int c0 = blockIdx.x * TPR * V + tc * V;
  const bool cok = c0 < C;
  float mu[V], sg[V], sgx[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { mu[j] = 0.f; sg[j] = 0.f; sgx[j] = 0.f; }
  if (cok) {
    ld_f32v<T>(mean + c0, mu);
    const long stride = (long)gridDim.y * RPB;
    long r = (long)blockIdx.y * RPB + tr;
    auto body = [&](long rr) {
      float g[V], xv[V];
      load_vec<T, V>(dy + rr * C + c0, g);
      load_vec<T, V>(x + rr * C + c0, xv);
      if constexpr (RELU) {
        float yv[V];
        load_vec<T, V>(y + rr * C + c0, yv);
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < V; ++j) {
        sg[j] += g[j];
        sgx[j] = fmaf(g[j], xv[j] - mu[j], sgx[j]);
      }
    };
    for (; r + stride < M; r += 2 * stride) {
      body(r);
      body(r + stride);
    }
    if (r < M) body(r);
  }
  bn_block_reduce<T, TPR>(sg, sgx, part, C);
}

__global__ __launch_bounds__(kFinCh * kFinSl) void bn_bwd_final_kernel(
    const float* __restrict__ part, int gy, long M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ coef) {
  double sg, sgx;
  if (!bn_combine(part, gy, C, sg, sgx)) return;
  const int c = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  const float is = invstd[c];
  const float dg = (float)(sgx * is);
  const float db = (float)sg;
  if (dgamma) dgamma[c] = dg;
  if (dbeta) dbeta[c] = db;
  // dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)) = A*g + B*x + Cc
  const float g = gamma ? gamma[c] : 1.f;
  const float A = g * is;
  const float B = -A * is * dg / (float)M;
  const float Cc = -A * db / (float)M - B * mean[c];
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = Cc;
}

template <typename T, int TPR, bool RELU, bool DRES>
__global__ __launch_bounds__(kBnBlock) void bn_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             const T* __restrict__ y, const float* __restrict__ coef,
                                                             T* __restrict__ dx, T* __restrict__ dz, long M, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int RPB = kBnBlock / TPR;
  const int tc = threadIdx.x % TPR, tr = threadIdx.x / TPR;
  const int c0 = blockIdx.x * TPR * V + tc * V;
  if (c0 >= C) return;
  float A[V], B[V], Cc[V];
  ld_f32v<T>(coef + c0, A);
  ld_f32v<T>(coef + C + c0, B);
  ld_f32v<T>(coef + 2 * C + c0, Cc);
  const long stride = (long)gridDim.y * RPB;
  for (long r = (long)blockIdx.y * RPB + tr; r < M; r += stride) {
    float g[V], xv[V];
    load_vec<T, V>(dy + r * C + c0, g);
    load_vec<T, V>(x + r * C + c0, xv);
    if constexpr (RELU) {
      float yv[V];
      load_vec<T, V>(y + r * C + c0, yv);
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    if constexpr (DRES) store_vec<T, V>(dz + r * C + c0, g);
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = fmaf(A[j], g[j], fmaf(B[j], xv[j], Cc[j]));
    store_vec<T, V>(dx + r * C + c0, o);
  }
}

// --------------------------------------------------------------------------- host helpers
struct BnGrid {
  int tpr, gx, gy;
};

template <typename T>
static BnGrid bn_grid(long M, int C) {
  constexpr int V = 16 / sizeof(T);
  int need = (C + V - 1) / V;  // lanes to cover one row
  int tpr = 8;
  while (tpr < need && tpr < 64) tpr *= 2;
  const int rpb = kBnBlock / tpr;
  const int gx = (C + tpr * V - 1) / (tpr * V);
  long gy = kBnTargetBlocks / gx;
  const long rows_groups = (M + rpb - 1) / rpb;
  if (gy > rows_groups) gy = rows_groups;
  if (gy < 1) gy = 1;
  return {tpr, gx, (int)gy};
}

#define PD_BN_TPR(tpr, TPR_, ...)                     \
  switch (tpr) {                                      \
    case 8: { constexpr int TPR_ = 8; __VA_ARGS__; break; }   \
    case 16: { constexpr int TPR_ = 16; __VA_ARGS__; break; } \
    case 32: { constexpr int TPR_ = 32; __VA_ARGS__; break; } \
    default: { constexpr int TPR_ = 64; __VA_ARGS__; break; } \
  }

}  // namespace pd

using namespace pd;

// Partial-sum workspace (floats) the caller allocates for a given shape: gy * 2 * C.
extern "C" long pd_bn_workspace(int dt, long M, int C) {
  BnGrid g = dt == kF32 ? bn_grid<float>(M, C) : bn_grid<bf16>(M, C);
  return (long)g.gy * 2 * C;
}

// Training forward.  x, z, y: [M, C] (channels last).  run_mean/run_var/gamma/beta fp32 [C].
// Outputs save_mean, save_invstd [C]; ws: workspace floats (pd_bn_workspace) + 2*C scratch.
extern "C" int pd_bn_fwd_train(int dt, const void* x, const void* z, void* y, long M, int C, float* run_mean,
                               float* run_var, const float* gamma, const float* beta, float momentum, float eps,
                               float* save_mean, float* save_invstd, float* ws, int relu, int update_running,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int V = dt == kF32 ? 4 : 8;
  if (C % V != 0) return -1;
  auto run = [&](auto tag) {
    using T = decltype(tag);
    BnGrid g = bn_grid<T>(M, C);
    float* part = ws;
    float* scale = ws + (long)g.gy * 2 * C;
    float* shift = scale + C;
    dim3 grid(g.gx, g.gy);
    PD_BN_TPR(g.tpr, TPR, bn_stats_kernel<T, TPR><<<grid, kBnBlock, 0, st>>>((const T*)x, run_mean, part, M, C));
    bn_stats_final_kernel<<<(C + kFinCh - 1) / kFinCh, kFinCh * kFinSl, 0, st>>>(part, g.gy, M, C, run_mean, run_var, gamma, beta, momentum,
                                                           eps, save_mean, save_invstd, scale, shift, update_running);
    PD_BN_TPR(g.tpr, TPR, {
      if (relu && z) bn_apply_kernel<T, TPR, true, true><<<grid, kBnBlock, 0, st>>>((const T*)x, (const T*)z, scale, shift, (T*)y, M, C);
      else if (relu) bn_apply_kernel<T, TPR, true, false><<<grid, kBnBlock, 0, st>>>((const T*)x, nullptr, scale, shift, (T*)y, M, C);
      else if (z) bn_apply_kernel<T, TPR, false, true><<<grid, kBnBlock, 0, st>>>((const T*)x, (const T*)z, scale, shift, (T*)y, M, C);
      else bn_apply_kernel<T, TPR, false, false><<<grid, kBnBlock, 0, st>>>((const T*)x, nullptr, scale, shift, (T*)y, M, C);
    });
  };
  if (dt == kF32) run(float{});
  else if (dt == kBF16) run(bf16{});
  else run(half16{});
  return (int)hipGetLastError();
}

// Inference forward with precomputed per-channel scale/shift (fp32 [C]).
extern "C" int pd_bn_apply(int dt, const void* x, const void* z, void* y, long M, int C, const float* scale,
                           const float* shift, int relu, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int V = dt == kF32 ? 4 : 8;
  if (C % V != 0) return -1;
  auto run = [&](auto tag) {
    using T = decltype(tag);
    BnGrid g = bn_grid<T>(M, C);
    dim3 grid(g.gx, g.gy);
    PD_BN_TPR(g.tpr, TPR, {
      if (relu && z) bn_apply_kernel<T, TPR, true, true><<<grid, kBnBlock, 0, st>>>((const T*)x, (const T*)z, scale, shift, (T*)y, M, C);
      else if (relu) bn_apply_kernel<T, TPR, true, false><<<grid, kBnBlock, 0, st>>>((const T*)x, nullptr, scale, shift, (T*)y, M, C);
      else if (z) bn_apply_kernel<T, TPR, false, true><<<grid, kBnBlock, 0, st>>>((const T*)x, (const T*)z, scale, shift, (T*)y, M, C);
      else bn_apply_kernel<T, TPR, false, false><<<grid, kBnBlock, 0, st>>>((const T*)x, nullptr, scale, shift, (T*)y, M, C);
    });
  };
  if (dt == kF32) run(float{});
  else if (dt == kBF16) run(bf16{});
  else run(half16{});
  return (int)hipGetLastError();
}

// Training backward.  y is the fused forward output (for the ReLU mask; may be null when relu=0).
// dz (optional) receives the gradient of the fused residual input.  dgamma/dbeta fp32 [C] (may be null).
extern "C" int pd_bn_bwd(int dt, const void* dy, const void* x, const void* y, const float* mean, const float* invstd,
                         const float* gamma, void* dx, void* dz, float* dgamma, float* dbeta, long M, int C, float* ws,
                         int relu, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int V = dt == kF32 ? 4 : 8;
  if (C % V != 0) return -1;
  if (relu && !y) return -2;
  auto run = [&](auto tag) {
    using T = decltype(tag);
    BnGrid g = bn_grid<T>(M, C);
    float* part = ws;
    float* coef = ws + (long)g.gy * 2 * C;  // 3*C
    dim3 grid(g.gx, g.gy);
    PD_BN_TPR(g.tpr, TPR, {
      if (relu) bn_bwd_reduce_kernel<T, TPR, true><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, (const T*)y, mean, part, M, C);
      else bn_bwd_reduce_kernel<T, TPR, false><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, nullptr, mean, part, M, C);
    });
    bn_bwd_final_kernel<<<(C + kFinCh - 1) / kFinCh, kFinCh * kFinSl, 0, st>>>(part, g.gy, M, C, mean, invstd, gamma, dgamma, dbeta, coef);
    PD_BN_TPR(g.tpr, TPR, {
      if (relu && dz) bn_bwd_dx_kernel<T, TPR, true, true><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, (const T*)y, coef, (T*)dx, (T*)dz, M, C);
      else if (relu) bn_bwd_dx_kernel<T, TPR, true, false><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, (const T*)y, coef, (T*)dx, nullptr, M, C);
      else if (dz) bn_bwd_dx_kernel<T, TPR, false, true><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, nullptr, coef, (T*)dx, (T*)dz, M, C);
      else bn_bwd_dx_kernel<T, TPR, false, false><<<grid, kBnBlock, 0, st>>>((const T*)dy, (const T*)x, nullptr, coef, (T*)dx, nullptr, M, C);
    });
  };
  if (dt == kF32) run(float{});
  else if (dt == kBF16) run(bf16{});
  else run(half16{});
  return (int)hipGetLastError();
}
