// Weight-only int8 / int4 GEMM for decode-sized token counts on gfx950:  Y[M,N] = X[M,K] . dequant(W)^T
//
// Reference behaviour: phi/kernels/fusion/gpu/weight_only_linear_kernel.cu (CUTLASS mixed-input
// GEMM / weight-only GEMV) and python/paddle/nn/quant/quantized_linear.py:183.  MI355X-first design:
//  * W is [N, K] int8 (each output channel's K weights contiguous) or [N/2, K] int4 (channel 2p in
//    the low nibble, 2p+1 in the high nibble); scales per channel [N] or per group [K/G, N];
//  * the kernel streams W from HBM exactly once: each lane loads 16 contiguous K-bytes of one
//    channel per 64-wide K step, sign-extends + converts them to bf16 in registers (integers up
//    to 8 bits are exact in bf16) and feeds v_mfma_f32_16x16x32_bf16 twice — the dot product is
//    permutation-invariant, so the k order inside the step only has to match X's;
//  * X[M, Kblk] (M <= 64) is staged once per block in LDS with a padded row pitch (conflict-free
//    16-byte reads; lanes of rows >= M feed zeros); the dequantized W fragment is reused across
//    the M tiles, and each wave keeps 2*D*RT 16-byte W loads in flight (double-buffered chunks);
//  * 4 waves x 16 channels = 64 channels per block, split-K over gridDim.y so decode shapes put
//    >= 1024 blocks (M <= 16) on the 256 CUs; fp32 partials go to a workspace and a second kernel
//    sums them, applies the per-channel scale, adds the bias and writes bf16 (deterministic).
//  * per-group scales are applied in the main loop: each group's MFMA partial is scaled into the
//    running accumulator at the group boundary.
#include "common.h"

namespace pd {

typedef __bf16 wo_bf16x8 __attribute__((ext_vector_type(8)));
typedef float wo_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWoWaves = 4;
constexpr int kWoRows = 16 * kWoWaves;  // output channels per block
constexpr int kWoPad = 8;               // bf16 elements of LDS row padding

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  // exact for small integers: the low 16 bits of the f32 are zero
  return (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
}

// 16 signed int8 (one uint4) -> two bf16x8 fragments (bytes 0-7, 8-15)
__device__ __forceinline__ void i8x16_to_bf16(uint4 w, wo_bf16x8& f0, wo_bf16x8& f1) {
  unsigned d[4] = {w.x, w.y, w.z, w.w};
  unsigned p[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = (int)d[i];
    const float b0 = (float)((v << 24) >> 24), b1 = (float)((v << 16) >> 24);
    const float b2 = (float)((v << 8) >> 24), b3 = (float)(v >> 24);
    p[2 * i] = pack_bf16x2(b0, b1);
    p[2 * i + 1] = pack_bf16x2(b2, b3);
  }
  uint4 a = make_uint4(p[0], p[1], p[2], p[3]), b = make_uint4(p[4], p[5], p[6], p[7]);
  f0 = __builtin_bit_cast(wo_bf16x8, a);
  f1 = __builtin_bit_cast(wo_bf16x8, b);
}

// 16 bytes holding one nibble per byte for this lane's channel -> two bf16x8 fragments
__device__ __forceinline__ void i4x16_to_bf16(uint4 w, int hi, wo_bf16x8& f0, wo_bf16x8& f1) {
  unsigned d[4] = {w.x, w.y, w.z, w.w};
  unsigned p[8];
  const int sh = hi ? 4 : 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = (int)(d[i] >> sh);
    const float b0 = (float)((v << 28) >> 28), b1 = (float)((v << 20) >> 28);
    const float b2 = (float)((v << 12) >> 28), b3 = (float)((v << 4) >> 28);
    p[2 * i] = pack_bf16x2(b0, b1);
    p[2 * i + 1] = pack_bf16x2(b2, b3);
  }
  uint4 a = make_uint4(p[0], p[1], p[2], p[3]), b = make_uint4(p[4], p[5], p[6], p[7]);
  f0 = __builtin_bit_cast(wo_bf16x8, a);
  f1 = __builtin_bit_cast(wo_bf16x8, b);
}

// grid: (N / (64*RT), S). block: 256 = 4 waves; wave w owns RT 16-channel row tiles
// (channels 64*RT*bx + 16*(w + 4*r) + lane&15) over its block's share of the K units.  RT > 1
// amortises the per-block X staging (X bytes / W bytes = 2M / (64 RT)) and keeps RT independent
// 16-byte W loads in flight per lane.
template <bool INT4, int MT, int RT, int GSTEPS>
__global__ __launch_bounds__(256) void wo_gemm_kernel(const unsigned short* __restrict__ X, const int8_t* __restrict__ W,
                                                      const float* __restrict__ gscale, float* __restrict__ ws,
                                                      int M, int N, int K, int unit, int kmax) {
  extern __shared__ unsigned short xs[];  // [M][kmax + kWoPad] (rows >= M are never read)
  const int pitch = kmax + kWoPad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // uneven split-K in whole units (64 or the scale group): block y owns units [U*y/S, U*(y+1)/S)
  const int U = K / unit, S = gridDim.y;
  const int k0 = (int)((long)U * blockIdx.y / S) * unit;
  const int Kblk = (int)((long)U * (blockIdx.y + 1) / S) * unit - k0;
  // ---- stage X[:M, k0:k0+Kblk]
  const int vpr = Kblk / 8;  // 16-byte vectors per row
  for (int i = tid; i < M * vpr; i += 256) {
    const int r = i / vpr, c = (i % vpr) * 8;
    *reinterpret_cast<uint4*>(xs + r * pitch + c) = *reinterpret_cast<const uint4*>(X + (long)r * K + k0 + c);
  }
  __syncthreads();

  const int g = lane >> 4;  // k sub-block of the step
  const int nbase = blockIdx.x * kWoRows * RT + wave * 16;
  const int8_t* wrow[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int n = nbase + r * kWoRows + (lane & 15);  // this lane's channel (A row) in tile r
    wrow[r] = (INT4 ? W + (long)(n >> 1) * K : W + (long)n * K) + k0 + 16 * g;
  }
  const int hi = lane & 1;  // channel parity (row tiles start at multiples of 16)
  wo_f32x4 acc[RT][MT], part[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[r][t] = wo_f32x4{0.f, 0.f, 0.f, 0.f};
      part[r][t] = acc[r][t];
    }
  const int nsteps = Kblk / 64;
  // W prefetch: chunks of D steps, double-buffered -> 2*D*RT 16-byte loads in flight per lane
  constexpr int D = RT == 1 ? 4 : 2;
  uint4 wb[RT][D];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int d = 0; d < D; ++d)
      wb[r][d] = d < nsteps ? *reinterpret_cast<const uint4*>(wrow[r] + d * 64) : make_uint4(0, 0, 0, 0);
  for (int c = 0; c < nsteps; c += D) {
    uint4 nb[RT][D];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int d = 0; d < D; ++d)
        nb[r][d] = c + D + d < nsteps ? *reinterpret_cast<const uint4*>(wrow[r] + (c + D + d) * 64)
                                      : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = c + d;
      if (s >= nsteps) break;
      const int kk = s * 64 + 16 * g;
      wo_bf16x8 b0[MT], b1[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = t * 16 + (lane & 15);
        const unsigned short* xr = xs + m * pitch + kk;
        const wo_bf16x8 z = {};
        b0[t] = m < M ? *reinterpret_cast<const wo_bf16x8*>(xr) : z;
        b1[t] = m < M ? *reinterpret_cast<const wo_bf16x8*>(xr + 8) : z;
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        wo_bf16x8 a0, a1;
        if constexpr (INT4) i4x16_to_bf16(wb[r][d], hi, a0, a1);
        else i8x16_to_bf16(wb[r][d], a0, a1);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          wo_f32x4& dst = GSTEPS ? part[r][t] : acc[r][t];
          dst = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[t], dst, 0, 0, 0);
          dst = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[t], dst, 0, 0, 0);
        }
      }
      if constexpr (GSTEPS > 0) {
        if ((s + 1) % GSTEPS == 0) {
          // C rows (lane>>4)*4 + i are channels; scale row-wise with this group's scales
          const int grp = (k0 + s * 64) / (64 * GSTEPS);
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            const int nb2 = nbase + r * kWoRows + (lane >> 4) * 4;
            const float4 sc = *reinterpret_cast<const float4*>(gscale + (long)grp * N + nb2);
#pragma unroll
            for (int t = 0; t < MT; ++t) {
              acc[r][t][0] = fmaf(part[r][t][0], sc.x, acc[r][t][0]);
              acc[r][t][1] = fmaf(part[r][t][1], sc.y, acc[r][t][1]);
              acc[r][t][2] = fmaf(part[r][t][2], sc.z, acc[r][t][2]);
              acc[r][t][3] = fmaf(part[r][t][3], sc.w, acc[r][t][3]);
              part[r][t] = wo_f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int d = 0; d < D; ++d) wb[r][d] = nb[r][d];
  }
  // ---- partial tiles -> ws[by][m][n]: lane holds col m = lane&15, rows (lane>>4)*4 + i
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int nb = nbase + r * kWoRows + (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + (lane & 15);
      if (m < M)
        *reinterpret_cast<float4*>(ws + ((long)blockIdx.y * M + m) * N + nb) =
            make_float4(acc[r][t][0], acc[r][t][1], acc[r][t][2], acc[r][t][3]);
    }
  }
}

// bf16 weights (the serving decode GEMM on the cached [N, K] projection weights): the same schedule with each lane
// streaming 32 contiguous K-bytes of its channel per 64-wide K step (two 16-B loads = the two MFMA fragments), no
// conversion.  Y[M, N] = X[M, K] . W^T, M <= 64, fp32 split-K partials into ws (summed by wo_reduce_kernel).
// GLU (the Llama MLP's down projection at decode): X is the gate|up GEMM output gu [M, 2K] and the staged row is
// silu(gate) * up, rounded to bf16 once like swiglu_fwd_kernel — the SwiGLU pass folds into the X staging (the
// whole X tile goes through LDS anyway), one launch less per layer.
__device__ __forceinline__ float dec_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }   // as swiglu_fwd

// cnt (optional): one int per column block, zero between calls.  The last of the S split-K workgroups of a column
// block to finish (atomic arrival count) sums the S partials in split order — bit-identical to wo_reduce_kernel —
// adds the bias and writes bf16 out, then re-arms its counter.  That drops the reduce launch (~5 us per projection
// at decode batch 1, where the step is a chain of small kernels).  Nobody waits on the counter, so no workgroup can
// stall another.
template <int MT, int RT, bool GLU = false>
__global__ __launch_bounds__(256) void dec_gemm_kernel(const unsigned short* __restrict__ X,
                                                       const unsigned short* __restrict__ W, float* __restrict__ ws,
                                                       int M, int N, int K, int kmax, int* __restrict__ cnt,
                                                       const unsigned short* __restrict__ bias,
                                                       unsigned short* __restrict__ out) {
  extern __shared__ unsigned short xs[];  // [M][kmax + kWoPad]
  const int pitch = kmax + kWoPad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int U = K / 64, S = gridDim.y;
  const int k0 = (int)((long)U * blockIdx.y / S) * 64;
  const int Kblk = (int)((long)U * (blockIdx.y + 1) / S) * 64 - k0;
  const int vpr = Kblk / 8;
  for (int i = tid; i < M * vpr; i += 256) {
    const int r = i / vpr, c = (i % vpr) * 8;
    if constexpr (GLU) {
      const uint4 gv = *reinterpret_cast<const uint4*>(X + (long)r * 2 * K + k0 + c);
      const uint4 uv = *reinterpret_cast<const uint4*>(X + (long)r * 2 * K + K + k0 + c);
      const unsigned gw[4] = {gv.x, gv.y, gv.z, gv.w}, uw[4] = {uv.x, uv.y, uv.z, uv.w};
      unsigned ow[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g0 = __uint_as_float(gw[j] << 16), g1 = __uint_as_float(gw[j] & 0xffff0000u);
        const float u0 = __uint_as_float(uw[j] << 16), u1 = __uint_as_float(uw[j] & 0xffff0000u);
        ow[j] = (unsigned)f2bf(g0 * dec_sigmoid(g0) * u0) | ((unsigned)f2bf(g1 * dec_sigmoid(g1) * u1) << 16);
      }
      *reinterpret_cast<uint4*>(xs + r * pitch + c) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    } else {
      *reinterpret_cast<uint4*>(xs + r * pitch + c) = *reinterpret_cast<const uint4*>(X + (long)r * K + k0 + c);
    }
  }
  __syncthreads();

  const int g = lane >> 4;
  const int nbase = blockIdx.x * kWoRows * RT + wave * 16;
  const unsigned short* wrow[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) wrow[r] = W + (long)(nbase + r * kWoRows + (lane & 15)) * K + k0 + 16 * g;
  wo_f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = wo_f32x4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = Kblk / 64;
  constexpr int D = RT == 1 ? 4 : 2;
  uint4 wb[RT][D][2];
  auto ld = [&](int r, int s, uint4 (&o)[2]) {
    if (s < nsteps) {
      const uint4* p = reinterpret_cast<const uint4*>(wrow[r] + s * 64);
      o[0] = p[0];
      o[1] = p[1];
    } else {
      o[0] = o[1] = make_uint4(0, 0, 0, 0);
    }
  };
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int d = 0; d < D; ++d) ld(r, d, wb[r][d]);
  for (int c = 0; c < nsteps; c += D) {
    uint4 nb[RT][D][2];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int d = 0; d < D; ++d) ld(r, c + D + d, nb[r][d]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = c + d;
      if (s >= nsteps) break;
      const int kk = s * 64 + 16 * g;
      wo_bf16x8 b0[MT], b1[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = t * 16 + (lane & 15);
        const unsigned short* xr = xs + m * pitch + kk;
        const wo_bf16x8 z = {};
        b0[t] = m < M ? *reinterpret_cast<const wo_bf16x8*>(xr) : z;
        b1[t] = m < M ? *reinterpret_cast<const wo_bf16x8*>(xr + 8) : z;
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const wo_bf16x8 a0 = __builtin_bit_cast(wo_bf16x8, wb[r][d][0]);
        const wo_bf16x8 a1 = __builtin_bit_cast(wo_bf16x8, wb[r][d][1]);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[t], acc[r][t], 0, 0, 0);
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[t], acc[r][t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        wb[r][d][0] = nb[r][d][0];
        wb[r][d][1] = nb[r][d][1];
      }
  }
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int nb = nbase + r * kWoRows + (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + (lane & 15);
      if (m >= M) continue;
      float* dst = ws + ((long)blockIdx.y * M + m) * N + nb;
      if (cnt == nullptr) {
        *reinterpret_cast<float4*>(dst) = make_float4(acc[r][t][0], acc[r][t][1], acc[r][t][2], acc[r][t][3]);
      } else {
        // write-through (system-scope) stores: the partials reach memory, not just this XCD's L2, so the reducing
        // workgroup on any XCD reads them without a whole-L2 writeback / invalidate fence (measured 3x slower)
#pragma unroll
        for (int j = 0; j < 4; ++j) __hip_atomic_store(dst + j, acc[r][t][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (cnt == nullptr) return;
  __shared__ int is_last;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // this wave's stores complete (vmcnt 0)
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    is_last = prev == S - 1;
    if (is_last) __hip_atomic_store(cnt + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);   // re-arm
  }
  __syncthreads();
  if (!is_last) return;
  const int ncol = kWoRows * RT, n0 = blockIdx.x * ncol, q = ncol / 4;
  auto ld4 = [&](const float* p) {   // system-scope loads: from memory, past any stale cached line
    return make_float4(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  };
  for (int i = tid; i < M * q; i += 256) {
    const int m = i / q, n = n0 + (i % q) * 4;
    float4 a = ld4(ws + (long)m * N + n);
    for (int sp = 1; sp < S; ++sp) {
      const float4 b = ld4(ws + ((long)sp * M + m) * N + n);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    unsigned short o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (bias) v[j] += bf2f(bias[n + j]);
      o[j] = f2bf(v[j]);
    }
    *reinterpret_cast<uint2*>(out + (long)m * N + n) =
        make_uint2((unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16));
  }
}

// Decode GEMM for 16 < M <= 64 tokens (the batched serving step): out[M, N] = X[M, K] . W[N, K]^T (+ bias), bf16.
// One workgroup = 16 * RT output channels (W rows) x the WHOLE K, split over its KW waves (no cross-workgroup split-K:
// the split-K kernel above moves S x M x N fp32 partials through HBM, which at M = 64 costs 25-100 % of the weight
// bytes); the KW wave partials meet once in LDS.  Per 64-wide K step a lane streams 32 contiguous bytes of each of
// its RT channels (two MFMA A fragments per channel tile) from HBM, DW steps ahead (DW x RT x 32 B in flight per
// lane), and reads its MT X row fragments (X: 64 x K bf16, L2-resident, shared by every workgroup) one step ahead;
// v_mfma_f32_16x16x32_bf16 gives D[channel][token] = out^T.  RT sets the X reuse: every X fragment a wave loads
// feeds RT channel tiles, so X's L2 -> CU traffic is MT / RT times the weight bytes (RT = 1: 4x at M = 64, which
// capped the kernel at 1.5-1.7 TB/s of weights; profiles/r5_decode_serving.md).  X rows >= M and K past the wave's
// range read as zeros through the buffer descriptors' range check.  grid = N / (16 RT) workgroups, block = 64 * KW.
template <int MT, int KW, int DW, int RT>
__global__ __launch_bounds__(64 * KW) void dec64_kernel(const unsigned short* __restrict__ X,
                                                        const unsigned short* __restrict__ W,
                                                        const unsigned short* __restrict__ bias,
                                                        unsigned short* __restrict__ out, int M, int N, int K) {
  __shared__ wo_f32x4 red[KW][MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.x * 16 * RT;
  const int U = K / 64;
  const int s0 = U * wave / KW, s1 = U * (wave + 1) / KW;   // this wave's 64-wide K steps
  const int ns = s1 - s0;
  // buffer descriptors (wave-uniform bases) with EXACT extents: W from the wave's first K step of row n0 to the end
  // of row n0 + 16 RT - 1, X to the end of row M - 1.  Prefetches past the wave's range use the offset kSkip, which
  // is beyond both extents, so the range check returns zeros (an earlier form bounded W at 0x7fffffff and skipped
  // with 0x7ffffff0 — INSIDE that range — and the tail prefetches read ~2 GiB past the weight: a GPU fault)
  constexpr int kSkip = (int)0x7fffff00;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(W + (long)n0 * K + (long)s0 * 64), (short)0,
      (int)((16L * RT * K - (long)s0 * 64) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(X + (long)s0 * 64), (short)0, (int)(((long)M * K - (long)s0 * 64) * 2), 0x00020000);
  const int wvo = (r16 * K + 16 * g) * 2;                      // lane's W byte offset at step 0 (row n0 + r16)
  const int rstride = 16 * K * 2;                              // bytes between channel tiles
  int xvo[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xvo[t] = ((t * 16 + r16) * K + 16 * g) * 2;
  auto ldw = [&](int s, uint4 (&o)[RT][2]) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int v = s < ns ? wvo + r * rstride + s * 128 : kSkip;   // past the wave's range: beyond the extent
      o[r][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, v, 0, 0));
      o[r][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, v + 16, 0, 0));
    }
  };
  auto ldx = [&](int s, uint4 (&o)[MT][2]) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int v = s < ns ? xvo[t] + s * 128 : kSkip;
      o[t][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, v, 0, 0));
      o[t][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, v + 16, 0, 0));
    }
  };
  wo_f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = wo_f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 wb[DW][RT][2], xb[2][MT][2];
#pragma unroll
  for (int d = 0; d < DW; ++d) ldw(d, wb[d]);
  ldx(0, xb[0]);
  // DW-deep W ring (compile-time slot index: the loop is unrolled by DW) and a 2-deep X ring
  for (int c = 0; c < ns; c += DW) {
#pragma unroll
    for (int d = 0; d < DW; ++d) {
      const int s = c + d;
      if (s >= ns) break;
      ldx(s + 1, xb[(d + 1) & 1]);
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const wo_bf16x8 a0 = __builtin_bit_cast(wo_bf16x8, wb[d][r][0]);
        const wo_bf16x8 a1 = __builtin_bit_cast(wo_bf16x8, wb[d][r][1]);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, __builtin_bit_cast(wo_bf16x8, xb[d & 1][t][0]),
                                                              acc[r][t], 0, 0, 0);
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, __builtin_bit_cast(wo_bf16x8, xb[d & 1][t][1]),
                                                              acc[r][t], 0, 0, 0);
        }
      }
      ldw(s + DW, wb[d]);
    }
  }
  // per channel tile: the KW partials through LDS, then wave t (< MT) sums token tile t and stores it
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (r) __syncthreads();   // the previous tile's readers are done with red
#pragma unroll
    for (int t = 0; t < MT; ++t) red[wave][t][lane] = acc[r][t];
    __syncthreads();
    if (wave < MT) {
      const int t = wave;
      wo_f32x4 v = red[0][t][lane];
#pragma unroll
      for (int w = 1; w < KW; ++w) {
        const wo_f32x4 o = red[w][t][lane];
        v[0] += o[0]; v[1] += o[1]; v[2] += o[2]; v[3] += o[3];
      }
      // D[channel 4g + e][token 16t + r16] -> out[token][n0 + 16 r + 4g .. + 3]
      const int m = t * 16 + r16;
      const int n = n0 + 16 * r + 4 * g;
      if (m < M) {
        float o[4] = {v[0], v[1], v[2], v[3]};
        if (bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += bf2f(bias[n + e]);
        }
        const uint2 pk = make_uint2((unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16),
                                    (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16));
        *reinterpret_cast<uint2*>(out + (long)m * N + n) = pk;
      }
    }
  }
}

// Decode GEMM for 16 < M <= 64, X through LDS (dec64s_kernel): the fix for dec64_kernel's limit.  vmcnt retires
// VMEM loads in issue order, so dec64_kernel's one-step X prefetch made every wait also wait for the W loads issued
// before it: its 8-step W ring worked like a 1-step one.  Here the waves of a workgroup split the CHANNELS (wave w:
// channels n0 + 16 RT w ..) and walk the same 64-wide K steps together; each step's X tile [64 tokens][64 k] (8 KiB)
// arrives by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction, 8 / KW per wave) into a DW-slot LDS ring
// and is read by every wave (ds_read_b128, lgkmcnt), so the only VMEM traffic is the DW - 1 steps of W and X
// pieces in flight, all issued together per step: one counted `vmcnt` + `s_barrier` per step.
// LDS image of a step tile: row r (token) at 128 r, 16-B chunk c (k 8c .. 8c + 7) at position c ^ (r & 7) (the
// swizzle is applied on the DMA source side: lane i of a piece fetches chunk (i & 7) ^ (i >> 3)), so the 16-lane
// ds_read_b128 groups (same chunk pair, 8 consecutive rows) are conflict-free.
// Split-K over gridDim.y (S): S == 1 writes bf16 (+ bias) directly; S > 1 writes fp32 partials into ws [S][M][N]
// for wo_reduce_kernel.  grid = (N / (16 RT KW), S), block = 64 KW.
// one 16-B-per-lane LDS-DMA piece (1 KiB per wave) at the wave-uniform LDS address dst
__device__ __forceinline__ void dec_lds_dma16(const __amdgpu_buffer_rsrc_t& rs, unsigned dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(size_t)dst, 16, voff, 0, 0, 0);
}

template <int MT, int KW, int RT, int DW>
__global__ __launch_bounds__(64 * KW) void dec64s_kernel(const unsigned short* __restrict__ X,
                                                         const unsigned short* __restrict__ W,
                                                         const unsigned short* __restrict__ bias,
                                                         unsigned short* __restrict__ out, float* __restrict__ ws,
                                                         int M, int N, int K) {
  constexpr int D = DW - 1;                 // prefetch distance (steps in flight)
  constexpr int P = 8 / KW;                 // X pieces per wave per step
  constexpr int C = P + 2 * RT;             // VMEM instructions per wave per step
  static_assert((D - 1) * C <= 63, "vmcnt immediate");
  __shared__ __attribute__((aligned(1024))) char xs[DW * 8192];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform: SGPR descriptors
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = (blockIdx.x * KW + wave) * 16 * RT;   // this wave's first channel
  const int U = K / 64, S = gridDim.y;
  const int s0 = (int)((long)U * blockIdx.y / S), ns = (int)((long)U * (blockIdx.y + 1) / S) - s0;
  // Prefetches past the split's last step read whatever the offset lands on (the next row's K, or zeros beyond the
  // extent through the range check) — never used: the step loop stops at ns.  No select, no branch per issue.
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(W + (long)n0 * K + (long)s0 * 64), (short)0,
      (int)((16L * RT * K - (long)s0 * 64) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(X + (long)s0 * 64), (short)0, (int)(((long)M * K - (long)s0 * 64) * 2), 0x00020000);
  const int wvo = (r16 * K + 16 * g) * 2;   // lane's W byte offset at step 0 (channel n0 + r16, k 16 g)
  const int rstride = 16 * K * 2;
  // X piece j of this wave: rows 8 (wave + KW j) + (lane >> 3), source chunk (lane & 7) ^ (lane >> 3)
  int xvo[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int row = 8 * (wave + KW * j) + (lane >> 3);
    xvo[j] = (row * K + 8 * ((lane & 7) ^ (lane >> 3))) * 2;
  }
  const unsigned xbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)xs;
  auto issue = [&](int s, int slot, uint4 (&o)[RT][2]) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const unsigned dst = xbase + slot * 8192 + (wave + KW * j) * 1024;
      dec_lds_dma16(rx, dst, (unsigned)(xvo[j] + s * 128));
    }
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int v = wvo + r * rstride + s * 128;
      o[r][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, v, 0, 0));
      o[r][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, v + 16, 0, 0));
    }
  };
  wo_f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = wo_f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 wb[DW][RT][2];
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d, wb[d]);
  // lane's X read offsets inside a slot: token row 16 t + r16, chunks 2g / 2g + 1 at their swizzled positions
  const int xr0 = r16 * 128 + ((2 * g) ^ (r16 & 7)) * 16, xr1 = r16 * 128 + ((2 * g + 1) ^ (r16 & 7)) * 16;
  for (int c = 0; c < ns; c += DW) {
#pragma unroll
    for (int d = 0; d < DW; ++d) {
      const int s = c + d;
      if (s >= ns) break;
      // step s's pieces (this wave's) landed: D - 1 later steps may stay in flight; then everyone's
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * C) : "memory");
      __builtin_amdgcn_s_barrier();
      // every wave is past step s - 1: its slot (d - 1) takes step s + D
      issue(s + D, (d + DW - 1) % DW, wb[(d + DW - 1) % DW]);
      const char* xt = xs + d * 8192;
      wo_bf16x8 b0[MT], b1[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        b0[t] = *reinterpret_cast<const wo_bf16x8*>(xt + t * 16 * 128 + xr0);
        b1[t] = *reinterpret_cast<const wo_bf16x8*>(xt + t * 16 * 128 + xr1);
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const wo_bf16x8 a0 = __builtin_bit_cast(wo_bf16x8, wb[d][r][0]);
        const wo_bf16x8 a1 = __builtin_bit_cast(wo_bf16x8, wb[d][r][1]);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[t], acc[r][t], 0, 0, 0);
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[t], acc[r][t], 0, 0, 0);
        }
      }
    }
  }
  // drain the tail prefetches (zero-filled, past the range) before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // D[channel 4g + e][token 16t + r16]
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int n = n0 + 16 * r + 4 * g;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + r16;
      if (m >= M) continue;
      if (S == 1) {
        float o[4] = {acc[r][t][0], acc[r][t][1], acc[r][t][2], acc[r][t][3]};
        if (bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += bf2f(bias[n + e]);
        }
        *reinterpret_cast<uint2*>(out + (long)m * N + n) =
            make_uint2((unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16),
                       (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16));
      } else {
        *reinterpret_cast<float4*>(ws + ((long)blockIdx.y * M + m) * N + n) =
            make_float4(acc[r][t][0], acc[r][t][1], acc[r][t][2], acc[r][t][3]);
      }
    }
  }
}

// out[m, n] = (sum_s ws[s, m, n]) * cscale[n] + bias[n]   (bf16 out / bias)
__global__ __launch_bounds__(256) void wo_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                        const float* __restrict__ cscale,
                                                        const unsigned short* __restrict__ bias,
                                                        unsigned short* __restrict__ out) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= (long)M * N) return;
  float4 a = *reinterpret_cast<const float4*>(ws + i);
  // unrolled so the S partial loads are issued together (same summation order): at decode M = 1 the launch is a few
  // workgroups and its time is this chain's latency
#pragma unroll 8
  for (int s = 1; s < S; ++s) {
    const float4 b = *reinterpret_cast<const float4*>(ws + (long)s * M * N + i);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  const int n = (int)(i % N);
  float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (cscale) v[j] *= cscale[n + j];
    if (bias) v[j] += bf2f(bias[n + j]);
    out[i + j] = f2bf(v[j]);
  }
}

}  // namespace pd

using namespace pd;

// Split-K factor for a shape: enough blocks to fill the chip, X tile within the LDS budget.
static inline int wo_unit(int group) { return group > 64 ? group : 64; }
static inline int wo_kcap(int M) {
  // X tile [M][Kblk] bf16 <= ~32 KB of LDS so several blocks fit per CU
  int cap = 2048;
  while (cap > 512 && (long)M * cap * 2 > 64 * 1024) cap >>= 1;
  return cap;
}

static inline int wo_mt(int M) {
  const int mt = (M + 15) / 16;
  return mt <= 1 ? 1 : (mt <= 2 ? 2 : 4);
}
static inline int wo_rt(int M, int N) {
  int rt = wo_mt(M);
  while (rt > 1 && N % (kWoRows * rt)) rt >>= 1;
  return rt;
}

extern "C" int pd_wo_splits(int M, int N, int K, int group) {
  const int unit = wo_unit(group), U = K / unit;
  const int nblk = N / (kWoRows * wo_rt(M, N));
  int S = (K + wo_kcap(M) - 1) / wo_kcap(M);
  // workgroups to aim for.  M <= 16: 768 (3 per CU; profiles/r6_decode_partials.md: 1024 / 896 / 640 / 512 lose
  // 1-3 % at b1, 2048 loses 4 %); PADDLE2_AMD_DEC_WG_TARGET overrides it (read once).
  static const char* te = getenv("PADDLE2_AMD_DEC_WG_TARGET");
  const int target = M <= 16 ? (te ? atoi(te) : 768) : 384;
  const int fill = (target + nblk - 1) / nblk;
  if (S < fill) S = fill;
  if (S > U) S = U;
  return S < 1 ? 1 : S;
}

// ws: S*M*N floats of split-K partials.  (fp32 atomics into one [M, N] buffer were tried: the
// device-scope fences a last-block epilogue needs write back the per-XCD L2s and cost ~10x.)
extern "C" long pd_wo_workspace(int M, int N, int S) { return (long)S * M * N; }

extern "C" int pd_wo_gemm(int int4, const void* X, const void* W, const float* cscale, const float* gscale, int group,
                          const void* bias, void* out, float* ws, int M, int N, int K, int S, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int unit = wo_unit(group);
  if (M < 1 || M > 64 || N % kWoRows || K % unit || S < 1 || S > K / unit) return -1;
  if (group > 0 && group != 64 && group != 128) return -2;
  const int kmax = ((K / unit + S - 1) / S) * unit;  // largest block K range
  const int MT = wo_mt(M), RT = wo_rt(M, N);
  const size_t lds = (size_t)M * (kmax + kWoPad) * 2;
  if (lds > 160 * 1024) return -3;
  dim3 grid(N / (kWoRows * RT), S);
  const int gsteps = group > 0 ? group / 64 : 0;
  auto launch = [&](auto kern) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, 256, lds, st>>>((const unsigned short*)X, (const int8_t*)W, gscale, ws, M, N, K, unit, kmax);
  };
#define PD_WO_G(I4, MT_, RT_)                                                  \
  if (gsteps == 0) launch(wo_gemm_kernel<I4, MT_, RT_, 0>);                    \
  else if (gsteps == 1) launch(wo_gemm_kernel<I4, MT_, RT_, 1>);               \
  else launch(wo_gemm_kernel<I4, MT_, RT_, 2>);
#define PD_WO_R(I4, MT_)                                                       \
  if (RT == 1) { PD_WO_G(I4, MT_, 1) } else if (RT == 2) { PD_WO_G(I4, MT_, 2) } else { PD_WO_G(I4, MT_, 4) }
  if (int4) {
    if (MT == 1) { PD_WO_R(true, 1) } else if (MT == 2) { PD_WO_R(true, 2) } else { PD_WO_R(true, 4) }
  } else {
    if (MT == 1) { PD_WO_R(false, 1) } else if (MT == 2) { PD_WO_R(false, 2) } else { PD_WO_R(false, 4) }
  }
#undef PD_WO_R
#undef PD_WO_G
  const long total = (long)M * N;
  wo_reduce_kernel<<<(int)((total / 4 + 255) / 256), 256, 0, st>>>(ws, S, M, N, group > 0 ? nullptr : cscale,
                                                                 (const unsigned short*)bias, (unsigned short*)out);
  return (int)hipGetLastError();
}

// The whole-K decode GEMM for 16 < M <= 64 (dec64_kernel): N % 16 == 0, K % 64 == 0, 16-B aligned rows.  kw: waves
// per workgroup (4 or 8); rt: channel tiles per workgroup (1, 2 or 4; N % (16 rt) == 0), 0 = auto: 4 for the wide
// projections (N >= 8192: 1.6 -> 2.7-3.5 TB/s at M = 64 even at 128-192 workgroups), 1 below (N = 4096 needs its
// 256 workgroups; rt 4 there halves the rate).  Measured: profiles/r5_decode_serving.md.  Returns -1 outside the
// domain.
extern "C" int pd_dec64_rt(int N) { return (N >= 8192 && N % 64 == 0) ? 4 : 1; }

extern "C" int pd_dec64_gemm(const void* X, const void* W, const void* bias, void* out, int M, int N, int K, int kw,
                             int rt, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (rt == 0) rt = pd_dec64_rt(N);
  if (M < 1 || M > 64 || N % 16 || K % 64 || (kw != 4 && kw != 8) || (size_t)X % 16 || (size_t)W % 16) return -1;
  if ((rt != 1 && rt != 2 && rt != 4) || N % (16 * rt)) return -1;
  // byte offsets (incl. the skip offset kSkip = 0x7fffff00 and its +16) stay below 2^31 and beyond every extent
  if ((long)N * K * 2 >= 0x7fffff00L || (long)M * K * 2 >= 0x7fffff00L) return -1;
  const dim3 grid(N / (16 * rt));
  // DW x RT = 8: the same 256 B of W in flight per lane at every RT
#define PD_D64(MT_, KW_, RT_) \
  dec64_kernel<MT_, KW_, 8 / RT_, RT_><<<grid, 64 * KW_, 0, st>>>((const unsigned short*)X, (const unsigned short*)W, \
                                                                  (const unsigned short*)bias, (unsigned short*)out, M, N, K)
#define PD_D64_RT(MT_, KW_) \
  if (rt == 1) PD_D64(MT_, KW_, 1); else if (rt == 2) PD_D64(MT_, KW_, 2); else PD_D64(MT_, KW_, 4);
  const int mt = (M + 15) / 16;
  if (kw == 8) {
    if (mt <= 2) { PD_D64_RT(2, 8) } else { PD_D64_RT(4, 8) }
  } else {
    if (mt <= 2) { PD_D64_RT(2, 4) } else { PD_D64_RT(4, 4) }
  }
#undef PD_D64_RT
#undef PD_D64
  return (int)hipGetLastError();
}

// The LDS-X decode GEMM (dec64s_kernel) for 16 < M <= 64: N % (64 rt) == 0, K % 64 == 0, 16-B aligned rows.
// cfg = (dw, rt, S): dw LDS ring slots (rt 1: 8 / 16, rt 2: 8 / 11); 0 fields = auto (pd_dec64s_cfg).
// ws: S * M * N floats when S > 1 (fp32 partials summed by wo_reduce_kernel).  Returns -1 outside the domain.
extern "C" void pd_dec64s_cfg(int M, int N, int K, int* dw, int* rt, int* S) {
  // ~24 MiB of weight bytes in flight chip-wide (HBM latency x bandwidth) from S x N x (DW - 1) x 128 B, and
  // enough workgroups to reach most CUs
  if (*rt == 0) *rt = (N % 128 == 0 && N >= 16384) ? 2 : 1;
  if (*dw == 0) *dw = *rt == 1 ? 16 : 11;   // the vmcnt immediate caps (DW - 2) x (2 + 2 RT) at 63
  if (*S == 0) {
    const long per = (long)N * (*dw - 1) * 128;
    int s = (int)((24L << 20) / per);
    const int wgs = N / (64 * *rt);
    while (s > 1 && wgs * s > 512) --s;
    if (s < 1) s = 1;
    if (s > K / 64) s = K / 64;
    *S = s;
  }
}

extern "C" long pd_dec64s_workspace(int M, int N, int K, int dw, int rt, int S) {
  pd_dec64s_cfg(M, N, K, &dw, &rt, &S);
  return S > 1 ? (long)S * M * N : 0;
}

extern "C" int pd_dec64s_gemm(const void* X, const void* W, const void* bias, void* out, float* ws, int M, int N,
                              int K, int dw, int rt, int S, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  pd_dec64s_cfg(M, N, K, &dw, &rt, &S);
  if (M < 1 || M > 64 || K % 64 || (size_t)X % 16 || (size_t)W % 16) return -1;
  const bool dw_ok = rt == 1 ? (dw == 8 || dw == 16) : (dw == 8 || dw == 11);
  if ((rt != 1 && rt != 2) || !dw_ok || N % (64 * rt) || S < 1 || S > K / 64) return -1;
  if (S > 1 && ws == nullptr) return -1;
  if ((long)N * K * 2 >= 0x7fffff00L || (long)M * K * 2 >= 0x7fffff00L) return -1;
  const dim3 grid(N / (64 * rt), S);
#define PD_D64S(MT_, RT_, DW_)                                                                                  \
  dec64s_kernel<MT_, 4, RT_, DW_><<<grid, 256, 0, st>>>((const unsigned short*)X, (const unsigned short*)W,     \
                                                       (const unsigned short*)bias, (unsigned short*)out, ws, M, \
                                                       N, K)
#define PD_D64S_RT(MT_)                                   \
  if (rt == 1) {                                          \
    if (dw == 8) PD_D64S(MT_, 1, 8); else PD_D64S(MT_, 1, 16); \
  } else {                                                \
    if (dw == 8) PD_D64S(MT_, 2, 8); else PD_D64S(MT_, 2, 11); \
  }
  if (M <= 32) { PD_D64S_RT(2) } else { PD_D64S_RT(4) }
#undef PD_D64S_RT
#undef PD_D64S
  if (S > 1) {
    const long total = (long)M * N;
    wo_reduce_kernel<<<(int)((total / 4 + 255) / 256), 256, 0, st>>>(ws, S, M, N, nullptr,
                                                                   (const unsigned short*)bias, (unsigned short*)out);
  }
  return (int)hipGetLastError();
}

// Decode GEMM on bf16 weights: out[M, N] = X[M, K] . W[N, K]^T (+ bias), M <= 64, split-K S (pd_dec_splits).
extern "C" int pd_dec_splits(int M, int N, int K) { return pd_wo_splits(M, N, K, 0); }

// glu: X is the gate|up output [M, 2K] and the GEMM runs on silu(gate) * up (the SwiGLU folded into X staging).
// cnt: nullable int[N / 64] zeroed counters (the fused last-arriver reduction; nullptr = separate reduce launch).
// noreduce: leave the S fp32 partials [S, M, N] in ws for the consumer to sum (pd_norm_fwd_part; pd_dec_reduce);
// `out` / `bias` unused then
extern "C" int pd_dec_gemm(const void* X, const void* W, const void* bias, void* out, float* ws, int M, int N, int K,
                           int S, int glu, int* cnt, void* stream, int noreduce) {
  hipStream_t st = (hipStream_t)stream;
  if (M < 1 || M > 64 || N % kWoRows || K % 64 || S < 1 || S > K / 64) return -1;
  const int kmax = ((K / 64 + S - 1) / S) * 64;
  const int MT = wo_mt(M), RT = wo_rt(M, N);
  const size_t lds = (size_t)M * (kmax + kWoPad) * 2;
  if (lds > 160 * 1024) return -3;
  dim3 grid(N / (kWoRows * RT), S);
  auto launch = [&](auto kern) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, 256, lds, st>>>((const unsigned short*)X, (const unsigned short*)W, ws, M, N, K, kmax, cnt,
                                 (const unsigned short*)bias, (unsigned short*)out);
  };
#define PD_DEC_R(MT_, G_)                                                                     \
  if (RT == 1) launch(dec_gemm_kernel<MT_, 1, G_>);                                          \
  else if (RT == 2) launch(dec_gemm_kernel<MT_, 2, G_>);                                     \
  else launch(dec_gemm_kernel<MT_, 4, G_>);
  if (glu) {
    if (MT == 1) { PD_DEC_R(1, true) } else if (MT == 2) { PD_DEC_R(2, true) } else { PD_DEC_R(4, true) }
  } else {
    if (MT == 1) { PD_DEC_R(1, false) } else if (MT == 2) { PD_DEC_R(2, false) } else { PD_DEC_R(4, false) }
  }
#undef PD_DEC_R
  if (cnt == nullptr && !noreduce) {
    const long total = (long)M * N;
    wo_reduce_kernel<<<(int)((total / 4 + 255) / 256), 256, 0, st>>>(ws, S, M, N, nullptr,
                                                                   (const unsigned short*)bias, (unsigned short*)out);
  }
  return (int)hipGetLastError();
}

// The reduce of a pd_dec_gemm(noreduce) call on its own: out[M, N] bf16 = sum of the S partials (+ bias)
extern "C" int pd_dec_reduce(const float* ws, int S, int M, int N, const void* bias, void* out, void* stream) {
  if (M < 1 || N % 4 || S < 1) return -1;
  const long total = (long)M * N;
  wo_reduce_kernel<<<(int)((total / 4 + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      ws, S, M, N, nullptr, (const unsigned short*)bias, (unsigned short*)out);
  return (int)hipGetLastError();
}
