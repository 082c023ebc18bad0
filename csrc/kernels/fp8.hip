// FP8 (OCP e4m3fn / e5m2) casting for delayed-scaling fp8 GEMMs on gfx950.
//
// Reference behaviour: the fp8 GEMM path of the reference (tensor/linalg.py:329
// fp8_fp8_half_gemm_fused; phi/kernels/fusion/gpu/fp8_*) quantizes activations/weights with a
// per-tensor scale.  The MI355X design follows the delayed-scaling recipe: the scale used for
// this step's cast comes from the amax HISTORY (known before the cast), and the cast kernel
// computes this tensor's amax in the same pass (one read of the bf16 tensor), so quantization
// is a single fused pass:
//   * cast_amax:            y = sat(x * scale) -> fp8, amax = max|x|            (row-major)
//   * cast_transpose_amax:  y = sat(x * scale) and yT = y^T -> fp8, amax       (bf16: in-register 8x8 byte
//                           transposes, cast_transpose_amax_v2_kernel; other types: 64x64 LDS tiles)
// amax is kAmaxSlots floats per tensor role (sharded same-address atomics), folded by update_scale.
// The transposed copy is what the column-major B operand of the fp8 GEMM wants for the weight
// (forward) and for x / dy (weight-gradient GEMM).  Conversion uses v_cvt_pk_fp8_f32 /
// v_cvt_pk_bf8_f32 (OCP encodings on gfx950) after saturating to the format's max finite value.
#include "common.h"

namespace pd {
namespace fp8 {

template <bool E5M2>
__device__ __forceinline__ unsigned pack4(float a, float b, float c, float d) {
  constexpr float kMax = E5M2 ? 57344.f : 448.f;
  a = fminf(fmaxf(a, -kMax), kMax);
  b = fminf(fmaxf(b, -kMax), kMax);
  c = fminf(fmaxf(c, -kMax), kMax);
  d = fminf(fmaxf(d, -kMax), kMax);
  int w;
  if (E5M2) {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  }
  return (unsigned)w;
}

// non-negative floats order like their bit patterns -> integer atomicMax
__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  atomicMax(reinterpret_cast<unsigned*>(addr), __float_as_uint(v));
}

// A tensor role's amax lives in kAmaxSlots floats: workgroup b adds into slot b % kAmaxSlots (same-address atomics
// serialise at ~12 ns each — a 1k-workgroup cast spent ~12 us on its ONE amax word); update_scale folds the slots.
constexpr int kAmaxSlots = 64;

// block-wide max, then ONE atomic per workgroup into its slot
__device__ __forceinline__ void block_amax(float m, float* amax) {
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0 && amax)
    atomic_max_pos(amax + (blockIdx.x % kAmaxSlots), fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// 4 x 4 byte transpose: rows a..d (each 4 fp8 of consecutive columns) -> 4 words, word j = column j's 4 rows
__device__ __forceinline__ void tr4x4(unsigned a, unsigned b, unsigned c, unsigned d, unsigned (&o)[4]) {
  const unsigned ab0 = __builtin_amdgcn_perm(b, a, 0x05010400u), ab1 = __builtin_amdgcn_perm(b, a, 0x07030602u);
  const unsigned cd0 = __builtin_amdgcn_perm(d, c, 0x05010400u), cd1 = __builtin_amdgcn_perm(d, c, 0x07030602u);
  o[0] = __builtin_amdgcn_perm(cd0, ab0, 0x05040100u);
  o[1] = __builtin_amdgcn_perm(cd0, ab0, 0x07060302u);
  o[2] = __builtin_amdgcn_perm(cd1, ab1, 0x05040100u);
  o[3] = __builtin_amdgcn_perm(cd1, ab1, 0x07060302u);
}

// x [R, C] bf16 (C % 8 == 0, R % 8 == 0) -> y [R, C] (optional) and yT [C, R], LDS-free: a lane quantises an 8 x 8 block
// (8 rows x one 16-B load each), writes its 8 row words of y (8 B each) and, after an in-register byte transpose
// (v_perm), its 8 column words of yT (8 B each: rows 8rb..8rb+7 of one column).  A wave covers 64 rows x 64 columns
// (lane: rb = lane & 7, cb = lane >> 3 -> the 8 lanes of a row block read one 128-B row segment, the 8 lanes of a
// column write one 64-B yT segment); a workgroup 64 rows x 256 columns.  Replaces the 64 x 64 fp32 LDS-tile kernel
// (two barriers per tile, 4-B stores; ~57 us per [4096, 5120] cast in the GPT-3 13B fp8 step).
// colpart (optional, the fp8 linear's dY cast): the unscaled column sums of each 64-row block, fp32 [ceil(R/64), C],
// for the bias gradient (colsum_kernel folds the row blocks) — the bias-grad pass no longer re-reads dY.
template <bool E5M2>
__global__ __launch_bounds__(256) void cast_transpose_amax_v2_kernel(const unsigned short* __restrict__ x,
                                                                     uint8_t* __restrict__ y, uint8_t* __restrict__ yT,
                                                                     int R, int C, const float* __restrict__ scale,
                                                                     float* __restrict__ amax,
                                                                     float* __restrict__ colpart) {
  const float s = scale[0];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rb = lane & 7, cb = lane >> 3;
  const int tilesC = (C + 255) / 256;
  const int r = (blockIdx.x / tilesC) * 64 + 8 * rb;
  const int c = (blockIdx.x % tilesC) * 256 + wave * 64 + 8 * cb;
  float m = 0.f;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < R && c < C) {
    unsigned lo[8], hi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v[8];
      load_vec<bf16, 8>(reinterpret_cast<const bf16*>(x) + (long)(r + i) * C + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
      if (colpart) {
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] += v[j];
      }
      lo[i] = pack4<E5M2>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
      hi[i] = pack4<E5M2>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    }
    if (y) {
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<uint2*>(y + (long)(r + i) * C + c) = make_uint2(lo[i], hi[i]);
    }
    unsigned t0[4], t1[4], t2[4], t3[4];
    tr4x4(lo[0], lo[1], lo[2], lo[3], t0);   // columns 0-3, rows 0-3
    tr4x4(lo[4], lo[5], lo[6], lo[7], t1);   // columns 0-3, rows 4-7
    tr4x4(hi[0], hi[1], hi[2], hi[3], t2);   // columns 4-7, rows 0-3
    tr4x4(hi[4], hi[5], hi[6], hi[7], t3);   // columns 4-7, rows 4-7
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<uint2*>(yT + (long)(c + j) * R + r) = make_uint2(t0[j], t1[j]);
      *reinterpret_cast<uint2*>(yT + (long)(c + 4 + j) * R + r) = make_uint2(t2[j], t3[j]);
    }
  }
  if (colpart) {
    // the 8 lanes of a column block (rb = 0..7: consecutive lanes) hold 8 rows each: fold them, lane rb = 0 stores
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cs[j] += __shfl_xor(cs[j], 1);
      cs[j] += __shfl_xor(cs[j], 2);
      cs[j] += __shfl_xor(cs[j], 4);
    }
    if (rb == 0 && c < C) {
      float* dst = colpart + (long)(blockIdx.x / tilesC) * C + c;
      *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
  block_amax(m, amax);
}

template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_amax_kernel(const T* __restrict__ x, uint8_t* __restrict__ y, long n,
                                                        const float* __restrict__ scale, float* __restrict__ amax) {
  const float s = scale[0];
  float m = 0.f;
  const long n8 = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    constexpr int W = 16 / sizeof(T);  // 8 bf16 or 4 fp32 per 16-B load
#pragma unroll
    for (int j = 0; j < 8; j += W) {
      float t[W];
      load_vec<T, W>(x + i * 8 + j, t);
#pragma unroll
      for (int q = 0; q < W; ++q) v[j + q] = t[q];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    uint2 o;
    o.x = pack4<E5M2>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    o.y = pack4<E5M2>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    *reinterpret_cast<uint2*>(y + i * 8) = o;
  }
  for (long i = n8 * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {  // tail
    const float v = Elt<T>::ld(x + i);
    m = fmaxf(m, fabsf(v));
    y[i] = (uint8_t)(pack4<E5M2>(v * s, 0.f, 0.f, 0.f) & 0xff);
  }
  block_amax(m, amax);
}

// x [R, C] -> y [R, C] (optional) and yT [C, R].  Grid-stride over 64x64 tiles: each thread loads
// 2 x 16 B of bf16 along a row, the scaled tile is staged in LDS as fp32 ([64][65], conflict-free
// column reads), then written row-major and transposed as 4-byte fp8 words.
template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_transpose_amax_kernel(const T* __restrict__ x, uint8_t* __restrict__ y,
                                                                  uint8_t* __restrict__ yT, int R, int C,
                                                                  const float* __restrict__ scale,
                                                                  float* __restrict__ amax) {
  __shared__ float tile[64][65];
  const float s = scale[0];
  const int tilesC = (C + 63) / 64, tilesR = (R + 63) / 64;
  const int ntiles = tilesC * tilesR;
  float m = 0.f;
  const bool vec = (C % 8) == 0 && sizeof(T) == 2;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r0 = (t / tilesC) * 64, c0 = (t % tilesC) * 64;
    if (vec) {
      // 64 rows x 8 chunks of 8 elements; 256 threads -> 2 chunks each
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int idx = threadIdx.x + 256 * k, rr = idx >> 3, cc = (idx & 7) * 8;
        const int r = r0 + rr, c = c0 + cc;
        float v[8];
        if (r < R && c + 7 < C) {
          if constexpr (sizeof(T) == 2) load_vec<T, 8>(x + (long)r * C + c, v);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (r < R && c + j < C) ? Elt<T>::ld(x + (long)r * C + c + j) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          m = fmaxf(m, fabsf(v[j]));
          tile[rr][cc + j] = v[j] * s;
        }
      }
    } else {
      const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int r = r0 + ty + 4 * k, c = c0 + tx;
        float v = 0.f;
        if (r < R && c < C) v = Elt<T>::ld(x + (long)r * C + c);
        m = fmaxf(m, fabsf(v));
        tile[ty + 4 * k][tx] = v * s;
      }
    }
    __syncthreads();
    if (y) {
      const int row = threadIdx.x >> 4, cq = (threadIdx.x & 15) * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rr = row + 16 * k, r = r0 + rr, c = c0 + cq;
        if (r < R) {
          const unsigned w = pack4<E5M2>(tile[rr][cq], tile[rr][cq + 1], tile[rr][cq + 2], tile[rr][cq + 3]);
          if (c + 3 < C) *reinterpret_cast<unsigned*>(y + (long)r * C + c) = w;
          else
            for (int j = 0; j < 4 && c + j < C; ++j) y[(long)r * C + c + j] = (uint8_t)((w >> (8 * j)) & 0xff);
        }
      }
    }
    {
      const int col = threadIdx.x >> 4, rq = (threadIdx.x & 15) * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cc = col + 16 * k, c = c0 + cc, r = r0 + rq;
        if (c < C) {
          const unsigned w = pack4<E5M2>(tile[rq][cc], tile[rq + 1][cc], tile[rq + 2][cc], tile[rq + 3][cc]);
          if (r + 3 < R) *reinterpret_cast<unsigned*>(yT + (long)c * R + r) = w;
          else
            for (int j = 0; j < 4 && r + j < R; ++j) yT[(long)c * R + r + j] = (uint8_t)((w >> (8 * j)) & 0xff);
        }
      }
    }
    __syncthreads();  // tile reused by the next iteration
  }
  block_amax(m, amax);
}

// delayed-scaling bookkeeping on device: roll the amax history, new scale = fp8_max / max(history)
// / 2^margin (kept when the history is all zero), and the matching inverse scale for the GEMM.  One wave, one
// element per lane (kAmaxSlots == 64, history length <= 64): the slot fold, the roll and the history max are lane
// loads + a wave max, not the serial single-lane loops of the first form (8 us per call, 480 calls = 4 ms of the
// GPT-3 13B fp8 step); longer histories take the serial loop.
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// up to kMaxMetas tensor roles in one launch (workgroup b = role b; ops/fp8.py batches the deferred updates of
// several linears).  The dequant factor each cast used is snapshotted into snap[b] (nullable) before the roll —
// the backward's copy, in the same launch instead of a separate 4-byte device copy per role (320 copyBuffer launches per GPT-3 13B step)
constexpr int kMaxMetas = 16;
struct UpdArgs {
  float* hist[kMaxMetas];
  float* amax[kMaxMetas];
  float* scale[kMaxMetas];
  float* inv[kMaxMetas];
  float* snap[kMaxMetas];
  int len[kMaxMetas];
  float fp8_max[kMaxMetas];
  float margin_pow2[kMaxMetas];
};

__global__ __launch_bounds__(64) void update_scale_kernel(UpdArgs u) {
  static_assert(kAmaxSlots == 64, "one amax slot per lane");
  const int b = blockIdx.x, i = threadIdx.x;
  float* __restrict__ hist = u.hist[b];
  float* __restrict__ amax = u.amax[b];
  const int len = u.len[b];
  const float a = wave_max(amax[i]);
  float m;
  if (len <= 64) {
    const float prev = (i > 0 && i < len) ? hist[i - 1] : 0.f;   // every lane reads before any lane writes
    const float h = i == 0 ? a : prev;
    m = wave_max(i < len ? h : 0.f);
    if (i < len) hist[i] = h;
  } else {
    m = 0.f;
    if (i == 0) {
      for (int j = len - 1; j > 0; --j) hist[j] = hist[j - 1];
      hist[0] = a;
      for (int j = 0; j < len; ++j) m = fmaxf(m, hist[j]);
    }
  }
  amax[i] = 0.f;
  if (i == 0) {
    if (u.snap[b]) u.snap[b][0] = u.inv[b][0];
    float s = u.scale[b][0];
    if (m > 0.f && isfinite(m)) s = u.fp8_max[b] / m / u.margin_pow2[b];
    u.scale[b][0] = s;
    u.inv[b][0] = 1.f / s;
  }
}

}  // namespace fp8
}  // namespace pd

using namespace pd;

// colpart: optional fp32 [ceil(R / 64), C] column sums of x per 64-row block (bf16 x with a transposed copy only:
// the LDS-free v2 path); -5 when requested on another path (the caller then sums the columns itself).
extern "C" int pd_fp8_cast(int dt, int e5m2, const void* x, void* y, void* yT, long R, long C, const float* scale,
                           float* amax, float* colpart, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v2 = yT != nullptr && dt == kBF16 && C % 8 == 0 && R % 8 == 0 && (size_t)x % 16 == 0 &&
                  (size_t)yT % 8 == 0 && (!y || (size_t)y % 8 == 0) && R * C < (1L << 31);
  if (colpart && (!v2 || (size_t)colpart % 16 != 0)) return -5;
  if (yT == nullptr) {
    const long n = R * C;
    long g = (n / 8 + 255) / 256;
    if (g < 1) g = 1;
    if (g > 1024) g = 1024;
#define PD_FP8_CAST(E)                                                                                           \
  PD_DISPATCH_FLOAT(dt, T, fp8::cast_amax_kernel<T, E><<<(int)g, 256, 0, st>>>((const T*)x, (uint8_t*)y, n, scale, \
                                                                               amax))
    if (e5m2) { PD_FP8_CAST(true); } else { PD_FP8_CAST(false); }
#undef PD_FP8_CAST
  } else if (v2) {
    const long wgs = ((C + 255) / 256) * ((R + 63) / 64);
    if (e5m2)
      fp8::cast_transpose_amax_v2_kernel<true><<<(unsigned)wgs, 256, 0, st>>>(
          (const unsigned short*)x, (uint8_t*)y, (uint8_t*)yT, (int)R, (int)C, scale, amax, colpart);
    else
      fp8::cast_transpose_amax_v2_kernel<false><<<(unsigned)wgs, 256, 0, st>>>(
          (const unsigned short*)x, (uint8_t*)y, (uint8_t*)yT, (int)R, (int)C, scale, amax, colpart);
  } else {
    long tiles = ((C + 63) / 64) * ((R + 63) / 64);
    dim3 grid((unsigned)(tiles < 1024 ? tiles : 1024));
#define PD_FP8_CT(E)                                                                                        \
  PD_DISPATCH_FLOAT(dt, T, fp8::cast_transpose_amax_kernel<T, E><<<grid, 256, 0, st>>>(                        \
                               (const T*)x, (uint8_t*)y, (uint8_t*)yT, (int)R, (int)C, scale, amax))
    if (e5m2) { PD_FP8_CT(true); } else { PD_FP8_CT(false); }
#undef PD_FP8_CT
  }
  return (int)hipGetLastError();
}

extern "C" int pd_fp8_update_scale(int n, float* const* hist, const int* len, float* const* amax, float* const* scale,
                                   float* const* inv_scale, float* const* snap, const float* fp8_max,
                                   const float* margin_pow2, void* stream) {
  if (n < 1 || n > fp8::kMaxMetas) return -1;
  fp8::UpdArgs u{};
  for (int b = 0; b < n; ++b) {
    u.hist[b] = hist[b];
    u.amax[b] = amax[b];
    u.scale[b] = scale[b];
    u.inv[b] = inv_scale[b];
    u.snap[b] = snap[b];
    u.len[b] = len[b];
    u.fp8_max[b] = fp8_max[b];
    u.margin_pow2[b] = margin_pow2[b];
  }
  fp8::update_scale_kernel<<<n, 64, 0, (hipStream_t)stream>>>(u);
  return (int)hipGetLastError();
}
