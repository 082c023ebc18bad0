// Shared pieces of the hand-written gfx950 MFMA GEMMs (gemm.hip: v2 / v4 / v6, gemm7.hip: v7): parameter
// block, XCD-aware tile order, buffer descriptors, LDS-DMA lane set-up, fragment reads and the epilogues.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "common.h"

namespace pd {
namespace gm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = 256 * BK * 2;        // one operand tile, 32 KiB
constexpr int B_OFF = 2 * TILE_BYTES;           // LDS: [A stage 0 | A stage 1 | B stage 0 | B stage 1]
constexpr int LDS_BYTES = 4 * TILE_BYTES;       // 2-stage ring, 128 KiB (stage delta 32 KiB fits a ds immediate)
constexpr unsigned kOOB = 0x80000000u;          // voffset beyond num_records -> the load returns 0
constexpr int kRecords = 0x7fffffff;

// kEpiGeLU: C = gelu(acc + bias), C2 = acc + bias (the pre-activation the backward reads); kEpiDGeLU: C = acc *
// gelu'(C2) with C2 = that saved pre-activation (reference funcs/fused_gemm_epilogue.h:382 GELU_AUX_BIAS forward,
// :580 the gelu_grad backward).  Both: p.H = 1 for the tanh approximation, 0 for erf.
// kEpiRope (v7 only): bf16 out with rotate-half RoPE applied to the 128-wide heads of columns < rope_cols
// (position = row % rope_seq; fp32 cos / sin tables [rope_seq, 128]) — the QKV projection's q / k heads.
// kEpiDSwiGLU: the down projection's input gradient d_a = acc is never stored: with gate = C2[r, c], up =
// C2[r, H + c] (the SwiGLU forward's saved pre-activations) the epilogue writes C[r, c] = d_a * up * silu'(gate)
// and C[r, H + c] = d_a * silu(gate) — the SwiGLU backward (C may alias C2: every element is read, then written,
// by the same lane).
enum Epi : int { kEpiBF16 = 0, kEpiF32 = 1, kEpiSwiGLU = 2, kEpiGeLU = 3, kEpiDGeLU = 4, kEpiRope = 5,
                 kEpiDSwiGLU = 6 };

struct Params {
  const unsigned short* A;
  const unsigned short* B;
  void* C;                      // bf16 [M, ldc] or fp32 [M, ldc] (main grad) or swiglu out [M, H]
  unsigned short* C2;           // swiglu: pre-activation gu [M, 2H]
  const unsigned short* bias;   // bf16 [N] or null
  long lda, ldb, ldc, ldc2;
  int M, N, K;
  int tiles_m, tiles_n, group_m;
  float beta;
  int H;                        // swiglu: gate/up split (columns of the packed weight); gelu: 1 = tanh form
  const void* zero;             // (ablation 7) 16 zero bytes for out-of-range global_load_lds lanes
  // grouped GEMM (MoE experts): goff [ngroups + 1] device offsets, never read back by the host.
  //  gmode 0 (fwd / dgrad): group g owns rows [goff[g], goff[g+1]) of A and C; B (and bias) advance by gsb
  //          (gsbias) elements per group; tiles_m is an upper bound (sum of ceil(rows_g / 256) <= it), so a
  //          workgroup maps its row tile to (group, local tile) and leaves if it has none;
  //  gmode 1 (wgrad): group g reduces over rows [goff[g], goff[g+1]) of both operands (A M-major, B
  //          N-major) into its own C slab (C advances by gsc elements); grid = ngroups x the tile grid.
  const int* goff;
  int ngroups, gmode;
  long gsb, gsc, gsbias;
  // tail split-K (v2 kernel, not grouped): each XCD runs its full waves of tiles whole, and its last partial
  // wave's tiles as ksplit K-slices of kchunk K-tiles into fp32 slabs `part` ([8][tail_cap][ksplit][BM*BN]);
  // splitk_reduce_kernel sums the slices in order into C.  cpx = CUs (= workgroup slots) per XCD.
  float* part;
  int ksplit, kchunk, tail_cap, cpx;
  // one past the last byte of each operand (v4: the buffer descriptors' num_records), null = unbounded
  const void* a_end;
  const void* b_end;
  // fp8 GEMM (gemm8.hip): device dequant factors of A and B (the product is scaled by *sa * *sb), null = 1
  const float* sa;
  const float* sb;
  // implicit-GEMM convolution (gemm7.hip SCHED bit 11): K-tiles per tap (log2), taps, kernel width, padded row pitch,
  // padding and the shift's sign (+1 forward, -1 input gradient)
  int cv_kpb_log2, cv_taps;
  long cv_off[16];   // implicit-GEMM conv: byte offset of tap t's A rows (host-computed)
  // RoPE epilogue (kEpiRope)
  const float* rope_cos;
  const float* rope_sin;
  int rope_cols, rope_seq;
};

// Tiles [t0, t0 + n) of the grouped order belong to XCD x (the chunking xcd_remap uses); the first `full`
// of them fill whole waves of the XCD's cpx CUs, the last `tail` run in its final, partial wave.
struct XPlan {
  int t0, n, full, tail;
};
__host__ __device__ __forceinline__ XPlan xcd_plan(int nwg, int x, int cpx) {
  const int q = nwg / 8, r = nwg % 8;
  XPlan o;
  o.n = q + (x < r ? 1 : 0);
  o.t0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  o.tail = o.n % cpx;
  o.full = o.n - o.tail;
  return o;
}

// grouped tile order: group_m row-tiles sweep the column tiles together (L2 reuse within an XCD)
__device__ __forceinline__ void tile_of(const Params& p, int bid, int& tm, int& tn) {
  const int per_group = p.group_m * p.tiles_n;
  const int first_m = (bid / per_group) * p.group_m;
  const int gsz = min(p.tiles_m - first_m, p.group_m);
  tm = first_m + (bid % per_group) % gsz;
  tn = (bid % per_group) / gsz;
}

// Grouped-GEMM set-up: rebase `p` onto this workgroup's group; returns false if the workgroup has no tile.
// `bx` is the block index the tile decode below uses (gmode 1 strips the group part off it).
template <int EPI>
__device__ __forceinline__ bool group_setup(Params& p, int& bx) {
  if (p.gmode == 1) {
    const int per = p.tiles_m * p.tiles_n;
    const int g = bx / per;
    bx -= g * per;
    const int r0 = p.goff[g];
    p.K = p.goff[g + 1] - r0;
    p.A += (long)r0 * p.lda;
    p.B += (long)r0 * p.ldb;
    p.C = (char*)p.C + g * p.gsc * (EPI == kEpiF32 ? 4 : 2);
    // this group's token rows only (both operands MN-major): k past the group reads zeros (v4 range check)
    p.a_end = p.A + (p.K > 0 ? (long)(p.K - 1) * p.lda + p.M : 0);
    p.b_end = p.B + (p.K > 0 ? (long)(p.K - 1) * p.ldb + p.N : 0);
    return true;
  }
  return true;  // gmode 0 is resolved after the tile decode (it needs the row tile)
}

template <int EPI>
__device__ __forceinline__ bool group_rows(Params& p, int& tm) {
  int cum = 0, g = 0;
  for (; g < p.ngroups; ++g) {
    const int rows = p.goff[g + 1] - p.goff[g];
    const int nt = (rows + BM - 1) / BM;
    if (tm < cum + nt) break;
    cum += nt;
  }
  if (g == p.ngroups) return false;
  const int r0 = p.goff[g];
  tm -= cum;
  p.M = p.goff[g + 1] - r0;
  p.A += (long)r0 * p.lda;  // gmode 0: A is K-major (rows = tokens)
  p.C = (char*)p.C + (long)r0 * p.ldc * (EPI == kEpiF32 ? 4 : 2);
  if (EPI == kEpiSwiGLU) p.C2 += (long)r0 * p.ldc2;
  p.B += g * p.gsb;
  if (p.bias) p.bias += g * p.gsbias;
  // this group's rows / this expert's weight only: rows past the group read zeros (v4 range check)
  p.a_end = p.A + (p.M > 0 ? (long)(p.M - 1) * p.lda + p.K : 0);
  p.b_end = p.B + p.gsb;
  return true;
}

__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int q = n / 8, r = n % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// MN-major image row swizzle (8 distinct values over the rows one 32-lane half reads)
__device__ __forceinline__ int hsw(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, kRecords, 0x00020000);
}
// descriptor whose range check stops at `nbytes` past `base` (clamped to [0, 2^31 - 1]; 0 = every load is 0).
// The inputs go through readfirstlane: they are wave-uniform, and hipcc otherwise keeps a descriptor built from
// a select in VGPRs and wraps every buffer op in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, long nbytes) {
  const int n = __builtin_amdgcn_readfirstlane((int)(nbytes < 0 ? 0L : (nbytes > (long)kRecords ? (long)kRecords : nbytes)));
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, n, 0x00020000);
}

// Column remap of the B operand for the SwiGLU epilogue: tile column c (0..255) of output tile tn
// -> packed-weight column.  Wave wn's 64 columns = 32 gate + the 32 matching up columns.
template <int EPI>
__device__ __forceinline__ int bcol(int tn, int c, int H) {
  if constexpr (EPI == kEpiSwiGLU) {
    const int base = tn * 128 + (c >> 6) * 32 + (c & 31);
    return (c & 32) ? H + base : base;
  } else {
    return tn * BN + c;
  }
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA staging.  A 256 (rows = the M or N index) x 64 (k) operand tile = 32 x 1 KiB blocks; each
// thread issues 4 (blk = 8i + wave).  (Measured: giving A to waves 0-3 and B to waves 4-7 at different
// points of the K-tile is slower — profiles/r2_gemm_native.md.)
// KMAJ: element (r, k) at r*ld + k -> image [256][64] (128-B rows), 16-B chunk swizzle ^((r>>1)&7);
//       lane: row r = 64i + 8*wave + (lane>>3), chunk lc (same for all i)
// else: element (r, k) at k*ld + r -> image [64][256] (512-B rows), 32-B pair swizzle ^hsw(k);
//       lane: k = 16i + 2*wave + (lane>>5), column chunk lc (same for all i: hsw(k) ignores bit 4)
// Per lane the offset (relative to the tile's base pointer) is computed once, with the column bound
// folded in as an out-of-range offset; per K-tile only the base pointer moves (SGPRs), and rows / k are
// checked only in a ragged tile.
struct Ld {
  unsigned voff;   // byte offset of instruction 0 (column bound folded in for MN-major)
  unsigned rmask;  // K-major: bit i = row of instruction i in range
  int kl;          // K-major: lane's first k inside the tile; MN-major: lane's k for i = 0 (instr i: +16i)
};

template <bool KMAJ, bool ISB, int EPI>
__device__ __forceinline__ Ld lane_setup(long ld, int R, int t0, int H, int wave, int lane) {
  Ld o;
  if constexpr (KMAJ) {
    const int r = 8 * wave + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    o.kl = lc * 8;
    const int r0 = ISB ? t0 * BN : t0 * BM;
    o.rmask = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) o.rmask |= (unsigned)(r0 + r + 64 * i < R) << i;
    o.voff = (unsigned)(((long)r * ld + lc * 8) * 2);
  } else {
    const int kk = 2 * wave + (lane >> 5);
    const int lc = (lane & 31) ^ (hsw(kk) << 1);
    const int gc = ISB ? bcol<EPI>(t0, lc * 8, H) : t0 * BM + lc * 8;
    const int c0 = ISB ? (EPI == kEpiSwiGLU ? 0 : t0 * BN) : t0 * BM;
    o.kl = kk;
    o.rmask = 15;
    o.voff = (unsigned)(((long)kk * ld + (gc - c0)) * 2) | ((unsigned)(gc >= R) << 31);
  }
  return o;
}

// Issue DMA instruction I of a tile whose base pointer is in `rs`.  istride = byte distance between
// instructions (K-major: 64 rows, MN-major: 16 k-rows).  `full`: every row in range and k0+64 <= K.
template <bool KMAJ, int I, bool GLDS = false>
__device__ __forceinline__ void dma(const __amdgpu_buffer_rsrc_t& rs, const Ld& L, unsigned istride, lds_char* dst,
                                    int wave, bool full, int krem, const char* gbase = nullptr,
                                    const char* zero = nullptr) {
  const bool ok = full || (KMAJ ? (((L.rmask >> I) & 1) && L.kl < krem) : (L.kl + 16 * I < krem));
  if constexpr (GLDS) {
    // global_load_lds_dwordx4 variant (ablation): per-lane 64-bit address, out-of-range lanes read zeros
    const unsigned v = L.voff + I * istride;
    const char* src = (ok && !(v >> 31)) ? gbase + v : zero;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + (8 * I + wave) * 1024),
                                     16, 0, 0);
  } else {
    const unsigned voff = (L.voff + I * istride) | ((unsigned)(!ok) << 31);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (8 * I + wave) * 1024),
                                             16, voff, 0, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------------
// Fragment reads (inline asm).  hipcc models the transposed-read builtin as aliasing the in-flight
// LDS-DMA and drains vmcnt(0) before it (serialising the prefetch), and its counted lgkmcnt waits
// for builtin reads would also count asm reads issued after them.  So every fragment read is asm
// with a per-lane base VGPR (computed once per stage) + a compile-time immediate, and the kernel
// retires them itself: lgkmcnt(0) at the start of the consuming sub-phase (`sync_frags`).
template <int IMM>
__device__ __forceinline__ bf16x8 rd128(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(IMM));
  return v;
}
template <int IMM>
__device__ __forceinline__ s16x4 rdtr(unsigned addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(IMM));
  return v;
}
__device__ __forceinline__ bf16x8 cat(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ void sync_frags() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ f32x4v mfma(bf16x8 a, bf16x8 b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// D = A.B + D with D pinned to AGPRs (v4); see the note at its use
__device__ __forceinline__ void mfma_agpr(f32x4v& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// v_rcp_f32 (1 ulp) instead of the IEEE divide sequence: the epilogue is exposed VALU time
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// GELU and its derivative in fp32 (torch's two forms: erf, and tanh with approximate = True)
__device__ __forceinline__ float gelu_f(float x, int tanh_form) {
  if (tanh_form) return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x)));
  return 0.5f * x * (1.f + erff(x * 0.70710678118f));
}
__device__ __forceinline__ float dgelu_f(float x, int tanh_form) {
  if (tanh_form) {
    const float x2 = x * x, t = tanhf(0.7978845608f * (x + 0.044715f * x2 * x));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608f * (1.f + 0.134145f * x2);
  }
  return 0.5f * (1.f + erff(x * 0.70710678118f)) + x * 0.3989422804f * __expf(-0.5f * x * x);
}

// bf16 output value of the bf16-producing epilogues from the fp32 accumulator: the plain / bias value, gelu of the
// (bf16-rounded, stored) pre-activation, or acc * gelu'(saved pre-activation `aux`)
template <int EPI>
__device__ __forceinline__ unsigned short epi_out(float acc, float bv, unsigned short aux, int tanh_form,
                                                  unsigned short& pre) {
  if constexpr (EPI == kEpiDGeLU) {
    return f2bf(acc * dgelu_f(bf2f(aux), tanh_form));
  } else {
    pre = f2bf(acc + bv);
    if constexpr (EPI == kEpiGeLU) return f2bf(gelu_f(bf2f(pre), tanh_form));
    return pre;
  }
}

template <int N, typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl<N>(f, std::make_integer_sequence<int, N>{});
}

// Per-lane fragment-read bases of one operand (stage 0; stage 1 is +TILE_BYTES in the immediate).
//  K-major: 2 bases (k32 step s); fragment (tile u of the wave's rows, step s) = b[s] + u*16*128.
//  MN-major: base x + ((F + u) ^ h) * 32 for wave-local 16-column tile u, with F = the wave's first
//  tile; the XOR is recomputed per read (2 VALU beside the MFMAs) instead of holding 4-8 bases.
template <bool KMAJ>
struct RdB {
  unsigned b[2];  // K-major: per-step bases; MN-major: b[0] = x, b[1] = h
  int f;          // MN-major: first 16-column tile of the wave
};

template <bool KMAJ>
__device__ __forceinline__ RdB<KMAJ> rd_setup(unsigned img, int first, int lane) {
  // img: LDS byte address of the operand tile; first: wave's first row (K-major) / column (MN-major)
  RdB<KMAJ> o;
  if constexpr (KMAJ) {
    const int rl = lane & 15;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = (4 * s + (lane >> 4)) ^ ((rl >> 1) & 7);
      o.b[s] = img + (first + rl) * 128 + ch * 16;
    }
    o.f = 0;
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    o.b[0] = img + (8 * g + q) * 512 + (pp >> 1) * 16 + (pp & 1) * 8;
    o.b[1] = q | ((g & 1) << 2);
    o.f = first >> 4;
  }
  return o;
}

// fragment of wave-local 16-row/col tile U (0..7 for A, 0..3 for B) at k32 step S out of stage ST
template <bool KMAJ, int U, int S, int ST>
__device__ __forceinline__ bf16x8 read_frag(const RdB<KMAJ>& r) {
  if constexpr (KMAJ) {
    return rd128<ST * TILE_BYTES + U * 16 * 128>(r.b[S]);
  } else {
    unsigned h = r.b[1];
    asm volatile("" : "+v"(h));  // opaque: keep the per-tile base out of loop-invariant hoisting
    const unsigned a = r.b[0] + (((unsigned)(r.f + U) ^ h) << 5);
    return cat(rdtr<ST * TILE_BYTES + S * 16384>(a), rdtr<ST * TILE_BYTES + S * 16384 + 2048>(a));
  }
}

// Epilogue from the accumulators.  acc[i][j]: rows arow + 16i + 4*(lane>>4) + e, tile column
// bcolw + 16j + (lane&15) (v_mfma_f32_16x16x32_bf16 C layout).
template <int EPI>
__device__ __forceinline__ void epilogue(const Params& p, f32x4v (&acc)[8][4], int tm, int tn, int arow, int bcolw,
                                         int wn, int lane) {
  const int row0 = tm * BM + arow + 4 * (lane >> 4);
  if constexpr (EPI == kEpiSwiGLU) {
    // gate = acc[i][0..1], up = acc[i][2..3] at the same lane position
    unsigned short* out = (unsigned short*)p.C;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gc = tn * 128 + wn * 32 + 16 * j + (lane & 15);  // gate column == output column
      if (gc >= p.H) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = row0 + 16 * i + e;
          if (r < p.M) {
            const float g = bf2f(f2bf(acc[i][j][e]));
            const float u = bf2f(f2bf(acc[i][2 + j][e]));
            p.C2[(long)r * p.ldc2 + gc] = f2bf(g);
            p.C2[(long)r * p.ldc2 + p.H + gc] = f2bf(u);
            out[(long)r * p.ldc + gc] = f2bf(silu(g) * u);
          }
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tn * BN + bcolw + 16 * j + (lane & 15);
      if (c >= p.N) continue;
      float bv = 0.f;
      if constexpr (EPI == kEpiBF16 || EPI == kEpiGeLU) {
        if (p.bias) bv = bf2f(p.bias[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = row0 + 16 * i + e;
          if (r < p.M) {
            if constexpr (EPI != kEpiF32) {
              unsigned short pre;
              const unsigned short aux = EPI == kEpiDGeLU ? p.C2[(long)r * p.ldc2 + c] : 0;
              ((unsigned short*)p.C)[(long)r * p.ldc + c] = epi_out<EPI>(acc[i][j][e], bv, aux, p.H, pre);
              if constexpr (EPI == kEpiGeLU) p.C2[(long)r * p.ldc2 + c] = pre;
            } else {
              float* cp = (float*)p.C + (long)r * p.ldc + c;
              *cp = p.beta != 0.f ? acc[i][j][e] + p.beta * *cp : acc[i][j][e];
            }
          }
        }
    }
  }
}

// LDS images, swizzles, range checks and epilogues are v2's (the DMA lane mapping of v2's 8 waves is
// kept: wave w issues the pieces of v2 waves w and w + 4).  Per CU and K-tile the piece count and LDS
// bytes equal v2's; what changes is that the MFMA pipe of each SIMD is fed by one wave that issues its
// DMA spread out, and B fragments are shared by 128 rows instead of 64 (1/3 fewer LDS reads per MFMA).
// Epilogue of the transposed accumulator layout (v4): acc[i][j][e] = C[row 16i + (lane & 15)][col 16j + 4 * (lane
// >> 4) + e] relative to (arow, bcolw) of tile (tm, tn).  One 8-B (bf16) / 16-B (fp32) access per (i, j) when the
// 4 columns are in range and aligned, element-wise at the ragged right edge.  SwiGLU: gate = columns j in {0, 1},
// up = j + 2 at the same lane position (the B column remap of bcol<>).
template <int EPI>
__device__ __forceinline__ void epilogue_t(const Params& p, f32x4v (&acc)[8][4], int tm, int tn, int arow, int bcolw,
                                           int lane) {
  const int row0 = tm * BM + arow + (lane & 15);
  const int cq = 4 * (lane >> 4);
  if constexpr (EPI == kEpiSwiGLU) {
    const int wn = bcolw >> 6;  // 64-column half of the tile: 32 gate + 32 up columns
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gc = tn * 128 + wn * 32 + 16 * j + cq;  // first of the lane's 4 gate (== output) columns
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = row0 + 16 * i;
        if (r >= p.M) continue;
        unsigned short g[4], u[4], o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[e] = f2bf(acc[i][j][e]);
          u[e] = f2bf(acc[i][2 + j][e]);
          o[e] = f2bf(silu(bf2f(g[e])) * bf2f(u[e]));
        }
        unsigned short* gp = p.C2 + (long)r * p.ldc2 + gc;
        unsigned short* op = (unsigned short*)p.C + (long)r * p.ldc + gc;
        if (gc + 3 < p.H) {
          *(uint2*)gp = make_uint2(g[0] | (unsigned)g[1] << 16, g[2] | (unsigned)g[3] << 16);
          *(uint2*)(gp + p.H) = make_uint2(u[0] | (unsigned)u[1] << 16, u[2] | (unsigned)u[3] << 16);
          *(uint2*)op = make_uint2(o[0] | (unsigned)o[1] << 16, o[2] | (unsigned)o[3] << 16);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (gc + e < p.H) {
              gp[e] = g[e];
              gp[p.H + e] = u[e];
              op[e] = o[e];
            }
        }
      }
    }
  } else if constexpr (EPI == kEpiDSwiGLU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tn * BN + bcolw + 16 * j + cq;   // d_a column = gate column; up at c + H
      if (c >= p.N) continue;
      const bool vec = c + 3 < p.N;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = row0 + 16 * i;
        if (r >= p.M) continue;
        const unsigned short* gp = p.C2 + (long)r * p.ldc2 + c;
        unsigned short* dp = (unsigned short*)p.C + (long)r * p.ldc + c;
        unsigned short g[4], u[4], dg[4], du[4];
        if (vec) {
          const uint2 g2 = *(const uint2*)gp, u2 = *(const uint2*)(gp + p.H);
          g[0] = g2.x & 0xffff; g[1] = g2.x >> 16; g[2] = g2.y & 0xffff; g[3] = g2.y >> 16;
          u[0] = u2.x & 0xffff; u[1] = u2.x >> 16; u[2] = u2.y & 0xffff; u[3] = u2.y >> 16;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            g[e] = c + e < p.N ? gp[e] : 0;
            u[e] = c + e < p.N ? gp[p.H + e] : 0;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = bf2f(g[e]), uv = bf2f(u[e]), da = acc[i][j][e];
          const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-gv));
          dg[e] = f2bf(da * uv * sg * (1.f + gv * (1.f - sg)));
          du[e] = f2bf(da * gv * sg);
        }
        if (vec) {
          *(uint2*)dp = make_uint2(dg[0] | (unsigned)dg[1] << 16, dg[2] | (unsigned)dg[3] << 16);
          *(uint2*)(dp + p.H) = make_uint2(du[0] | (unsigned)du[1] << 16, du[2] | (unsigned)du[3] << 16);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < p.N) {
              dp[e] = dg[e];
              dp[p.H + e] = du[e];
            }
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tn * BN + bcolw + 16 * j + cq;
      if (c >= p.N) continue;
      const bool vec = c + 3 < p.N;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == kEpiBF16 || EPI == kEpiGeLU) {
        if (p.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[e] = c + e < p.N ? bf2f(p.bias[c + e]) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = row0 + 16 * i;
        if (r >= p.M) continue;
        if constexpr (EPI != kEpiF32) {
          unsigned short* cp = (unsigned short*)p.C + (long)r * p.ldc + c;
          unsigned short* ap = EPI == kEpiBF16 ? nullptr : p.C2 + (long)r * p.ldc2 + c;
          unsigned short o[4], pre[4], aux[4] = {0, 0, 0, 0};
          if constexpr (EPI == kEpiDGeLU) {
            if (vec) {
              const uint2 a2 = *(const uint2*)ap;
              aux[0] = a2.x & 0xffff; aux[1] = a2.x >> 16; aux[2] = a2.y & 0xffff; aux[3] = a2.y >> 16;
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) aux[e] = c + e < p.N ? ap[e] : 0;
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = epi_out<EPI>(acc[i][j][e], bv[e], aux[e], p.H, pre[e]);
          if (vec) {
            *(uint2*)cp = make_uint2(o[0] | (unsigned)o[1] << 16, o[2] | (unsigned)o[3] << 16);
            if constexpr (EPI == kEpiGeLU)
              *(uint2*)ap = make_uint2(pre[0] | (unsigned)pre[1] << 16, pre[2] | (unsigned)pre[3] << 16);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c + e < p.N) {
                cp[e] = o[e];
                if constexpr (EPI == kEpiGeLU) ap[e] = pre[e];
              }
          }
        } else {
          float* cp = (float*)p.C + (long)r * p.ldc + c;
          if (vec) {
            float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
            if (p.beta != 0.f) {
              const float4 o = *(const float4*)cp;
              v.x += p.beta * o.x; v.y += p.beta * o.y; v.z += p.beta * o.z; v.w += p.beta * o.w;
            }
            *(float4*)cp = v;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c + e < p.N) cp[e] = p.beta != 0.f ? acc[i][j][e] + p.beta * cp[e] : acc[i][j][e];
          }
        }
      }
    }
  }
}

constexpr int NTHR4 = 256;

// Per-lane fragment-read bases (stage 0, k32 step 0).  K-major: one base per k32 step, fragment u at an
// immediate +u*2048.  MN-major: one base per 16-column tile u with the pair swizzle folded in (512 registers
// leave room for 8 bases), step / stage / the second 4-row half as immediates — no VALU per read.
template <bool KMAJ>
struct Rd4 {
  unsigned b[KMAJ ? 2 : 8];
};

template <bool KMAJ>
__device__ __forceinline__ Rd4<KMAJ> rd4_setup(unsigned img, int first, int lane) {
  Rd4<KMAJ> o;
  if constexpr (KMAJ) {
    const int rl = lane & 15;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = (4 * s + (lane >> 4)) ^ ((rl >> 1) & 7);
      o.b[s] = img + (first + rl) * 128 + ch * 16;
    }
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const unsigned x = img + (8 * g + q) * 512 + (pp >> 1) * 16 + (pp & 1) * 8;
    const unsigned h = q | ((g & 1) << 2);
    const int f = first >> 4;
#pragma unroll
    for (int u = 0; u < 8; ++u) o.b[u] = x + (((unsigned)(f + u) ^ h) << 5);
  }
  return o;
}

template <bool KMAJ, int U, int S, int ST>
__device__ __forceinline__ bf16x8 frag4(const Rd4<KMAJ>& r) {
  if constexpr (KMAJ) {
    return rd128<ST * TILE_BYTES + U * 16 * 128>(r.b[S]);
  } else {
    return cat(rdtr<ST * TILE_BYTES + S * 16384>(r.b[U]), rdtr<ST * TILE_BYTES + S * 16384 + 2048>(r.b[U]));
  }
}

// Per-lane DMA source offsets of this wave's 8 pieces of one operand (piece 4h + I = instruction I of v2 wave
// wave + 4h), column bound folded in as bit 31 (MN-major); kl[h]: K-major lane's first k in the tile (masked
// mode only).
struct Pc4 {
  unsigned v[8];
  int kl[2];
};

template <bool KMAJ, bool ISB, int EPI>
__device__ __forceinline__ Pc4 pc4_setup(long ld, int R, int t0, int H, int wave, int lane, unsigned istride) {
  Pc4 o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const Ld L = lane_setup<KMAJ, ISB, EPI>(ld, R, t0, H, wave + 4 * h, lane);
    o.kl[h] = L.kl;
#pragma unroll
    for (int i = 0; i < 4; ++i) o.v[4 * h + i] = L.voff + i * istride;
  }
  return o;
}

// FAST: no per-lane k masks — every operand is bounded by the hardware range check alone (exact extents, and
// descriptors of tiles past K carry num_records 0); otherwise a K-major operand's last, partial K-tile masks the

}  // namespace gm
}  // namespace pd
