// Shared pieces of the TN (both operands K-major) persistent GEMMs: gemm7.hip (bf16 MFMA, v7) and gemm8.hip
// (fp8 / bf8 MFMA): LDS-DMA piece offsets, counted waits, DMA-behind-MFMA asm, 16-B epilogue stores.
#pragma once
#include "gemm_core.h"

namespace pd {
namespace gm {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

// Per-lane source offsets of this wave's 8 LDS-DMA pieces of a K-major operand (v4's image): piece j fills LDS
// block 8(j&3) + 4(j>>2) + wave = rows 64(j&3) + 8(wave + 4(j>>2)) + (lane>>3), 16-B chunk (lane&7) ^ ((row>>1)&7).
// SwiGLU: tile row r of the packed gate|up weight (read as [2H, K] rows) is gate row (r>>6)*32 + (r&31) or the
// matching up row H + ... (bit 5), relative to the tile's first gate row.
template <bool SWI>
__device__ __forceinline__ void kk_offsets(unsigned (&v)[8], long ld, int H, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 64 * (j & 3) + 8 * (wave + 4 * (j >> 2)) + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    const long row = SWI ? (long)((r >> 6) * 32 + (r & 31) + ((r & 32) ? H : 0)) : (long)r;
    v[j] = (unsigned)((row * ld + lc * 8) * 2);
  }
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// one MFMA with an LDS-DMA piece behind it: M0 (LDS destination = wb + IMM) is written before the MFMA, which
// covers the M0 -> buffer_load ... lds hazard.  POL = the load's cache policy (SCHED bits 2-3 for A, 4-5 for B):
// 0 default, 1 sc0 sc1 (L1 bypass), 2 nt (streaming), 3 sc1.
#define PD_V7_MFMA_DMA(POLSTR)                                        \
  asm volatile(                                                      \
      "s_add_u32 m0, %1, %2\n\t"                                     \
      "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\t"                  \
      "buffer_load_dwordx4 %5, %6, 0 offen" POLSTR " lds"             \
      : "+a"(c)                                                      \
      : "s"(wb), "i"(IMM), "v"(a), "v"(b), "v"(voff), "s"(srd)       \
      : "memory")
#define PD_V7_DMA_ONLY(POLSTR)                                        \
  asm volatile(                                                      \
      "s_add_u32 m0, %0, %1\n\t"                                     \
      "s_nop 0\n\t"                                                  \
      "buffer_load_dwordx4 %2, %3, 0 offen" POLSTR " lds"             \
      :                                                              \
      : "s"(wb), "i"(IMM), "v"(voff), "s"(srd)                       \
      : "memory")
template <int IMM, int POL = 0>
__device__ __forceinline__ void mfma_dma(f32x4v& c, const bf16x8& a, const bf16x8& b, unsigned wb, unsigned voff,
                                         const i32x4& srd) {
  if constexpr (POL == 1) PD_V7_MFMA_DMA(" sc0 sc1");
  else if constexpr (POL == 2) PD_V7_MFMA_DMA(" nt");
  else if constexpr (POL == 3) PD_V7_MFMA_DMA(" sc1");
  else PD_V7_MFMA_DMA("");
}
template <int IMM, int POL = 0>
__device__ __forceinline__ void dma_only(unsigned wb, unsigned voff, const i32x4& srd) {
  if constexpr (POL == 1) PD_V7_DMA_ONLY(" sc0 sc1");
  else if constexpr (POL == 2) PD_V7_DMA_ONLY(" nt");
  else if constexpr (POL == 3) PD_V7_DMA_ONLY(" sc1");
  else PD_V7_DMA_ONLY("");
}
#undef PD_V7_MFMA_DMA
#undef PD_V7_DMA_ONLY

// LDS byte offset (from the wave's piece base) of piece j of operand B? in stage ST
template <bool ISB, int ST, int J>
constexpr int piece_dst() {
  return ST * TILE_BYTES + (8 * (J & 3) + 4 * (J >> 2)) * 1024 + (ISB ? B_OFF : 0);
}

// bf16 epilogue of an interior tile with 16-B stores (SCHED bit 8).  A lane holds 4 consecutive columns of one row
// per 16x16 accumulator (transposed MFMA tile: row = lane & 15, columns 4 (lane >> 4) ..); packing two row blocks
// (2q, 2q + 1) and swapping lanes 16-31 / 48-63 of the first with lanes 0-15 / 32-47 of the second
// (v_permlane16_swap) gives every lane 8 consecutive columns of one row: lanes 0-15 block 2q columns 0-7, 16-31
// block 2q+1 columns 0-7, 32-47 block 2q columns 8-15, 48-63 block 2q+1 columns 8-15 — one dwordx4 store per pair
// of row blocks and column tile instead of two dwordx2 (cdna_hip_programming.md T21, with the 16-lane swap that
// matches the 16x16 layout).  Bias is added before the packing.
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void st16(void* ptr, unsigned a, unsigned b, unsigned c, unsigned d) {
  const u32x4v v = {a, b, c, d};
  if constexpr (NT) __builtin_nontemporal_store(v, (u32x4v*)ptr);
  else *(u32x4v*)ptr = v;
}
template <bool NT = false>
__device__ __forceinline__ void epilogue_v7_x4(const Params& p, f32x4v (&acc)[8][4], int tm, int tn, int arow,
                                               int bcolw, int lane) {
  unsigned short* C = (unsigned short*)p.C;
  const int sub = (lane >> 4) & 1;                // which block of the pair this lane stores
  const int r = lane & 15;
  const int ch = 8 * (lane >> 5);                 // column half of the 16-column tile
  const long row_base = (long)tm * BM + arow + r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c0 = tn * BN + bcolw + 16 * j;      // first column of tile j
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
      const int cb = c0 + 4 * (lane >> 4);        // this lane's 4 columns before the swap
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = bf2f(p.bias[cb + e]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4v& a = acc[2 * q][j];
      const f32x4v& b = acc[2 * q + 1][j];
      unsigned x0 = pack_bf2(a[0] + bv[0], a[1] + bv[1]), x1 = pack_bf2(a[2] + bv[2], a[3] + bv[3]);
      unsigned y0 = pack_bf2(b[0] + bv[0], b[1] + bv[1]), y1 = pack_bf2(b[2] + bv[2], b[3] + bv[3]);
      auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      const long row = row_base + 16 * (2 * q + sub);
      st16<NT>(C + row * p.ldc + c0 + ch, s0[0], s1[0], s0[1], s1[1]);
    }
  }
}

// ---------------------------------------------------------------------------------------------------- tail split-K
// Persistent TN GEMMs (v7, fp8) run tiles_m * tiles_n tiles on G workgroups; the last partial wave of R = tiles % G
// tiles keeps R CUs busy for one whole tile time while the rest idle (M = 4096, N = 5120: 320 tiles, 64 in the
// tail).  The split: the whole-tile launch skips the last tail_cap = R tiles, a second launch runs each of them
// as ksplit K-slices (one per workgroup, fp32 partials into slabs of the workspace p.part), and tail_reduce_kernel
// sums the slabs into C.  The slice count: ks = min(G / R, 8) lowered until the K-tile count nt splits into even
// slices of >= 8 K-tiles; 0 = no split (R > G / 2, too short a K, or the slabs do not fit the workspace).
inline int tail_plan(int nwg, int G, int nt, long ws_bytes) {
  const int R = nwg % G;
  // >= 8 waves: the tail is <= 1/16 of the run and the second launch's seam costs about what the split saves
  // (Llama M = 32768 shapes measured 0-1.5 % slower with it, profiles/r4_gemm_tail_splitk.md)
  if (R == 0 || ws_bytes <= 0 || nwg >= 8 * G) return 0;
  int ks = std::min(G / R, 8);
  while (ks > 1 && (nt % (2 * ks) || nt / ks < 8)) --ks;
  return ks >= 2 && (long)R * ks * BM * BN * 4 <= ws_bytes ? ks : 0;
}

// The fp32 partial of one K-slice of a tail tile, plain row-major [BM][BN] in its slab (tile-relative rows /
// columns of epilogue_t's lane mapping)
__device__ __forceinline__ void store_partial(float* slab, const f32x4v (&acc)[8][4], int arow, int bcolw, int lane) {
  const int cq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(float4*)(slab + (arow + 16 * i + (lane & 15)) * BN + bcolw + 16 * j + cq) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
}

// Fix-up: tail tile r's C = the sum of its ksplit fp32 slabs (r * ksplit ..): bf16 (+ bias) or fp32 (+ beta * C).
// grid (BM * BN / 1024, tail_cap), 256 threads x 4 consecutive columns.
template <int EPI>
__global__ __launch_bounds__(256) void tail_reduce_kernel(Params p, int whole) {
  const int r = blockIdx.y;
  int tm, tn;
  tile_of(p, whole + r, tm, tn);
  const int e0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int row = e0 / BN, col = e0 - row * BN;
  const long gr = (long)tm * BM + row;
  const int gc = tn * BN + col;
  if (gr >= p.M || gc >= p.N) return;
  const float* sp = p.part + (long)r * p.ksplit * (BM * BN) + e0;
  float4 v = *(const float4*)sp;
  for (int k = 1; k < p.ksplit; ++k) {
    const float4 o = *(const float4*)(sp + (long)k * (BM * BN));
    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
  }
  float a[4] = {v.x, v.y, v.z, v.w};
  const bool vec = gc + 3 < p.N;
  if constexpr (EPI == kEpiF32) {
    float* cp = (float*)p.C + gr * p.ldc + gc;
    for (int e = 0; e < 4; ++e)
      if (p.beta != 0.f && gc + e < p.N) a[e] += p.beta * cp[e];
    if (vec) {
      *(float4*)cp = make_float4(a[0], a[1], a[2], a[3]);
    } else {
      for (int e = 0; e < 4; ++e)
        if (gc + e < p.N) cp[e] = a[e];
    }
  } else {
    unsigned short o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(a[e] + (p.bias && gc + e < p.N ? bf2f(p.bias[gc + e]) : 0.f));
    unsigned short* cp = (unsigned short*)p.C + gr * p.ldc + gc;
    if (vec) {
      *(uint2*)cp = make_uint2(o[0] | (unsigned)o[1] << 16, o[2] | (unsigned)o[3] << 16);
    } else {
      for (int e = 0; e < 4; ++e)
        if (gc + e < p.N) cp[e] = o[e];
    }
  }
}

}  // namespace gm
}  // namespace pd
