// v7: the TN MFMA GEMM — both operands K-major.  dgrad dx = dy . W^T reads W as [N, K] rows in place; the
// forward y = x . W runs on W^T (one HBM-speed transpose of the weight per forward, ops/gemm.py), so every
// fragment read is a conflict-free ds_read_b128 and no transposed LDS read is needed.
//
// Reference parity: paddle/phi/kernels/impl/matmul_kernel_impl.h:108 (matmul / matmul_grad) and
// paddle/phi/kernels/funcs/fused_gemm_epilogue.h:397 (bias epilogue); the SwiGLU epilogue fuses the
// reference's separate swiglu op (paddle/phi/kernels/fusion/gpu/swiglu_kernel.cu) into the gate|up GEMM.
//
// Tile, LDS images and ring are v4's (gemm.hip): 256x256x64 tile, 4 waves x 128x128 wave tiles with the
// accumulators pinned in AGPRs, a 2-stage LDS-DMA ring (tile t+2 streamed into the stage of tile t once every
// wave holds its fragments), persistent static schedule as v6 (grid = min(tiles, CUs), XCD-chunked tile slots).
// What v7 changes is the instruction schedule of a K-tile (128 MFMAs per wave):
//  * the next K-tile's buffer descriptors are a handful of SALU ops placed between MFMAs (records = end - base
//    in 32 bits: operand extents are < 2 GiB, host-checked) instead of a serial 64-bit clamp block in front of
//    the K-tile's first MFMA;
//  * each LDS-DMA piece is one asm statement `s_add m0 / v_mfma / buffer_load ... lds`: the MFMA covers the
//    M0 -> LDS-DMA hazard, where the compiler's form puts an s_nop in front of every piece;
//  * fragment reads go one per two MFMAs (v4 issued them one per MFMA in 16-read bursts), and the MFMA order is
//    A-fragment-major so a K-tile can start after 9 of its 16 step-0 reads;
//  * SCHED bit 0: per-operand barriers (4 per K-tile: B's stage is released after B's step-1 reads and A's after
//    A's; tile t+1's B is waited for before its A) instead of 2;  bit 1: s_setprio 1 around the MFMA stream.
//  * SCHED bits 15 / 16 (spread schedule only): A / B MN-major — v4's MN-major LDS images and transposed fragment
//    reads on this persistent kernel: the weight gradient on X and dY as stored (both bits, fp32 main grad stored
//    from the AGPRs) and the forward on W as stored (bit 16), so no W^T pass (profiles/r6_gemm_mn_major.md).
#include "gemm_tn.h"

namespace pd {
namespace gm {

// SwiGLU epilogue of an interior tile with 16-B stores (SCHED bit 8): the same row-block pairing + v_permlane16_swap
// as epilogue_v7_x4, applied to the gate, up and silu(gate) * up values (gate / up = column tiles j and j + 2 of
// the wave's 64-column half: bcol<kEpiSwiGLU>).  Rounding as epilogue_t: the activation uses the bf16-rounded gate
// and up, exactly what the backward reads back from gu.
template <bool NT = false>
__device__ __forceinline__ void epilogue_v7_swi_x4(const Params& p, f32x4v (&acc)[8][4], int tm, int tn, int arow,
                                                   int bcolw, int lane) {
  const int wsub = bcolw >> 6;                    // 64-column half of the tile: 32 gate + 32 up columns
  const int sub = (lane >> 4) & 1;
  const int r = lane & 15;
  const int ch = 8 * (lane >> 5);
  const long row_base = (long)tm * BM + arow + r;
  unsigned short* out = (unsigned short*)p.C;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int gc0 = tn * 128 + wsub * 32 + 16 * j;   // first gate (== output) column of this 16-column tile
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned g2[2][2], u2[2][2], o2[2][2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const f32x4v& ga = acc[2 * q + b][j];
        const f32x4v& ua = acc[2 * q + b][2 + j];
        float gv[4], uv[4], ov[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gv[e] = bf2f(f2bf(ga[e]));
          uv[e] = bf2f(f2bf(ua[e]));
          ov[e] = silu(gv[e]) * uv[e];
        }
        g2[b][0] = pack_bf2(gv[0], gv[1]);
        g2[b][1] = pack_bf2(gv[2], gv[3]);
        u2[b][0] = pack_bf2(uv[0], uv[1]);
        u2[b][1] = pack_bf2(uv[2], uv[3]);
        o2[b][0] = pack_bf2(ov[0], ov[1]);
        o2[b][1] = pack_bf2(ov[2], ov[3]);
      }
      auto g0 = __builtin_amdgcn_permlane16_swap(g2[0][0], g2[1][0], false, false);
      auto g1 = __builtin_amdgcn_permlane16_swap(g2[0][1], g2[1][1], false, false);
      auto u0 = __builtin_amdgcn_permlane16_swap(u2[0][0], u2[1][0], false, false);
      auto u1 = __builtin_amdgcn_permlane16_swap(u2[0][1], u2[1][1], false, false);
      auto o0 = __builtin_amdgcn_permlane16_swap(o2[0][0], o2[1][0], false, false);
      auto o1 = __builtin_amdgcn_permlane16_swap(o2[0][1], o2[1][1], false, false);
      const long row = row_base + 16 * (2 * q + sub);
      const int c = gc0 + ch;
      st16<NT>(p.C2 + row * p.ldc2 + c, g0[0], g1[0], g0[1], g1[1]);
      st16<NT>(p.C2 + row * p.ldc2 + p.H + c, u0[0], u1[0], u0[1], u1[1]);
      st16<NT>(out + row * p.ldc + c, o0[0], o1[0], o0[1], o1[1]);
    }
  }
}

// RoPE epilogue (kEpiRope, whole 256 x 256 tiles): the wave's 128 columns are one head when they lie below
// rope_cols, and its two 64-column halves h = 0 / 1 hold head dims d and d + 64 at the same lane position, so every
// rotate-half pair is in one lane: out_0 = x_0 cos - x_1 sin, out_1 = x_1 cos + x_0 sin on the fp32 accumulators
// (cos / sin[d + 64] = [d] for rotate-half tables), fused into the 16-B-store epilogue.  Each half's pass reads
// its partner half's accumulators in place — the pass structure of the plain epilogue; rotating the accumulator
// set first (or both halves per group) kept hundreds of extra values alive next to the next tile's prefetched
// fragments and spilled 468-780 B/lane to scratch, this form leaves ~100 B/lane outside the MFMA loop.
template <bool NT>
__device__ __forceinline__ void epilogue_v7_rope_x4(const Params& p, f32x4v (&acc)[2][8][4], int tm, int tn,
                                                    int arow, int bcolw, int lane) {
  unsigned short* C = (unsigned short*)p.C;
  const int sub = (lane >> 4) & 1;
  const int r = lane & 15;
  const int ch = 8 * (lane >> 5);
  const long row_base = (long)tm * BM + arow + r;
  const float sgn_lo = tn * BN + bcolw < p.rope_cols ? 1.f : 0.f;   // 0: v heads, stored unrotated
  // token position of row block i: one 32-bit remainder, then p0 + 16 i with one conditional wrap (the host
  // requires rope_seq >= 128 > 16 * 7)
  const unsigned seq = (unsigned)p.rope_seq;
  const unsigned p0 = (unsigned)row_base % seq;
  auto pos = [&](int i) -> long {
    const unsigned t = p0 + 16u * i;
    return (long)(t >= seq ? t - seq : t);
  };
  // the same pass structure as the plain 16-B epilogue (half h outer): out_h = x_h cos + (h ? x_0 : -x_1) sin,
  // reading the partner half's accumulators in place; tables are L1 hits on the second half's pass
  sfor<2>([&](auto H) {
    constexpr int h = decltype(H)::value;
    sfor<4>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int d = 16 * j + 4 * (lane >> 4);
      sfor<4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const f32x4v& a = acc[h][2 * q][j];
        const f32x4v& b = acc[h][2 * q + 1][j];
        const f32x4v& pa = acc[1 - h][2 * q][j];
        const f32x4v& pb = acc[1 - h][2 * q + 1][j];
        const float4 ca = *(const float4*)(p.rope_cos + pos(2 * q) * 128 + d);
        const float4 sa = *(const float4*)(p.rope_sin + pos(2 * q) * 128 + d);
        const float4 cb = *(const float4*)(p.rope_cos + pos(2 * q + 1) * 128 + d);
        const float4 sb = *(const float4*)(p.rope_sin + pos(2 * q + 1) * 128 + d);
        const float sg = (h ? 1.f : -1.f) * sgn_lo;
        // rotated (or, for v heads, cos = 1 / sin = 0 equivalent) values of this half
        const float c0 = sgn_lo ? ca.x : 1.f, c1 = sgn_lo ? ca.y : 1.f, c2 = sgn_lo ? ca.z : 1.f,
                    c3 = sgn_lo ? ca.w : 1.f;
        const float d0 = sgn_lo ? cb.x : 1.f, d1 = sgn_lo ? cb.y : 1.f, d2 = sgn_lo ? cb.z : 1.f,
                    d3 = sgn_lo ? cb.w : 1.f;
        const float x0 = a[0] * c0 + sg * pa[0] * sa.x, x1 = a[1] * c1 + sg * pa[1] * sa.y;
        const float x2 = a[2] * c2 + sg * pa[2] * sa.z, x3 = a[3] * c3 + sg * pa[3] * sa.w;
        const float y0 = b[0] * d0 + sg * pb[0] * sb.x, y1 = b[1] * d1 + sg * pb[1] * sb.y;
        const float y2 = b[2] * d2 + sg * pb[2] * sb.z, y3 = b[3] * d3 + sg * pb[3] * sb.w;
        unsigned u0 = pack_bf2(x0, x1), u1 = pack_bf2(x2, x3);
        unsigned w0 = pack_bf2(y0, y1), w1 = pack_bf2(y2, y3);
        auto s0 = __builtin_amdgcn_permlane16_swap(u0, w0, false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(u1, w1, false, false);
        const long row = row_base + 16 * (2 * q + sub);
        st16<NT>(C + row * p.ldc + tn * BN + bcolw + 64 * h + 16 * j + ch, s0[0], s1[0], s0[1], s1[1]);
      });
    });
  });
}

// SCHED bits 15 / 16: operand A / B MN-major — the weight gradient dW = X^T . dY on X [tokens, K] and dY [tokens, N] as
// stored (both; tokens = the reduction), the forward y = x . W on W [K, N] as stored (B).  Per MN-major operand, the
// LDS image is v4's (gemm_core.h lane_setup / rd4_setup): piece
// (h, i) of a wave fills k rows 16 i + 2 (wave + 4 h) + (lane >> 5) of the [64 k][256] image, 16-B column chunk
// (lane & 31) ^ (hsw(k) << 1); fragments are two ds_read_b64_tr_b16 each.  Columns past M / N inside a row are read
// (unused accumulator columns, never stored); the descriptor extent still bounds the operand's last row.
__device__ __forceinline__ void mn_offsets(unsigned (&v)[8], long ld, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int h = j >> 2, i = j & 3;
    const int kk = 2 * (wave + 4 * h) + (lane >> 5);
    const int lc = (lane & 31) ^ (hsw(kk) << 1);
    v[j] = (unsigned)((((long)kk + 16 * i) * ld + lc * 8) * 2);
  }
}

// fp32 main-grad epilogue of the MN-major weight gradient: C = acc (beta 0, the step's first write of the gradient)
// or C += acc (beta 1, accumulation) with each accumulator taken straight from its AGPRs (gfx950 memory ops take AGPR
// data), so no accumulator is copied into the VGPRs that hold the next tile's prefetched fragments — the generic form
// (epilogue_t) spilled 112-153 VGPRs.  beta 1 adds by no-return fp32 atomics: one add per element, so the result is
// exactly round(C + acc), the read-modify-write's value.  Rows past M are skipped per lane; N % 8 == 0 (host-checked)
// keeps every 4-column group whole.  Other beta values are declined by the host (v4's spread kernel runs them).
__device__ __forceinline__ void st_f4_agpr(float* ptr, const f32x4v& a) {
  asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(ptr), "a"(a) : "memory");
}
__device__ __forceinline__ void add_f4_agpr(float* ptr, const f32x4v& a) {
  asm volatile("global_atomic_add_f32 %0, %1, off\n\t"
               "global_atomic_add_f32 %0, %2, off offset:4\n\t"
               "global_atomic_add_f32 %0, %3, off offset:8\n\t"
               "global_atomic_add_f32 %0, %4, off offset:12"
               ::"v"(ptr), "a"(a[0]), "a"(a[1]), "a"(a[2]), "a"(a[3]) : "memory");
}
__device__ __forceinline__ void epilogue_v7_f32(const Params& p, f32x4v (&acc)[8][4], int tm, int tn, int arow, int bcolw,
                                                int lane) {
  float* C = (float*)p.C;
  const int row0 = tm * BM + arow + (lane & 15);
  const int c0 = tn * BN + bcolw + 4 * (lane >> 4);
  float* base = C + (long)row0 * p.ldc + c0;
  const bool add = p.beta != 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c0 + 16 * j >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (row0 + 16 * i >= p.M) continue;
      float* cp = base + (long)(16 * i) * p.ldc + 16 * j;
      if (add) add_f4_agpr(cp, acc[i][j]);
      else st_f4_agpr(cp, acc[i][j]);
    }
  }
}

// fragment U of k32 step S from stage ST: K-major one ds_read_b128, MN-major two transposed reads (ds_read_b64_tr_b16)
// off one of 8 per-lane bases with the pair swizzle folded in — step / stage / half as immediates, no VALU per read
// (a per-read recomputed swizzle, 2 bases instead of 8, ran the Llama weight gradients 10-14 % slower)
template <bool MN, int U, int S, int ST>
__device__ __forceinline__ bf16x8 fragx(const Rd4<!MN>& r) {
  return frag4<!MN, U, S, ST>(r);
}
template <bool MN>
using RdX = Rd4<!MN>;
template <bool MN>
__device__ __forceinline__ RdX<MN> rdx_setup(unsigned img, int first, int lane) {
  return rd4_setup<!MN>(img, first, lane);
}

template <int EPI, int SCHED>
__global__ __launch_bounds__(NTHR4, 1) void gemm_v7_kernel(Params p) {
  constexpr bool BAR4 = SCHED & 1, PRIO = (SCHED & 2) != 0;
  constexpr int PA = (SCHED >> 2) & 3, PB = (SCHED >> 4) & 3;  // LDS-DMA cache policy of A / B (see mfma_dma)
  constexpr int PLVL = (SCHED & 64) ? 3 : 1;                    // s_setprio level around the MFMA stream
  constexpr bool VS = (SCHED & 128) != 0;                        // the three-barrier spread schedule (ktile_v)
  constexpr bool X4 = (SCHED & 256) != 0;                        // 16-B epilogue stores on interior tiles
  constexpr bool ROT = (SCHED & 512) != 0;                       // odd slots start their K loop half way
  constexpr bool NTS = (SCHED & 1024) != 0;                      // non-temporal epilogue stores (X4 path)
  constexpr bool CONV = (SCHED & 2048) != 0;                     // implicit-GEMM convolution (row-shifted A taps)
  // tail split-K (a launch of its own after the whole tiles' launch, which skips the last tail_cap tiles): the last
  // partial wave's tail_cap tiles run as ksplit K-slices, one per workgroup (slot = tail tile * ksplit + slice),
  // into fp32 slabs that v7_tail_reduce_kernel sums (an in-loop tail unit spilled 700 B/lane to scratch)
  constexpr bool TSK = (SCHED & 4096) != 0;
  // experiment bits (variant 64 + SCHED, bf16 epilogue only): 8192 = epilogue stores ablated (accumulators kept
  // live, the tile's output never written) — the cost of the store burst; 16384 = XCD-phase stagger: the
  // workgroups of XCD x sleep x * p.kchunk * ~8k cycles before their first tile, so the XCDs' tile boundaries (and
  // their epilogue store bursts) fall at different times
  constexpr bool NOST = (SCHED & 8192) != 0;
  constexpr bool XDLY = (SCHED & 16384) != 0;
  constexpr bool SWI = EPI == kEpiSwiGLU;
  // bits 15 / 16: A / B MN-major (the weight gradient: both; the forward on W as stored: B)
  constexpr bool MNA = (SCHED & 32768) != 0, MNB = (SCHED & 65536) != 0, MN = MNA || MNB;
  static_assert(!MN || (VS && !CONV && !ROT && !SWI && EPI != kEpiRope), "MN-major: the spread schedule, plain epilogues");
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  const unsigned sbase = (unsigned)(size_t)(lds_char*)smem_raw;

  const int nwg = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  // tail_cap > 0: the whole-tile launch leaves the last tail_cap tiles to the TSK launch (one slice per workgroup)
  const int whole = nwg - p.tail_cap, nwhole = 0;
  const int ntile = TSK ? (slot < p.tail_cap * p.ksplit ? 1 : 0) : (slot < whole ? (whole - slot + G - 1) / G : 0);
  if (ntile == 0) return;

  if constexpr (XDLY) {
    const int xs = (blockIdx.x & 7) * p.kchunk;
    for (int i = 0; i < xs; ++i) __builtin_amdgcn_s_sleep(127);
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = p.K / BK;  // even, K % 128 == 0 (host-checked)
  const int ntc = TSK ? nt / p.ksplit : nt;   // K-tiles of a tail slice (even, host-checked)
  int ntu = TSK && nwhole == 0 ? ntc : nt;    // K-tiles of the current unit

  f32x4v acc[2][8][4];
  // zero the accumulators of a tile; the zeros are pinned (asm operands) in front of an s_nop so the VALU writes
  // keep their wait states before the first MFMA reads them as src C (the compiler would otherwise re-place the
  // zeroing at the tile-loop head, right in front of the asm MFMAs whose operands it cannot see)
  auto zero_acc = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[h][i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
          asm volatile("" : "+a"(acc[h][i][j]));
        }
    asm volatile("s_nop 4" ::: "memory");
  };

  unsigned va[8], vb[8];
  if constexpr (MNA) mn_offsets(va, p.lda, wave, lane);
  else kk_offsets<false>(va, p.lda, 0, wave, lane);
  if constexpr (MNB) mn_offsets(vb, p.ldb, wave, lane);
  else kk_offsets<SWI>(vb, p.ldb, p.H, wave, lane);
  const int arow = wm * 128, bcolw = wn * 128;
  const RdX<MNA> ra = rdx_setup<MNA>(sbase, arow, lane);
  const RdX<MNB> rb = rdx_setup<MNB>(sbase + B_OFF, bcolw, lane);
  // bytes per K-tile along each operand: 64 k-columns (K-major) or 64 k-rows (MN-major)
  const unsigned kst_a = MNA ? (unsigned)(p.lda * (BK * 2)) : 128u, kst_b = MNB ? (unsigned)(p.ldb * (BK * 2)) : 128u;
  const unsigned wdst = __builtin_amdgcn_readfirstlane(sbase + wave * 1024);

  // stream state: bases of the current tile (c*) and of this workgroup's next tile (n*, live if nlive)
  const unsigned a_end = (unsigned)(size_t)p.a_end, b_end = (unsigned)(size_t)p.b_end;
  auto a_base = [&](int tm) { return (u64)(size_t)(p.A + (MNA ? (long)tm * BM : (long)tm * BM * p.lda)); };
  auto b_base = [&](int tn) {
    return (u64)(size_t)(p.B + (MNB ? (long)tn * BN : (long)tn * (SWI ? 128 : BN) * p.ldb));
  };
  // unit u of this workgroup: tile slot + u * G, or (TSK, u == nwhole) its tail slice, whose bases start at the
  // slice's first K-tile
  auto unit_tile = [&](int u, int& tm, int& tn) {
    if (TSK && u == nwhole) tile_of(p, whole + slot / p.ksplit, tm, tn);
    else tile_of(p, slot + u * G, tm, tn);
  };
  auto unit_koff = [&](int u, unsigned kst) -> u64 {
    return (TSK && u == nwhole) ? (u64)(unsigned)((slot % p.ksplit) * ntc) * kst : 0;
  };
  int ctm, ctn;
  unit_tile(0, ctm, ctn);
  u64 ca = a_base(ctm) + unit_koff(0, kst_a), cb = b_base(ctn) + unit_koff(0, kst_b), na = ca, nb = cb;
  bool nlive = false;
  auto set_next = [&](int u) {
    nlive = u + 1 < ntile;
    if (nlive) {
      int tm, tn;
      unit_tile(u + 1, tm, tn);
      na = a_base(tm) + unit_koff(u + 1, kst_a);
      nb = b_base(tn) + unit_koff(u + 1, kst_b);
    }
  };
  set_next(0);
  // descriptors of stream K-tile kk (0 <= kk < nt + 2; kk >= nt: the next tile's K-tile kk - nt)
  // (bases are < 2^48: the descriptor's high word is the address's high 16 bits, stride 0)
  // SCHED bit 9: every workgroup of an odd slot runs its K-tiles rotated by nt / 2 (same products, another
  // summation order), so the persistent grid's tiles end — and their epilogue stores burst — in two interleaved
  // phases instead of all 256 CUs at once
  const int rot = (ROT && (slot & 1)) ? nt / 2 : 0;
  auto desc = [&](int kk, u64 cur, u64 nxt, unsigned end, unsigned kst) {
    const int ntx = TSK ? ntu : nt;
    const bool nx = kk >= ntx;
    int kt = nx ? kk - ntx : kk;
    if constexpr (ROT) kt = kt + rot >= nt ? kt + rot - nt : kt + rot;
    const unsigned off = MN ? (unsigned)kt * kst : (unsigned)kt << 7;  // K-major: * BK * 2 bytes (kst = 128)
    const u64 b = (nx ? nxt : cur) + off;
    const bool live = !nx || nlive;
    return i32x4{(int)(unsigned)b, (int)(unsigned)(b >> 32), live ? (int)(end - (unsigned)b) : 0, 0x00020000};
  };
  // SCHED bit 11, implicit-GEMM convolution over a zero-bordered NHWC input (ops/conv_gemm.py): K = taps x C, and
  // K-tile kt of tap t = kt >> cv_kpb_log2 reads the A rows shifted by the tap's host-computed byte offset
  // cv_off[t] — only the descriptor base moves, per lane nothing changes (taps past cv_taps read the centre rows
  // and meet zero weight columns).  The offset is picked by a select chain over the kernarg table: scalar ops only
  // (an indexed kernarg array would be copied to scratch; an in-kernel tap / kw division put VALU + a branch into
  // the descriptor code, and that build lost K-tile 1's contribution on gfx950)
  auto desc_a = [&](int kk) {
    if constexpr (!CONV) {
      return desc(kk, ca, na, a_end, kst_a);
    } else {
      const bool nx = kk >= nt;
      const int kt = nx ? kk - nt : kk;
      const int tap = kt >> p.cv_kpb_log2;
      const unsigned coff = (unsigned)(kt & ((1 << p.cv_kpb_log2) - 1)) << 7;
      long roff = 0;
#pragma unroll
      for (int t = 0; t < 16; ++t) roff = tap == t ? p.cv_off[t] : roff;
      const u64 b = (nx ? na : ca) + (u64)roff + (u64)coff;
      const bool live = !nx || nlive;
      return i32x4{(int)(unsigned)b, (int)(unsigned)(b >> 32), live ? (int)(a_end - (unsigned)b) : 0, 0x00020000};
    }
  };
  auto descs = [&](int kk, i32x4& sa, i32x4& sb) {
    sa = desc_a(kk);
    sb = desc(kk, cb, nb, b_end, kst_b);
  };

  bf16x8 xa[8], xb[8], ya[8], yb[8];  // k32 step 0 / step 1 fragments of the current K-tile

  // prologue: K-tiles 0 and 1 of the first tile in flight, wait for K-tile 0 (everyone's), read its step 0
  {
    i32x4 sa, sb;
    descs(0, sa, sb);
    sfor<8>([&](auto J) {
      constexpr int j = decltype(J)::value;
      dma_only<piece_dst<true, 0, j>(), PB>(wdst, vb[j], sb);
    });
    sfor<8>([&](auto J) {
      constexpr int j = decltype(J)::value;
      dma_only<piece_dst<false, 0, j>(), PA>(wdst, va[j], sa);
    });
    descs(1, sa, sb);
    sfor<8>([&](auto J) {
      constexpr int j = decltype(J)::value;
      dma_only<piece_dst<true, 1, j>(), PB>(wdst, vb[j], sb);
    });
    sfor<8>([&](auto J) {
      constexpr int j = decltype(J)::value;
      dma_only<piece_dst<false, 1, j>(), PA>(wdst, va[j], sa);
    });
  }
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  sfor<8>([&](auto U) { xb[decltype(U)::value] = fragx<MNB, decltype(U)::value, 0, 0>(rb); });
  sfor<8>([&](auto U) { xa[decltype(U)::value] = fragx<MNA, decltype(U)::value, 0, 0>(ra); });
  if constexpr (VS) {
    wait_lgkm<0>();
    __builtin_amdgcn_sched_barrier(0);
  }

  // slot positions (MFMA index q of the K-tile, 0..127)
  constexpr int REL_B = BAR4 ? 16 : 32, REL_A = 32;        // stage release barriers (before MFMA q)
  constexpr int DMA_B = REL_B + 1, DMA_A = BAR4 ? 33 : 49;  // first piece slots (then every 2 MFMAs)
  constexpr int LND_B = BAR4 ? 80 : 96, LND_A = 96;        // tile t+1 landed barriers
  constexpr int XRD_B = LND_B, XRD_A = BAR4 ? 96 : 112;    // first x-read slots (then every 2 MFMAs)

  auto ktile = [&](auto ST, int k) {
    constexpr int st = decltype(ST)::value;
    i32x4 sa, sb;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
    sfor<128>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      constexpr int qq = q & 63, i = qq >> 3, j = qq & 7;
      // ---- waits / barriers in front of MFMA q
      if constexpr (q < 64 && q % 8 == 0 && q != REL_B && q != REL_A) {
        // step-0 read order [b0..b7, a0..a7]: MFMAs 8i.. need b0..b7 and a_i; y reads issued so far: ceil(q/2)
        constexpr int ny = q / 2 < 16 ? q / 2 : 16;
        constexpr int n = 7 - i + ny;
        wait_lgkm<(n > 15 ? 15 : n)>();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q == REL_B || q == REL_A) {
        // every wave holds its step-1 fragments of this stage (B at REL_B, A at REL_A): release it
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        wait_lgkm<0>();
        __builtin_amdgcn_s_barrier();
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q == LND_B || q == LND_A) {
        // K-tile t+1 landed: B alone (its A + t+2's 16 pieces may stay in flight) or everything of t+1
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (q == LND_B && BAR4) wait_vm<24>();
        else wait_vm<16>();
        __builtin_amdgcn_s_barrier();
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- MFMA q (A-fragment-major; B fragment as src0: the transposed tile, 4 columns per lane)
      const bf16x8(&fa)[8] = q < 64 ? xa : ya;
      const bf16x8(&fb)[8] = q < 64 ? xb : yb;
      f32x4v& c = acc[j >> 2][i][j & 3];
      constexpr bool pb_ = q >= DMA_B && q < DMA_B + 16 && (q - DMA_B) % 2 == 0;
      constexpr bool pa_ = q >= DMA_A && q < DMA_A + 16 && (q - DMA_A) % 2 == 0;
      if constexpr (pb_) {
        constexpr int pj = (q - DMA_B) / 2;
        mfma_dma<piece_dst<true, st, pj>(), PB>(c, fb[j], fa[i], wdst, vb[pj], sb);
      } else if constexpr (pa_) {
        constexpr int pj = (q - DMA_A) / 2;
        mfma_dma<piece_dst<false, st, pj>(), PA>(c, fb[j], fa[i], wdst, va[pj], sa);
      } else {
        mfma_agpr(c, fb[j], fa[i]);
      }
      // ---- work behind MFMA q
      if constexpr (q == 1 || q == 3) {
        // K-tile t+2's descriptors (B behind MFMA 1, A behind MFMA 3): SALU between MFMAs — kk made opaque
        // here so none of it is hoisted into a serial block at the loop head, and the result pinned after
        int kk = k + 2;
        asm volatile("" : "+s"(kk));
        if constexpr (q == 1) {
          sb = desc(kk, cb, nb, b_end, kst_b);
          asm volatile("" : "+s"(sb));
        } else {
          sa = desc_a(kk);
          asm volatile("" : "+s"(sa));
        }
      }
      if constexpr (q <= 30 && q % 2 == 0) {
        // step-1 fragments of this stage
        constexpr int r = q / 2;
        if constexpr (r < 8) yb[r] = frag4<true, r, 1, st>(rb);
        else ya[r - 8] = frag4<true, r - 8, 1, st>(ra);
      }
      if constexpr (q >= XRD_B && q < XRD_B + 16 && (q - XRD_B) % 2 == 0) {
        constexpr int r = (q - XRD_B) / 2;
        xb[r] = frag4<true, r, 0, st ^ 1>(rb);  // K-tile t+1's step-0 fragments
      }
      if constexpr (q >= XRD_A && q < XRD_A + 16 && (q - XRD_A) % 2 == 0) {
        constexpr int r = (q - XRD_A) / 2;
        xa[r] = frag4<true, r, 0, st ^ 1>(ra);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // SCHED bit 7: the spread schedule — per K-tile (MFMA index n = 0..127, B-fragment-major order, "before MFMA n"):
  //   step-1 A fragments at n = 1, 3, .., 15; lgkmcnt(0) + barrier at 21 (A's half of the stage released);
  //   A pieces 0-4 of tile t+2 at 23, 26, .., 35 beside the step-1 B fragments (25 .. 43); lgkmcnt(0) + barrier at
  //   51 (B released); A pieces 5-7 at 53, 56, 59, B pieces 0-4 at 62, 65, 86, 88, 90; vmcnt(13) + barrier at 92
  //   (tile t+1 landed: only this tile's 13 pieces stay in flight); tile t+1's step-0 fragments from 94 (A) and
  //   106 (B) with B pieces 5-7 at 97, 101, 125 in between; lgkmcnt(0) at 127.  Three barriers, no counted
  //   lgkmcnt waits: every fragment is read at least 8 MFMAs (~128 cycles) before its first use, and the 16
  //   LDS-DMA pieces are spread over 100 MFMAs instead of one burst.
  auto ktile_v = [&](auto ST, int k) {
    constexpr int st = decltype(ST)::value;
    i32x4 sa, sb;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
    sfor<128>([&](auto Q) {
      constexpr int n = decltype(Q)::value;
      constexpr int RA1[8] = {1, 3, 5, 7, 9, 11, 13, 15};
      constexpr int RB1[8] = {25, 28, 31, 34, 37, 39, 41, 43};
      constexpr int PA_[8] = {23, 26, 29, 32, 35, 53, 56, 59};
      constexpr int PB_[8] = {62, 65, 86, 88, 90, 97, 101, 125};
      constexpr int XA[8] = {94, 95, 96, 98, 99, 103, 104, 105};
      constexpr int XB[8] = {106, 107, 110, 113, 115, 118, 121, 124};
      auto idx = [](const int (&t)[8], int v) constexpr {
        int r = -1;
        for (int i = 0; i < 8; ++i)
          if (t[i] == v) r = i;
        return r;
      };
      constexpr int ra1 = idx(RA1, n), rb1 = idx(RB1, n), pa = idx(PA_, n), pb = idx(PB_, n), xa_ = idx(XA, n),
                    xb_ = idx(XB, n);
      // ---- in front of MFMA n
      if constexpr (n == 21 || n == 51) {
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        wait_lgkm<0>();
        __builtin_amdgcn_s_barrier();
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (n == 92) {
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        wait_vm<13>();
        __builtin_amdgcn_s_barrier();
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PLVL);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (n == 127) {
        wait_lgkm<0>();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (ra1 >= 0) ya[ra1] = fragx<MNA, (ra1 < 0 ? 0 : ra1), 1, st>(ra);
      if constexpr (rb1 >= 0) yb[rb1] = fragx<MNB, (rb1 < 0 ? 0 : rb1), 1, st>(rb);
      if constexpr (xa_ >= 0) xa[xa_] = fragx<MNA, (xa_ < 0 ? 0 : xa_), 0, st ^ 1>(ra);
      if constexpr (xb_ >= 0) xb[xb_] = fragx<MNB, (xb_ < 0 ? 0 : xb_), 0, st ^ 1>(rb);
      // ---- MFMA n (B fragment outer, A inner; B as src0: the transposed tile, 4 columns per lane)
      constexpr int nn = n & 63, j = nn >> 3, i = nn & 7;
      const bf16x8(&fa)[8] = n < 64 ? xa : ya;
      const bf16x8(&fb)[8] = n < 64 ? xb : yb;
      f32x4v& c = acc[j >> 2][i][j & 3];
      if constexpr (pa >= 0) {
        mfma_dma<piece_dst<false, st, (pa < 0 ? 0 : pa)>(), PA>(c, fb[j], fa[i], wdst, va[pa < 0 ? 0 : pa], sa);
      } else if constexpr (pb >= 0) {
        mfma_dma<piece_dst<true, st, (pb < 0 ? 0 : pb)>(), PB>(c, fb[j], fa[i], wdst, vb[pb < 0 ? 0 : pb], sb);
      } else {
        mfma_agpr(c, fb[j], fa[i]);
      }
      // ---- behind MFMA n: tile t+2's descriptors (SALU between MFMAs), A before its first piece at 23
      if constexpr (n == 2 || n == 10) {
        int kk = k + 2;
        asm volatile("" : "+s"(kk));
        if constexpr (n == 2) {
          sa = desc_a(kk);
          asm volatile("" : "+s"(sa));
        } else {
          sb = desc(kk, cb, nb, b_end, kst_b);
          asm volatile("" : "+s"(sb));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  for (int u = 0; u < ntile; ++u) {
    zero_acc();
    for (int k = 0; k < (TSK ? ntu : nt); k += 2) {
      if constexpr (VS) {
        ktile_v(std::integral_constant<int, 0>{}, k);
        ktile_v(std::integral_constant<int, 1>{}, k + 1);
      } else {
        ktile(std::integral_constant<int, 0>{}, k);
        ktile(std::integral_constant<int, 1>{}, k + 1);
      }
    }
    // tile done: accumulators out while the next tile's first K-tiles stream / sit in LDS
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
    if constexpr (EPI == kEpiRope) epilogue_v7_rope_x4<NTS>(p, acc, ctm, ctn, arow, bcolw, lane);   // whole tiles
    if constexpr (EPI == kEpiGeLU || EPI == kEpiDGeLU || EPI == kEpiDSwiGLU) {
      // compile-time halves (sfor): with a runtime h — the unroller gives up on the large GELU / dGELU bodies —
      // acc[h] was indexed dynamically and all 256 accumulators were demoted to scratch (1040 B/lane)
      sfor<2>([&](auto H) {
        constexpr int h = decltype(H)::value;
        epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
      });
    } else if constexpr (TSK) {
      // tail slice: the fp32 partial into its slab
      sfor<2>([&](auto H) {
        constexpr int h = decltype(H)::value;
        store_partial(p.part + (long)slot * (BM * BN), acc[h], arow, bcolw + 64 * h, lane);
      });
    } else if constexpr (EPI != kEpiRope) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (NOST) {
          // never true at run time (ablation): the stores are skipped, the accumulators stay live
          if (p.beta == -1234.5f) epilogue_v7_x4<NTS>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"a"(acc[h][i][j]));
        } else if constexpr (X4 && EPI == kEpiBF16) {
          // interior tile, 16-B aligned rows: the widened stores; otherwise the element-checked epilogue
          if ((ctm + 1) * BM <= p.M && (ctn + 1) * BN <= p.N && (p.ldc & 7) == 0 && ((size_t)p.C & 15) == 0)
            epilogue_v7_x4<NTS>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
          else
            epilogue_t<kEpiBF16>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        } else if constexpr (X4 && EPI == kEpiSwiGLU) {
          if ((ctm + 1) * BM <= p.M && (ctn + 1) * 128 <= p.H && (p.ldc & 7) == 0 && (p.ldc2 & 7) == 0 &&
              (p.H & 7) == 0 && ((size_t)p.C & 15) == 0 && ((size_t)p.C2 & 15) == 0)
            epilogue_v7_swi_x4<NTS>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
          else
            epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        } else if constexpr (EPI == kEpiF32) {
          epilogue_v7_f32(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        } else {
          epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        }
      }
    }
    if (u + 1 < ntile) {
      unit_tile(u + 1, ctm, ctn);
      ca = na;
      cb = nb;
      if constexpr (TSK) ntu = u + 1 == nwhole ? ntc : nt;
      set_next(u + 1);
    }
  }
  // the dead prefetches past the last tile (num_records 0) must land before the workgroup's LDS goes away
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace gm
}  // namespace pd

// Launch v7 (called by pd_gemm for variants 7..10 = SCHED 0..3).  Returns false if the problem is outside v7's
// domain (the caller then runs v6): both operands K-major, bf16 (+bias) or SwiGLU epilogue, K % 128 == 0, every
// operand extent < 2 GiB, 8-B-aligned output rows.
bool pd_gemm_v7(const pd::gm::Params& p_in, int layout, int epi, int sched, int cus, long ws_bytes, hipStream_t st) {
  using namespace pd::gm;
  Params p = p_in;
  const long a_bytes = (long)((const char*)p.a_end - (const char*)p.A);
  const long b_bytes = (long)((const char*)p.b_end - (const char*)p.B);
  if (a_bytes <= 0 || b_bytes <= 0 || a_bytes >= 0x7fffffffL || b_bytes >= 0x7fffffffL) return false;
  if (p.ldc % 4 || (size_t)p.C % 16 || (p.C2 && (p.ldc2 % 4 || (size_t)p.C2 % 16))) return false;
  const dim3 grid(std::min(p.tiles_m * p.tiles_n, cus));
  if (sched & (32768 | 65536)) {
    // MN-major operands on the persistent spread schedule (bit 15: A, bit 16: B): the weight gradient (layout 0, fp32
    // main-grad C = product + beta C with beta 0 / 1, or bf16) and the forward on W as stored (layout 1: x K-major, W
    // N-major; bf16 + bias); every 64-k-row K-tile stride in 32 bits; tail split-K as the TN forward
    const bool mna = sched & 32768, mnb = sched & 65536;
    if ((layout & 1) == mna || ((layout >> 1) & 1) == mnb || p.K % 128 || p.C2) return false;
    if (epi != kEpiF32 && epi != kEpiBF16) return false;
    if (epi == kEpiF32 && (p.bias || (p.beta != 0.f && p.beta != 1.f))) return false;
    if (mna && (p.lda % 8 || p.M % 8 || (long)p.lda * 128 * (p.K / BK) >= 0xffffffffL)) return false;
    if (mnb && (p.ldb % 8 || p.N % 8 || (long)p.ldb * 128 * (p.K / BK) >= 0xffffffffL)) return false;
    const int nwg = p.tiles_m * p.tiles_n, G = cus, R = nwg % G;
    const int ks = p.part && ws_bytes > 0 ? tail_plan(nwg, G, p.K / BK, ws_bytes) : 0;
    if (ks >= 2) {
      p.ksplit = ks;
      p.tail_cap = R;
    }
    const dim3 wgrid(ks >= 2 ? std::min(nwg - R, G) : grid.x), tgrid(R * ks);
    const bool whole = ks < 2 || nwg > R;
#define PD_V7_MN(E, S)                                                                   \
  {                                                                                      \
    if (whole) gemm_v7_kernel<E, S><<<wgrid, NTHR4, 0, st>>>(p);                         \
    if (ks >= 2) {                                                                       \
      gemm_v7_kernel<E, S | 4096><<<tgrid, NTHR4, 0, st>>>(p);                           \
      tail_reduce_kernel<E><<<dim3(BM * BN / 1024, R), 256, 0, st>>>(p, nwg - R);        \
    }                                                                                    \
  }
    if (mna && mnb) {
      if (epi == kEpiF32) PD_V7_MN(kEpiF32, 384 | 32768 | 65536)
      else PD_V7_MN(kEpiBF16, 384 | 32768 | 65536)
    } else if (mnb) {
      PD_V7_MN(kEpiBF16, 384 | 65536)
    } else {
      return false;
    }
#undef PD_V7_MN
    return true;
  }
  if (layout != 3 || epi == kEpiF32 || p.K % 128) return false;
  if (sched & 16384) {   // XCD-stagger experiment: the per-XCD delay unit from the environment
    const char* d = getenv("PD_GEMM_XCD_DELAY");
    p.kchunk = d ? atoi(d) : 1;
  }
  // SCHED 0..3 = variants 7..10; the experiment configurations (cache policy / priority level, variant 64 + cfg)
  // are instantiated for the bf16 epilogue only
#define PD_V7_CASE(E, S) \
  case S: gemm_v7_kernel<E, S><<<grid, NTHR4, 0, st>>>(p); break;
#define PD_V7(E)                                                        \
  switch (sched) {                                                      \
    PD_V7_CASE(E, 0) PD_V7_CASE(E, 1) PD_V7_CASE(E, 2) PD_V7_CASE(E, 3) \
    default: return false;                                              \
  }
  if (epi == kEpiSwiGLU && sched > 3) {   // the spread schedule with the SwiGLU epilogue
    switch (sched) {
      PD_V7_CASE(kEpiSwiGLU, 128) PD_V7_CASE(kEpiSwiGLU, 384) PD_V7_CASE(kEpiSwiGLU, 896)
      PD_V7_CASE(kEpiSwiGLU, 1408) PD_V7_CASE(kEpiSwiGLU, 1920)
      default: return false;
    }
    return true;
  }
  if (epi == kEpiRope) {   // RoPE epilogue: the spread schedule only, bias-free
    // whole tiles only (M, N multiples of 256, 16-B rows): the kernel carries just the streaming 16-B-store form
    if (sched != 384 || p.bias || !p.rope_cos || !p.rope_sin || p.rope_seq < 128 || p.rope_cols % 128 ||
        p.M % BM || p.N % BN || (p.ldc & 7) || ((size_t)p.C & 15))
      return false;
    gemm_v7_kernel<kEpiRope, 384><<<grid, NTHR4, 0, st>>>(p);
    return true;
  }
  if (epi == kEpiDSwiGLU) {   // SwiGLU backward in the down projection's dgrad: the spread schedule only
    if (sched != 384 || p.bias || !p.C2 || p.H != p.N) return false;
    gemm_v7_kernel<kEpiDSwiGLU, 384><<<grid, NTHR4, 0, st>>>(p);
    return true;
  }
  if (epi == kEpiGeLU || epi == kEpiDGeLU) {   // the GELU epilogues: the spread schedule only
    if (sched != 384) return false;
    if (epi == kEpiGeLU)
      gemm_v7_kernel<kEpiGeLU, 384><<<grid, NTHR4, 0, st>>>(p);
    else
      gemm_v7_kernel<kEpiDGeLU, 384><<<grid, NTHR4, 0, st>>>(p);
    return true;
  }
  if (epi == kEpiBF16 && sched == 384 && p.part && ws_bytes > 0) {
    // tail split-K plan: with G = cus persistent workgroups the last partial wave holds R = tiles % G tiles; when
    // R <= G / 2 they run as ks = G / R (<= 8) K-slices of >= 8 K-tiles each (one slice per workgroup) instead
    // of one whole tile on R CUs while the rest idle — e.g. M = 4096, N = 5120: 320 tiles, 64 of them in 4
    // slices, 1.25 instead of 2 tile times + a ~64 MiB fp32 fix-up read
    const int nwg = p.tiles_m * p.tiles_n, G = cus, R = nwg % G;
    const int ks = tail_plan(nwg, G, p.K / BK, ws_bytes);
    if (ks >= 2) {
      p.ksplit = ks;
      p.tail_cap = R;
      if (nwg > R) gemm_v7_kernel<kEpiBF16, 384><<<dim3(std::min(nwg - R, G)), NTHR4, 0, st>>>(p);   // whole tiles
      gemm_v7_kernel<kEpiBF16, 384 | 4096><<<dim3(R * ks), NTHR4, 0, st>>>(p);                     // tail slices
      tail_reduce_kernel<kEpiBF16><<<dim3(BM * BN / 1024, R), 256, 0, st>>>(p, nwg - R);
      return true;
    }
  }
  if (epi == kEpiBF16 && sched > 3) {
    switch (sched) {
      PD_V7_CASE(kEpiBF16, 6) PD_V7_CASE(kEpiBF16, 18) PD_V7_CASE(kEpiBF16, 22) PD_V7_CASE(kEpiBF16, 10)
      PD_V7_CASE(kEpiBF16, 42) PD_V7_CASE(kEpiBF16, 66) PD_V7_CASE(kEpiBF16, 86) PD_V7_CASE(kEpiBF16, 20)
      PD_V7_CASE(kEpiBF16, 14) PD_V7_CASE(kEpiBF16, 128) PD_V7_CASE(kEpiBF16, 130) PD_V7_CASE(kEpiBF16, 194)
      PD_V7_CASE(kEpiBF16, 384) PD_V7_CASE(kEpiBF16, 896) PD_V7_CASE(kEpiBF16, 1408) PD_V7_CASE(kEpiBF16, 1920)
      PD_V7_CASE(kEpiBF16, 384 | 8192) PD_V7_CASE(kEpiBF16, 384 | 16384)
      default: return false;
    }
    return true;
  }
  if (epi == kEpiBF16) {
    PD_V7(kEpiBF16)
  } else {
    PD_V7(kEpiSwiGLU)
  }
#undef PD_V7_CASE
#undef PD_V7
  return true;
}

// Implicit-GEMM convolution on the spread TN schedule (ops/conv_gemm.py): C[M, N] = sum over taps t of
// A[r + shift_t, :] . B[:, t*Cin : (t+1)*Cin]^T with A the zero-bordered NHWC input flattened to [pixels, lda]
// (A points at padded pixel 0; [a_lo, a_hi) is the allocation, guard rows included) and B the tap-major weight
// [N, K] (K = taps x Cin rounded up to an even number of 64-wide K-tiles, zero columns past the taps).
// Returns -1 outside the kernel's domain.
extern "C" int pd_gemm_conv(const void* A, long lda, const void* a_lo, const void* a_hi, const void* B, long ldb,
                            void* C, long ldc, int M, int N, int K, int taps, int kw, int pitch, int pad_h, int pad_w,
                            int sign, int kpb_log2, int group_m, int cus, void* stream) {
  using namespace pd::gm;
  if (M <= 0 || N <= 0 || K % 128 || lda % 8 || ldb % 8 || ldc % 4 || (size_t)C % 16) return -1;
  if ((64L << kpb_log2) != lda) return -1;   // one tap = one row of channels = 2^kpb_log2 K-tiles
  if (taps < 1 || taps > 16 || kw < 1) return -1;
  // every tap's shifted rows must stay inside [a_lo, a_hi)
  long lo_rows = 0, hi_rows = 0;
  for (int t = 0; t < taps; ++t) {
    const int kh = t / kw, kx = t - kh * kw;
    const long r = (long)sign * ((long)(kh - pad_h) * pitch + (kx - pad_w));
    lo_rows = std::min(lo_rows, r);
    hi_rows = std::max(hi_rows, r);
  }
  const char* a = (const char*)A;
  if (a + lo_rows * lda * 2 < (const char*)a_lo) return -1;
  if (a + (long)(M + hi_rows) * lda * 2 > (const char*)a_hi) return -1;
  const long a_bytes = (const char*)a_hi - a, b_bytes = ((long)(N - 1) * ldb + K) * 2;
  if (a_bytes >= 0x7fffffffL || b_bytes >= 0x7fffffffL || (const char*)a_lo < a - 0x3fffffffL) return -1;
  Params p;
  p.A = (const unsigned short*)A;
  p.B = (const unsigned short*)B;
  p.C = C;
  p.C2 = nullptr;
  p.bias = nullptr;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldc2 = 0;
  p.M = M; p.N = N; p.K = K; p.beta = 0.f; p.H = 0;
  p.zero = nullptr;
  p.goff = nullptr; p.ngroups = 0; p.gmode = 0; p.gsb = p.gsc = p.gsbias = 0;
  p.part = nullptr; p.ksplit = 1; p.kchunk = 0; p.tail_cap = 0; p.cpx = cus / 8;
  p.a_end = a_hi;
  p.b_end = (const char*)B + b_bytes;
  p.sa = p.sb = nullptr;
  p.cv_kpb_log2 = kpb_log2; p.cv_taps = taps;
  for (int t = 0; t < 16; ++t) {
    const int kh = t / kw, kx = t - kh * kw;
    p.cv_off[t] = t < taps ? (long)sign * ((long)(kh - pad_h) * pitch + (kx - pad_w)) * lda * 2 : 0;
  }
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + BN - 1) / BN;
  p.group_m = group_m > 0 ? group_m : 4;
  const dim3 grid(std::min(p.tiles_m * p.tiles_n, cus));
  gemm_v7_kernel<kEpiBF16, 384 | 2048><<<grid, NTHR4, 0, (hipStream_t)stream>>>(p);
  return (int)hipGetLastError();
}
