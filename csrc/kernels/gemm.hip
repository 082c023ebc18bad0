// Hand-written CDNA4 (gfx950) bf16 GEMM on MFMA: C[M,N] = A[M,K] . B[K,N] with fused epilogues.
//
// Reference parity: paddle/phi/kernels/impl/matmul_kernel_impl.h:108 (MatMulFunction, the cuBLAS
// call behind matmul / matmul_grad), paddle/phi/kernels/funcs/fused_gemm_epilogue.h:397 (bias / act
// epilogues) and paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu:282 (dW += x^T dy
// into an fp32 main grad).  Not a translation: one MI355X-native kernel template serves every
// operand layout, so a Linear's three GEMMs run without any transpose pass:
//   forward  y  = x . W      A K-major (x [M,K]),      B N-major (W [K,N], Paddle layout)
//   dgrad    dx = dy . W^T   A K-major (dy [M,N]),     B K-major (W read as [N,K] rows)
//   wgrad    dW = x^T . dy   A M-major (x read as [K,M] columns), B N-major (dy [M,N])
//
// Design (cdna_hip_programming.md §5, §5.5):
//  * 256x256 output tile per workgroup, BK = 64, 8 waves (2 along M x 4 along N), each wave a
//    128x64 sub-tile as 8x4 v_mfma_f32_16x16x32_bf16 accumulators (128 acc VGPRs);
//  * operands staged global -> LDS with buffer_load ... lds (LDS-DMA, 16 B per lane, no VGPR
//    round trip) into a 2-stage ring (2 x (32 + 32) KiB = 128 KiB, one __shared__ array); the
//    buffer descriptor's range check returns zeros for rows / k beyond the matrix, so any M, N, K
//    work with no edge code in the loop (16-B chunks: K % 8 for K-major operands, M/N % 8 for
//    M/N-major ones);
//  * LDS images are XOR-swizzled on the SOURCE address (LDS-DMA writes lane-linearly, rule 21):
//    K-major [256][64] tiles (128-B rows) by chunk ^ ((row>>1)&7) -> conflict-free ds_read_b128
//    fragment reads; MN-major [64][256] tiles (512-B rows) by pair ^ h(k) -> conflict-free
//    ds_read_b64_tr_b16 (T10) transposed reads, which deliver the K-packed MFMA fragment of an
//    M/N-contiguous operand with no transpose pass;
//  * 4 phases per K-tile (quadrants A0B0, A0B1, A1B1, A1B0 of the wave tile); each phase issues
//    the NEXT phase's fragment reads before its 16 MFMAs; ONE barrier per K-tile (before phase 3)
//    retires tile t+1's LDS-DMA and all reads of tile t, then tile t+2 is streamed into the freed
//    stage during phases 3-4 — every LDS-DMA has ~one K-tile of MFMA work to land under;
//  * XCD-aware bijective block remap (T1) + grouped tile order so the 32 concurrent tiles of an
//    XCD share A/B panels in its L2;
//  * epilogues: bf16 (+bias), fp32 main-grad (C = acc + beta*C), and SwiGLU for the packed
//    gate|up projection (the B tile's columns are remapped so each wave holds matching gate and
//    up columns; it writes the pre-activation gu for the backward and silu(g)*u).
#include "gemm_core.h"

namespace pd {
namespace gm {

template <bool AK, bool BKM, int EPI, int DBG = 0>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  const unsigned sbase = (unsigned)(size_t)smem;

  int bx = blockIdx.x;
  if (p.goff) group_setup<EPI>(p, bx);
  const int nwg = p.tiles_m * p.tiles_n;
  int bid, kpart = -1, slab = 0;
  if (p.ksplit > 1) {
    const int x = bx % 8, local = bx / 8;
    const XPlan xp = xcd_plan(nwg, x, p.cpx);
    if (local >= xp.full + xp.tail * p.ksplit) return;  // whole workgroup: this XCD has fewer blocks
    if (local < xp.full) {
      bid = xp.t0 + local;
    } else {
      const int r = local - xp.full;
      bid = xp.t0 + xp.full + r / p.ksplit;
      kpart = r % p.ksplit;
      slab = (x * p.tail_cap + r / p.ksplit) * p.ksplit + kpart;
    }
  } else {
    bid = xcd_remap(bx, nwg);
  }
  int tm, tn;
  tile_of(p, bid, tm, tn);
  if (p.goff && p.gmode == 0 && !group_rows<EPI>(p, tm)) return;  // whole workgroup: no tile of any group
  // a K-slice of a tail tile: rebase K so the loop below sees a problem of kchunk K-tiles
  const int kt0 = kpart >= 0 ? kpart * p.kchunk : 0;
  if (kpart >= 0) p.K = min(p.K - kt0 * BK, p.kchunk * BK);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int Ncols = (EPI == kEpiSwiGLU) ? 2 * p.H : p.N;
  // K-tiles, rounded up to an even count: the loop body is two tiles (stage 0, stage 1) of
  // straight-line MFMA chains; a padding tile past K loads zeros through the range check
  const int nt = (((p.K + BK - 1) / BK) + 1) & ~1;

  f32x4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const Ld LA = lane_setup<AK, false, EPI>(p.lda, p.M, tm, p.H, wave, lane);
  const Ld LB = lane_setup<BKM, true, EPI>(p.ldb, Ncols, tn, p.H, wave, lane);
  // tile base pointers (element units) at k0 = 0; per K-tile they advance by a_step / b_step elements
  const int tma = DBG == 6 ? 0 : tm, tnb = DBG == 6 ? 0 : tn;  // (ablation 6: every tile loads tile (0,0))
  const long a_step = AK ? BK : (long)BK * p.lda;
  const long b_step = BKM ? BK : (long)BK * p.ldb;
  const unsigned short* a_t0 = (AK ? p.A + (long)tma * BM * p.lda : p.A + (long)tma * BM) + a_step * kt0;
  const unsigned short* b_t0 =
      (BKM ? p.B + (long)tnb * BN * p.ldb : (EPI == kEpiSwiGLU ? p.B : p.B + (long)tnb * BN)) + b_step * kt0;
  const unsigned a_is = (unsigned)(AK ? 64 * p.lda * 2 : 16 * p.lda * 2);
  const unsigned b_is = (unsigned)(BKM ? 64 * p.ldb * 2 : 16 * p.ldb * 2);
  const bool a_rows_full = !AK || (tm + 1) * BM <= p.M;
  const bool b_rows_full = !BKM || (tn + 1) * BN <= Ncols;

  const int arow = wm * 128;  // wave's first row in the A tile
  const int bcolw = wn * 64;  // wave's first column in the B tile
  const RdB<AK> ra = rd_setup<AK>(sbase, arow, lane);
  const RdB<BKM> rb = rd_setup<BKM>(sbase + B_OFF, bcolw, lane);

  // stream DMA instruction I (0..3) of tile t's A / B into stage `st`
  constexpr bool GL = DBG == 7;
  auto dmaA = [&](int t, int st, auto I) {
    const auto* pa = a_t0 + a_step * t;   // range check ends at the operand's last byte (p.a_end), not 2 GiB on
    const __amdgpu_buffer_rsrc_t rs =      // (a stray read past the tensor returns 0 instead of touching memory)
        p.a_end ? make_rsrc_n(pa, (long)((const char*)p.a_end - (const char*)pa)) : make_rsrc(pa);
    const int krem = p.K - t * BK;
    dma<AK, decltype(I)::value, GL>(rs, LA, a_is, smem + st * TILE_BYTES, wave, a_rows_full && krem >= BK, krem,
                                    (const char*)(a_t0 + a_step * t), (const char*)p.zero);
  };
  auto dmaB = [&](int t, int st, auto I) {
    const auto* pb = b_t0 + b_step * t;
    const __amdgpu_buffer_rsrc_t rs =
        p.b_end ? make_rsrc_n(pb, (long)((const char*)p.b_end - (const char*)pb)) : make_rsrc(pb);
    const int krem = p.K - t * BK;
    dma<BKM, decltype(I)::value, GL>(rs, LB, b_is, smem + B_OFF + st * TILE_BYTES, wave,
                                     b_rows_full && krem >= BK, krem, (const char*)(b_t0 + b_step * t),
                                     (const char*)p.zero);
  };

  // prologue: tiles 0 and 1 in flight, wait for tile 0
  sfor<4>([&](auto I) { dmaA(0, 0, I); dmaB(0, 0, I); });
  sfor<4>([&](auto I) { dmaA(1, 1, I); dmaB(1, 1, I); });
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // Fragment sets (A half = 4 m16 tiles, B half = 2 n16 tiles).  A0/B0 of the two k32 steps have
  // their own names (x: step 0, y: step 1) so no fragment is ever copied between registers.
  bf16x8 a0x[4], b0x[2], a0y[4], b0y[2], a1[4], b1[2];

  // One sub-phase: 8 MFMAs on quadrant (MI, NI) with fragments fa/fb; after MFMA k the read/DMA
  // work item k (if any) is issued, pinned in place so the LDS traffic spreads over the MFMAs.
  auto sub = [&](auto MI, auto NI, const bf16x8 (&fa)[4], const bf16x8 (&fb)[2], auto&& work) {
    constexpr int mi = decltype(MI)::value, ni = decltype(NI)::value;
    if constexpr (DBG != 2) sync_frags();
    __builtin_amdgcn_s_setprio(1);
    sfor<8>([&](auto K) {
      constexpr int k = decltype(K)::value;
      acc[4 * mi + k / 2][2 * ni + k % 2] = mfma(fa[k / 2], fb[k % 2], acc[4 * mi + k / 2][2 * ni + k % 2]);
      work(K);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_setprio(0);
  };
  auto none = [&](auto) {};
  // read A half H (m16 tiles 4H..4H+3) at step S: 4 fragments, issued one per MFMA slot 0..3
  auto rdA = [&](bf16x8 (&dst)[4], auto ST, auto H, auto S) {
    return [&, ST, H, S](auto K) {
      constexpr int k = decltype(K)::value;
      if constexpr (k < 4 && DBG != 5)
        dst[k] = read_frag<AK, 4 * decltype(H)::value + k, decltype(S)::value, decltype(ST)::value>(ra);
    };
  };
  auto rdB = [&](bf16x8 (&dst)[2], auto ST, auto H, auto S) {
    return [&, ST, H, S](auto K) {
      constexpr int k = decltype(K)::value;
      if constexpr (k < 2 && DBG != 5)
        dst[k] = read_frag<BKM, 2 * decltype(H)::value + k, decltype(S)::value, decltype(ST)::value>(rb);
    };
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;

  {
    sfor<4>([&](auto K) { rdA(a0x, C0{}, C0{}, C0{})(K); });
    sfor<2>([&](auto K) { rdB(b0x, C0{}, C0{}, C0{})(K); });
  }

  // One K-tile out of stage ST (compile-time) with tile t+2 streamed into it after the barrier.
  auto ktile = [&](auto ST, int t) {
    constexpr int st = decltype(ST)::value;
    using SC = std::integral_constant<int, st>;
    using SN = std::integral_constant<int, st ^ 1>;
    const bool stage2 = t + 2 < nt;
    // ---- k32 step 0: sub-phases A0B0, A0B1, A1B1, A1B0; each issues the next one's reads
    sub(C0{}, C0{}, a0x, b0x, rdB(b1, SC{}, C1{}, C0{}));
    sub(C0{}, C1{}, a0x, b1, rdA(a1, SC{}, C1{}, C0{}));
    sub(C1{}, C1{}, a1, b1, rdA(a0y, SC{}, C0{}, C1{}));
    sub(C1{}, C0{}, a1, b0x, rdB(b0y, SC{}, C0{}, C1{}));
    // ---- k32 step 1
    sub(C0{}, C0{}, a0y, b0y, rdB(b1, SC{}, C1{}, C1{}));
    sub(C0{}, C1{}, a0y, b1, rdA(a1, SC{}, C1{}, C1{}));
    // barrier: tile t+1 landed (own DMA drained, then everyone's); every read of stage `st` retired
    if constexpr (DBG == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    if constexpr (DBG != 3) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // stream tile t+2 into the freed stage (one DMA per two MFMAs) and read tile t+1's A0/B0
    sub(C1{}, C1{}, a1, b1, [&](auto K) {
      constexpr int k = decltype(K)::value;
      if constexpr (k % 2 == 0) {
        if (DBG != 4 && stage2) dmaA(t + 2, st, std::integral_constant<int, k / 2>{});
      }
      rdA(a0x, SN{}, C0{}, C0{})(K);
    });
    sub(C1{}, C0{}, a1, b0y, [&](auto K) {
      constexpr int k = decltype(K)::value;
      if constexpr (k % 2 == 0) {
        if (DBG != 4 && stage2) dmaB(t + 2, st, std::integral_constant<int, k / 2>{});
      }
      rdB(b0x, SN{}, C0{}, C0{})(K);
    });
  };

  for (int t = 0; t < nt; t += 2) {
    ktile(C0{}, t);
    ktile(C1{}, t + 1);
  }

  if constexpr (EPI != kEpiSwiGLU) {
    if (kpart >= 0) {  // K-slice of a tail tile: the raw fp32 partial into its slab (tile-local, unmasked)
      float* sp = p.part + (long)slab * (BM * BN);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sp[(arow + 16 * i + 4 * (lane >> 4) + e) * BN + bcolw + 16 * j + (lane & 15)] = acc[i][j][e];
      return;
    }
  }
  epilogue<EPI>(p, acc, tm, tn, arow, bcolw, wn, lane);
}

// Sum the K-slices of every tail tile in slice order (deterministic) and apply the epilogue: fp32 main grad
// C = sum + beta*C, or bf16 C = sum (+ bias).  grid (BM*BN/1024, 8*tail_cap), 256 threads x 4 elements.
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(Params p) {
  const int x = blockIdx.y / p.tail_cap, j = blockIdx.y % p.tail_cap;
  const XPlan xp = xcd_plan(p.tiles_m * p.tiles_n, x, p.cpx);
  if (j >= xp.tail) return;
  int tm, tn;
  tile_of(p, xp.t0 + xp.full + j, tm, tn);
  const int e0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int r = tm * BM + e0 / BN, c = tn * BN + e0 % BN;
  if (r >= p.M) return;
  const float* sp = p.part + (long)(x * p.tail_cap + j) * p.ksplit * (BM * BN) + e0;
  float4 s = *(const float4*)sp;
  for (int k = 1; k < p.ksplit; ++k) {
    const float4 v = *(const float4*)(sp + (long)k * (BM * BN));
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (c + q >= p.N) break;
    if constexpr (EPI == kEpiF32) {
      float* cp = (float*)p.C + (long)r * p.ldc + c + q;
      *cp = p.beta != 0.f ? sv[q] + p.beta * *cp : sv[q];
    } else {
      const float bv = p.bias ? bf2f(p.bias[c + q]) : 0.f;
      ((unsigned short*)p.C)[(long)r * p.ldc + c + q] = f2bf(sv[q] + bv);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// v4: 4 waves (2 x 2), one wave per SIMD (512-register budget: the 8x8 accumulator grid of a 128x128
// wave tile lives in the 256 AGPRs), LDS-DMA staging, and a K-tile's COMPLETE fragment set held in
// VGPRs (2 k32 steps x (8 A + 8 B) fragments = 128 VGPRs) so a stage is released a quarter of the way
// into the tile.  Per K-tile and wave:
//   step 0 (64 MFMAs, j-major: B fragment j outer, A fragment i inner, so MFMAs 0-7 need 9 of the 16 x reads
//     and each later group of 8 one more — counted lgkmcnt waits, no drain at the tile start): the step-1
//     fragments are read behind MFMAs 0-15; after MFMA 23 lgkmcnt(0) +
//     barrier (every wave has its reads of this stage) and the 16 LDS-DMA pieces of tile t+2 are
//     streamed into the freed stage one per 5 MFMAs (MFMAs 24-99: a piece's ~60-cycle issue cost hides
//     under 80 MFMA cycles instead of stalling a dense DMA burst);
//   step 1 (64 MFMAs): after MFMA 111 vmcnt(16) (this wave's pieces of tile t+1 landed; tile t+2's 16
//     stay in flight) + barrier (everyone's), then tile t+1's step-0 fragments are read behind the
//     last 16 MFMAs.
// lanes whose 16-B chunk starts at or past K (K % 64 != 0).
// SP: the spread three-barrier K-tile schedule of v7 (gemm7.hip ktile_v) on any operand layout — fragments of an
// MN-major operand are two ds_read_b64_tr_b16 each; used for the wgrad (both operands MN-major, fp32 main grad).
template <bool AK, bool BKM, int EPI, bool FAST, bool SP = false>
__global__ __launch_bounds__(NTHR4, 1) void gemm_v4_kernel(Params p) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  const unsigned sbase = (unsigned)(size_t)smem;

  int bx = blockIdx.x;
  if (p.goff) group_setup<EPI>(p, bx);
  const int nwg = p.tiles_m * p.tiles_n;
  int bid, kpart = -1, slab = 0;
  if (p.ksplit > 1) {
    const int x = bx % 8, local = bx / 8;
    const XPlan xp = xcd_plan(nwg, x, p.cpx);
    if (local >= xp.full + xp.tail * p.ksplit) return;
    if (local < xp.full) {
      bid = xp.t0 + local;
    } else {
      const int r = local - xp.full;
      bid = xp.t0 + xp.full + r / p.ksplit;
      kpart = r % p.ksplit;
      slab = (x * p.tail_cap + r / p.ksplit) * p.ksplit + kpart;
    }
  } else {
    bid = xcd_remap(bx, nwg);
  }
  int tm, tn;
  tile_of(p, bid, tm, tn);
  if (p.goff && p.gmode == 0 && !group_rows<EPI>(p, tm)) return;
  const int kt0 = kpart >= 0 ? kpart * p.kchunk : 0;
  if (kpart >= 0) p.K = min(p.K - kt0 * BK, p.kchunk * BK);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int Ncols = (EPI == kEpiSwiGLU) ? 2 * p.H : p.N;
  const int ktiles = (p.K + BK - 1) / BK;
  const int nt = (ktiles + 1) & ~1;

  f32x4v acc[2][8][4];  // [column half h][row tile i][column tile j]: column tile 4h + j of the wave
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const long a_step = AK ? BK : (long)BK * p.lda;
  const long b_step = BKM ? BK : (long)BK * p.ldb;
  const unsigned short* a_t0 = (AK ? p.A + (long)tm * BM * p.lda : p.A + (long)tm * BM) + a_step * kt0;
  const unsigned short* b_t0 =
      (BKM ? p.B + (long)tn * BN * p.ldb : (EPI == kEpiSwiGLU ? p.B : p.B + (long)tn * BN)) + b_step * kt0;
  const unsigned a_is = (unsigned)(AK ? 64 * p.lda * 2 : 16 * p.lda * 2);
  const unsigned b_is = (unsigned)(BKM ? 64 * p.ldb * 2 : 16 * p.ldb * 2);
  const Pc4 PA = pc4_setup<AK, false, EPI>(p.lda, p.M, tm, p.H, wave, lane, a_is);
  const Pc4 PB = pc4_setup<BKM, true, EPI>(p.ldb, Ncols, tn, p.H, wave, lane, b_is);
  // byte extent of each operand from its tile-0 base: the descriptors' num_records, so the hardware range check
  // bounds every DMA to the operand (rows past M / N and k past K read as zero)
  const long a_bytes = (long)((const char*)p.a_end - (const char*)a_t0);
  const long b_bytes = (long)((const char*)p.b_end - (const char*)b_t0);
  auto desc = [&](const unsigned short* t0, long step, long bytes, int t) {
    const long off = step * t;
    return make_rsrc_n(t0 + off, t < ktiles ? bytes - 2 * off : 0L);
  };

  const int arow = wm * 128, bcolw = wn * 128;
  const Rd4<AK> ra = rd4_setup<AK>(sbase, arow, lane);
  const Rd4<BKM> rb = rd4_setup<BKM>(sbase + B_OFF, bcolw, lane);
  const unsigned wdst = sbase + wave * 1024;  // this wave's first LDS-DMA piece slot

  // DMA piece k (0..15) of tile t into stage st: operand k >> 3, v2 wave (wave + 4 * ((k >> 2) & 1)),
  // instruction k & 3; `wb` is the opaque per-tile copy of wdst (the 32 slot addresses are one s_add each
  // instead of 32 loop-invariant SGPRs)
  auto piece = [&](auto Kc, int st, const __amdgpu_buffer_rsrc_t& rsa, const __amdgpu_buffer_rsrc_t& rsb,
                   unsigned wb, int krem) {
    constexpr int k = decltype(Kc)::value, I = k & 3, h = (k >> 2) & 1, j = 4 * h + I;
    constexpr bool isB = k >= 8;
    constexpr bool kmaj = isB ? BKM : AK;
    const unsigned dst = wb + st * TILE_BYTES + (8 * I + 4 * h) * 1024 + (isB ? B_OFF : 0);
    unsigned v = isB ? PB.v[j] : PA.v[j];
    if constexpr (!FAST && kmaj) v |= (unsigned)((isB ? PB.kl[h] : PA.kl[h]) >= krem) << 31;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isB ? rsb : rsa, (__attribute__((address_space(3))) void*)(size_t)dst,
                                             16, v, 0, 0, 0);
  };

  bf16x8 xa[8], xb[8], ya[8], yb[8];  // k32 step 0 / step 1 fragment sets of the current K-tile
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;

  // prologue: tiles 0 and 1 in flight, wait for tile 0 (everyone's), read its step-0 fragments
  {
    const __amdgpu_buffer_rsrc_t a0 = desc(a_t0, a_step, a_bytes, 0), b0 = desc(b_t0, b_step, b_bytes, 0);
    const __amdgpu_buffer_rsrc_t a1 = desc(a_t0, a_step, a_bytes, 1), b1 = desc(b_t0, b_step, b_bytes, 1);
    sfor<16>([&](auto K) { piece(K, 0, a0, b0, wdst, p.K); });
    sfor<16>([&](auto K) { piece(K, 1, a1, b1, wdst, p.K - BK); });
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  // fragment-set read order R = [b0, a0..a7, b1..b7]: the j-major MFMA order (B tile j outer, A tile i inner)
  // can start after 9 reads and needs one more read per 8 MFMAs (counted lgkmcnt, not a full drain)
  auto rd_set = [&](auto Q, auto S, auto ST, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    constexpr int q = decltype(Q)::value, s_ = decltype(S)::value, st_ = decltype(ST)::value;
    if constexpr (q == 0) fb[0] = frag4<BKM, 0, s_, st_>(rb);
    else if constexpr (q <= 8) fa[q - 1] = frag4<AK, q - 1, s_, st_>(ra);
    else fb[q - 8] = frag4<BKM, q - 8, s_, st_>(rb);
  };
  sfor<16>([&](auto Q) { rd_set(Q, C0{}, C0{}, xa, xb); });

  // MFMAs as asm on "+a" accumulators: with builtins hipcc re-shuffles the 256 accumulator registers between
  // AGPRs and VGPRs at the loop header (hundreds of v_accvgpr moves per K-tile pair); pinned to AGPRs they stay
  // put.  Hazards hipcc no longer sees: the fragments come straight from asm ds_reads (waited by lgkmcnt, no
  // VALU writes in between) and the accumulators are read only after the s_nop at the end of the loop.
  // Operands swapped (B fragment as src0): the MFMA computes the TRANSPOSED 16x16 tile, so each lane holds 4
  // consecutive COLUMNS of one row (row 16i + (lane & 15), columns 16j + 4 * (lane >> 4) + e): the epilogue
  // stores 8 B (bf16) / 16 B (fp32) per lane instead of 2 / 4 B.
  auto mm = [&](auto Q, const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
    constexpr int q = decltype(Q)::value, j = q / 8, i = q % 8;
    mfma_agpr(acc[j >> 2][i][j & 3], fb[j], fa[i]);
  };

  // The loop has no branches: past K every piece reads zeros through a num_records-0 descriptor (no memory
  // traffic), so tiles nt and nt+1 are "streamed" into stages nobody reads again, and vmcnt(16) always retires
  // tile t+1.
  auto ktile = [&](auto ST, int t) {
    constexpr int st = decltype(ST)::value;
    const __amdgpu_buffer_rsrc_t rsa = desc(a_t0, a_step, a_bytes, t + 2), rsb = desc(b_t0, b_step, b_bytes, t + 2);
    const int krem = p.K - (t + 2) * BK;
    unsigned wb = wdst;
    asm volatile("" : "+s"(wb));
    __builtin_amdgcn_s_setprio(1);
    sfor<64>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      // x set (read order R, issued behind the previous tile's last 16 MFMAs): MFMAs 0-7 need R[0..8],
      // MFMAs 8-15 R[9] (outstanding then: R[10..15] + the 8 y reads issued so far); from MFMA 16 on at most 15
      // LDS ops can be outstanding, so R[10+] are retired by the time each is needed
      if constexpr (q == 0) {
        asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q == 8) {
        asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q >= 16 && q < 24 && q % 8 == 0) {
        asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(Q, xa, xb);
      if constexpr (q < 16) rd_set(Q, C1{}, ST, ya, yb);
      if constexpr (q == 23) {
        // every wave holds all its fragments of this stage: release it
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
      }
      if constexpr (q >= 24 && (q - 24) % 5 == 0)
        piece(std::integral_constant<int, (q - 24) / 5>{}, st, rsa, rsb, wb, krem);
      __builtin_amdgcn_sched_barrier(0);
    });
    sfor<64>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      mm(Q, ya, yb);
      if constexpr (q + 64 >= 24 && (q + 64 - 24) % 5 == 0 && (q + 64 - 24) / 5 < 16)
        piece(std::integral_constant<int, (q + 64 - 24) / 5>{}, st, rsa, rsb, wb, krem);
      if constexpr (q == 47) {
        // tile t+1 landed (own pieces, then everyone's)
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
      }
      if constexpr (q >= 48) rd_set(std::integral_constant<int, q - 48>{}, C0{}, std::integral_constant<int, st ^ 1>{}, xa, xb);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_setprio(0);
  };

  // the spread schedule (SP): see gemm7.hip ktile_v for the per-MFMA positions
  auto ktile_sp = [&](auto ST, int t) {
    constexpr int st = decltype(ST)::value;
    const __amdgpu_buffer_rsrc_t rsa = desc(a_t0, a_step, a_bytes, t + 2), rsb = desc(b_t0, b_step, b_bytes, t + 2);
    const int krem = p.K - (t + 2) * BK;
    unsigned wb = wdst;
    asm volatile("" : "+s"(wb));
    sfor<128>([&](auto Q) {
      constexpr int n = decltype(Q)::value;
      constexpr int RA1[8] = {1, 3, 5, 7, 9, 11, 13, 15};
      constexpr int RB1[8] = {25, 28, 31, 34, 37, 39, 41, 43};
      constexpr int PA_[8] = {23, 26, 29, 32, 35, 53, 56, 59};
      constexpr int PB_[8] = {62, 65, 86, 88, 90, 97, 101, 125};
      constexpr int XA[8] = {94, 95, 96, 98, 99, 103, 104, 105};
      constexpr int XB[8] = {106, 107, 110, 113, 115, 118, 121, 124};
      auto idx = [](const int (&tb)[8], int v) constexpr {
        int r = -1;
        for (int i = 0; i < 8; ++i)
          if (tb[i] == v) r = i;
        return r;
      };
      constexpr int ra1 = idx(RA1, n), rb1 = idx(RB1, n), pa = idx(PA_, n), pb = idx(PB_, n), xa_ = idx(XA, n),
                    xb_ = idx(XB, n);
      if constexpr (n == 21 || n == 51) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (n == 92) {
        asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (n == 127) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (ra1 >= 0) ya[ra1] = frag4<AK, (ra1 < 0 ? 0 : ra1), 1, st>(ra);
      if constexpr (rb1 >= 0) yb[rb1] = frag4<BKM, (rb1 < 0 ? 0 : rb1), 1, st>(rb);
      if constexpr (xa_ >= 0) xa[xa_] = frag4<AK, (xa_ < 0 ? 0 : xa_), 0, st ^ 1>(ra);
      if constexpr (xb_ >= 0) xb[xb_] = frag4<BKM, (xb_ < 0 ? 0 : xb_), 0, st ^ 1>(rb);
      constexpr int nn = n & 63;
      if constexpr (n < 64) mm(std::integral_constant<int, nn>{}, xa, xb);
      else mm(std::integral_constant<int, nn>{}, ya, yb);
      // pieces behind the MFMA (a buffer_load ... lds after an MFMA: the compiler covers the M0 hazard itself)
      if constexpr (pa >= 0) piece(std::integral_constant<int, (pa < 0 ? 0 : pa)>{}, st, rsa, rsb, wb, krem);
      if constexpr (pb >= 0) piece(std::integral_constant<int, 8 + (pb < 0 ? 0 : pb)>{}, st, rsa, rsb, wb, krem);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  if constexpr (SP) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the prologue's step-0 reads (no counted waits in SP)
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < nt; t += 2) {
      ktile_sp(C0{}, t);
      ktile_sp(C1{}, t + 1);
    }
  } else {
    for (int t = 0; t < nt; t += 2) {
      ktile(C0{}, t);
      ktile(C1{}, t + 1);
    }
  }
  // drain the masked tail pieces and the last (unused) fragment reads before the workgroup's LDS goes away;
  // the s_nops cover the MFMA-write -> accumulator-read wait states of the last MFMAs
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 7" ::: "memory");

  if constexpr (EPI != kEpiSwiGLU) {
    if (kpart >= 0) {
      float* sp = p.part + (long)slab * (BM * BN);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              sp[(arow + 16 * i + (lane & 15)) * BN + bcolw + 64 * h + 16 * j + 4 * (lane >> 4) + e] = acc[h][i][j][e];
      return;
    }
  }
  if constexpr (EPI == kEpiGeLU || EPI == kEpiDGeLU) {
    // compile-time halves: a runtime h (the unroller gives up on the GELU bodies) indexed acc[h]
    // dynamically, which demoted every accumulator to scratch -- inside the MFMA loop
    sfor<2>([&](auto H) {
      constexpr int h = decltype(H)::value;
      epilogue_t<EPI>(p, acc[h], tm, tn, arow, bcolw + 64 * h, lane);
    });
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) epilogue_t<EPI>(p, acc[h], tm, tn, arow, bcolw + 64 * h, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// v6: v4's K-loop made persistent.  grid = min(tiles, CUs); workgroup w takes tiles slot(w), slot(w) + G, ...
// (slot = the XCD-chunked remap, so the G tiles in flight at any time are the grouped-order block each XCD's
// L2 shares, as in a one-wave launch).  The K-tile stream of all its tiles is one pipeline: the LDS-DMA two
// K-tiles ahead runs across tile boundaries, so the next tile's first K-tiles land while the previous tile's
// epilogue stores (no per-tile prologue bubble), and the workgroup's LDS / register setup happens once.
// No tail split-K: the last round may be partial.  (A dynamically scheduled form — per-XCD atomic tile queues
// with stealing — measured 3-8 % slower than this static one: it loses the grouped L2 block per XCD.)
template <bool AK, bool BKM, int EPI, bool FAST>
__global__ __launch_bounds__(NTHR4, 1) void gemm_v6_kernel(Params p) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  const unsigned sbase = (unsigned)(size_t)(lds_char*)smem_raw;

  const int nwg = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  const int ntile = slot < nwg ? (nwg - slot + G - 1) / G : 0;
  if (ntile == 0) return;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ktiles = (p.K + BK - 1) / BK;
  const int nt = (ktiles + 1) & ~1;

  f32x4v acc[2][8][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const long a_step = AK ? BK : (long)BK * p.lda;
  const long b_step = BKM ? BK : (long)BK * p.ldb;
  const unsigned a_is = (unsigned)(AK ? 64 * p.lda * 2 : 16 * p.lda * 2);
  const unsigned b_is = (unsigned)(BKM ? 64 * p.ldb * 2 : 16 * p.ldb * 2);
  // lane offsets relative to the tile base: tile-independent (no per-tile column flags — with exact operand
  // extents the rows / columns past M / N of an edge tile read either zeros or bytes of the operand that only
  // feed output rows / columns the epilogue never stores)
  const Pc4 PA = pc4_setup<AK, false, EPI>(p.lda, 1 << 30, 0, p.H, wave, lane, a_is);
  const Pc4 PB = pc4_setup<BKM, true, EPI>(p.ldb, 1 << 30, 0, p.H, wave, lane, b_is);
  const char* a_end = (const char*)p.a_end;
  const char* b_end = (const char*)p.b_end;
  auto a_base = [&](int tm) { return AK ? p.A + (long)tm * BM * p.lda : p.A + (long)tm * BM; };
  auto b_base = [&](int tn) {
    return BKM ? p.B + (long)tn * BN * p.ldb : (EPI == kEpiSwiGLU ? p.B + (long)tn * 128 : p.B + (long)tn * BN);
  };

  const int arow = wm * 128, bcolw = wn * 128;
  const Rd4<AK> ra = rd4_setup<AK>(sbase, arow, lane);
  const Rd4<BKM> rb = rd4_setup<BKM>(sbase + B_OFF, bcolw, lane);
  const unsigned wdst = sbase + wave * 1024;

  // prefetch cursor: tile (sequence index pu) and K-tile pk of the next K-tile to stream; descriptors of tiles
  // past this workgroup's last carry num_records 0
  int pu = 0, pk = 0, ptm = 0, ptn = 0;
  const unsigned short* pa0 = nullptr;
  const unsigned short* pb0 = nullptr;
  auto set_tile = [&](int u) {
    const int L = slot + u * G;
    if (u < ntile) tile_of(p, L, ptm, ptn);
    pa0 = a_base(ptm);
    pb0 = b_base(ptn);
  };
  set_tile(0);
  auto next_desc = [&](__amdgpu_buffer_rsrc_t& rsa, __amdgpu_buffer_rsrc_t& rsb, int& krem) {
    const bool live = pu < ntile && pk < ktiles;
    const long ao = a_step * pk, bo = b_step * pk;
    rsa = make_rsrc_n(pa0 + ao, live ? (long)(a_end - (const char*)(pa0 + ao)) : 0L);
    rsb = make_rsrc_n(pb0 + bo, live ? (long)(b_end - (const char*)(pb0 + bo)) : 0L);
    krem = p.K - pk * BK;
    if (++pk == nt) {
      pk = 0;
      ++pu;
      set_tile(pu);
    }
  };

  auto piece = [&](auto Kc, int st, const __amdgpu_buffer_rsrc_t& rsa, const __amdgpu_buffer_rsrc_t& rsb,
                   unsigned wb, int krem) {
    constexpr int k = decltype(Kc)::value, I = k & 3, h = (k >> 2) & 1, j = 4 * h + I;
    constexpr bool isB = k >= 8;
    constexpr bool kmaj = isB ? BKM : AK;
    const unsigned dst = wb + st * TILE_BYTES + (8 * I + 4 * h) * 1024 + (isB ? B_OFF : 0);
    unsigned v = isB ? PB.v[j] : PA.v[j];
    if constexpr (!FAST && kmaj) v |= (unsigned)((isB ? PB.kl[h] : PA.kl[h]) >= krem) << 31;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isB ? rsb : rsa, (__attribute__((address_space(3))) void*)(size_t)dst,
                                             16, v, 0, 0, 0);
  };

  bf16x8 xa[8], xb[8], ya[8], yb[8];
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  auto rd_set = [&](auto Q, auto S, auto ST, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    constexpr int q = decltype(Q)::value, s_ = decltype(S)::value, st_ = decltype(ST)::value;
    if constexpr (q == 0) fb[0] = frag4<BKM, 0, s_, st_>(rb);
    else if constexpr (q <= 8) fa[q - 1] = frag4<AK, q - 1, s_, st_>(ra);
    else fb[q - 8] = frag4<BKM, q - 8, s_, st_>(rb);
  };

  // prologue: the first two K-tiles of the first tile
  {
    __amdgpu_buffer_rsrc_t rsa, rsb;
    int krem;
    next_desc(rsa, rsb, krem);
    sfor<16>([&](auto K) { piece(K, 0, rsa, rsb, wdst, krem); });
    next_desc(rsa, rsb, krem);
    sfor<16>([&](auto K) { piece(K, 1, rsa, rsb, wdst, krem); });
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  sfor<16>([&](auto Q) { rd_set(Q, C0{}, C0{}, xa, xb); });

  auto mm = [&](auto Q, const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
    constexpr int q = decltype(Q)::value, j = q / 8, i = q % 8;
    mfma_agpr(acc[j >> 2][i][j & 3], fb[j], fa[i]);
  };

  auto ktile = [&](auto ST) {
    constexpr int st = decltype(ST)::value;
    __amdgpu_buffer_rsrc_t rsa, rsb;
    int krem;
    next_desc(rsa, rsb, krem);
    unsigned wb = wdst;
    asm volatile("" : "+s"(wb));
    __builtin_amdgcn_s_setprio(1);
    sfor<64>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      if constexpr (q == 0) {
        asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q == 8) {
        asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (q >= 16 && q < 24 && q % 8 == 0) {
        asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(Q, xa, xb);
      if constexpr (q < 16) rd_set(Q, C1{}, ST, ya, yb);
      if constexpr (q == 23) {
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
      }
      if constexpr (q >= 24 && (q - 24) % 5 == 0) piece(std::integral_constant<int, (q - 24) / 5>{}, st, rsa, rsb, wb, krem);
      __builtin_amdgcn_sched_barrier(0);
    });
    sfor<64>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      mm(Q, ya, yb);
      if constexpr (q + 64 >= 24 && (q + 64 - 24) % 5 == 0 && (q + 64 - 24) / 5 < 16)
        piece(std::integral_constant<int, (q + 64 - 24) / 5>{}, st, rsa, rsb, wb, krem);
      if constexpr (q == 47) {
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
      }
      if constexpr (q >= 48) rd_set(std::integral_constant<int, q - 48>{}, C0{}, std::integral_constant<int, st ^ 1>{}, xa, xb);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_setprio(0);
  };

  int ctm, ctn;
  tile_of(p, slot, ctm, ctn);
  for (int u = 0; u < ntile; ++u) {
    for (int t = 0; t < nt; t += 2) {
      ktile(C0{});
      ktile(C1{});
    }
    // tile done: its accumulators out (the next tile's first K-tiles are already streaming / being read)
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
    if constexpr (EPI == kEpiGeLU || EPI == kEpiDGeLU) {
      // compile-time halves: a runtime h (the unroller gives up on the GELU bodies) indexed acc[h]
      // dynamically, which demoted every accumulator to scratch -- inside the MFMA loop
      sfor<2>([&](auto H) {
        constexpr int h = decltype(H)::value;
        epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
      });
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_nop 4" ::: "memory");
    if (u + 1 < ntile) tile_of(p, slot + (u + 1) * G, ctm, ctn);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace gm
}  // namespace pd

bool pd_gemm_v7(const pd::gm::Params& p, int layout, int epi, int sched, int cus, long ws_bytes, hipStream_t st);  // gemm7.hip

// layout: bit0 = A K-major, bit1 = B K-major.  epi: 0 bf16 (+bias), 1 fp32 main grad (beta), 2 swiglu.
// CUs per XCD of the current device (workgroup slots of the 128 KiB-LDS kernel), cached per device
static int cus_per_xcd() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 32;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8) n = 256;
    cache[dev] = n / 8;
  }
  return cache[dev];
}

// Tail split-K plan: an XCD's last, partial wave of `tail` tiles takes one full tile time; cut into s
// K-slices (at least 8 K-tiles each) it takes ceil(tail*s / cpx) / s of one.  The smallest s (2..4) with the
// shortest tail time wins if it saves at least 1/8 of a tile time and its slabs fit the workspace (8 *
// tail_cap * s slabs of BM*BN fp32).  Returns the grid size (0 = no split).
static int plan_splitk(pd::gm::Params& p, long ws_bytes) {
  using namespace pd::gm;
  const int nwg = p.tiles_m * p.tiles_n, cpx = p.cpx;
  int maxtail = 0;
  for (int x = 0; x < 8; ++x) maxtail = std::max(maxtail, xcd_plan(nwg, x, cpx).tail);
  const int ktiles = (p.K + BK - 1) / BK;
  if (maxtail == 0) return 0;
  int s = 1;
  double best = 1.0;
  for (int c = 2; c <= 4; ++c) {
    if (ktiles / c < 8 || 8L * maxtail * c * BM * BN * 4 > ws_bytes) continue;
    const double t = (double)((maxtail * c + cpx - 1) / cpx) / c;
    if (t < best - 0.125) { best = t; s = c; }
  }
  if (s < 2) return 0;
  const int kchunk = (((ktiles + s - 1) / s) + 1) & ~1;  // even: the loop body is two K-tiles
  s = (ktiles + kchunk - 1) / kchunk;
  if (s < 2 || 8L * maxtail * s * BM * BN * 4 > ws_bytes) return 0;
  p.ksplit = s;
  p.kchunk = kchunk;
  p.tail_cap = maxtail;
  int blocks = 0;
  for (int x = 0; x < 8; ++x) {
    const XPlan xp = xcd_plan(nwg, x, cpx);
    blocks = std::max(blocks, xp.full + xp.tail * s);
  }
  return 8 * blocks;
}

// RoPE-epilogue tables of the next pd_gemm call on this thread (pd_gemm_set_rope; consumed by the call)
static thread_local const float* t_rope_cos = nullptr;
static thread_local const float* t_rope_sin = nullptr;
static thread_local int t_rope_cols = 0, t_rope_seq = 0;
extern "C" void pd_gemm_set_rope(const float* cos, const float* sin, int cols, int seq) {
  t_rope_cos = cos; t_rope_sin = sin; t_rope_cols = cols; t_rope_seq = seq;
}

extern "C" int pd_gemm(int layout, int epi, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                       void* C2, long ldc2, const void* bias, int M, int N, int K, float beta, int H, int group_m,
                       int variant, void* ws, long ws_bytes, void* stream) {
  using namespace pd::gm;
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if (epi == kEpiRope && (layout != 3 || !t_rope_cos)) return -3;   // RoPE: TN layout, tables set first
  if ((layout & 3) && K % 8) return -1;   // K-major operands move 16-B chunks along k
  Params p;
  p.A = (const unsigned short*)A;
  p.B = (const unsigned short*)B;
  p.C = C;
  p.C2 = (unsigned short*)C2;
  p.bias = (const unsigned short*)bias;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldc2 = ldc2;
  p.M = M; p.N = N; p.K = K; p.beta = beta; p.H = H;
  p.zero = bias;  // ablation 7 only: the caller passes a zeroed buffer in `bias`
  p.goff = nullptr; p.ngroups = 0; p.gmode = 0; p.gsb = p.gsc = p.gsbias = 0;
  p.part = (float*)ws; p.ksplit = 1; p.kchunk = 0; p.tail_cap = 0; p.cpx = cus_per_xcd();
  p.rope_cos = t_rope_cos; p.rope_sin = t_rope_sin; p.rope_cols = t_rope_cols; p.rope_seq = t_rope_seq;
  t_rope_cos = t_rope_sin = nullptr;
  {
    // operand extents: K-major [rows][ld] with K valid per row, MN-major [k][ld] with rows / cols valid per k
    const bool ak = layout & 1, bk = (layout >> 1) & 1;
    const long ncols = epi == kEpiSwiGLU ? 2L * H : (long)N;
    const long a_el = ak ? (long)(M - 1) * lda + K : (long)(K - 1) * lda + M;
    const long b_el = bk ? (ncols - 1) * ldb + K : (long)(K - 1) * ldb + ncols;
    p.a_end = (const unsigned short*)A + a_el;
    p.b_end = (const unsigned short*)B + b_el;
  }
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = epi == kEpiSwiGLU ? (H + 127) / 128 : (N + BN - 1) / BN;
  p.group_m = group_m > 0 ? group_m : 8;
  const bool ak = layout & 1, bk = (layout >> 1) & 1;
  if (!ak && (lda % 8 || M % 8)) return -2;   // MN-major operands move whole 16-B column chunks
  if (!bk && (ldb % 8 || (epi == kEpiSwiGLU ? (2 * H) % 8 : N % 8))) return -2;
  if (epi == kEpiSwiGLU && H % 32) return -3;
  if ((epi == kEpiGeLU || epi == kEpiDGeLU) && (!C2 || ldc2 < N)) return -3;   // the pre-activation operand
  if (epi == kEpiDSwiGLU && (!C2 || H != N || ldc2 < 2L * N || ldc < 2L * N)) return -3;   // gate | up, 2N wide
  hipStream_t st = (hipStream_t)stream;
  // v7 (gemm7.hip): the TN schedule, variants 7..10 = its SCHED 0..3; problems outside its domain run v6
  if ((variant >= 7 && variant <= 10) || variant >= 64) {
    const int sched = variant >= 64 ? variant - 64 : variant - 7;
    if (pd_gemm_v7(p, layout, epi, sched, 8 * p.cpx, ws ? ws_bytes : 0, st)) return (int)hipGetLastError();
    const bool mn = variant >= 64 && (sched & (32768 | 65536));
    // an MN-major schedule asked for a problem whose operands are both K-major: the same schedule on the TN kernel
    if (mn && layout == 3 && pd_gemm_v7(p, layout, epi, sched & ~(32768 | 65536), 8 * p.cpx, ws ? ws_bytes : 0, st))
      return (int)hipGetLastError();
    // outside the kernel's domain: the persistent v6, or for the MN-major schedules v4's spread kernel (any layout)
    variant = mn ? 5 : 6;
  }
  if (epi == kEpiRope || epi == kEpiDSwiGLU) return -3;   // the spread TN schedule only (RoPE / SwiGLU backward)
  if (epi == kEpiSwiGLU && bk) return -3;  // K-major gate|up weight: v7 only
  // v4+ store 4 consecutive output columns per lane (8-B bf16 / 16-B fp32 accesses): rows must keep that alignment
  if (variant >= 4 && (ldc % 4 || (size_t)C % 16 || (C2 && (ldc2 % 4 || (size_t)C2 % 16)))) variant = 0;
  dim3 grid(p.tiles_m * p.tiles_n);
  if (ws && (variant == 0 || variant == 4 || variant == 5) && (epi == kEpiBF16 || epi == kEpiF32)) {
    const int g = plan_splitk(p, ws_bytes);
    if (g) grid = dim3(g);
  }
  const dim3 rgrid(BM * BN / 1024, 8 * p.tail_cap);
  const bool fast = !(ak || bk) || K % BK == 0;  // v4: no K-major operand has a partial last K-tile
  const dim3 pgrid(std::min(p.tiles_m * p.tiles_n, 8 * p.cpx));  // v6: one persistent workgroup per CU
#define PD_GEMM_LAUNCH(AKV, BKV, EPIV)                                          \
  if (variant == 5) {                                                            \
    if (fast)                                                                    \
      gemm_v4_kernel<AKV, BKV, EPIV, true, true><<<grid, NTHR4, 0, st>>>(p);    \
    else                                                                         \
      gemm_v4_kernel<AKV, BKV, EPIV, false, true><<<grid, NTHR4, 0, st>>>(p);   \
    if (p.ksplit > 1) splitk_reduce_kernel<EPIV><<<rgrid, 256, 0, st>>>(p);     \
  } else if (variant == 4) {                                                     \
    if (fast)                                                                    \
      gemm_v4_kernel<AKV, BKV, EPIV, true><<<grid, NTHR4, 0, st>>>(p);          \
    else                                                                         \
      gemm_v4_kernel<AKV, BKV, EPIV, false><<<grid, NTHR4, 0, st>>>(p);         \
    if (p.ksplit > 1) splitk_reduce_kernel<EPIV><<<rgrid, 256, 0, st>>>(p);     \
  } else if (variant == 6) {                                                     \
    if (fast)                                                                    \
      gemm_v6_kernel<AKV, BKV, EPIV, true><<<pgrid, NTHR4, 0, st>>>(p);         \
    else                                                                         \
      gemm_v6_kernel<AKV, BKV, EPIV, false><<<pgrid, NTHR4, 0, st>>>(p);        \
  } else {                                                                       \
    gemm_kernel<AKV, BKV, EPIV><<<grid, NTHR, 0, st>>>(p);                      \
    if (p.ksplit > 1) splitk_reduce_kernel<EPIV><<<rgrid, 256, 0, st>>>(p);     \
  }
  switch (epi * 4 + layout) {
    case 0 * 4 + 0: PD_GEMM_LAUNCH(false, false, kEpiBF16); break;
    case 0 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiBF16); break;
    case 0 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiBF16); break;
    case 1 * 4 + 0: PD_GEMM_LAUNCH(false, false, kEpiF32); break;
    case 1 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiF32); break;
    case 1 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiF32); break;
    case 2 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiSwiGLU); break;
    case 3 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiGeLU); break;
    case 3 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiGeLU); break;
    case 4 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiDGeLU); break;
#ifdef PD_GEMM_DEBUG_VARIANTS
    // timing-only ablations (WRONG results): 16+: no vmcnt at the barrier, 20+: no lgkm syncs, 24+: no barrier
    case 16 + 3: gemm_kernel<true, true, kEpiBF16, 1><<<grid, NTHR, 0, st>>>(p); break;
    case 20 + 3: gemm_kernel<true, true, kEpiBF16, 2><<<grid, NTHR, 0, st>>>(p); break;
    case 24 + 3: gemm_kernel<true, true, kEpiBF16, 3><<<grid, NTHR, 0, st>>>(p); break;
    case 28 + 3: gemm_kernel<true, true, kEpiBF16, 4><<<grid, NTHR, 0, st>>>(p); break;   // no DMA in the loop
    case 32 + 3: gemm_kernel<true, true, kEpiBF16, 5><<<grid, NTHR, 0, st>>>(p); break;   // no LDS reads in the loop
    case 36 + 3: gemm_kernel<true, true, kEpiBF16, 6><<<grid, NTHR, 0, st>>>(p); break;   // all tiles load tile (0,0)
    case 40 + 3: gemm_kernel<true, true, kEpiBF16, 7><<<grid, NTHR, 0, st>>>(p); break;   // global_load_lds staging
#endif
    default: return -4;
  }
#undef PD_GEMM_LAUNCH
  return (int)hipGetLastError();
}

// Grouped GEMM over expert-sorted rows (MoE): ONE launch for every group, offsets read on the device.
//  gmode 0: C[goff[g]:goff[g+1], :N] = A[goff[g]:goff[g+1], :K] . B_g (+ bias_g), B_g = B + g*gsb
//           (fwd: layout AK, B N-major [K, N]; dgrad: layout AK|BK, B_g read as [N, K] rows); max_rows = total
//           rows (sizes the grid: ceil(max_rows / 256) + ngroups row tiles bound every split)
//  gmode 1: C_g[M, N] (+)= A[goff[g]:goff[g+1], :M]^T . B[goff[g]:goff[g+1], :N], C_g = C + g*gsc (fp32 epilogue
//           for main grads, bf16 otherwise); layout 0 (both operands token-major)
extern "C" int pd_gemm_grouped(int layout, int epi, const void* A, long lda, const void* B, long ldb, long gsb,
                               void* C, long ldc, long gsc, void* C2, long ldc2, const void* bias, long gsbias,
                               const int* goff, int ngroups, int gmode, int M, int N, int K, int max_rows, float beta,
                               int H, int group_m, void* stream) {
  using namespace pd::gm;
  if (ngroups <= 0 || !goff || N <= 0) return -1;
  Params p;
  p.A = (const unsigned short*)A;
  p.B = (const unsigned short*)B;
  p.C = C;
  p.C2 = (unsigned short*)C2;
  p.bias = (const unsigned short*)bias;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldc2 = ldc2;
  p.N = N; p.beta = beta; p.H = H; p.zero = nullptr;
  p.goff = goff; p.ngroups = ngroups; p.gmode = gmode; p.gsb = gsb; p.gsc = gsc; p.gsbias = gsbias;
  p.part = nullptr; p.ksplit = 1; p.kchunk = 0; p.tail_cap = 0; p.cpx = 32;
  p.a_end = nullptr; p.b_end = nullptr;
  p.group_m = group_m > 0 ? group_m : 8;
  p.tiles_n = epi == kEpiSwiGLU ? (H + 127) / 128 : (N + BN - 1) / BN;
  const bool ak = layout & 1, bk = (layout >> 1) & 1;
  dim3 grid;
  if (gmode == 0) {
    if (!ak || K <= 0 || K % 8 || max_rows <= 0) return -1;
    p.M = max_rows; p.K = K;
    p.tiles_m = (max_rows + BM - 1) / BM + ngroups;
    grid = dim3(p.tiles_m * p.tiles_n);
    if (!bk && (ldb % 8 || (epi == kEpiSwiGLU ? (2 * H) % 8 : N % 8))) return -2;
    if (epi == kEpiSwiGLU && (bk || H % 32)) return -3;
  } else if (gmode == 1) {
    if (layout != 0 || M <= 0 || M % 8 || N % 8 || lda % 8 || ldb % 8 || epi == kEpiSwiGLU) return -1;
    p.M = M; p.K = 0;
    p.tiles_m = (M + BM - 1) / BM;
    grid = dim3(p.tiles_m * p.tiles_n * ngroups);
  } else {
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  switch (epi * 4 + layout) {
    case 0 * 4 + 0: gemm_kernel<false, false, kEpiBF16><<<grid, NTHR, 0, st>>>(p); break;
    case 0 * 4 + 1: gemm_kernel<true, false, kEpiBF16><<<grid, NTHR, 0, st>>>(p); break;
    case 0 * 4 + 3: gemm_kernel<true, true, kEpiBF16><<<grid, NTHR, 0, st>>>(p); break;
    case 1 * 4 + 0: gemm_kernel<false, false, kEpiF32><<<grid, NTHR, 0, st>>>(p); break;
    case 2 * 4 + 1: gemm_kernel<true, false, kEpiSwiGLU><<<grid, NTHR, 0, st>>>(p); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}
