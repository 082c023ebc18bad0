// fp8 / bf8 TN GEMM on gfx950's K = 128 matrix instruction (v_mfma_f32_16x16x128_f8f6f4): twice the bf16 MFMA
// rate per clock, fp32 accumulation, per-tensor dequant factors read from the device (delayed scaling keeps them
// there), bf16 (+bias) or fp32 output.  Both operands K-major — the three GEMMs of an fp8 linear:
//   forward  y  = x[M, K] . W^T[N, K]            e4m3 x e4m3
//   dgrad    dx = dy[M, N] . W[K, N] (rows of W)  e5m2 x e4m3
//   wgrad    dW = x^T[K, M] . dy^T[N, M]          e4m3 x e5m2
// Reference parity: paddle/phi/kernels/fusion/fp8_gemm/fp8_gemm_with_cublasLt/fp8_fp8_half_gemm.cu:28-58
// (cublasLt fp8 GEMM with a scale, half / bf16 out, optional bias).
//
// The LDS side is v7's unchanged (gemm7.hip): a K-tile is 128 B of every row — 64 bf16 there, 128 fp8 here — so
// the 256 x 128-B operand images, the 2-stage LDS-DMA ring, the XOR swizzle, the persistent XCD-chunked tile
// slots and the fragment reads are byte-for-byte v7's; the kernel sees the fp8 matrices as 2-byte-unit matrices
// (lda / 2, K / 2).  One 16x16x128 MFMA takes a row's whole 128-B K-tile: the lane's two 16-B chunks (v7's k32
// step-0 and step-1 fragments, chunks g and 4 + g of the row for lane group g) concatenated, the same k order for
// both operands, so the sum over k is the GEMM's.  64 MFMAs per K-tile and wave, each twice a bf16 MFMA's cycles.
//
// K-tile schedule (MFMA n = 0..63, B-fragment-major: column block j = n / 8 outer, row block i = n % 8 inner):
//   before n = 0: vmcnt(0) + lgkmcnt(0) + barrier — tile t+1 landed (every wave's pieces) and every wave holds all
//     of tile t's fragments, so stage(t) is free;
//   n = 1..16: the 16 LDS-DMA pieces of tile t+2 into stage(t), one behind each MFMA (last piece >= 48 MFMAs before
//     the wait that needs it);
//   n = 2, 4, .., 32: tile t+1's A fragments into the other A register set (A is used by every MFMA, so it is
//     double-buffered: 2 x 64 VGPRs);
//   n = 8j + 8, 8j + 9: tile t+1's B_j (j < 7) into B_j's registers right after B_j's last MFMA of tile t;
//   n = 36, 37: tile t+1's B_7 into the other B_7 register set.
// One barrier and no counted lgkmcnt waits per K-tile: every fragment is read a full K-tile ahead.
#include "gemm_tn.h"

namespace pd {
namespace gm {

typedef int i32x8 __attribute__((ext_vector_type(8)));

// a row block's 32 fp8 of the K-tile: the two 16-B chunks as one 8-VGPR operand (the register allocator places
// the two reads' destinations adjacently; no copies)
__device__ __forceinline__ i32x8 pair(const bf16x8& x, const bf16x8& y) {
  const i32x4 a = __builtin_bit_cast(i32x4, x), b = __builtin_bit_cast(i32x4, y);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// D += src0 x src1 (src0 = the B fragment: the transposed output tile, as v7); cbsz / blgp = the formats of
// src0 / src1 (0 e4m3, 1 e5m2)
template <int F0, int F1>
__device__ __forceinline__ void mfma8(f32x4v& c, const i32x8& b, const i32x8& a) {
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 cbsz:%3 blgp:%4"
               : "+a"(c)
               : "v"(b), "v"(a), "i"(F0), "i"(F1));
}
// the same with an LDS-DMA piece behind it (M0 written before the MFMA, which covers the M0 -> lds-load hazard)
template <int IMM, int F0, int F1>
__device__ __forceinline__ void mfma8_dma(f32x4v& c, const i32x8& b, const i32x8& a, unsigned wb, unsigned voff,
                                          const i32x4& srd) {
  asm volatile(
      "s_add_u32 m0, %1, %2\n\t"
      "v_mfma_f32_16x16x128_f8f6f4 %0, %3, %4, %0 cbsz:%7 blgp:%8\n\t"
      "buffer_load_dwordx4 %5, %6, 0 offen lds"
      : "+a"(c)
      : "s"(wb), "i"(IMM), "v"(b), "v"(a), "v"(voff), "s"(srd), "i"(F0), "i"(F1)
      : "memory");
}

// SCHED 1 (the late-wait K-tile): the one barrier at n = 0 becomes two — lgkmcnt(0) + barrier at n = 0 (every wave
// holds tile t's fragments: stage(t) may take tile t+2's pieces) and vmcnt(13) + barrier before MFMA 14 (tile t+1
// landed; this tile's first 13 pieces stay in flight) — and tile t+1's fragments are read from MFMA 14 on (B_7's
// second set at 14-15, A at 16-31, B_j at >= 8j + 8: 32-41, 48-49, 56-57).  A piece of tile t+1 then has ~62
// MFMAs (instead of ~48) between its issue and the wait that needs it.
// SCHED 2 (spread pieces): SCHED 1's waits and fragment reads, but tile t+2's 16 LDS-DMA pieces go one per two MFMAs
// (A at n = 1, 5, .., 29, B at n = 3, 7, .., 31) instead of one behind each of MFMAs 1..16: a piece's issue costs
// tens of cycles beside MFMAs (MI355X_MICROARCH 'LDS-DMA piece issue cost'), so 16 back-to-back pieces starve the
// matrix pipe for part of the burst; the late wait at n = 14 then leaves the 7 pieces issued before it in flight.
template <int SCHED>
__device__ constexpr int f8_piece_a(int n) {   // A piece index issued behind MFMA n, or -1
  if constexpr (SCHED == 2) return (n >= 1 && n <= 29 && (n - 1) % 4 == 0) ? (n - 1) / 4 : -1;
  else return (n >= 1 && n <= 8) ? n - 1 : -1;
}
template <int SCHED>
__device__ constexpr int f8_piece_b(int n) {
  if constexpr (SCHED == 2) return (n >= 3 && n <= 31 && (n - 3) % 4 == 0) ? (n - 3) / 4 : -1;
  else return (n >= 9 && n <= 16) ? n - 9 : -1;
}
template <int SCHED>
__device__ constexpr int f8_pieces_before(int n) {   // pieces issued behind MFMAs 0 .. n-1 of a K-tile
  int c = 0;
  for (int i = 0; i < n; ++i) c += (f8_piece_a<SCHED>(i) >= 0) + (f8_piece_b<SCHED>(i) >= 0);
  return c;
}

template <int FA, int FB, int EPI, bool TSK = false, int SCHED = 0>
__global__ __launch_bounds__(NTHR4, 1) void gemm_f8_kernel(Params p) {
  constexpr bool LATE = SCHED >= 1;   // SCHED 1 / 2: the late-wait K-tile
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  const unsigned sbase = (unsigned)(size_t)(lds_char*)smem_raw;

  const int nwg = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  // tail split-K (gemm_tn.h): the whole-tile launch skips the last tail_cap tiles, the TSK launch runs them as
  // ksplit K-slices (slot = tail tile * ksplit + slice), one per workgroup
  const int whole = nwg - p.tail_cap;
  const int ntile = TSK ? (slot < p.tail_cap * p.ksplit ? 1 : 0) : (slot < whole ? (whole - slot + G - 1) / G : 0);
  if (ntile == 0) return;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = TSK ? p.K / BK / p.ksplit : p.K / BK;  // K-tiles of 128 fp8 (p.K counts 2-byte units); even
  const float scale = (p.sa ? *p.sa : 1.f) * (p.sb ? *p.sb : 1.f);

  f32x4v acc[2][8][4];
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
  kk_offsets<false>(va, p.lda, 0, wave, lane);
  kk_offsets<false>(vb, p.ldb, 0, wave, lane);
  const int arow = wm * 128, bcolw = wn * 128;
  const Rd4<true> ra = rd4_setup<true>(sbase, arow, lane);
  const Rd4<true> rb = rd4_setup<true>(sbase + B_OFF, bcolw, lane);
  const unsigned wdst = __builtin_amdgcn_readfirstlane(sbase + wave * 1024);

  // stream state as v7: bases of the current tile (c*) and of this workgroup's next tile (n*, live if nlive)
  const unsigned a_end = (unsigned)(size_t)p.a_end, b_end = (unsigned)(size_t)p.b_end;
  auto a_base = [&](int tm) { return (u64)(size_t)(p.A + (long)tm * BM * p.lda); };
  auto b_base = [&](int tn) { return (u64)(size_t)(p.B + (long)tn * BN * p.ldb); };
  int ctm, ctn;
  tile_of(p, TSK ? whole + slot / p.ksplit : slot, ctm, ctn);
  const u64 koff = TSK ? (u64)(unsigned)((slot % p.ksplit) * nt) << 7 : 0;   // the slice's first K-tile
  u64 ca = a_base(ctm) + koff, cb = b_base(ctn) + koff, na = ca, nb = cb;
  bool nlive = false;
  auto set_next = [&](int u) {
    nlive = u + 1 < ntile;
    if (nlive) {
      int tm, tn;
      tile_of(p, slot + (u + 1) * G, tm, tn);
      na = a_base(tm);
      nb = b_base(tn);
    }
  };
  set_next(0);
  // descriptors of stream K-tile kk (0 <= kk < nt + 2; kk >= nt: the next tile's K-tile kk - nt)
  auto desc = [&](int kk, u64 cur, u64 nxt, unsigned end) {
    const bool nx = kk >= nt;
    const int kt = nx ? kk - nt : kk;
    const u64 b = (nx ? nxt : cur) + ((unsigned)kt << 7);
    const bool live = !nx || nlive;
    return i32x4{(int)(unsigned)b, (int)(unsigned)(b >> 32), live ? (int)(end - (unsigned)b) : 0, 0x00020000};
  };

  bf16x8 ax[2][8], ay[2][8];  // A row blocks (chunk g / 4 + g of the K-row), one set per stage
  bf16x8 bx[9], by[9];        // B column blocks: j < 7 shared by the stages, j = 7 at 7 + stage

  // prologue: K-tiles 0 and 1 of the first tile in flight, wait for K-tile 0 (everyone's), read all of it
  {
    const i32x4 sa0 = desc(0, ca, na, a_end), sb0 = desc(0, cb, nb, b_end);
    sfor<8>([&](auto J) { dma_only<piece_dst<true, 0, decltype(J)::value>()>(wdst, vb[decltype(J)::value], sb0); });
    sfor<8>([&](auto J) { dma_only<piece_dst<false, 0, decltype(J)::value>()>(wdst, va[decltype(J)::value], sa0); });
    const i32x4 sa1 = desc(1, ca, na, a_end), sb1 = desc(1, cb, nb, b_end);
    sfor<8>([&](auto J) { dma_only<piece_dst<true, 1, decltype(J)::value>()>(wdst, vb[decltype(J)::value], sb1); });
    sfor<8>([&](auto J) { dma_only<piece_dst<false, 1, decltype(J)::value>()>(wdst, va[decltype(J)::value], sa1); });
  }
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  sfor<8>([&](auto U) {
    constexpr int u = decltype(U)::value;
    ax[0][u] = frag4<true, u, 0, 0>(ra);
    ay[0][u] = frag4<true, u, 1, 0>(ra);
    bx[u] = frag4<true, u, 0, 0>(rb);
    by[u] = frag4<true, u, 1, 0>(rb);
  });

  auto ktile = [&](auto ST, int k) {
    constexpr int st = decltype(ST)::value, nx = st ^ 1;
    i32x4 sa, sb;
    sfor<64>([&](auto Q) {
      constexpr int n = decltype(Q)::value;
      constexpr int j = n >> 3, i = n & 7;
      if constexpr (LATE) {
        if constexpr (n == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (n == 14) {
          constexpr int inflight = f8_pieces_before<SCHED>(14);
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(inflight) : "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (n == 14) bx[7 + nx] = frag4<true, 7, 0, nx>(rb);
        if constexpr (n == 15) by[7 + nx] = frag4<true, 7, 1, nx>(rb);
        if constexpr (n >= 16 && n <= 31) {
          constexpr int r = n - 16, u = r >> 1;
          if constexpr (r & 1)
            ay[nx][u] = frag4<true, u, 1, nx>(ra);
          else
            ax[nx][u] = frag4<true, u, 0, nx>(ra);
        }
        constexpr int bj = (n >= 32 && n <= 41) ? (n - 32) >> 1 : (n == 48 || n == 49) ? 5 : (n == 56 || n == 57) ? 6 : -1;
        if constexpr (bj >= 0) {
          if constexpr ((n & 1) == 0)
            bx[bj < 0 ? 0 : bj] = frag4<true, (bj < 0 ? 0 : bj), 0, nx>(rb);
          else
            by[bj < 0 ? 0 : bj] = frag4<true, (bj < 0 ? 0 : bj), 1, nx>(rb);
        }
      }
      if constexpr (!LATE && n == 0) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- tile t+1's fragments (stage nx)
      if constexpr (!LATE && n >= 2 && n <= 32 && n % 2 == 0) {
        constexpr int r = (n - 2) / 2, u = r >> 1;
        if constexpr (r & 1)
          ay[nx][u] = frag4<true, u, 1, nx>(ra);
        else
          ax[nx][u] = frag4<true, u, 0, nx>(ra);
      }
      if constexpr (!LATE && n >= 8 && n <= 57 && (n % 8) < 2) {
        constexpr int jb = n / 8 - 1;
        if constexpr (n % 8 == 0)
          bx[jb] = frag4<true, jb, 0, nx>(rb);
        else
          by[jb] = frag4<true, jb, 1, nx>(rb);
      }
      if constexpr (!LATE && n == 36) bx[7 + nx] = frag4<true, 7, 0, nx>(rb);
      if constexpr (!LATE && n == 37) by[7 + nx] = frag4<true, 7, 1, nx>(rb);
      // ---- MFMA n, with piece n - 1 of tile t+2 behind it for n = 1..16 (A pieces, then B)
      constexpr int jj = j < 7 ? j : 7 + st;
      f32x4v& c = acc[j >> 2][i][j & 3];
      const i32x8 fb = pair(bx[jj], by[jj]), fa = pair(ax[st][i], ay[st][i]);
      constexpr int pa = f8_piece_a<SCHED>(n), pb = f8_piece_b<SCHED>(n);
      if constexpr (pa >= 0) {
        mfma8_dma<piece_dst<false, st, (pa & 7)>(), FB, FA>(c, fb, fa, wdst, va[pa & 7], sa);
      } else if constexpr (pb >= 0) {
        mfma8_dma<piece_dst<true, st, (pb & 7)>(), FB, FA>(c, fb, fa, wdst, vb[pb & 7], sb);
      } else {
        mfma8<FB, FA>(c, fb, fa);
      }
      // ---- behind MFMA 0: tile t+2's descriptors (SALU beside the MFMA; kk opaque so it is not hoisted)
      if constexpr (n == 0) {
        int kk = k + 2;
        asm volatile("" : "+s"(kk));
        sa = desc(kk, ca, na, a_end);
        sb = desc(kk, cb, nb, b_end);
        asm volatile("" : "+s"(sa), "+s"(sb));
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  for (int u = 0; u < ntile; ++u) {
    zero_acc();
    for (int k = 0; k < nt; k += 2) {
      ktile(std::integral_constant<int, 0>{}, k);
      ktile(std::integral_constant<int, 1>{}, k + 1);
    }
    // MFMA -> accumulator-read wait states of the last (16-pass) MFMAs, then dequantise and store
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] *= scale;
    if constexpr (TSK) {
      sfor<2>([&](auto H) {
        constexpr int h = decltype(H)::value;
        store_partial(p.part + (long)slot * (BM * BN), acc[h], arow, bcolw + 64 * h, lane);
      });
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (EPI == kEpiBF16) {
          if ((ctm + 1) * BM <= p.M && (ctn + 1) * BN <= p.N && (p.ldc & 7) == 0 && ((size_t)p.C & 15) == 0)
            epilogue_v7_x4<false>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
          else
            epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        } else {
          epilogue_t<EPI>(p, acc[h], ctm, ctn, arow, bcolw + 64 * h, lane);
        }
      }
    }
    if (u + 1 < ntile) {
      tile_of(p, slot + (u + 1) * G, ctm, ctn);
      ca = na;
      cb = nb;
      set_next(u + 1);
    }
  }
  // the dead prefetches past the last tile (num_records 0) must land before the workgroup's LDS goes away
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace gm
}  // namespace pd

// C[M, N] = (A[M, K] . B[N, K]^T) * (*sa) * (*sb) (+ bias[N]), A / B fp8 (fa / fb: 0 e4m3, 1 e5m2) with row
// strides lda / ldb in bytes; epi 0: bf16 C (+ bias), 1: fp32 C (+ beta * C).  Returns -1 outside the kernel's
// domain (K % 256, 16-B rows, operand extents >= 2 GiB, unsupported format pair): the caller takes another path.
extern "C" int pd_gemm_f8(int fa, int fb, int epi, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                          const void* bias, const float* sa, const float* sb, int M, int N, int K, float beta,
                          int group_m, int cus, void* ws, long ws_bytes, void* stream) {
  using namespace pd::gm;
  if (M <= 0 || N <= 0 || K <= 0 || K % 256 || lda % 16 || ldb % 16 || lda < K || ldb < K) return -1;
  if ((size_t)A % 16 || (size_t)B % 16 || (size_t)C % 16 || ldc % 4 || ldc < N) return -1;
  const long a_bytes = (long)(M - 1) * lda + K, b_bytes = (long)(N - 1) * ldb + K;
  if (a_bytes >= 0x7fffffffL || b_bytes >= 0x7fffffffL) return -1;
  if (epi != kEpiBF16 && epi != kEpiF32) return -1;
  Params p;
  p.A = (const unsigned short*)A;
  p.B = (const unsigned short*)B;
  p.C = C;
  p.C2 = nullptr;
  p.bias = epi == kEpiBF16 ? (const unsigned short*)bias : nullptr;
  p.lda = lda / 2; p.ldb = ldb / 2; p.ldc = ldc; p.ldc2 = 0;
  p.M = M; p.N = N; p.K = K / 2; p.beta = beta; p.H = 0;
  p.zero = nullptr;
  p.goff = nullptr; p.ngroups = 0; p.gmode = 0; p.gsb = p.gsc = p.gsbias = 0;
  p.part = nullptr; p.ksplit = 1; p.kchunk = 0; p.tail_cap = 0; p.cpx = cus / 8;
  p.a_end = (const char*)A + a_bytes;
  p.b_end = (const char*)B + b_bytes;
  p.sa = sa; p.sb = sb;
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + BN - 1) / BN;
  p.group_m = group_m > 0 ? group_m : 4;
  hipStream_t st = (hipStream_t)stream;
  const int nwg = p.tiles_m * p.tiles_n;
  const int ks = ws ? tail_plan(nwg, cus, p.K / BK, ws_bytes) : 0;
  const int R = ks ? nwg % cus : 0;
  if (ks) {
    p.part = (float*)ws; p.ksplit = ks; p.tail_cap = R;
  }
  const dim3 grid(std::min(nwg - R, cus)), tgrid(R * ks), rgrid(BM * BN / 1024, R);
  // K-tile schedule: PADDLE2_AMD_FP8_SCHED (0 = one barrier per K-tile, 1 = the late-wait schedule, 2 = late wait +
  // spread pieces, the default: +9-19% over 0 at the GPT-3 13B shapes, profiles/r5_fp8_schedules.md), read per call
  const char* se = getenv("PADDLE2_AMD_FP8_SCHED");
  const int sched = se ? atoi(se) : 2;
#define PD_F8(FA_, FB_, E_)                                                                   \
  if (nwg > R) {                                                                              \
    if (sched == 1) gemm_f8_kernel<FA_, FB_, E_, false, 1><<<grid, NTHR4, 0, st>>>(p);       \
    else if (sched == 2) gemm_f8_kernel<FA_, FB_, E_, false, 2><<<grid, NTHR4, 0, st>>>(p);  \
    else gemm_f8_kernel<FA_, FB_, E_><<<grid, NTHR4, 0, st>>>(p);                             \
  }                                                                                           \
  if (ks) {                                                                                   \
    if (sched == 1) gemm_f8_kernel<FA_, FB_, E_, true, 1><<<tgrid, NTHR4, 0, st>>>(p);       \
    else if (sched == 2) gemm_f8_kernel<FA_, FB_, E_, true, 2><<<tgrid, NTHR4, 0, st>>>(p);  \
    else gemm_f8_kernel<FA_, FB_, E_, true><<<tgrid, NTHR4, 0, st>>>(p);                      \
    tail_reduce_kernel<E_><<<rgrid, 256, 0, st>>>(p, nwg - R);                               \
  }
  switch (fa * 100 + fb * 10 + epi) {
    case 0: PD_F8(0, 0, kEpiBF16) break;    // forward
    case 100: PD_F8(1, 0, kEpiBF16) break;  // dgrad
    case 10: PD_F8(0, 1, kEpiBF16) break;   // wgrad, bf16 dW
    case 11: PD_F8(0, 1, kEpiF32) break;    // wgrad, fp32 dW
    default: return -1;
  }
#undef PD_F8
  return (int)hipGetLastError();
}
