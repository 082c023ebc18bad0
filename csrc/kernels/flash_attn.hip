// Flash attention forward + backward on CDNA4 MFMA (gfx950), bf16 or fp16 in / fp32 accumulate,
// head dims 64 / 128 / 256 (other D <= 256 are zero-padded to the next one by the host wrapper).
//
// Reference behaviour: phi/kernels/gpu/flash_attn_kernel.cu / flash_attn_grad_kernel.cu
// (q/k/v [b, s, nh, hd], causal, GQA via num_heads_k, returns softmax_lse [b, nh, s]).  The
// reference dlopens an external flash-attn fork; this is a from-scratch CDNA4 design:
//
// Forward (per workgroup: 4 waves x 32 query rows = 128 rows of one (b, head)):
//  * swapped product S^T = K . Q^T with v_mfma_f32_32x32x16_bf16 so each lane owns ONE query
//    row's scores (16 keys per lane-half): the softmax row max/sum is 16 in-register ops plus
//    one lane^32 exchange — no LDS round trip for P;
//  * the S^T accumulator feeds the P.V product directly as the MFMA B operand (guide §3
//    "accumulator tile as the next MFMA's operand"), with V^T fragments read by
//    ds_read_b64_tr_b16 (T10) from a row-major V tile;
//  * K/V tiles (64 keys) are register-staged global->LDS with the issue-early/write-late split
//    (T14), double-buffered, one barrier per tile; every LDS image uses the dual-use XOR swizzle
//    off = 256*row + 16*(ch ^ ((row&3)<<2 | (row>>2)&3)) so both ds_read_b128 row reads and
//    ds_read_b64_tr_b16 column reads are conflict-free (T10 (b));
//  * O^T accumulators are per-lane (lane = query) so the online-softmax rescale is a scalar
//    multiply; exp2 with the 1/sqrt(d)*log2(e) scale folded into one multiply;
//  * 1-D grid with an XCD-aware bijective remap (T1): all query blocks of a KV head land on one
//    XCD so K/V are served from that XCD's L2; causal grids start with the heaviest blocks.
//
// Backward (per workgroup: 8 waves x 32 keys = 256 keys of one (b, kv-head); two waves per SIMD so
// one wave's LDS/VALU phases hide under the other's MFMAs):
//  * key on the lane: S = Q.K^T and dP = dO.V^T have the key as the accumulator column, so
//    P and dS are directly the B operands of dV^T += dO^T.P and dK^T += Q^T.dS (tr-reads of the
//    Q / dO tiles give the A operands); V fragments stay in VGPRs for the whole sweep, K is read
//    from its one LDS image both by rows (S) and by columns (dQ), keeping the wave under 256 VGPRs;
//  * the workgroup sweeps every query head of its GQA group x every 32-row query tile, so dK/dV
//    are complete in registers and written once (no cross-workgroup sum for dK/dV);
//  * dS goes through LDS once for dQ = dS.K (4 waves split D).  Dense mode (default): every key block
//    adds its dQ tile into ONE zeroed fp32 slab with buffer fp32 atomics (fa_dq_atomic; the slab is then
//    converted by dq_reduce_kernel) — at B8 S4096 the per-key-block slabs cost more HBM than the atomics;
//    deterministic mode (FLAGS_cudnn_deterministic / PADDLE2_AMD_FA_DQ_ATOMIC=0) and the varlen / FlashMask
//    modes write per-key-block slabs with plain stores, summed in a fixed order by dq_reduce_kernel
//    (bitwise reproducible);
//  * the next (head, q-tile) step's Q / dO / lse / delta are prefetched into registers while the
//    current step computes (T14 issue-early / write-late).
#include "common.h"

#include <algorithm>
#include <cstring>
#include <type_traits>

namespace pd {
namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kDefer = 8.f;  // fwd defer-max threshold (log2 units)
constexpr float kBig = 32.f;   // two-row-block fwd: base / running-max gap that triggers the exact second pass

__device__ __forceinline__ int swz(int row, int ch, int nch) {
  return ch ^ ((((row & 3) << 2) | ((row >> 2) & 3)) & (nch - 1));
}

// byte offset of element (row, col) (16-bit elements) in a swizzled [rows][D] tile
template <int D>
__device__ __forceinline__ int tile_off(int row, int col) {
  constexpr int NCH = D / 8;
  return row * (D * 2) + swz(row, col >> 3, NCH) * 16 + (col & 7) * 2;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not its global memory ops.
// __syncthreads() is a release fence as well, so hipcc puts s_waitcnt vmcnt(0) in front of it — every in-flight
// global load (prefetch) and store of the wave would drain at each barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}

__device__ __forceinline__ s16x4 lds_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)((lds_char*)base + off));
}

__device__ __forceinline__ bf16x8 cat4(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Operand fragments travel as 16-byte bf16x8 bit containers for both element types; F16 selects the
// fp16 conversions and the f16 MFMA (same 32x32x16 shape and operand layout, so every LDS image,
// swizzle and lane mapping below is shared).
template <bool F16>
__device__ __forceinline__ unsigned short cvt16(float f) {
  if constexpr (F16) return __builtin_bit_cast(unsigned short, (_Float16)f);
  else return f2bf(f);
}

// Pack 8 fp32 accumulator registers [8s, 8s+8) into an MFMA operand fragment.
template <bool F16>
__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int s) {
  if constexpr (F16) {
    f16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (_Float16)acc[8 * s + j];
    return __builtin_bit_cast(bf16x8, r);
  } else {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
    return r;
  }
}

template <bool F16>
__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// O^T += V^T . P^T with the accumulator pinned to AGPRs (the two-row-block forward: its 128 O registers per lane must
// live in the accumulator file, which the compiler's own allocation did not find — 270 v_accvgpr copies per tile).
// NOP: the P operand was just written by VALU (pack8); two wait states before an MFMA reads it (the hazard
// recognizer does not look inside an asm statement).
template <bool F16, bool NOP>
__device__ __forceinline__ void mfma_acc(f32x16& c, bf16x8 a, bf16x8 b) {
  if constexpr (F16) {
    if constexpr (NOP) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  } else {
    if constexpr (NOP) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
}
// wait states between the last asm MFMA writing an AGPR accumulator and a VALU / v_accvgpr read of it (16-pass XDL
// write -> VALU read: 18)
__device__ __forceinline__ void mfma_acc_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

// XCD-aware bijective remap of a 1-D block id (cdna guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int q = n / 8, r = n % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Sequence-layout / mask extensions (template MODE):
//   kDense   - q/k/v [B, S, H, D], lse [B, H, Sq]
//   kVarlen  - packed q/k/v [total, H, D] with cumulative offsets cu_q/cu_k [B+1] (flash_attn_unpadded,
//              reference flash_attn_kernel.cu FlashAttnUnpaddedKernel); lse [H, total_q]; bottom-right causal
//              alignment per sequence
//   kMask    - FlashMask (reference flash_attn_kernel.cu:445-494 startend_row_indices): per key column two row
//              intervals [a1, b1) U [a2, b2) are masked (host normalises LTS/LTE/UTS/UTE to this form).  A host
//              plan classifies every (query block x key tile) product as unmasked / partial / fully masked from
//              per-tile min/max summaries, so fully masked products are never visited (not even scanned), and
//              element masks run only on partial ones
enum Mode : int { kDense = 0, kVarlen = 1, kMask = 2 };
struct Ext {
  const int* cu_q;      // kVarlen
  const int* cu_k;
  int total_q;
  const int4* fm;       // kMask: [B, Hm, Sk] (a1, b1, a2, b2)
  const int* fm_t64;    // kMask fwd plan: [B*Hm, ceil(Sq/128), 2 + ceil(Sk/64)] = first tile, end tile, class/tile
  const int* fm_t256;   // kMask bwd plan: [B*Hm, ceil(Sq/32), ceil(Sk/256)] class per (32-row q tile, key block)
  int fm_hm;            // mask heads: 1 or Hq
  unsigned drop_seed;   // DROP: per-call seed (Paddle's seed/offset pair folded on the host)
  unsigned drop_thresh; // DROP: element dropped iff hash < p * 2^32
  float drop_rscale;    // DROP: 1 / (1 - p)
  int dq_atomic;        // dense bwd: dQ partials fp32-atomically added into ONE zeroed slab (pslab = 0)
  int wave_skip;        // fwd, causal: a wave skips the key tiles that lie wholly above its last row
  // dense bwd, D = 128: q / k were rotate-half RoPE'd in the producing GEMM's epilogue; dK (bwd epilogue) and dQ
  // (dq_reduce) leave as RoPE^T of their gradients, i.e. gradients of the PRE-rotation q / k.  fp32 [S, 128]
  // tables (first 64 columns used), position = token index within its sequence.
  const float* rope_cos;
  const float* rope_sin;
  // split-dQ mode (dense): the backward stores dS (bf16, unscaled) per (q tile, key block) into this compact
  // buffer instead of running the dQ phase; dq_gemm_kernel then computes dQ = scale * dS . K.  Layout per
  // (b, hq): key block kb owns tiles t >= tb(kb) (tb = q_begin / 32), one [BNK/32 key slices][32 q][32 keys] block
  // each (slice w = wave w's keys, written as 2 KB contiguous), key blocks in order:
  // elem = (b*Hq + hq) * ds_per_bh + base(kb) + (t - tb(kb)) * 32 * BNK + (key / 32) * 1024 + [fragment order:
  // ((key % 32) / 16) * 512 + ((key / 8) & 1) * 256 + row * 8 + key % 8]
  bf16* ds_out;
  long ds_per_bh;
  int pair_order;       // bwd: dispatch a (b, kv head) pair's key blocks together on one XCD (needs Hk*B % 8 == 0)
  // bwd, 8 waves (PADDLE2_AMD_FA_BWD_OPT): bit 0 = waves 4-7 at s_setprio 1 (the second-dispatched half loses every
  // arbitration otherwise, MI355X_MICROARCH "Two waves per SIMD" item 4); bit 1 = the dQ slices run on waves 4-7
  // instead of 0-3 (the half that finishes its S / dP / dV / dK MFMAs later takes the dQ tail)
  int bwd_opt;
};

// Counter-based dropout mask: a stateless 32-bit hash of (seed, batch*head, query, key), so the backward
// regenerates exactly the forward's mask with no stored bitmask (the reference uses Philox seed/offset,
// flash_attn_kernel.cu; the stream differs but the contract -- same (seed, offset) => same mask -- holds)
__device__ __forceinline__ bool drop_keep(const Ext& ex, unsigned bh, unsigned q, unsigned k) {
  unsigned x = ex.drop_seed ^ (bh * 0x27D4EB2Du);
  x += q * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x += k * 0xC2B2AE3Du;
  x ^= x >> 13;
  x *= 0x27D4EB2Fu;
  x ^= x >> 16;
  return x >= ex.drop_thresh;
}

// plan classes: 0 = unmasked, 1 = partial, 2 = fully masked

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// raw buffer resource over [p, p + bytes): out-of-range offsets read 0 / drop stores (gfx9 dword3)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes > 0 ? bytes : 0, 0x00020000);
}
// the same for a base / extent the compiler cannot PROVE wave-uniform although it is (derived from loop state that
// lives in VGPRs): the inputs go through readfirstlane, so the descriptor sits in SGPRs and each buffer op is one
// instruction — otherwise hipcc wraps every op in a waterfall loop (cdna_hip_programming.md T20; the dQ atomics of
// the backward were 32 such loops per step)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes > 0 ? bytes : 0);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, n, 0x00020000);
}
__device__ __forceinline__ bool fm_masked(int4 m, int row) {
  return (row >= m.x && row < m.y) || (row >= m.z && row < m.w);
}

// Transposed-read address for the A operand V^T / dO^T / Q^T / K^T-column fragments:
// 32x16 operand whose row = column `c0 + (lane&31)` of a row-major tile, k rows = `r0 + k`.
// PERM selects the permuted k order required when the B operand is an accumulator tile.
template <int D, bool PERM>
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int r0, int c0, int lane) {
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int h = g >> 1;
  const int col = c0 + ((g & 1) << 4) + 4 * pp;
  int ra, rb;
  if (PERM) { ra = r0 + 4 * h + qq; rb = ra + 8; }       // keys 16s + 8(j>>2) + 4h + (j&3)
  else { ra = r0 + 8 * h + qq; rb = ra + 4; }            // natural k = 8h + j
  return cat4(lds_tr(tile, tile_off<D>(ra, col)), lds_tr(tile, tile_off<D>(rb, col)));
}

// =====================================================================================
//                                       FORWARD
// =====================================================================================
// NW waves x 32 query rows per workgroup: NW = 4 (two workgroups per CU for D <= 128) or NW = 8 (one 512-thread
// workgroup per CU: every K/V tile is staged once for 256 query rows, half the global->LDS traffic and staging VALU
// per MFMA; causal tiles above a wave's last row are skipped by that wave).  NW = 8 excludes FlashMask (its plans
// are built for 128-row query blocks).
// RB = 2 (NW = 4, D = 128, dense / varlen, no dropout): every wave owns TWO 32-row query blocks (rows m0 + 32 wv and
// m0 + 128 + 32 wv of a 256-row workgroup, one workgroup per CU with the whole 512-register file): each K fragment
// (ds_read_b128) and each V^T fragment (2 x ds_read_b64_tr_b16) feeds two MFMAs instead of one, a K/V tile is staged
// once for 256 rows, and the two blocks' softmax chains are independent VALU work the scheduler can place beside
// the other block's MFMAs (one wave per SIMD: no partner wave's MFMAs compete for the matrix pipe).
template <int D, bool CAUSAL, int MODE, bool DROP, bool F16, int NW, int RB = 1>
__global__ __launch_bounds__(NW * 64, (NW == 8 || D > 128 || RB == 2 ? 1 : 2)) void fwd_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ Vv, bf16* __restrict__ O,
                                                     float* __restrict__ LSE, int B, int SqMax, int SkMax, int Hq,
                                                     int Hk, long sq, long sk, long sv, long so, float scale, Ext ex) {
  constexpr int BM = 32 * NW * RB, BN = 64, NCH = D / 8, KS = D / 16, DT = D / 32, NT = NW * 64;
  constexpr int TILE = BN * D * 2;
  constexpr int NLOAD = BN * NCH / NT;
  static_assert(NLOAD * NT == BN * NCH, "tile copy must divide over the workgroup");
  static_assert(NW == 4 || MODE != kMask, "FlashMask plans assume 128-row query blocks");
  static_assert(RB == 1 || (NW == 4 && D <= 128 && MODE != kMask && !DROP), "two row blocks: 4 waves, no mask / dropout");
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][K|V]
  __shared__ int4 fm_s[MODE == kMask ? 2 * BN : 1];              // [buf][key] FlashMask intervals
  // RB = 2: the workgroup's 256 Q rows stay in LDS (same swizzled row image as K) and are read per tile — 64 VGPRs of
  // Q fragments did not fit beside 2 x 32 score and 2 x 64 output registers per lane
  __shared__ __attribute__((aligned(16))) char qsm[RB == 2 ? BM * D * 2 : 16];

  const int nmb = (SqMax + BM - 1) / BM;
  const int total = nmb * Hq * B;
  const int w_id = xcd_remap(blockIdx.x, total);
  int mb = w_id % nmb;
  const int hq = (w_id / nmb) % Hq;
  const int b = w_id / (nmb * Hq);
  if (CAUSAL) mb = nmb - 1 - mb;  // heaviest query blocks first
  const int hk = hq / (Hq / Hk);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int m0 = mb * BM;

  // per-sequence extents: token offsets of this sequence's first q / k row and its LSE row base
  int Sq = SqMax, Sk = SkMax;
  long qt0 = (long)b * SqMax, kt0 = (long)b * SkMax;
  long lse0 = ((long)b * Hq + hq) * SqMax;
  if constexpr (MODE == kVarlen) {
    qt0 = ex.cu_q[b];
    kt0 = ex.cu_k[b];
    Sq = ex.cu_q[b + 1] - (int)qt0;
    Sk = ex.cu_k[b + 1] - (int)kt0;
    lse0 = (long)hq * ex.total_q + qt0;
    if (m0 >= Sq) return;  // whole workgroup: this sequence is shorter than max_seqlen
  }
  const int off = Sk - Sq;  // bottom-right causal alignment

  const bf16* Qb = Q + qt0 * sq + hq * D;
  const bf16* Kb = K + kt0 * sk + hk * D;
  const bf16* Vb = Vv + kt0 * sv + hk * D;
  // FlashMask: this head's per-key intervals and 64-key tile summaries
  const int4* fmk = nullptr;
  const int* plan = nullptr;
  if constexpr (MODE == kMask) {
    const long mh = (long)b * ex.fm_hm + (ex.fm_hm == 1 ? 0 : hq);
    const int nt_all = (Sk + BN - 1) / BN;
    fmk = ex.fm + mh * Sk;
    plan = ex.fm_t64 + (mh * nmb + mb) * (nt_all + 2);
  }

  // Q fragments (B operand of S^T = K.Q^T): lane holds Q[q][16ks + 8h .. +8]; row block j = rows m0 + 32 NW j + 32 wv
  int qrow[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) qrow[j] = m0 + j * 32 * NW + wv * 32 + r;
  constexpr int QF = RB == 1 ? KS : 1;
  bf16x8 qf[QF];
  if constexpr (RB == 1) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (qrow[0] < Sq) qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (long)qrow[0] * sq + ks * 16 + 8 * h);
      else qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    // settle the Q fragment loads before the loop (see bwd_kernel: keeps vmcnt(0) out of the tile loop)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(qf[ks]));
  } else {
    // Q block [BM rows][D] -> LDS image (rows past Sq read as zero through the buffer extent); the first tile's
    // barrier publishes it
    const int nq = max(0, min(Sq - m0, BM));
    const __amdgpu_buffer_rsrc_t rq = make_rsrc_u(Qb + (long)m0 * sq, nq * (int)sq * 2);
    constexpr int NQL = BM * NCH / NT;
#pragma unroll
    for (int i = 0; i < NQL; ++i) {
      const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
      const u16x8 v = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, row * (int)sq * 2 + ch * 16, 0, 0));
      *reinterpret_cast<u16x8*>(qsm + row * (D * 2) + swz(row, ch, NCH) * 16) = v;
    }
  }

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + BM + off);
  int ntiles = n_end > 0 ? (n_end + BN - 1) / BN : 0;
  int t = 0;
  if constexpr (MODE == kMask) {
    t = plan[0];                    // first / end key tile that is not fully masked
    ntiles = min(ntiles, plan[1]);
  }

  u16x8 stk[NLOAD], stv[NLOAD];
  int voff_k[NLOAD], voff_v[NLOAD];
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) {
    const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
    voff_k[i] = row * (int)sk * 2 + ch * 16;
    voff_v[i] = row * (int)sv * 2 + ch * 16;
  }
  int stm = 0;  // kMask: one int of the tile's [64 keys][4] interval image per thread
  auto gload = [&](int n0) {
    if constexpr (MODE == kMask) {
      const int key = n0 + (tid >> 2);
      stm = key < Sk ? reinterpret_cast<const int*>(fmk + key)[tid & 3] : 0;
    }
    // SRSRC buffer loads (T8): the tile base is scalar (SGPRs), each lane's byte offset is a loop-invariant
    // VGPR, and keys past Sk fall outside num_records and read as zero — no per-load 64-bit address math,
    // compare or select
    const int nrows = min(Sk - n0, BN);
    const __amdgpu_buffer_rsrc_t rk = make_rsrc_u(Kb + (long)n0 * sk, nrows * (int)sk * 2);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc_u(Vb + (long)n0 * sv, nrows * (int)sv * 2);
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) {
      stk[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, voff_k[i], 0, 0));
      stv[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, voff_v[i], 0, 0));
    }
  };
  auto lstore = [&](int buf) {
    char* kt = smem + buf * 2 * TILE;
    char* vt = kt + TILE;
    if constexpr (MODE == kMask) reinterpret_cast<int*>(fm_s + buf * BN)[tid] = stm;
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) {
      const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
      const int o = row * (D * 2) + swz(row, ch, NCH) * 16;
      *reinterpret_cast<u16x8*>(kt + o) = stk[i];
      *reinterpret_cast<u16x8*>(vt + o) = stv[i];
    }
  };

  f32x16 oacc[RB][DT];
#pragma unroll
  for (int j = 0; j < RB; ++j)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      oacc[j][dt] = f32x16{};
      if constexpr (RB == 2) asm volatile("" : "+a"(oacc[j][dt]));
    }
  if constexpr (RB == 2) asm volatile("s_nop 4" ::: "memory");
  float m_i[RB], l_i[RB];
  // RB = 2: no O rescale inside the loop (a VALU multiply of the AGPR-pinned accumulators made hipcc home them in
  // VGPRs and copy 128 registers per tile).  m_i is the exponent base, set once at the row's first finite tile (O and l
  // are still zero there, so no rescale is needed); m_run tracks the true running max.  A row whose max later climbs
  // more than kBig above its base (P > 2^kBig; the bases are otherwise exact, P only ranges wider than with kDefer)
  // flags the workgroup, which then repeats the sweep with every base fixed at the row's final maximum (pass 1: no
  // growth possible) — a rare second pass in place of a per-tile rescale path.
  float m_run[RB];
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    m_i[j] = -INFINITY;
    l_i[j] = 0.f;
    m_run[j] = -INFINITY;
  }
  const float sl2 = scale * kLog2e;

  // next key tile >= t that is not fully masked (FlashMask); identity otherwise
  auto next_tile = [&](int t) {
    if constexpr (MODE == kMask) {
      while (t < ntiles && plan[2 + t] == 2) ++t;
    }
    return t;
  };
  const int t_first = t;
  __shared__ int wg_ovf;
  if constexpr (RB == 2) {
    if (tid == 0) wg_ovf = 0;
  }
  if (t < ntiles) {
    gload(t * BN);
    lstore(0);
  }
  __syncthreads();
  // static priority for the second-dispatched half of an 8-wave workgroup (MI355X_MICROARCH "Two waves per SIMD"
  // item 4): it is the arbitration loser on every segment otherwise
  if constexpr (NW == 8) {
    if (wv >= 4) __builtin_amdgcn_s_setprio(1);
  }
  // causal: the last key this wave's rows (its last row block) can see; tiles past it are all masked for the wave
  const int wave_last_key = m0 + (RB - 1) * 32 * NW + wv * 32 + 31 + off;

  // Per-lane LDS read bases (D <= 128; cdna guide T20-style address hygiene): every K row read and V^T transposed
  // read is one precomputed lane base + a compile-time immediate (buffer / key sub-block / 16-row step), so the tile
  // body carries no per-read swizzle arithmetic.
  //  K row read (key row kb*32 + r, 16-B chunk 2ks + h): chunk ^ m(r) = (2ks) ^ (h ^ m(r)) -> o_k ^ (ks << 5)
  //  V^T tr read (rows r0 + 4hh + qq (+8), 16-B chunk 4dt + cbits): -> o_va / o_vb ^ (dt << 6)
  constexpr bool PRE = D <= 128;
  int o_k = 0, o_va = 0, o_vb = 0;   // three lane bases; one v_xor per read (all-precomputed spilled: 256 VGPRs)
  if constexpr (PRE) {
    auto mm = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
    o_k = r * (D * 2) + (((h ^ mm(r)) & (NCH - 1)) << 4);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, hh = g >> 1;
    const int cbits = ((g & 1) << 1) | (pp >> 1);
    const int ra = 4 * hh + qq, rb = ra + 8;
    o_va = ra * (D * 2) + (((cbits ^ mm(ra)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
    o_vb = rb * (D * 2) + (((cbits ^ mm(rb)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  }

  // One key tile.  MASKED (compile time): the boundary / causal-diagonal / FlashMask-partial tiles run the element
  // masks; every other tile runs a body with no mask code at all (a runtime branch inside one body was if-converted
  // by hipcc: ~100 compares / selects per tile on every tile).  BUF: the LDS stage (a compile-time stage doubled the
  // bodies and spilled 264 B/lane).
  auto tile = [&](auto MASKED_, int BUF, int n0, bool has_next, int tn, bool rt_mask) {
    constexpr bool MASKED = decltype(MASKED_)::value;
    const char* kt = smem + BUF * 2 * TILE;
    const char* vt = kt + TILE;
    // opaque per tile: the XOR-ed read offsets are recomputed (1 VALU each) instead of hoisted out of the loop as
    // ~50 live registers (which spilled)
    if constexpr (PRE) asm volatile("" : "+v"(o_k), "+v"(o_va), "+v"(o_vb));
    // ---- S^T = K . Q^T for two 32-key sub-blocks (each K fragment feeds every row block)
    f32x16 s[RB][2];
    if constexpr (RB == 1) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        s[0][kb] = f32x16{};
        const int krow = kb * 32 + r;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          bf16x8 a;
          if constexpr (PRE) a = lds_b128(kt + kb * 32 * (D * 2), o_k ^ (ks << 5));
          else a = lds_b128(kt, krow * (D * 2) + swz(krow, 2 * ks + h, NCH) * 16);
          s[0][kb] = mfma<F16>(a, qf[ks], s[0][kb]);
        }
      }
    } else {
      // ks outer: per step one fragment read per row block (Q) and per key sub-block (K), four MFMAs
#pragma unroll
      for (int j = 0; j < RB; ++j) s[j][0] = s[j][1] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 bq[RB], a[2];
#pragma unroll
        for (int j = 0; j < RB; ++j) bq[j] = lds_b128(qsm + (j * 32 * NW + wv * 32) * (D * 2), o_k ^ (ks << 5));
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) a[kb] = lds_b128(kt + kb * 32 * (D * 2), o_k ^ (ks << 5));
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int j = 0; j < RB; ++j) s[j][kb] = mfma<F16>(a[kb], bq[j], s[j][kb]);
      }
    }
    // next tile's K/V loads issue after QK^T (T14): softmax + PV cover their flight, lstore waits at the end
    if (has_next) gload(tn * BN);
    // ---- mask, online softmax (lane owns query qrow; 32 of the 64 keys).  The max is taken on raw scores and the
    // 1/sqrt(d)*log2(e) scale is folded into one FMA feeding v_exp_f32.
    auto apply_mask = [&]() {
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        // key = n0 + 4h + c with the compile-time c = 32kb + (i&3) + 8(i>>2): masked iff c >= lim (key >= Sk, or
        // key > qrow + off when causal) — one compare against an immediate per score, nothing hoisted per lane
        int lim = Sk - n0 - 4 * h;
        if constexpr (CAUSAL) lim = min(lim, qrow[j] + off - n0 - 4 * h + 1);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = kb * 32 + (i & 3) + 8 * (i >> 2);
            s[j][kb][i] = c >= lim ? -INFINITY : s[j][kb][i];
          }
        }
      }
      if constexpr (MODE == kMask) {
        if (plan[2 + n0 / BN] == 1) {
          // 4 consecutive keys per group from the LDS image; the sched barrier keeps only one group's
          // intervals live (the D=128 accumulators leave no room for all 32)
          const int4* fmt_s = fm_s + BUF * BN;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                const int4 m = fmt_s[kb * 32 + 8 * g + 4 * h + jj];
                s[0][kb][4 * g + jj] = fm_masked(m, qrow[0]) ? -INFINITY : s[0][kb][4 * g + jj];
              }
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      }
    };
    if constexpr (MASKED) apply_mask();
    else if constexpr (RB == 2) {
      // one body for both tile kinds with two row blocks (two bodies made the register allocator disagree on
      // the loop-carried accumulators' homes at the join: 600 B/lane of spills); a real branch, not if-converted
      if (rt_mask) {
        asm volatile("" ::: "memory");
        apply_mask();
      }
    }
    // row max: four independent max3 chains (one 16-deep chain was a serial latency path), then the lane-half
    // exchange by v_permlane32_swap (no LDS round trip: ds_bpermute + lgkmcnt wait)
    float m_cand[RB];
    bool grow = false;
    (void)m_cand;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      float mxa[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) mxa[i & 3] = fmaxf(mxa[i & 3], s[j][kb][i]);
      }
      float mx = fmaxf(fmaxf(mxa[0], mxa[1]), fmaxf(mxa[2], mxa[3]));
      {
        const unsigned mu = __builtin_bit_cast(unsigned, mx);
        const auto sw = __builtin_amdgcn_permlane32_swap(mu, mu, false, false);
        mx = fmaxf(__builtin_bit_cast(float, (unsigned)sw[0]), __builtin_bit_cast(float, (unsigned)sw[1]));
      }
      if constexpr (RB == 2) {
        m_run[j] = fmaxf(m_run[j], mx * sl2);
        m_i[j] = m_i[j] == -INFINITY ? m_run[j] : m_i[j];   // first finite tile: O, l still zero
        ovf = ovf || (m_run[j] > m_i[j] + kBig);
      } else {
        m_cand[j] = fmaxf(m_i[j], mx * sl2);
        grow = grow || (m_cand[j] > m_i[j] + kDefer);
      }
    }
    // defer-max (T13): the running base moves only when some row of the wave grew past it by more than
    // 2^kDefer; otherwise P <= 2^kDefer (exact in fp32 / bf16) and the l / O rescale is skipped.  The branch is
    // wave-uniform and kept a real branch (the asm statement cannot be speculated): if-converted, its DT*16
    // multiplies and copies ran on every tile.  With two row blocks one branch moves both bases (moving a base
    // that did not need it is exact: the defer is only a skip)
    if constexpr (RB == 1) {
      if (__builtin_expect(__any(grow), 0)) {
        asm volatile("" ::: "memory");
        const float alpha = __builtin_amdgcn_exp2f(m_i[0] - (m_cand[0] == -INFINITY ? 0.f : m_cand[0]));
        l_i[0] *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) oacc[0][dt] *= alpha;
        m_i[0] = m_cand[0];
      }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const float base = m_i[j] == -INFINITY ? 0.f : m_i[j];
      float lsa[4] = {0.f, 0.f, 0.f, 0.f};   // four independent add chains (a 32-deep serial chain before)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[j][kb][i], sl2, -base));
          s[j][kb][i] = p;
          lsa[i & 3] += p;
        }
      }
      l_i[j] += (lsa[0] + lsa[1]) + (lsa[2] + lsa[3]);  // per lane-half partial; halves combined at the end
    }
    if constexpr (DROP) {  // row sums keep the undropped P; only the P.V operand is masked
      const unsigned bh = (unsigned)(b * Hq + hq);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = n0 + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (!drop_keep(ex, bh, (unsigned)qrow[0], (unsigned)key)) s[0][kb][i] = 0.f;
        }
      }
    }

    // ---- O^T += V^T . P^T (each V^T fragment feeds every row block)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 pb[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) pb[j] = pack8<F16>(s[j][kb], ss);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          bf16x8 a;
          if constexpr (PRE) {
            const char* vr = vt + (kb * 32 + 16 * ss) * (D * 2);
            a = cat4(lds_tr(vr, o_va ^ (dt << 6)), lds_tr(vr, o_vb ^ (dt << 6)));
          } else {
            a = tr_frag<D, true>(vt, kb * 32 + 16 * ss, dt * 32, lane);
          }
          if constexpr (RB == 2) {
            // dt = 0: the first reads of this step's VALU-packed P fragments
            if (dt == 0) {
              mfma_acc<F16, true>(oacc[0][dt], a, pb[0]);
              mfma_acc<F16, true>(oacc[RB - 1][dt], a, pb[RB - 1]);
            } else {
              mfma_acc<F16, false>(oacc[0][dt], a, pb[0]);
              mfma_acc<F16, false>(oacc[RB - 1][dt], a, pb[RB - 1]);
            }
          } else {
            oacc[0][dt] = mfma<F16>(a, pb[0], oacc[0][dt]);
          }
        }
      }
    }
    if (has_next) lstore(BUF ^ 1);  // write late (T14)
    __syncthreads();
  };

  // RB = 2 tile, software-ordered so each row block's softmax runs beside the other block's MFMAs (one wave per SIMD
  // has no partner wave to fill the MFMA pipe while it exponentiates):
  //   QK0 | mask0? | QK1 || softmax0 | mask1? | PV0 || softmax1 | PV1
  // The rare causal / boundary masks are real (uniform) branches placed where they do not split an overlapped pair.
  auto tile2 = [&](int BUF, int n0, bool has_next, int tn, bool rt_mask) {
    const char* kt = smem + BUF * 2 * TILE;
    const char* vt = kt + TILE;
    if constexpr (PRE) asm volatile("" : "+v"(o_k), "+v"(o_va), "+v"(o_vb));
    f32x16 s0[2], s1[2];
    auto qk = [&](f32x16 (&sb)[2], int j) {
      sb[0] = sb[1] = f32x16{};
      const char* qb = qsm + (j * 32 * NW + wv * 32) * (D * 2);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 bq = lds_b128(qb, o_k ^ (ks << 5));
        const bf16x8 a0 = lds_b128(kt, o_k ^ (ks << 5));
        const bf16x8 a1 = lds_b128(kt + 32 * (D * 2), o_k ^ (ks << 5));
        sb[0] = mfma<F16>(a0, bq, sb[0]);
        sb[1] = mfma<F16>(a1, bq, sb[1]);
      }
    };
    auto mask = [&](f32x16 (&sb)[2], int j) {
      if (rt_mask) {
        asm volatile("" ::: "memory");
        int lim = Sk - n0 - 4 * h;
        if constexpr (CAUSAL) lim = min(lim, qrow[j] + off - n0 - 4 * h + 1);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = kb * 32 + (i & 3) + 8 * (i >> 2);
            sb[kb][i] = c >= lim ? -INFINITY : sb[kb][i];
          }
      }
    };
    auto softmax = [&](f32x16 (&sb)[2], int j) {
      float mxa[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) mxa[i & 3] = fmaxf(mxa[i & 3], sb[kb][i]);
      float mx = fmaxf(fmaxf(mxa[0], mxa[1]), fmaxf(mxa[2], mxa[3]));
      {
        const unsigned mu = __builtin_bit_cast(unsigned, mx);
        const auto sw = __builtin_amdgcn_permlane32_swap(mu, mu, false, false);
        mx = fmaxf(__builtin_bit_cast(float, (unsigned)sw[0]), __builtin_bit_cast(float, (unsigned)sw[1]));
      }
      m_run[j] = fmaxf(m_run[j], mx * sl2);
      m_i[j] = m_i[j] == -INFINITY ? m_run[j] : m_i[j];
      ovf = ovf || (m_run[j] > m_i[j] + kBig);
      const float base = m_i[j] == -INFINITY ? 0.f : m_i[j];
      float lsa[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pp = __builtin_amdgcn_exp2f(fmaf(sb[kb][i], sl2, -base));
          sb[kb][i] = pp;
          lsa[i & 3] += pp;
        }
      l_i[j] += (lsa[0] + lsa[1]) + (lsa[2] + lsa[3]);
    };
    auto pv = [&](f32x16 (&sb)[2], int j) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const bf16x8 pb = pack8<F16>(sb[kb], ss);
          const char* vr = vt + (kb * 32 + 16 * ss) * (D * 2);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const bf16x8 a = cat4(lds_tr(vr, o_va ^ (dt << 6)), lds_tr(vr, o_vb ^ (dt << 6)));
            if (dt == 0) mfma_acc<F16, true>(oacc[j][dt], a, pb);
            else mfma_acc<F16, false>(oacc[j][dt], a, pb);
          }
        }
    };
    qk(s0, 0);
    mask(s0, 0);
    qk(s1, 1);
    // unconditional (no branch between QK1 and softmax0): past the last tile the buffer extent is 0 and the loads
    // read zeros into a stage nobody reads
    gload(tn * BN);
    softmax(s0, 0);
    // interleave: per QK1 MFMA up to 2 LDS reads and 6 VALU of softmax0
#pragma unroll
    for (int g = 0; g < 2 * KS; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, 6, 0);
    }
    // pin P0 here: otherwise its exps are sunk past the mask1 branch into PV0's block, out of QK1's MFMA stream
    asm volatile("" : "+v"(s0[0]), "+v"(s0[1]));
    mask(s1, 1);
    softmax(s1, 1);
    pv(s0, 0);
#pragma unroll
    for (int g = 0; g < 2 * DT; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      __builtin_amdgcn_sched_group_barrier(0x402, 8, 1);
    }
    pv(s1, 1);
    lstore(BUF ^ 1);  // write late (T14)
    (void)has_next;
    __syncthreads();
  };

  using FalseT = std::integral_constant<bool, false>;
  using TrueT = std::integral_constant<bool, true>;
  for (int pass = 0;; ++pass) {
  for (int buf = 0; t < ntiles; buf ^= 1) {
    const int n0 = t * BN;
    const int tn = next_tile(t + 1);
    const bool has_next = tn < ntiles;
    if (CAUSAL && (NW == 8 || RB == 2 || ex.wave_skip) && n0 > wave_last_key) {  // wave-uniform: only stage the next tile for the others
      if (has_next) {
        gload(tn * BN);
        lstore(buf ^ 1);
      }
      __syncthreads();
      t = tn;
      continue;
    }
    bool masked = (n0 + BN > Sk) || (CAUSAL && (n0 + BN - 1 > m0 + off));
    if constexpr (MODE == kMask) masked = masked || plan[2 + t] == 1;
    if constexpr (RB == 2) tile2(buf, n0, has_next, tn, masked);
    else if (masked) tile(TrueT{}, buf, n0, has_next, tn, true);
    else tile(FalseT{}, buf, n0, has_next, tn, false);
    t = tn;
  }
  if constexpr (RB == 1) {
    break;
  } else {
    if (pass == 1) break;
    if (__any(ovf) && lane == 0) wg_ovf = 1;
    __syncthreads();
    if (__builtin_expect(wg_ovf == 0, 1)) break;
    // rare: repeat the sweep with every row's base at its final maximum (P <= 1, no growth)
    mfma_acc_drain();
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      m_i[j] = m_run[j];
      l_i[j] = 0.f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        oacc[j][dt] = f32x16{};
        asm volatile("" : "+a"(oacc[j][dt]));
      }
    }
    asm volatile("s_nop 4" ::: "memory");
    t = t_first;
    if (t < ntiles) {
      gload(t * BN);
      lstore(0);
    }
    __syncthreads();
  }
  }

  // ---- epilogue: normalise, store O and LSE.  A row's 8 consecutive d of a 32-column group sit 4 + 4 in lanes i and
  // i + 32; one v_permlane32_swap per dword pairs groups (c, c + 1) so each lane stores 16 contiguous bytes (lanes < 32
  // group c, lanes >= 32 group c + 1): 8 dwordx4 stores per row block instead of 16 dwordx2 (the store tail is
  // issue-bound: cdna guide T21).  The swaps run with every lane active, before the row-bound check.
  if constexpr (RB == 2) mfma_acc_drain();
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const float l_tot = l_i[j] + __shfl_xor(l_i[j], 32, 64);
    float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if constexpr (DROP) inv *= ex.drop_rscale;
    unsigned pk[DT][4][2];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          pk[dt][c][e] = (unsigned)cvt16<F16>(oacc[j][dt][4 * c + 2 * e] * inv) |
                         ((unsigned)cvt16<F16>(oacc[j][dt][4 * c + 2 * e + 1] * inv) << 16);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; c += 2)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(pk[dt][c][e], pk[dt][c + 1][e], false, false);
          pk[dt][c][e] = sw[0];
          pk[dt][c + 1][e] = sw[1];
        }
    if (qrow[j] < Sq) {
      char* orow = reinterpret_cast<char*>(O + (qt0 + qrow[j]) * so + hq * D) + (h ? 16 : 0);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int c = 0; c < 4; c += 2)
          *reinterpret_cast<uint4*>(orow + 64 * dt + 16 * c) =
              make_uint4(pk[dt][c][0], pk[dt][c][1], pk[dt][c + 1][0], pk[dt][c + 1][1]);
      if (h == 0) {
        LSE[lse0 + qrow[j]] = l_tot > 0.f ? (m_i[j] + log2f(l_tot)) * kLn2 : INFINITY;
      }
    }
  }
}

// =====================================================================================
//                                       BACKWARD
// =====================================================================================
// delta[b, h, q] = sum_d dO . O  (fp32).  D/8 lanes per row (16 for D = 128), so a wave covers 64*8/D rows and
// every lane moves 2 x 16 B — the one-wave-per-row form left 3/4 of the lanes idle.
template <bool F16>
__global__ __launch_bounds__(256) void bwd_delta_kernel(const bf16* __restrict__ O, const bf16* __restrict__ dO,
                                                        float* __restrict__ delta, int B, int Sq, int Hq, int D,
                                                        long so) {
  const int lpr = D / 8;                       // lanes per row (power of two: 8 or 16)
  const long rowid = (blockIdx.x * 256L + threadIdx.x) / lpr;
  const long total = (long)B * Hq * Sq;
  const int sub = threadIdx.x & (lpr - 1);
  float acc = 0.f;
  if (rowid < total) {
    const int q = (int)(rowid % Sq);
    const int hq = (int)((rowid / Sq) % Hq);
    const int b = (int)(rowid / ((long)Sq * Hq));
    const long base = ((long)b * Sq + q) * so + (long)hq * D + sub * 8;
    float a[8], c[8];
    if constexpr (F16) {
      load_vec<half16, 8>(reinterpret_cast<const half16*>(O + base), a);
      load_vec<half16, 8>(reinterpret_cast<const half16*>(dO + base), c);
    } else {
      load_vec<bf16, 8>(O + base, a);
      load_vec<bf16, 8>(dO + base, c);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * c[j];
  }
  for (int m = lpr / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if (rowid < total && sub == 0) delta[rowid] = acc;
}

// D = 256 runs 4 waves x 32 keys (128-key blocks): the dK/dV accumulators alone are 256 VGPRs per lane, so
// one wave per SIMD with the whole 512-entry register file; D <= 128 runs 8 waves (two per SIMD).
template <int D>
constexpr int bwd_waves() { return D > 128 ? 4 : 8; }

// NWB = 4 at D = 128 (dense, atomic dQ): 128-key blocks, two 256-thread workgroups per CU instead of one 512-thread
// one — the two workgroups' barriers are independent, so SIMD partners drift apart and one wave's exp / dS VALU runs
// beside the other's MFMAs instead of colliding with them; every wave takes a dQ slice (4 slices, 4 waves)
template <int D, bool CAUSAL, int MODE, bool DROP, bool F16, int NWB = bwd_waves<D>(), bool DQS = false>
__global__ __launch_bounds__(NWB * 64, (NWB == 4 && D <= 128) ? 2 : 1) void bwd_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ Vv, const bf16* __restrict__ dO,
                                                     const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                     float* __restrict__ dQP, bf16* __restrict__ dK,
                                                     bf16* __restrict__ dV, int B, int SqMax, int SkMax, int Hq,
                                                     int Hk, long sq, long sk, long sv, long so, long sdk, long sdv,
                                                     long pslab, float scale, Ext ex) {
  constexpr int NW = NWB, BNK = NW * 32, BMQ = 32, NCH = D / 8, KS = D / 16, DT = D / 32;
  constexpr int KTILE = BNK * D * 2;     // K block image: B operand of S (row reads) and of dQ (tr reads)
  constexpr int QTILE = BMQ * D * 2;     // Q / dO tile image
  constexpr int STILE = BMQ * BNK * 2;   // dS tile [32 q][256 keys]
  // small, per-step images first so every ds_* address is a lane base + a 16-bit immediate (an LDS offset
  // >= 64 KiB cost one v_add per read); the K image sits at a 256-B-aligned KOFF so XOR-ed row offsets
  // compose with its base
  constexpr int KOFF = (2 * QTILE + STILE + 2 * BMQ * 4 + 255) / 256 * 256;
  __shared__ __attribute__((aligned(16))) char smem[KOFF + KTILE];
  // deferred dQ atomics (dense atomic mode): a step's dQ tile is parked here ([slice][16][64 lanes], conflict-free
  // b32 accesses) and added at the NEXT step's head, after that step's staging wait.  CDNA counts atomics in
  // vmcnt, so atomics issued at a step's end made the next head's wait for its prefetched Q/dO (vmcnt(0)) wait
  // out the atomic round trips: 0.94 ms of the 4.63 ms layer (profiles/r3_flash_bwd_dq_ablation.md)
  __shared__ float dq_stash[MODE == kDense ? DT * 16 * 64 : 1];
  char* qimg = smem;
  char* doimg = qimg + QTILE;
  char* simg = doimg + QTILE;
  float* lse_s = reinterpret_cast<float*>(simg + STILE);
  float* del_s = lse_s + BMQ;
  char* kimg = smem + KOFF;

  // heaviest (lowest, under the causal mask) key blocks first, round-robin over the XCDs.  Ext::pair_order: the key
  // blocks of one (b, kv head) pair are dispatched together onto one XCD (pair = (bid / 8 / nkb) * 8 + bid % 8), so
  // the pair's Q / dO tiles are re-read from that XCD's L2 instead of from HBM by every key block
  int kblk = blockIdx.x / (Hk * B);
  int rest = blockIdx.x % (Hk * B);
  if (ex.pair_order) {
    const int nkb_all = gridDim.x / (Hk * B);
    const int j = blockIdx.x / 8;
    rest = (j / nkb_all) * 8 + blockIdx.x % 8;
    kblk = j % nkb_all;
  }
  const int hk = rest % Hk;
  const int b = rest / Hk;
  const int group = Hq / Hk;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // the wave's dQ slice index base (wave-uniform): wv, or with bwd_opt bit 1 and 8 waves wv ^ 4 (waves 4-7 take the
  // slices; waves 0-3 start at >= DT and skip the dQ loop)
  const int wq = (NW == 8 && (ex.bwd_opt & 2)) ? (wv ^ 4) : wv;
  if (NW == 8 && (ex.bwd_opt & 1) && wv >= 4) __builtin_amdgcn_s_setprio(1);
  const int k0 = kblk * BNK;
  int Sq = SqMax, Sk = SkMax;
  long qt0 = (long)b * SqMax, kt0 = (long)b * SkMax;
  long lse_b = (long)b * Hq * SqMax, lse_hs = SqMax;  // LSE/delta index = lse_b + hq * lse_hs + q
  if constexpr (MODE == kVarlen) {
    qt0 = ex.cu_q[b];
    kt0 = ex.cu_k[b];
    Sq = ex.cu_q[b + 1] - (int)qt0;
    Sk = ex.cu_k[b + 1] - (int)kt0;
    lse_b = qt0;
    lse_hs = ex.total_q;
    if (k0 >= Sk) return;  // whole workgroup: key block past this sequence's end
  }
  const int off = Sk - Sq;
  const int lkey = wv * 32 + r;          // key (within the block) owned by this lane's accumulator column
  const int mykey = k0 + lkey;

  const bf16* Kb = K + kt0 * sk + hk * D;
  const bf16* Vb = Vv + kt0 * sv + hk * D;

  for (int c = tid; c < BNK * NCH; c += NW * 64) {
    const int row = c / NCH, ch = c % NCH, key = k0 + row;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (key < Sk) v = *reinterpret_cast<const u16x8*>(Kb + (long)key * sk + ch * 8);
    *reinterpret_cast<u16x8*>(kimg + row * (D * 2) + swz(row, ch, NCH) * 16) = v;
  }
  bf16x8 vf[KS];  // V fragments of this lane's key stay in VGPRs (B operand of dP)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (mykey < Sk) vf[ks] = *reinterpret_cast<const bf16x8*>(Vb + (long)mykey * sv + ks * 16 + 8 * h);
    else vf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  // settle the V fragment loads here: a VMEM result still in flight at the loop header makes the compiler's
  // waitcnt pass fence the first in-loop use with vmcnt(0) — which would also drain every step's prefetch
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(vf[ks]));
  f32x16 dkacc[DT], dvacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dkacc[dt] = f32x16{}; dvacc[dt] = f32x16{}; }
  const float sl2 = scale * kLog2e;
  const float inv_scale = 1.f / scale;

  int q_begin = 0;
  if (CAUSAL) q_begin = max(0, k0 - off) / BMQ * BMQ;
  const int nqt = Sq > q_begin ? (Sq - q_begin + BMQ - 1) / BMQ : 0;
  constexpr int NL = (BMQ * NCH + NW * 64 - 1) / (NW * 64);  // 16-B chunks per thread per tile
  const int ntot = nqt * group;        // (head, q-tile) steps, head-major
  // this workgroup's dQ partial slab: plain stores, summed by dq_reduce_kernel (no atomics)
  float* dQs = dQP + (long)kblk * pslab + qt0 * Hq * D;

  // FlashMask: this lane's key intervals; 256-key block summaries per mask head
  int4 mym = int4{0, 0, 0, 0};
  const int nkb = (Sk + BNK - 1) / BNK;
  auto fm_head = [&](int hq) -> long { return (long)b * ex.fm_hm + (ex.fm_hm == 1 ? 0 : hq); };
  auto step_cls = [&](int st) -> int {  // 0 unmasked, 1 partial, 2 fully masked
    if constexpr (MODE != kMask) return 0;
    const int hq = hk * group + st / nqt;
    const int q0 = q_begin + (st % nqt) * BMQ;
    return ex.fm_t256[(fm_head(hq) * ((Sq + BMQ - 1) / BMQ) + q0 / BMQ) * nkb + kblk];
  };
  // fully masked steps are skipped; dq_reduce skips the same (q tile, key block) slabs from the plan
  auto next_step = [&](int st) {
    if constexpr (MODE == kMask) {
      while (st < ntot && step_cls(st) == 2) ++st;
    }
    return st;
  };

  // register-staged prefetch of the next (head, q-tile) step (issue early / write late, T14)
  u16x8 pq[NL], pd[NL];
  float plse = INFINITY, pdel = 0.f;
  // Q / dO tiles by SRSRC buffer loads (scalar tile base, loop-invariant lane offsets, rows past Sq read 0);
  // the row constants are loaded raw and only scaled / masked when staged into LDS, so no arithmetic
  // waits on the load inside this prefetch (that wait used to stall wave 0 — and with it the barrier)
  int voff_q[NL], voff_o[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + NW * 64 * i, row = c / NCH, ch = c % NCH;
    voff_q[i] = row * (int)sq * 2 + ch * 16;
    voff_o[i] = row * (int)so * 2 + ch * 16;
  }
  auto gload = [&](int step) {
    const int hq = hk * group + step / nqt;
    const int q0 = q_begin + (step % nqt) * BMQ;
    const int nrows = min(Sq - q0, BMQ);
    const __amdgpu_buffer_rsrc_t rq = make_rsrc_u(Q + (qt0 + q0) * sq + hq * D, nrows * (int)sq * 2);
    const __amdgpu_buffer_rsrc_t rd = make_rsrc_u(dO + (qt0 + q0) * so + hq * D, nrows * (int)so * 2);
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + NW * 64 * i;
      if (c < BMQ * NCH) {
        pq[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, voff_q[i], 0, 0));
        pd[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rd, voff_o[i], 0, 0));
      }
    }
    if (tid < BMQ) {
      const long li = lse_b + hq * lse_hs + min(q0 + tid, Sq - 1);
      plse = LSE[li];
      pdel = DELTA[li];
    }
  };
  int step = next_step(0);
  if (step < ntot) gload(step);

  // ---- per-lane LDS byte offsets.  Every operand address below is one of these bases XOR/plus a
  // compile-time constant (folded into the ds_* immediate offset where it is an add), so the loop
  // carries ~8 address VGPRs instead of ~50 hoisted per-(ks, dt) offsets (which spilled).
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, hh = g4 >> 1;
  const int cb = ((g4 & 1) << 1) | (pp >> 1);
  auto msk = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
  // row reads of Q / dO (row r) and K (row lkey): chunk (2ks + h) ^ m(row) = (h ^ m) ^ 2ks
  int o_qrow = r * (D * 2) + (((h ^ msk(r)) & (NCH - 1)) << 4);
  int o_krow = lkey * (D * 2) + (((h ^ msk(lkey)) & (NCH - 1)) << 4);
  // transposed A-operand reads (dV / dK, permuted k): rows 16ss + 4hh + qq (+8); chunk dt*4 + cb
  const int ra = 4 * hh + qq, rb = ra + 8;
  int o_trA = ra * (D * 2) + (((cb ^ msk(ra)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  int o_trB = rb * (D * 2) + (((cb ^ msk(rb)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  // transposed K^T reads for dQ (natural k): rows 16ks + 8hh + qq (+4); chunk wv*4 + cb
  const int rqa = 8 * hh + qq, rqb = rqa + 4;
  // (relative to smem: KOFF folded into the lane base, the per-ks step stays an immediate < 64 KiB)
  int o_kqA = KOFF + rqa * (D * 2) + ((((wq * 4 + cb) ^ msk(rqa)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  int o_kqB = KOFF + rqb * (D * 2) + ((((wq * 4 + cb) ^ msk(rqb)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  // dS image [32 q][BNK keys]: A-operand row reads and this lane's column writes
  constexpr int SNCH = BNK / 8;
  int o_srow = r * (BNK * 2) + (((h ^ msk(r)) & (SNCH - 1)) << 4);
  int o_scol = 4 * h * (BNK * 2) + ((((lkey >> 3) ^ h) & (SNCH - 1)) << 4) + ((lkey & 7) << 1);

  // split-dQ mode: this key block's first dS block within a (b, hq) region (sum over the earlier key blocks)
  // (a compile-time variant: as a runtime branch the two dQ paths shared one register allocation and one waitcnt
  // state at the loop head, and the split path's head waited for its own dS stores)
  static_assert(!DQS || MODE == kDense, "split dQ is a dense-mode path");
  constexpr bool ds_split = DQS;
  long ds_kb_base = 0;
  if constexpr (MODE == kDense) {
    if (ex.ds_out != nullptr) {
      const int nqt_all = (Sq + BMQ - 1) / BMQ;
      for (int k2 = 0; k2 < kblk; ++k2) {
        const int tb = CAUSAL ? max(0, k2 * BNK - off) / BMQ : 0;
        ds_kb_base += (long)max(0, nqt_all - tb) * (BMQ * BNK);
      }
    }
  }

  bf16* pend_ds = nullptr;        // split-dQ: this wave's parked dS slice goes here at the next step's head
  auto flush_ds = [&]() {
    if (pend_ds == nullptr) return;
    const char* wimg = simg + wv * (BMQ * 32 * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = lane + 64 * j;
      const u16x8 v = *reinterpret_cast<const u16x8*>(wimg + ((c ^ ((c >> 5) & 3)) << 4));
      __builtin_nontemporal_store(v, reinterpret_cast<u16x8*>(pend_ds + c * 8));
    }
    pend_ds = nullptr;
  };
  int pend_hq = -1, pend_q0 = 0;  // deferred dQ tile (wave-uniform); pend_hq < 0: none
  auto flush_dq = [&]() {
    if constexpr (MODE == kDense) {
      if (pend_hq < 0) return;
      const int hqd4 = Hq * D * 4;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc_u(dQs + (long)pend_q0 * Hq * D + (long)pend_hq * D, BMQ * hqd4);
#pragma unroll
      for (int dsl = wq; dsl < DT; dsl += NW) {
        const int vo = 4 * h * hqd4 + (dsl * 32 + r) * 4;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dq_stash[(dsl * 16 + i) * 64 + lane], rs, vo,
                                                         ((i & 3) + 8 * (i >> 2)) * hqd4, 0);
      }
      pend_hq = -1;
    }
  };
  while (step < ntot) {
    const int hq = hk * group + step / nqt;
    const int q0 = q_begin + (step % nqt) * BMQ;
    // keep the bases opaque per step so derived offsets are recomputed (1 VALU each), not hoisted
    asm volatile("" : "+v"(o_qrow), "+v"(o_krow), "+v"(o_trA), "+v"(o_trB));
    asm volatile("" : "+v"(o_kqA), "+v"(o_kqB), "+v"(o_srow), "+v"(o_scol));
    __syncthreads();  // previous step's readers are done
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + NW * 64 * i, row = c / NCH, ch = c % NCH;
      if (c < BMQ * NCH) {
        const int o = row * (D * 2) + swz(row, ch, NCH) * 16;
        *reinterpret_cast<u16x8*>(qimg + o) = pq[i];
        *reinterpret_cast<u16x8*>(doimg + o) = pd[i];
      }
    }
    if (tid < BMQ) {
      const bool ok = q0 + tid < Sq;
      lse_s[tid] = ok ? -plse * inv_scale : -INFINITY;
      del_s[tid] = ok ? -pdel : 0.f;
    }
    const int fm_cls = step_cls(step);
    if constexpr (MODE == kMask) {
      // consumed only after the S / dP MFMA chain, which hides the load
      // causal masks carry only [a1, b1) (host normalisation leaves interval 2 empty)
      if (fm_cls == 1 && mykey < Sk) {
        if (CAUSAL) {
          const int2 m2 = reinterpret_cast<const int2*>(ex.fm + fm_head(hq) * Sk + mykey)[0];
          mym = int4{m2.x, m2.y, 0, 0};
        } else {
          mym = ex.fm[fm_head(hq) * Sk + mykey];
        }
      }
    }
    __syncthreads();
    flush_ds();  // the previous step's dS slice (split-dQ; a step ahead of the next barrier's vmcnt(0) drain)
    flush_dq();  // the previous step's dQ atomics: issued after this step's staging wait, before the next prefetch
    const int step_next = next_step(step + 1);
    if (step_next < ntot) gload(step_next);  // lands while this step computes

    // S' = Q.K^T - lse/scale and dP' = dO.V^T - delta: the row constants are the accumulators'
    // initial values (loaded straight from LDS into the accumulator registers), so P = exp2(S' *
    // scale*log2e) and dS = P * dP' need no further per-element subtraction.
    f32x16 sacc, dpacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = (i & 3) + 8 * (i >> 2) + 4 * h;
      sacc[i] = lse_s[qi];
      dpacc[i] = del_s[qi];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int o = o_qrow ^ (ks << 5);
      sacc = mfma<F16>(lds_b128(qimg, o), lds_b128(kimg, o_krow ^ (ks << 5)), sacc);
      dpacc = mfma<F16>(lds_b128(doimg, o), vf[ks], dpacc);
    }
    // P = exp2(S*scale*log2e - lse*log2e), dS = P * (dP - delta).  Branch-free mask: row q0+qi is
    // masked for this lane's key iff dlim + qi < 0, dlim = q0 + off - key (causal; huge when the
    // step needs no mask), -huge for keys past Sk.
    const bool need_mask = (k0 + BNK > Sk) || (CAUSAL && (k0 + BNK - 1 > q0 + off));
    int dlim = (CAUSAL && need_mask) ? (q0 + off - mykey) : (1 << 30);
    if (mykey >= Sk) dlim = -(1 << 30);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = (i & 3) + 8 * (i >> 2) + 4 * h;
      const float p = __builtin_amdgcn_exp2f(sacc[i] * sl2);
      sacc[i] = (dlim + qi < 0) ? 0.f : p;
      if constexpr (MODE == kMask) {
        if (fm_cls == 1 && fm_masked(mym, q0 + qi)) sacc[i] = 0.f;
      }
      if constexpr (DROP) {
        // dS = P (keep * r * dP - delta), dV operand = keep * r * P; dpacc holds dP - delta, nd = -delta
        const float nd = del_s[qi];
        const bool keep = drop_keep(ex, (unsigned)(b * Hq + hq), (unsigned)(q0 + qi), (unsigned)mykey);
        dpacc[i] = sacc[i] * (keep ? fmaf(ex.drop_rscale, dpacc[i] - nd, nd) : nd);
        sacc[i] = keep ? sacc[i] * ex.drop_rscale : 0.f;
      } else {
        dpacc[i] = sacc[i] * dpacc[i];
      }
    }
    // dV^T += dO^T . P ; dK^T += Q^T . dS   (A operands by transposed reads, permuted k)
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pb = pack8<F16>(sacc, ss);
      const bf16x8 db = pack8<F16>(dpacc, ss);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int oa = (o_trA ^ (dt << 6)) + ss * 16 * (D * 2);
        const int ob = (o_trB ^ (dt << 6)) + ss * 16 * (D * 2);
        dvacc[dt] = mfma<F16>(cat4(lds_tr(doimg, oa), lds_tr(doimg, ob)), pb, dvacc[dt]);
        dkacc[dt] = mfma<F16>(cat4(lds_tr(qimg, oa), lds_tr(qimg, ob)), db, dkacc[dt]);
      }
    }
    if (MODE == kDense && ex.dq_atomic == 3) {  // ablation: no dQ phase
      step = step_next;
      continue;
    }
    if (ds_split && ex.dq_atomic == 5) {   // bench-only ablation: dS computed, never stored
      asm volatile("" ::"v"(dpacc));
      step = step_next;
      continue;
    }
    if (ds_split) {
      // split-dQ: the wave transposes its [32 q][32 keys] dS slice through a PRIVATE 2-KB LDS region (its share of
      // the dS image; no workgroup barrier); the 2 KB leave as 16-B stores at the NEXT step's head, after that
      // step's staging wait (stores count in vmcnt: issued here, they made the head's wait for the prefetched Q / dO
      // wait for them too) — no dQ MFMAs and no atomics in this kernel
      // slice layout (global = LDS up to the swizzle): MFMA-fragment order for dq_gemm_kernel's B operand — 16-B
      // unit u = (key / 16) * 64 + ((key / 8) & 1) * 32 + q holds keys 8 (u / 32) .. +8 of row q, so each of its
      // fragment loads is one contiguous 1-KB wave read; in LDS unit u sits at u ^ ((u >> 5) & 3) (the four
      // units one ds_write_b16 instruction touches land on different banks)
      char* wimg = simg + wv * (BMQ * 32 * 2);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = (i & 3) + 8 * (i >> 2) + 4 * h;
        const int u = (r >> 4) * 64 + ((r >> 3) & 1) * 32 + q;
        *reinterpret_cast<unsigned short*>(wimg + ((u ^ ((u >> 5) & 3)) << 4) + (r & 7) * 2) = cvt16<F16>(dpacc[i]);
      }
      if (ex.dq_atomic != 4)   // 4: bench-only ablation, LDS transpose without the global stores
        pend_ds = ex.ds_out + ((long)(b * Hq + hq)) * ex.ds_per_bh + ds_kb_base + (long)(step % nqt) * (BMQ * BNK) +
                  wv * (BMQ * 32);
      step = step_next;
      continue;
    }
    // dS -> LDS image [32 q][BNK keys] (bf16) for dQ: row qi = (i&3) + 8(i>>2) + 4h, column lkey
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int xc = ((((i & 3) << 2) | (((i >> 2) & 1) << 1)) << 4);
      const int ac = ((i & 3) + 8 * (i >> 2)) * (BNK * 2);
      *reinterpret_cast<unsigned short*>(simg + ((o_scol ^ xc) + ac)) = cvt16<F16>(dpacc[i]);
    }
    __syncthreads();
    // dQ[32 q][32-col slice] = dS[32 q][BNK keys] . K[BNK keys][d]; slice dsl on wave dsl % NW (one slice
    // per SIMD for D=128, so every SIMD's matrix pipe carries the same 16 MFMAs; two per wave at D=256).
    // Slice dsl's K^T chunk is (dsl*4 + cb) ^ m with m < 16: for dsl = wv + NW that is the wave's own
    // chunk + 16 (bit 4 untouched by the XOR), i.e. +256 B on the lane base
#pragma unroll
    for (int dsl = wq; dsl < DT; dsl += NW) {
      f32x16 dq = f32x16{};
      const int kq_shift = (dsl - wq) * 64;
#pragma unroll
      for (int ks = 0; ks < BNK / 16; ++ks) {
        const bf16x8 a = lds_b128(simg, o_srow ^ (ks << 5));
        const int kb16 = ks * 16 * (D * 2) + kq_shift;
        const bf16x8 bb = cat4(lds_tr(smem, o_kqA + kb16), lds_tr(smem, o_kqB + kb16));
        dq = mfma<F16>(a, bb, dq);
      }
      // accumulator: row q = (i&3)+8(i>>2)+4h, col d = wv*32 + r -> two 128-B row segments per store.
      // Full 32-row tiles: non-temporal buffer stores, the per-row offset in the scalar soffset (no VALU);
      // the tile that crosses Sq keeps the checked stores
      if (MODE == kDense && ex.dq_atomic == 2) continue;  // ablation: dQ computed, not stored
      if (MODE == kDense && ex.dq_atomic == 1 && q0 + BMQ <= Sq) {  // park for the next step's head
#pragma unroll
        for (int i = 0; i < 16; ++i) dq_stash[(dsl * 16 + i) * 64 + lane] = dq[i] * scale;
        pend_hq = hq;
        pend_q0 = q0;
        continue;
      }
      if (q0 + BMQ <= Sq) {
        const int hqd4 = Hq * D * 4;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc_u(dQs + (long)q0 * Hq * D + (long)hq * D, BMQ * hqd4);
        const int vo = 4 * h * hqd4 + (dsl * 32 + r) * 4;
        if (ex.dq_atomic) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dq[i] * scale, rs, vo, ((i & 3) + 8 * (i >> 2)) * hqd4, 0);
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dq[i] * scale), rs, vo,
                                                  ((i & 3) + 8 * (i >> 2)) * hqd4, 2);
        }
      } else {
        float* dqh = dQs + (long)hq * D + dsl * 32 + r;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (q < Sq) {
            if (ex.dq_atomic) unsafeAtomicAdd(dqh + (long)q * Hq * D, dq[i] * scale);
            else __builtin_nontemporal_store(dq[i] * scale, dqh + (long)q * Hq * D);
          }
        }
      }
    }
    step = step_next;
  }
  flush_dq();
  flush_ds();
  // write dK (scaled) and dV for this lane's key: accumulator row = d, column = key
  if (mykey < Sk) {
    bf16* dkr = dK + (kt0 + mykey) * sdk + hk * D;
    bf16* dvr = dV + (kt0 + mykey) * sdv + hk * D;
    bool rope_t = false;
    if constexpr (D == 128 && MODE == kDense) rope_t = ex.rope_cos != nullptr;
    if (rope_t) {
      // RoPE^T on dK: columns d and d + 64 of this lane's key sit in slices dt and dt + 2; each rotated pair is
      // stored at once (short live ranges: the epilogue runs with the whole dK / dV accumulator set live)
      const float* cr = ex.rope_cos + (long)mykey * 128;
      const float* sr = ex.rope_sin + (long)mykey * 128;
#pragma unroll
      for (int dt = 0; dt < DT / 2; ++dt) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int d = dt * 32 + 8 * c + 4 * h;
          const float4 cv = *reinterpret_cast<const float4*>(cr + d);
          const float4 sv = *reinterpret_cast<const float4*>(sr + d);
          const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, sn[4] = {sv.x, sv.y, sv.z, sv.w};
          unsigned short lo16[4], hi16[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = dkacc[dt][4 * c + e] * scale, hi = dkacc[dt + DT / 2][4 * c + e] * scale;
            lo16[e] = cvt16<F16>(lo * cc[e] + hi * sn[e]);
            hi16[e] = cvt16<F16>(hi * cc[e] - lo * sn[e]);
          }
          *reinterpret_cast<ushort4*>(dkr + d) = ushort4{lo16[0], lo16[1], lo16[2], lo16[3]};
          *reinterpret_cast<ushort4*>(dkr + d + D / 2) = ushort4{hi16[0], hi16[1], hi16[2], hi16[3]};
        }
      }
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int d = dt * 32 + 8 * c + 4 * h;
        ushort4 kv, vv;
        kv.x = cvt16<F16>(dkacc[dt][4 * c + 0] * scale); kv.y = cvt16<F16>(dkacc[dt][4 * c + 1] * scale);
        kv.z = cvt16<F16>(dkacc[dt][4 * c + 2] * scale); kv.w = cvt16<F16>(dkacc[dt][4 * c + 3] * scale);
        vv.x = cvt16<F16>(dvacc[dt][4 * c + 0]); vv.y = cvt16<F16>(dvacc[dt][4 * c + 1]);
        vv.z = cvt16<F16>(dvacc[dt][4 * c + 2]); vv.w = cvt16<F16>(dvacc[dt][4 * c + 3]);
        if (!rope_t) *reinterpret_cast<ushort4*>(dkr + d) = kv;
        *reinterpret_cast<ushort4*>(dvr + d) = vv;
      }
    }
  }
}

// Split-dQ second half (dense, D = 128, 256-key backward blocks): dQ = scale * dS . K from the compact dS buffer of
// the backward, summed over key blocks in registers (fp32, fixed order: bitwise reproducible, no atomics), RoPE^T
// and the bf16 store fused into the epilogue — no zeroed slab, no reduce pass.  Memory-bound on the dS read.
// Workgroup: 4 waves x 32 query rows (one 32-row dS tile per wave) of one (b, hq).  Per 64-key step the K tile is
// staged in LDS (register-staged, double-buffered, the forward's swizzled image, shared by the waves); each wave
// computes the swapped product dQ^T[d][q] += K^T[d][k] . dS^T[k][q]: K^T fragments by transposed LDS reads (natural
// k order), dS^T fragments straight from the wave's own dS rows (16 B per lane, one step ahead, buffer loads).
template <bool F16, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void dq_gemm_kernel(const bf16* __restrict__ dS, const bf16* __restrict__ K,
                                                        bf16* __restrict__ dQ, int B, int Sq, int Sk, int Hq, int Hk,
                                                        long sk, long sdq, long per_bh, float scale,
                                                        const float* __restrict__ rcos,
                                                        const float* __restrict__ rsin) {
  constexpr int D = 128, NCH = D / 8, BNK = 256, BN = 64, NT = 256, TILE = BN * D * 2;
  constexpr int NLOAD = BN * NCH / NT;   // 4 chunks of 16 B per thread per K tile
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];
  const int off = Sk - Sq;
  const int nqt_all = (Sq + 31) / 32;
  const int nmb = (Sq + 127) / 128;
  const int total = nmb * Hq * B;
  const int w_id = xcd_remap(blockIdx.x, total);
  int mb = w_id % nmb;
  const int hq = (w_id / nmb) % Hq;
  const int b = w_id / (nmb * Hq);
  if (CAUSAL) mb = nmb - 1 - mb;   // heaviest query blocks first
  const int hk = hq / (Hq / Hk);
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int t = mb * 4 + wv;       // this wave's dS tile (wave-uniform in SGPRs: scalar branches, buffer bases)
  const int nkb = (Sk + BNK - 1) / BNK;
  auto tb = [&](int kb) { return CAUSAL ? max(0, kb * BNK - off) / 32 : 0; };
  // key blocks that wrote tile tt: tb(kb) <= tt (tb is non-decreasing)
  auto nkb_of = [&](int tt) {
    int n = 0;
    for (int kb = 0; kb < nkb; ++kb)
      if (tb(kb) <= tt) n = kb + 1;
    return n;
  };
  const int my_nkb = t < nqt_all ? nkb_of(t) : 0;
  const int wg_nkb = nkb_of(min(mb * 4 + 3, nqt_all - 1));
  const int nsteps = wg_nkb * (BNK / BN);

  const bf16* Kb = K + (long)b * Sk * sk + hk * D;
  const bf16* dSb = dS + ((long)b * Hq + hq) * per_bh;

  // every load below is issued unconditionally (a dead one gets num_records 0 and reads zeros): loads under a
  // branch made the waitcnt pass merge states at the join and wait for the prefetch itself
  int voff_k[NLOAD];
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) {
    const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
    voff_k[i] = row * (int)sk * 2 + ch * 16;
  }
  auto gload = [&](int st, bool live, u16x8 (&stk)[NLOAD]) {
    const int n0 = st * BN;
    const int nrows = live ? min(Sk - n0, BN) : 0;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc_u(Kb + (long)(live ? n0 : 0) * sk, nrows * (int)sk * 2);
#pragma unroll
    for (int i = 0; i < NLOAD; ++i)
      stk[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, voff_k[i], 0, 0));
  };
  auto lstore = [&](int buf, const u16x8 (&stk)[NLOAD]) {
    char* kt = smem + buf * TILE;
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) {
      const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
      *reinterpret_cast<u16x8*>(kt + row * (D * 2) + swz(row, ch, NCH) * 16) = stk[i];
    }
  };
  // dS^T fragments of a step (two 32-key slices of the block, 4 KB contiguous, stored in fragment order by the
  // backward): k-slice ks of lane l is 16 B at ks * 1 KB + l * 16 — one contiguous 1-KB read per fragment
  int lkb = 0;
  long lbase = 0;   // load cursor: key block and its base in the (b, hq) region
  const int voff_ds = lane * 16;
  auto load_ds = [&](int st, bool live, bf16x8 (&dst)[4]) {
    const int kb = st / (BNK / BN);
    while (lkb < kb) {
      lbase += (long)max(0, nqt_all - tb(lkb)) * (32 * BNK);
      ++lkb;
    }
    const bool ok = live && kb < my_nkb;
    const bf16* p = dSb + (ok ? lbase + (long)(t - tb(kb)) * (32 * BNK) + (st % (BNK / BN)) * (BN * 32) : 0);
    const __amdgpu_buffer_rsrc_t rd = make_rsrc_u(p, ok ? BN * 32 * 2 : 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      dst[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rd, voff_ds + ks * 1024, 0, 0));
  };
  // transposed K^T reads, natural k order: rows 16 ks + 8 hh + qq (+4), 16-B chunk 4 dt + cbits
  auto mm = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, hh = g >> 1;
  const int cbits = ((g & 1) << 1) | (pp >> 1);
  const int ra = 8 * hh + qq, rb = ra + 4;
  int o_a = ra * (D * 2) + (((cbits ^ mm(ra)) & (NCH - 1)) << 4) + ((pp & 1) << 3);
  int o_b = rb * (D * 2) + (((cbits ^ mm(rb)) & (NCH - 1)) << 4) + ((pp & 1) << 3);

  f32x16 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x16{};
  // everything streams two steps ahead: K tiles in two register sets (tile st + 1 goes to LDS at the end of step st,
  // tile st + 2 is loaded during it), dS fragments in three sets (step st multiplies set st % 3 while st + 1 and
  // st + 2 are in flight) — named sets, no register copies (a copy would wait for the prefetch)
  bf16x8 dsa[4], dsb[4], dsc[4];
  u16x8 ka[NLOAD], kb2[NLOAD];
  gload(0, nsteps > 0, ka);
  gload(1, nsteps > 1, kb2);
  load_ds(0, nsteps > 0, dsa);
  load_ds(1, nsteps > 1, dsb);
  lstore(0, ka);
  lds_barrier();
  // one 64-key step: K tile st + 2 into `kn`, dS fragments of step st + 2 into `nxt2`, 16 MFMAs on `cur`
  // (accumulator-major: each K^T fragment is read one MFMA ahead), then K tile st + 1 (`k1`) into the other stage
  auto body = [&](int st, bf16x8 (&cur)[4], bf16x8 (&nxt2)[4], u16x8 (&k1)[NLOAD], u16x8 (&kn)[NLOAD]) {
    const int buf = st & 1;
    gload(st + 2, st + 2 < nsteps, kn);
    load_ds(st + 2, st + 2 < nsteps, nxt2);
    asm volatile("" : "+v"(o_a), "+v"(o_b));
    if (st / (BNK / BN) < my_nkb) {   // wave-uniform: this wave's tile was written by this key block
      const char* kt = smem + buf * TILE;
      auto rdA = [&](int dt, int ks) {
        const char* kr = kt + 16 * ks * (D * 2);
        return cat4(lds_tr(kr, o_a ^ (dt << 6)), lds_tr(kr, o_b ^ (dt << 6)));
      };
      bf16x8 af[2];
      af[0] = rdA(0, 0);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int dt = j >> 2, ks = j & 3;
        if (j < 15) af[(j + 1) & 1] = rdA((j + 1) >> 2, (j + 1) & 3);
        acc[dt] = mfma<F16>(af[j & 1], cur[ks], acc[dt]);
      }
    }
    lstore(buf ^ 1, k1);   // (dead on the last step: zeros into the idle stage)
    lds_barrier();         // the later K / dS loads stay in flight across it
  };
  // K set of step st + 1: ka for odd st + 1, kb2 for even ... (tile t lives in ka if t even, kb2 if t odd)
  for (int st = 0; st < nsteps; st += 6) {
    body(st, dsa, dsc, kb2, ka);
    if (st + 1 < nsteps) body(st + 1, dsb, dsa, ka, kb2);
    if (st + 2 < nsteps) body(st + 2, dsc, dsb, kb2, ka);
    if (st + 3 < nsteps) body(st + 3, dsa, dsc, ka, kb2);
    if (st + 4 < nsteps) body(st + 4, dsb, dsa, kb2, ka);
    if (st + 5 < nsteps) body(st + 5, dsc, dsb, ka, kb2);
  }

  // epilogue: lane = query row q, accumulator rows = d (32 dt + 8 c + 4 h + e)
  const int q = t * 32 + r;
  if (t >= nqt_all || q >= Sq) return;
  bf16* orow = dQ + ((long)b * Sq + q) * sdq + hq * D;
  if (rcos != nullptr) {
    // RoPE^T: dims d and d + 64 (slices dt and dt + 2) of this lane's row rotate back together
    const float* cr = rcos + (long)q * 128;
    const float* sr = rsin + (long)q * 128;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int d = dt * 32 + 8 * c + 4 * h;
        const float4 cv = *reinterpret_cast<const float4*>(cr + d);
        const float4 sv = *reinterpret_cast<const float4*>(sr + d);
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, sn[4] = {sv.x, sv.y, sv.z, sv.w};
        unsigned short lo16[4], hi16[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = acc[dt][4 * c + e] * scale, hi = acc[dt + 2][4 * c + e] * scale;
          lo16[e] = cvt16<F16>(lo * cc[e] + hi * sn[e]);
          hi16[e] = cvt16<F16>(hi * cc[e] - lo * sn[e]);
        }
        *reinterpret_cast<ushort4*>(orow + d) = ushort4{lo16[0], lo16[1], lo16[2], lo16[3]};
        *reinterpret_cast<ushort4*>(orow + d + 64) = ushort4{hi16[0], hi16[1], hi16[2], hi16[3]};
      }
    }
  } else {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int d = dt * 32 + 8 * c + 4 * h;
        ushort4 v;
        v.x = cvt16<F16>(acc[dt][4 * c + 0] * scale);
        v.y = cvt16<F16>(acc[dt][4 * c + 1] * scale);
        v.z = cvt16<F16>(acc[dt][4 * c + 2] * scale);
        v.w = cvt16<F16>(acc[dt][4 * c + 3] * scale);
        *reinterpret_cast<ushort4*>(orow + d) = v;
      }
    }
  }
}

// dQ[b, q, h, :] = sum over the key blocks that wrote row q of their partial slabs; bf16 out with row
// stride sdq.  Causal: key block kb wrote rows q >= qbegin(kb) = floor(max(0, kb*BNK - off) / BMQ) * BMQ.
// RoPE^T variant (dense, D = 128, Ext::rope_cos set): a thread takes 8 columns of a head's low half and the
// matching 8 of its high half, sums both over the slabs and rotates them back before the bf16 store.
template <bool F16>
__global__ __launch_bounds__(256) void dq_reduce_rope_kernel(const float* __restrict__ P, bf16* __restrict__ dq,
                                                             int B, int Sq, int Hq, int nkb, long pslab, long sdq,
                                                             int causal, int off, int bnk, Ext ex) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const long per_row = (long)Hq * 8;  // (head, 8-column chunk of the low half) per thread
  const long total = (long)B * Sq * per_row;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / per_row;
    const int j = (int)(i - row * per_row);
    const int d0 = (j & 7) * 8;
    const long e = (long)(j >> 3) * 128 + d0;
    const int q = (int)(row % Sq);
    int kb_end = nkb;
    if (causal) {
      const int lim = q + off;
      kb_end = lim < 0 ? 0 : min(nkb, lim / bnk + 1);
      while (kb_end < nkb && (max(0, kb_end * bnk - off) / 32) * 32 <= q) ++kb_end;
    }
    float lo[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hi[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const float* src = P + row * (long)Hq * 128 + e;
    for (int kb = 0; kb < kb_end; ++kb) {
      const float* sp = src + kb * pslab;
      const f32x4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sp));
      const f32x4 a1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sp + 4));
      const f32x4 b0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sp + 64));
      const f32x4 b1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sp + 68));
#pragma unroll
      for (int t = 0; t < 4; ++t) { lo[t] += a0[t]; lo[4 + t] += a1[t]; hi[t] += b0[t]; hi[4 + t] += b1[t]; }
    }
    const float* cr = ex.rope_cos + (long)q * 128 + d0;
    const float* sr = ex.rope_sin + (long)q * 128 + d0;
    float olo[8], ohi[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float c = cr[t], sn = sr[t];
      olo[t] = lo[t] * c + hi[t] * sn;
      ohi[t] = hi[t] * c - lo[t] * sn;
    }
    bf16* out = dq + row * sdq + e;
    if constexpr (F16) {
      store_vec<half16, 8>(reinterpret_cast<half16*>(out), olo);
      store_vec<half16, 8>(reinterpret_cast<half16*>(out + 64), ohi);
    } else {
      store_vec<bf16, 8>(out, olo);
      store_vec<bf16, 8>(out + 64, ohi);
    }
  }
}

template <int MODE, bool F16>
__global__ __launch_bounds__(256) void dq_reduce_kernel(const float* __restrict__ P, bf16* __restrict__ dq, int B,
                                                        int Sq, int Hq, int D, int nkb, long pslab, long sdq,
                                                        int causal, int off, int bnk, Ext ex) {
  const long per_row = (long)Hq * D / 8;  // 8 floats per thread
  const long total = (MODE == kVarlen ? (long)ex.total_q : (long)B * Sq) * per_row;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / per_row;              // token index (b*Sq + q when dense)
    const long e = (i - row * per_row) * 8;    // offset inside the [Hq*D] row
    int q;
    if constexpr (MODE == kVarlen) {
      int lo = 0, hi = B;                      // largest b with cu_q[b] <= row
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (ex.cu_q[mid] <= row) lo = mid; else hi = mid;
      }
      q = (int)(row - ex.cu_q[lo]);
      const int sk_b = ex.cu_k[lo + 1] - ex.cu_k[lo];
      off = sk_b - (ex.cu_q[lo + 1] - ex.cu_q[lo]);
      nkb = (sk_b + bnk - 1) / bnk;
    } else {
      q = (int)(row % Sq);
    }
    int kb_end = nkb;
    if (causal) {
      // last key block whose q_begin <= q
      const int lim = q + off;                 // max key index visible to this row
      kb_end = lim < 0 ? 0 : min(nkb, lim / bnk + 1);
      // rounding: block kb also wrote rows down to floor((kb*bnk-off)/32)*32
      while (kb_end < nkb && (max(0, kb_end * bnk - off) / 32) * 32 <= q) ++kb_end;
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const float* src = P + row * (long)Hq * D + e;
    const int* cls = nullptr;
    if constexpr (MODE == kMask) {
      const long mh = (row / Sq) * ex.fm_hm + (ex.fm_hm == 1 ? 0 : (int)(e / D));
      cls = ex.fm_t256 + (mh * ((Sq + 31) / 32) + q / 32) * nkb;
    }
    for (int kb = 0; kb < kb_end; ++kb) {
      if constexpr (MODE == kMask) {
        if (cls[kb] == 2) continue;  // the bwd kernel skipped (never wrote) this slab row
      }
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + kb * pslab));
      const f32x4 c = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + kb * pslab + 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[j] += a[j]; acc[4 + j] += c[j]; }
    }
    if constexpr (F16) store_vec<half16, 8>(reinterpret_cast<half16*>(dq + row * sdq + e), acc);
    else store_vec<bf16, 8>(dq + row * sdq + e, acc);
  }
}

}  // namespace fa
}  // namespace pd

using namespace pd;

#ifndef PD_FA_DEVICE_ONLY
namespace pd {
namespace fa {
// the two-row-block forward lives in flash_fwd2.hip (its own compile flags)
void launch_fwd_rb2(bool f16, bool causal, int mode, dim3 grid, hipStream_t st, const void* q, const void* k,
                    const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv,
                    long so, float scale, const Ext& ex);
// the 16x16x32-MFMA forward (flash_fwd2.hip; PADDLE2_AMD_FA_FWD_MFMA=16)
void launch_fwd_m16(bool f16, bool causal, int mode, dim3 grid, hipStream_t st, const void* q, const void* k,
                    const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv,
                    long so, float scale, const Ext& ex);
}  // namespace fa
}  // namespace pd

namespace {

// PADDLE2_AMD_FA_FWD_MFMA = 16: the forward on v_mfma_f32_16x16x32 (D = 128, dense / varlen, no dropout, 4 waves)
bool fa_fwd_m16() {
  const char* e = getenv("PADDLE2_AMD_FA_FWD_MFMA");
  return e && atoi(e) == 16;
}

template <int D, bool F16>
void launch_fwd(dim3 grid, hipStream_t st, const void* q, const void* k, const void* v, void* o, float* lse, int B,
                int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv, long so, float scale, bool causal, int mode,
                bool drop, const fa::Ext& ex, int nw, int rb) {
#define PD_FA_FWD_W(CC, MM, DR, W)                                                                                 \
  fa::fwd_kernel<D, CC, MM, DR, F16, W><<<grid, W * 64, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, \
                                                                 (bf16*)o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so, \
                                                                 scale, ex)
#define PD_FA_FWD(CC, MM, DR) PD_FA_FWD_W(CC, MM, DR, 4)
#define PD_FA_FWD_C(MM, DR) \
  if (causal) PD_FA_FWD(true, MM, DR); else PD_FA_FWD(false, MM, DR);
  if constexpr (D == 128) {
    if (nw == 4 && rb == 1 && mode != 2 && !drop && fa_fwd_m16()) {  // 16x16x32 MFMAs (opt-in)
      fa::launch_fwd_m16(F16, causal, mode, grid, st, q, k, v, o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so, scale, ex);
      return;
    }
    if (nw == 4 && rb == 2) {  // two row blocks per wave: dense / varlen without dropout
      fa::launch_fwd_rb2(F16, causal, mode, grid, st, q, k, v, o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so, scale, ex);
      return;
    }
    if (nw == 8) {  // dense / varlen without dropout
      if (mode == 0) { if (causal) PD_FA_FWD_W(true, fa::kDense, false, 8); else PD_FA_FWD_W(false, fa::kDense, false, 8); }
      else { if (causal) PD_FA_FWD_W(true, fa::kVarlen, false, 8); else PD_FA_FWD_W(false, fa::kVarlen, false, 8); }
      return;
    }
  }
  if (drop) {
    if (mode == 0) { PD_FA_FWD_C(fa::kDense, true) } else { PD_FA_FWD_C(fa::kVarlen, true) }
  } else if (mode == 0) { PD_FA_FWD_C(fa::kDense, false) }
  else if (mode == 1) { PD_FA_FWD_C(fa::kVarlen, false) }
  else if constexpr (D <= 128) { PD_FA_FWD_C(fa::kMask, false) }
#undef PD_FA_FWD_C
#undef PD_FA_FWD
#undef PD_FA_FWD_W
}

template <int D, bool F16>
void launch_bwd(dim3 grid, hipStream_t st, const void* q, const void* k, const void* v, const void* dout,
                const float* lse, const float* delta, float* dqp, void* dk, void* dv, int B, int Sq, int Sk, int Hq,
                int Hk, long sq, long sk, long sv, long so, long sdk, long sdv, long pslab, float scale, bool causal,
                int mode, bool drop, const fa::Ext& ex, int nwb) {
  constexpr int NT = fa::bwd_waves<D>() * 64;
  if constexpr (D == 128) {
    if (ex.ds_out != nullptr) {   // split dQ (dense, 8 waves): dS out, no dQ phase
#define PD_FA_BWDS(CC, DR)                                                                                         \
  fa::bwd_kernel<D, CC, fa::kDense, DR, F16, 8, true><<<grid, 512, 0, st>>>(                                      \
      (const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, dqp, (bf16*)dk, (bf16*)dv, B, \
      Sq, Sk, Hq, Hk, sq, sk, sv, so, sdk, sdv, pslab, scale, ex)
      if (drop) { if (causal) PD_FA_BWDS(true, true); else PD_FA_BWDS(false, true); }
      else { if (causal) PD_FA_BWDS(true, false); else PD_FA_BWDS(false, false); }
#undef PD_FA_BWDS
      return;
    }
  }
  if constexpr (D == 128) {
    if (nwb == 4) {   // dense, atomic dQ, no dropout (fa_bwd_waves)
#define PD_FA_BWD4(CC)                                                                                              \
  fa::bwd_kernel<D, CC, fa::kDense, false, F16, 4><<<grid, 256, 0, st>>>(                                          \
      (const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, dqp, (bf16*)dk, (bf16*)dv, B, \
      Sq, Sk, Hq, Hk, sq, sk, sv, so, sdk, sdv, pslab, scale, ex)
      if (causal) PD_FA_BWD4(true); else PD_FA_BWD4(false);
#undef PD_FA_BWD4
      return;
    }
  }
#define PD_FA_BWD(CC, MM, DR)                                                                                    \
  fa::bwd_kernel<D, CC, MM, DR, F16><<<grid, NT, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,       \
                                                          (const bf16*)dout, lse, delta, dqp, (bf16*)dk, (bf16*)dv, \
                                                          B, Sq, Sk, Hq, Hk, sq, sk, sv, so, sdk, sdv, pslab, scale, ex)
#define PD_FA_BWD_C(MM, DR) \
  if (causal) PD_FA_BWD(true, MM, DR); else PD_FA_BWD(false, MM, DR);
  if (drop) {
    if (mode == 0) { PD_FA_BWD_C(fa::kDense, true) } else { PD_FA_BWD_C(fa::kVarlen, true) }
  } else if (mode == 0) { PD_FA_BWD_C(fa::kDense, false) }
  else if (mode == 1) { PD_FA_BWD_C(fa::kVarlen, false) }
  else if constexpr (D <= 128) { PD_FA_BWD_C(fa::kMask, false) }
#undef PD_FA_BWD_C
#undef PD_FA_BWD
}

// shape / mode validation shared by fwd and bwd: dt bf16 or f16, D in {64, 128, 256}, FlashMask only for
// D <= 128 (its plans are built for 256-key backward blocks)
int check_args(int dt, int D, int Hq, int Hk, int mode, int drop, float pdrop, const int* cu_q, const int* cu_k,
               const int* fm, const int* plan, int fm_hm) {
  if ((dt != kBF16 && dt != kF16) || (D != 64 && D != 128 && D != 256) || Hq % Hk || mode < 0 || mode > 2) return -1;
  if (mode == 2 && D > 128) return -1;
  if (drop && (mode == 2 || !(pdrop > 0.f && pdrop < 1.f))) return -3;
  if (mode == 1 && (!cu_q || !cu_k)) return -2;
  if (mode == 2 && (!fm || !plan || (fm_hm != 1 && fm_hm != Hq))) return -2;
  return 0;
}

}  // namespace

// Dense backward dQ accumulation: fp32 atomics into one slab (default; the reference's flash bwd is likewise
// not bit-reproducible) or, with PADDLE2_AMD_FA_DQ_ATOMIC=0 (set by FLAGS_cudnn_deterministic), per-key-block
// slabs summed in a fixed order.  Read per call: the Python side sizes the workspace by the same rule.
static bool fa_dq_atomic() {
  const char* e = getenv("PADDLE2_AMD_FA_DQ_ATOMIC");
  return e ? atoi(e) != 0 : true;
}
extern "C" int pd_flash_dq_atomic() { return fa_dq_atomic() ? 1 : 0; }

// Forward workgroup width.  Measured (profiles/r3_flash_fwd_waves.md, B8 H32 D128): the 8-wave kernel wins on
// long non-causal rows (S4096: 982 vs 937 TF/s) and loses on causal S4096 (808 vs 821: the per-wave tile skip
// leaves SIMD partners unbalanced on the diagonal), D = 64 and short sequences.  PADDLE2_AMD_FA_FWD_WAVES = 4 / 8
// forces one kernel (8 only where it exists: D = 128, dense / varlen, no dropout).
static int fa_fwd_waves(int D, int Sq, int causal, int mode, int drop) {
  if (D != 128 || mode == 2 || drop) return 4;
  if (const char* e = getenv("PADDLE2_AMD_FA_FWD_WAVES")) {
    const int w = atoi(e);
    if (w == 4 || w == 8) return w;
  }
  return (!causal && Sq >= 2048) ? 8 : 4;
}

// Row blocks per wave of the 4-wave forward (D = 128, dense / varlen, no dropout): 1 = 32 rows per wave, two
// workgroups per CU; 2 = 64 rows per wave (two 32-row blocks sharing every K / V fragment read), one 256-row
// workgroup per CU.  PADDLE2_AMD_FA_FWD_RB = 1 / 2 forces one.
static int fa_fwd_rb(int D, int nw, int mode, int drop) {
  if (D != 128 || nw != 4 || mode == 2 || drop) return 1;
  if (const char* e = getenv("PADDLE2_AMD_FA_FWD_RB")) return atoi(e) == 2 ? 2 : 1;
  return 1;
}

// Key-block width of the backward (rows of the dQ partial slabs): 256 keys for D <= 128, 128 for D = 256.
// (The 4-wave D = 128 kernel's 128-key blocks run only in the dense atomic mode, whose dQ is one slab.)
extern "C" int pd_flash_bwd_block(int D) { return D > 128 ? 128 : 256; }

// Backward workgroup width at D = 128 for the dense atomic-dQ path: 8 waves (256 keys, one workgroup per CU) or 4
// (128 keys, two per CU).  PADDLE2_AMD_FA_BWD_WAVES = 4 / 8 forces one.
static int fa_bwd_waves(int D, int mode, bool atomic, int drop) {
  if (D != 128 || mode != 0 || !atomic || drop) return D > 128 ? 4 : 8;
  if (const char* e = getenv("PADDLE2_AMD_FA_BWD_WAVES")) {
    const int w = atoi(e);
    if (w == 4 || w == 8) return w;
  }
  return 8;
}

// mode: 0 dense, 1 varlen (B sequences, Sq/Sk = max_seqlen, rows located by cu_q/cu_k, lse [Hq, total_q]),
// 2 FlashMask (dense layout + fm [B, fm_hm, Sk] int4 intervals with the fm_t64 / fm_t256 fwd / bwd plans).
// dt: kBF16 or kF16 (q/k/v/o share it).
extern "C" int pd_flash_fwd_ext(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B,
                                int Sq, int Sk, int Hq, int Hk, int D, long sq, long sk, long sv, long so, float scale,
                                int causal, int mode, const int* cu_q, const int* cu_k, int total_q, const int* fm,
                                const int* fm_t64, const int* fm_t256, int fm_hm, int drop, unsigned seed, float pdrop,
                                void* stream) {
  if (int e = check_args(dt, D, Hq, Hk, mode, drop, pdrop, cu_q, cu_k, fm, fm_t64, fm_hm)) return e;
  hipStream_t st = (hipStream_t)stream;
  const int nw = fa_fwd_waves(D, Sq, causal, mode, drop);
  const int rb = fa_fwd_rb(D, nw, mode, drop);
  const int nmb = (Sq + 32 * nw * rb - 1) / (32 * nw * rb);
  dim3 grid(nmb * Hq * B);
  fa::Ext ex{cu_q, cu_k, total_q, (const int4*)fm, fm_t64, fm_t256, fm_hm, seed,
             drop ? (unsigned)fminf(pdrop * 4294967296.f, 4294967040.f) : 0u, drop ? 1.f / (1.f - pdrop) : 1.f};
  // per-wave causal tile skip: +0.7-1.9 % on the 4-wave kernel, bitwise-identical output
  // (profiles/r3_flash_fwd_waves.md); PADDLE2_AMD_FA_FWD_WAVE_SKIP=0 turns it off
  ex.wave_skip = 1;
  if (const char* e = getenv("PADDLE2_AMD_FA_FWD_WAVE_SKIP")) ex.wave_skip = atoi(e) != 0;
#define PD_FWD(DD, FF) \
  launch_fwd<DD, FF>(grid, st, q, k, v, o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so, scale, causal, mode, drop, ex, nw, rb)
  const bool f16 = dt == kF16;
  if (D == 128) { if (f16) PD_FWD(128, true); else PD_FWD(128, false); }
  else if (D == 64) { if (f16) PD_FWD(64, true); else PD_FWD(64, false); }
  else { if (f16) PD_FWD(256, true); else PD_FWD(256, false); }
#undef PD_FWD
  return (int)hipGetLastError();
}

extern "C" int pd_flash_fwd(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq,
                            int Sk, int Hq, int Hk, int D, long sq, long sk, long sv, long so, float scale, int causal,
                            void* stream) {
  return pd_flash_fwd_ext(dt, q, k, v, o, lse, B, Sq, Sk, Hq, Hk, D, sq, sk, sv, so, scale, causal, 0, nullptr,
                          nullptr, 0, nullptr, nullptr, nullptr, 1, 0, 0u, 0.f, stream);
}

// dqp: fp32 workspace of nkb * rows*Hq*D floats (nkb = ceil(Sk / pd_flash_bwd_block(D)), rows = B*Sq, or total_q
// for varlen) for per-key-block dQ partials (need not be zeroed; ONE slab for dense mode when pd_flash_dq_atomic()); delta a [B, Hq, Sq] ([Hq, total_q] varlen) fp32
// workspace.  q/k/v/o/dout and dq/dk/dv may all be row-strided views ([B, S, H, D] with token strides), e.g. slices
// of one fused QKV / dQKV buffer.
// RoPE^T tables for the next pd_flash_bwd_ext call on this thread (consumed by it; dense mode, D = 128 only)
static thread_local const float* t_bwd_rope_cos = nullptr;
static thread_local const float* t_bwd_rope_sin = nullptr;
extern "C" void pd_flash_bwd_set_rope(const float* cos, const float* sin) {
  t_bwd_rope_cos = cos;
  t_bwd_rope_sin = sin;
}

// Split-dQ workspace (dense, D = 128): bf16 elements of the compact dS buffer per (b, hq) — every key block's
// [32 q][256 keys] blocks for the 32-row query tiles it visits — or 0 where the split path does not apply.
// Opt-in (PADDLE2_AMD_FA_DQ_SPLIT=1): a deterministic dQ without atomics or fp32 slabs.  At B8 S4096 H32 D128
// causal it measured 4.5-5.2 ms per layer against 4.4-4.5 for the fused atomic path (profiles/r6_flash_dq_split.md):
// the 4.6 GB of dS stores cost the main kernel ~0.6 ms of memory traffic and dq_gemm_kernel reads them back in
// 1.1 ms, more than the atomics (0.8 ms) plus the fused dQ MFMAs (0.75 ms) they replace.
static long fa_ds_per_bh(int Sq, int Sk, int D, int causal) {
  if (D != 128) return 0;
  const int BNK = 256, nqt = (Sq + 31) / 32, nkb = (Sk + BNK - 1) / BNK, off = Sk - Sq;
  long n = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const int tb = causal ? std::max(0, kb * BNK - off) / 32 : 0;
    n += (long)std::max(0, nqt - tb) * 32 * BNK;
  }
  return n;
}
extern "C" long pd_flash_ds_elems(int B, int Sq, int Sk, int Hq, int D, int causal) {
  const char* e = getenv("PADDLE2_AMD_FA_DQ_SPLIT");
  if (!e || atoi(e) == 0) return 0;
  return (long)B * Hq * fa_ds_per_bh(Sq, Sk, D, causal);
}
// dS workspace for the next pd_flash_bwd_ext call on this thread (consumed by it; dense mode only)
static thread_local void* t_bwd_ds = nullptr;
extern "C" void pd_flash_bwd_set_ds(void* ds) { t_bwd_ds = ds; }

extern "C" int pd_flash_bwd_ext(int dt, const void* q, const void* k, const void* v, const void* o, const void* dout,
                                const float* lse, float* delta, void* dq, void* dk, void* dv, float* dqp, int B,
                                int Sq, int Sk, int Hq, int Hk, int D, long sq, long sk, long sv, long so, long sdq,
                                long sdk, long sdv, float scale, int causal, int mode, const int* cu_q, const int* cu_k,
                                int total_q, const int* fm, const int* fm_t64, const int* fm_t256, int fm_hm,
                                int drop, unsigned seed, float pdrop, void* stream) {
  void* ds = t_bwd_ds;
  t_bwd_ds = nullptr;
  if (int e = check_args(dt, D, Hq, Hk, mode, drop, pdrop, cu_q, cu_k, fm, fm_t256, fm_hm)) {
    t_bwd_rope_cos = t_bwd_rope_sin = nullptr;
    return e;
  }
  if (ds && (mode != 0 || D != 128)) {
    t_bwd_rope_cos = t_bwd_rope_sin = nullptr;
    return -5;
  }
  if (t_bwd_rope_cos && (mode != 0 || D != 128 || !t_bwd_rope_sin)) {
    t_bwd_rope_cos = t_bwd_rope_sin = nullptr;
    return -4;
  }
  hipStream_t st = (hipStream_t)stream;
  const bool f16 = dt == kF16;
  const long nrows = mode == 1 ? (long)total_q : (long)B * Sq;  // query tokens
  // delta shares the lse layout: [B, Hq, Sq] dense, [Hq, total_q] (= B 1, Sq total_q) varlen
  const int dB = mode == 1 ? 1 : B, dS = mode == 1 ? total_q : Sq;
  const long rows = (long)dB * Hq * dS;
  const long rows_per_blk = 256 / (D / 8);
  const int dgrid = (int)((rows + rows_per_blk - 1) / rows_per_blk);
  if (f16)
    fa::bwd_delta_kernel<true><<<dgrid, 256, 0, st>>>((const bf16*)o, (const bf16*)dout, delta, dB, dS, Hq, D, so);
  else
    fa::bwd_delta_kernel<false><<<dgrid, 256, 0, st>>>((const bf16*)o, (const bf16*)dout, delta, dB, dS, Hq, D, so);
  // dense mode, atomic dQ: every key block adds into one zeroed fp32 slab (one slab of workspace, a convert
  // pass instead of the slab reduce: 0.27 ms less per B8 S4096 H32 D128 layer)
  const bool split = ds != nullptr;   // dS out + dq_gemm_kernel (no dQ phase, no slab, no reduce)
  const bool atomic = !split && mode == 0 && fa_dq_atomic();
  const int nwb = split ? 8 : fa_bwd_waves(D, mode, atomic, drop);
  const int BNK = D == 128 && nwb == 4 ? 128 : pd_flash_bwd_block(D);
  const int nkb = (Sk + BNK - 1) / BNK;
  const long pslab = (atomic || split) ? 0 : nrows * Hq * D;
  if (atomic) hipMemsetAsync(dqp, 0, nrows * Hq * D * sizeof(float), st);
  dim3 grid(nkb * Hk * B);
  fa::Ext ex{cu_q, cu_k, total_q, (const int4*)fm, fm_t64, fm_t256, fm_hm, seed,
             drop ? (unsigned)fminf(pdrop * 4294967296.f, 4294967040.f) : 0u, drop ? 1.f / (1.f - pdrop) : 1.f,
             atomic ? 1 : 0};
  ex.rope_cos = t_bwd_rope_cos;
  ex.rope_sin = t_bwd_rope_sin;
  t_bwd_rope_cos = t_bwd_rope_sin = nullptr;
  // PADDLE2_AMD_FA_BWD_ORDER = pair: co-dispatch a pair's key blocks (L2 reuse of Q / dO) instead of heaviest first
  if (const char* e = getenv("PADDLE2_AMD_FA_BWD_ORDER"))
    ex.pair_order = (strcmp(e, "pair") == 0 && (Hk * B) % 8 == 0) ? 1 : 0;
  if (const char* e = getenv("PADDLE2_AMD_FA_BWD_OPT")) ex.bwd_opt = atoi(e) & 3;
  if (split) {
    ex.ds_out = (bf16*)ds;
    ex.ds_per_bh = fa_ds_per_bh(Sq, Sk, D, causal);
    // the dK epilogue applies RoPE^T itself (ex.rope_cos); dQ's RoPE^T moves into dq_gemm_kernel
  }
  // bench-only ablation (scripts/bench_flash_bwd.py; results are WRONG): 2 = compute dQ but skip its stores,
  // 3 = skip the whole dQ phase (dS image, barrier, dQ MFMAs, stores) — prices the dQ path in isolation
  if (const char* e = getenv("PADDLE2_AMD_FA_DEBUG_DQ_ABLATE")) {
    const int m = atoi(e);
    if (atomic && (m == 2 || m == 3)) ex.dq_atomic = m;
    if (split && (m == 4 || m == 5)) ex.dq_atomic = m;   // split: 4 = no dS stores, 5 = no dS LDS image either
  }
#define PD_BWD(DD, FF)                                                                                              \
  launch_bwd<DD, FF>(grid, st, q, k, v, dout, lse, delta, dqp, dk, dv, B, Sq, Sk, Hq, Hk, sq, sk, sv, so, sdk, sdv, \
                     pslab, scale, causal, mode, drop, ex, nwb)
  if (D == 128) { if (f16) PD_BWD(128, true); else PD_BWD(128, false); }
  else if (D == 64) { if (f16) PD_BWD(64, true); else PD_BWD(64, false); }
  else { if (f16) PD_BWD(256, true); else PD_BWD(256, false); }
#undef PD_BWD
  if (split) {
    const int nmb = (Sq + 127) / 128;
    const dim3 g2(nmb * Hq * B);
#define PD_DQG(FF, CC)                                                                                              \
  fa::dq_gemm_kernel<FF, CC><<<g2, 256, 0, st>>>((const bf16*)ds, (const bf16*)k, (bf16*)dq, B, Sq, Sk, Hq, Hk, sk, \
                                                 sdq, ex.ds_per_bh, scale, ex.rope_cos, ex.rope_sin)
    if (f16) { if (causal) PD_DQG(true, true); else PD_DQG(true, false); }
    else { if (causal) PD_DQG(false, true); else PD_DQG(false, false); }
#undef PD_DQG
    return (int)hipGetLastError();
  }
  long work = nrows * Hq * D / 8;
  long g = (work + 255) / 256;
  if (g > 8192) g = 8192;
#define PD_DQR(MM, FF)                                                                                             \
  fa::dq_reduce_kernel<MM, FF><<<(int)g, 256, 0, st>>>(dqp, (bf16*)dq, B, Sq, Hq, D, atomic ? 1 : nkb, pslab, sdq, \
                                                       atomic ? 0 : causal, Sk - Sq, BNK, ex)
  if (ex.rope_cos) {
    long gr = (nrows * Hq * 8 + 255) / 256;
    if (gr > 8192) gr = 8192;
    if (f16)
      fa::dq_reduce_rope_kernel<true><<<(int)gr, 256, 0, st>>>(dqp, (bf16*)dq, B, Sq, Hq, atomic ? 1 : nkb, pslab, sdq,
                                                               atomic ? 0 : causal, Sk - Sq, BNK, ex);
    else
      fa::dq_reduce_rope_kernel<false><<<(int)gr, 256, 0, st>>>(dqp, (bf16*)dq, B, Sq, Hq, atomic ? 1 : nkb, pslab,
                                                                sdq, atomic ? 0 : causal, Sk - Sq, BNK, ex);
  } else if (mode == 2) { if (f16) PD_DQR(fa::kMask, true); else PD_DQR(fa::kMask, false); }
  else if (mode == 1) { if (f16) PD_DQR(fa::kVarlen, true); else PD_DQR(fa::kVarlen, false); }
  else { if (f16) PD_DQR(fa::kDense, true); else PD_DQR(fa::kDense, false); }
#undef PD_DQR
  return (int)hipGetLastError();
}

extern "C" int pd_flash_bwd(int dt, const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, float* delta, void* dq, void* dk, void* dv, float* dqp, int B, int Sq,
                            int Sk, int Hq, int Hk, int D, long sq, long sk, long sv, long so, long sdq, long sdk,
                            long sdv, float scale, int causal, void* stream) {
  return pd_flash_bwd_ext(dt, q, k, v, o, dout, lse, delta, dq, dk, dv, dqp, B, Sq, Sk, Hq, Hk, D, sq, sk, sv, so, sdq,
                          sdk, sdv, scale, causal, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 1, 0, 0u, 0.f,
                          stream);
}
#endif  // PD_FA_DEVICE_ONLY
