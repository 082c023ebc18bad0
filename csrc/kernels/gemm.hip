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
#include <hip/hip_runtime.h>

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
constexpr int STAGE_BYTES = 2 * TILE_BYTES;     // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 2-stage ring, 128 KiB
constexpr unsigned kOOB = 0x80000000u;          // voffset beyond num_records -> the load returns 0
constexpr int kRecords = 0x7fffffff;

enum Epi : int { kEpiBF16 = 0, kEpiF32 = 1, kEpiSwiGLU = 2 };

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
  int H;                        // swiglu: gate/up split (columns of the packed weight)
};

__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int q = n / 8, r = n % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// MN-major image row swizzle (8 distinct values over the rows one 32-lane half reads)
__device__ __forceinline__ int hsw(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, kRecords, 0x00020000);
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

// Per-lane LDS-DMA source offsets of one operand, computed once per workgroup.
// A 256 (rows = the M or N index) x 64 (k) tile = 32 x 1 KiB blocks; thread issues 4 (blk = 8i + wave).
// KMAJ: element (r, k) at r*ld + k  ->  image [256][64], 16-B chunk swizzle ^((r>>1)&7)
//       lane: row r = 64i + 8*wave + (lane>>3) (rows of instruction i are 64i apart), chunk lc fixed
// else: element (r, k) at k*ld + r  ->  image [64][256], pair swizzle ^hsw(k)
//       lane: k = 16i + 2*wave + (lane>>5), column chunk lc fixed (hsw(k) does not depend on i)
struct Ld {
  unsigned voff;   // byte offset for instruction 0 relative to the tile's base (row/col bound folded in)
  int kl;          // this lane's k inside the tile (K-major: first k of its chunk)
  int rl;          // K-major: this lane's row inside the tile for i = 0; MN-major: unused
  bool rok;        // MN-major: column in range
};

template <bool KMAJ, bool ISB, int EPI>
__device__ __forceinline__ Ld lane_setup(long ld, int R, int t0, int H, int wave, int lane) {
  Ld o;
  if constexpr (KMAJ) {
    const int r = 8 * wave + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);
    o.kl = lc * 8;
    o.rl = r;
    o.rok = true;
    if constexpr (ISB && EPI == kEpiSwiGLU) {
      o.voff = 0;  // (not used: SwiGLU needs an N-major B)
    } else {
      o.voff = (unsigned)((long)r * ld * 2 + lc * 16);
    }
  } else {
    const int kk = 2 * wave + (lane >> 5);
    const int lc = (lane & 31) ^ (hsw(kk) << 1);
    const int gc = ISB ? bcol<EPI>(t0, lc * 8, H) : t0 * BM + lc * 8;
    const int c0 = ISB ? (EPI == kEpiSwiGLU ? 0 : t0 * BN) : t0 * BM;
    o.kl = kk;
    o.rl = 0;
    o.rok = gc < R;
    o.voff = (unsigned)((long)kk * ld * 2 + (long)(gc - c0) * 2);
  }
  return o;
}

// Stream instructions [2*part, 2*part+2) of a 256 x 64 operand tile (k0 = first k) into `dst`.
// `tbase` = the tile's element base (K-major: row t0*256, col k0; MN-major: row k0, col of tile).
template <bool KMAJ>
__device__ __forceinline__ void stage(const unsigned short* tbase, const Ld& L, long ld, int R, int rt0, int K,
                                      int k0, lds_char* dst, int wave, int part) {
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(tbase);
#pragma unroll
  for (int ii = 0; ii < 2; ++ii) {
    const int i = part * 2 + ii;
    unsigned voff;
    if constexpr (KMAJ) {
      const bool ok = (rt0 + L.rl + 64 * i < R) && (k0 + L.kl < K);
      voff = (L.voff + (unsigned)(64 * i) * (unsigned)(ld * 2)) | ((unsigned)(!ok) << 31);
    } else {
      const bool ok = L.rok && (k0 + L.kl + 16 * i < K);
      voff = (L.voff + (unsigned)(16 * i) * (unsigned)(ld * 2)) | ((unsigned)(!ok) << 31);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (8 * i + wave) * 1024),
                                             16, voff, 0, 0, 0);
  }
}

// Fragment reads.  K-major: one ds_read_b128 of 8 consecutive k for row rb + (lane&15).
// MN-major: two ds_read_b64_tr_b16 (rows k = 32s + 8g + q and +4, columns rb + 4p .. +3; lane receives
// column rb + (lane&15)).  All fragment reads are inline asm: hipcc models the transposed-read builtin
// as aliasing the in-flight LDS-DMA and drains vmcnt(0) before it (serialising the prefetch), and its
// counted lgkmcnt waits for builtin reads would also count the asm ones issued after them (waiting
// for the NEXT sub-phase's reads).  The kernel retires its reads itself: lgkmcnt(0) at the start of
// the consuming sub-phase (`sync_frags`), one sub-phase (8 MFMAs) after issue.
__device__ __forceinline__ s16x4 tr_read(const lds_char* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((unsigned)(size_t)p));
  return r;
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const lds_char* img, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rb + (lane & 15);
    const int ch = (4 * s + (lane >> 4)) ^ ((r >> 1) & 7);
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)(img + r * 128 + ch * 16)));
    return v;
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int ka = 32 * s + 8 * g + q;
    const int h = q | ((g & 1) << 2);
    const int off = ka * 512 + ((rb >> 4) ^ h) * 32 + (p >> 1) * 16 + (p & 1) * 8;
    const s16x4 lo = tr_read(img + off);
    const s16x4 hi = tr_read(img + off + 4 * 512);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// Retire every outstanding LDS read before a sub-phase's MFMAs consume the previous sub-phase's
// fragments (needed for the asm transposed reads; the sched_barrier keeps hipcc from hoisting the
// register-only MFMAs above the wait, cdna guide §5.4 rule 18).
__device__ __forceinline__ void sync_frags() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ f32x4v mfma(bf16x8 a, bf16x8 b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(NTHR, 1) void gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(1024))) char smem_raw[LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;

  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  // grouped order: group_m row-tiles sweep the column tiles together (L2 reuse within an XCD)
  const int per_group = p.group_m * p.tiles_n;
  const int gid = bid / per_group;
  const int first_m = gid * p.group_m;
  const int gsz = min(p.tiles_m - first_m, p.group_m);
  const int tm = first_m + (bid % per_group) % gsz;
  const int tn = (bid % per_group) / gsz;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int Ncols = (EPI == kEpiSwiGLU) ? 2 * p.H : p.N;
  const int nt = (p.K + BK - 1) / BK;

  f32x4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const Ld LA = lane_setup<AK, false, EPI>(p.lda, p.M, tm, p.H, wave, lane);
  const Ld LB = lane_setup<BKM, true, EPI>(p.ldb, Ncols, tn, p.H, wave, lane);
  const int a_r0 = tm * BM;                                     // A rows of this tile
  const int b_r0 = (EPI == kEpiSwiGLU) ? 0 : tn * BN;           // B rows/cols of this tile (remap: in LB)
  auto tile_ptr = [&](const unsigned short* g, long ld, bool kmaj, int r0, int k0) {
    return kmaj ? g + (long)r0 * ld + k0 : g + (long)k0 * ld + r0;
  };
  auto stageA = [&](int t, int buf, int part) {
    stage<AK>(tile_ptr(p.A, p.lda, AK, a_r0, t * BK), LA, p.lda, p.M, a_r0, p.K, t * BK, smem + buf * STAGE_BYTES,
              wave, part);
  };
  auto stageB = [&](int t, int buf, int part) {
    stage<BKM>(tile_ptr(p.B, p.ldb, BKM, b_r0, t * BK), LB, p.ldb, Ncols, b_r0, p.K, t * BK,
               smem + buf * STAGE_BYTES + TILE_BYTES, wave, part);
  };
  const int arow = wm * 128;  // wave's first row in the A tile
  const int bcolw = wn * 64;  // wave's first column in the B tile

  // prologue: tiles 0 and 1 in flight, wait for tile 0
  stageA(0, 0, 0); stageA(0, 0, 1); stageB(0, 0, 0); stageB(0, 0, 1);
  if (nt > 1) {
    stageA(1, 1, 0); stageA(1, 1, 1); stageB(1, 1, 0); stageB(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  // fragment sets: A half = 4 m16 tiles, B half = 2 n16 tiles.  A0/B0 of the two k32 steps of a tile
  // have their own names (x: step 0, y: step 1) so no fragment is ever copied between registers.
  bf16x8 a0x[4], b0x[2], a0y[4], b0y[2], a1[4], b1[2];
  auto readA = [&](bf16x8 (&dst)[4], const lds_char* img, int half, int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = frag<AK>(img, arow + 64 * half + 16 * i, s, lane);
  };
  auto readB = [&](bf16x8 (&dst)[2], const lds_char* img, int half, int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) dst[j] = frag<BKM>(img, bcolw + 32 * half + 16 * j, s, lane);
  };
  auto mm = [&](const bf16x8 (&a)[4], const bf16x8 (&b)[2], int mi, int ni) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[4 * mi + i][2 * ni + j] = mfma(a[i], b[j], acc[4 * mi + i][2 * ni + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  readA(a0x, smem, 0, 0);
  readB(b0x, smem + TILE_BYTES, 0, 0);

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const lds_char* ia = smem + cur * STAGE_BYTES;
    const lds_char* ib = ia + TILE_BYTES;
    const bool more = t + 1 < nt;
    const bool stage2 = t + 2 < nt;
    // ---- k32 step 0: sub-phases A0B0, A0B1, A1B1, A1B0; each issues the next one's reads first
    sync_frags();
    readB(b1, ib, 1, 0);
    mm(a0x, b0x, 0, 0);
    sync_frags();
    readA(a1, ia, 1, 0);
    mm(a0x, b1, 0, 1);
    sync_frags();
    mm(a1, b1, 1, 1);
    readA(a0y, ia, 0, 1);
    readB(b0y, ib, 0, 1);
    mm(a1, b0x, 1, 0);
    // ---- k32 step 1
    sync_frags();
    readB(b1, ib, 1, 1);
    mm(a0y, b0y, 0, 0);
    sync_frags();
    readA(a1, ia, 1, 1);
    mm(a0y, b1, 0, 1);
    // barrier: tile t+1 landed (own DMA drained, then everyone's); every read of stage `cur` retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (stage2) { stageA(t + 2, cur, 0); stageA(t + 2, cur, 1); }
    mm(a1, b1, 1, 1);
    if (stage2) { stageB(t + 2, cur, 0); stageB(t + 2, cur, 1); }
    if (more) {
      const lds_char* na = smem + (cur ^ 1) * STAGE_BYTES;
      readA(a0x, na, 0, 0);
      readB(b0x, na + TILE_BYTES, 0, 0);
    }
    mm(a1, b0y, 1, 0);
  }

  // ---- epilogue.  acc[i][j]: rows arow + 16i + 4*(lane>>4) + e, tile column bcolw + 16j + (lane&15)
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
      if constexpr (EPI == kEpiBF16) {
        if (p.bias) bv = bf2f(p.bias[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = row0 + 16 * i + e;
          if (r < p.M) {
            if constexpr (EPI == kEpiBF16) {
              ((unsigned short*)p.C)[(long)r * p.ldc + c] = f2bf(acc[i][j][e] + bv);
            } else {
              float* cp = (float*)p.C + (long)r * p.ldc + c;
              *cp = p.beta != 0.f ? acc[i][j][e] + p.beta * *cp : acc[i][j][e];
            }
          }
        }
    }
  }
}

}  // namespace gm
}  // namespace pd

// layout: bit0 = A K-major, bit1 = B K-major.  epi: 0 bf16 (+bias), 1 fp32 main grad (beta), 2 swiglu.
extern "C" int pd_gemm(int layout, int epi, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                       void* C2, long ldc2, const void* bias, int M, int N, int K, float beta, int H, int group_m,
                       void* stream) {
  using namespace pd::gm;
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if ((layout & 3) && K % 8) return -1;   // K-major operands move 16-B chunks along k
  Params p;
  p.A = (const unsigned short*)A;
  p.B = (const unsigned short*)B;
  p.C = C;
  p.C2 = (unsigned short*)C2;
  p.bias = (const unsigned short*)bias;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldc2 = ldc2;
  p.M = M; p.N = N; p.K = K; p.beta = beta; p.H = H;
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = epi == kEpiSwiGLU ? (H + 127) / 128 : (N + BN - 1) / BN;
  p.group_m = group_m > 0 ? group_m : 8;
  const bool ak = layout & 1, bk = (layout >> 1) & 1;
  if (!ak && (lda % 8 || M % 8)) return -2;   // MN-major operands move whole 16-B column chunks
  if (!bk && (ldb % 8 || (epi == kEpiSwiGLU ? (2 * H) % 8 : N % 8))) return -2;
  if (epi == kEpiSwiGLU && (bk || H % 32)) return -3;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(p.tiles_m * p.tiles_n);
#define PD_GEMM_LAUNCH(AKV, BKV, EPIV) \
  gemm_kernel<AKV, BKV, EPIV><<<grid, NTHR, 0, st>>>(p)
  switch (epi * 4 + layout) {
    case 0 * 4 + 0: PD_GEMM_LAUNCH(false, false, kEpiBF16); break;
    case 0 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiBF16); break;
    case 0 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiBF16); break;
    case 1 * 4 + 0: PD_GEMM_LAUNCH(false, false, kEpiF32); break;
    case 1 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiF32); break;
    case 1 * 4 + 3: PD_GEMM_LAUNCH(true, true, kEpiF32); break;
    case 2 * 4 + 1: PD_GEMM_LAUNCH(true, false, kEpiSwiGLU); break;
    default: return -4;
  }
#undef PD_GEMM_LAUNCH
  return (int)hipGetLastError();
}
