// Decode attention (one new query token per sequence) over a paged or contiguous KV cache.
//
// Reference behaviour: phi/kernels/fusion/gpu/masked_multihead_attention_kernel.cu (MMHA over a
// [2, b, nh, max_seq, hd] cache) and block_multihead_attention (paged cache + block tables).
// MI355X design (flash-decoding, memory-bound):
//  * grid = (batch, kv_head, split): each workgroup streams one contiguous chunk of the sequence's
//    keys ONCE and serves every query head of the GQA group from it (K/V bytes read once per
//    group, not once per q head);
//  * 256 threads = 16 key slots x 16 lanes; a key slot's lanes hold 8 consecutive head-dim
//    elements each (16-B loads, hd = 128; 8 lanes for hd = 64), dots are reduced with
//    __shfl_xor inside the slot; every slot keeps an online-softmax state (m, l, o[8]) per q head;
//  * slots are merged through LDS, and when the sequence is split across workgroups a second
//    kernel merges the per-split (m, l, o) partials in fp32 — long contexts fill all 256 CUs.
// Addressing covers both cache layouts: token t of sequence b lives at
//   block(b, t) * s_blk + (t % block_size) * s_tok + kv_head * s_head
// with block(b, t) = block_table[b][t / block_size] (paged) or b (contiguous, block_size = inf).
#include "common.h"

namespace pd {
namespace dec {


template <int HD, int G>
__global__ __launch_bounds__(256) void decode_kernel(const bf16* __restrict__ q, long sq_b, long sq_h,
                                                     const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                     long s_blk, long s_tok, long s_head,
                                                     const int* __restrict__ block_table, int max_blocks,
                                                     int block_size, const int* __restrict__ seq_lens,
                                                     float* __restrict__ part_o, float* __restrict__ part_ml,
                                                     bf16* __restrict__ out, long so_b, long so_h, int Hq, int Hk,
                                                     int splits, int chunk, float scale) {
  constexpr int L = HD / 8;             // lanes per key slot
  constexpr int SLOTS = 256 / L;        // keys processed per iteration
  const int hk = blockIdx.x, b = blockIdx.y, sp = blockIdx.z;   // kv heads fastest: a sequence's heads run together
  const int tid = threadIdx.x, slot = tid / L, ln = tid % L;
  const int len = seq_lens[b];
  const int k_begin = sp * chunk, k_end = min(len, k_begin + chunk);
  const float sl2 = scale * 1.4426950408889634f;

  // q slices of the G heads of this kv group (8 elements per lane)
  float qv[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16* qp = q + (long)b * sq_b + (long)(hk * G + g) * sq_h + ln * 8;
    load_vec<bf16, 8>(qp, qv[g]);
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
  }
  for (int t = k_begin + slot; t < k_end; t += SLOTS) {
    long blk = b;
    int off = t;
    if (block_table) {
      blk = block_table[(long)b * max_blocks + t / block_size];
      off = t % block_size;
    }
    const long base = blk * s_blk + (long)off * s_tok + (long)hk * s_head + ln * 8;
    float kv[8], vv[8];
    load_vec<bf16, 8>(kc + base, kv);
    load_vec<bf16, 8>(vc + base, vv);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) d += qv[g][j] * kv[j];
#pragma unroll
      for (int w = L / 2; w > 0; w >>= 1) d += __shfl_xor(d, w, 64);
      const float s = d * sl2;
      const float mn = fmaxf(m[g], s);
      const float a = exp2f(m[g] - mn), p = exp2f(s - mn);
      l[g] = l[g] * a + p;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] = o[g][j] * a + p * vv[j];
      m[g] = mn;
    }
  }
  // merge the SLOTS partial states of this workgroup through LDS, one head at a time
  __shared__ float sm_m[SLOTS], sm_l[SLOTS];
  __shared__ float sm_o[SLOTS][HD + 4];
  for (int g = 0; g < G; ++g) {
    if (ln == 0) {
      sm_m[slot] = m[g];
      sm_l[slot] = l[g];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sm_o[slot][ln * 8 + j] = o[g][j];
    __syncthreads();
    if (tid < HD) {
      float M = -INFINITY;
      for (int s2 = 0; s2 < SLOTS; ++s2) M = fmaxf(M, sm_m[s2]);
      float Lsum = 0.f, acc = 0.f;
      for (int s2 = 0; s2 < SLOTS; ++s2) {
        const float w = sm_m[s2] == -INFINITY ? 0.f : exp2f(sm_m[s2] - M);
        Lsum += sm_l[s2] * w;
        acc += sm_o[s2][tid] * w;
      }
      const int hq = hk * G + g;
      if (splits == 1) {
        const float v = Lsum > 0.f ? acc / Lsum : 0.f;
        out[(long)b * so_b + (long)hq * so_h + tid].x = f2bf(v);
      } else {
        const long pi = (((long)b * Hq + hq) * splits + sp);
        part_o[pi * HD + tid] = acc;
        if (tid == 0) {
          part_ml[pi * 2] = M;
          part_ml[pi * 2 + 1] = Lsum;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------------------
// MFMA decode (HD = 128): the G query heads of a kv group are the 16 (padded) rows of v_mfma_f32_16x16x32_bf16.
//  * each wave owns every 4th 32-key tile of the workgroup's chunk; a lane loads 16 B of K and of V per
//    (key, 32-wide d chunk): lane l -> key 16u + (l&15), d = 32c + 8(l>>4) (u = 0,1; c = 0..3) — exactly the
//    A-operand map of K for S^T = K.Q^T (rows = keys, k = d), so K never touches LDS; Q^T is the B operand,
//    loaded once;
//  * S^T's accumulator holds, per lane, 4 keys of column g = l&15: the online softmax runs per lane column
//    (tile max: 8 in-lane values + 2 cross-group shuffles), and the bf16 P fragment of the P.V MFMA is built in
//    place — its k order (keys 4h..4h+3, 16+4h..16+4h+3 for lane group h) is matched by the V operand, read from
//    a per-wave row-major LDS image with ds_read_b64_tr_b16 (T10, XOR-swizzled 256-B rows, conflict-free);
//  * the next tile's 16 loads are in flight while the current one computes (16 KiB per wave), and the row
//    addresses (paged block-table reads) run one more tile ahead;
//  * the 4 waves' (m, l, O) are merged through LDS; split partials go to the same merge kernel as the vector path.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;

__device__ __forceinline__ int voff(int row, int ch) {   // 16-B chunk ch of row `row` in a [32][128 bf16] image
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

constexpr int kMfmaLds = 4 * 32 * 256;                   // 4 waves x one 32-key V tile

template <int G, bool PAGED>
__global__ __launch_bounds__(256, 2) void decode_mfma_kernel(const bf16* __restrict__ q, long sq_b, long sq_h,
                                                             const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                             long s_blk, long s_tok, long s_head,
                                                             const int* __restrict__ block_table, int max_blocks,
                                                             int bs_shift, const int* __restrict__ seq_lens,
                                                             float* __restrict__ part_o, float* __restrict__ part_ml,
                                                             bf16* __restrict__ out, long so_b, long so_h, int Hq,
                                                             int splits, int chunk, float scale) {
  constexpr int HD = 128;
  __shared__ __attribute__((aligned(16))) char lds[kMfmaLds + 4 * 16 * 2 * 4];
  const int hk = blockIdx.x, b = blockIdx.y, sp = blockIdx.z;   // kv heads fastest: a sequence's heads run together
  const int tid = threadIdx.x, l = tid & 63, h = l >> 4, c16 = l & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile loops branch on SGPRs
  const int len = seq_lens[b];
  const int k_begin = sp * chunk, k_end = min(len, k_begin + chunk);
  const float sl2 = scale * 1.4426950408889634f;

  bf16x8 qf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c16 < G) qf[c] = *reinterpret_cast<const bf16x8*>(q + (long)b * sq_b + (long)(hk * G + c16) * sq_h + 32 * c + 8 * h);
    else qf[c] = bf16x8{};
  }
  f32x4 o[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, lsum = 0.f;
  char* vl = lds + w * (32 * 256);
  const int ntile = k_end > k_begin ? (k_end - k_begin + 31) / 32 : 0;

  // block of this lane's keys (u = 0, 1) in tile t; keys past the sequence are clamped so their (masked)
  // loads stay inside valid blocks
  auto blocks = [&](int t, int (&bk)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int key = min(k_begin + 32 * t + 16 * u + c16, len - 1);
      bk[u] = PAGED ? block_table[(long)b * max_blocks + (key >> bs_shift)] : b;
    }
  };
  bf16x8 kr[2][4], vr[2][4];
  auto load = [&](int t, const int (&bk)[2], bf16x8 (&kk)[2][4], bf16x8 (&vv)[2][4]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int key = min(k_begin + 32 * t + 16 * u + c16, len - 1);
      const int off = PAGED ? (key & ((1 << bs_shift) - 1)) : key;
      const long a = (long)bk[u] * s_blk + (long)off * s_tok + (long)hk * s_head + 8 * h;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        kk[u][c] = *reinterpret_cast<const bf16x8*>(kc + a + 32 * c);
        vv[u][c] = *reinterpret_cast<const bf16x8*>(vc + a + 32 * c);
      }
    }
  };
  // Issue order per iteration: block-table reads of tile t+8, then the K/V loads of tile t+4 (whose blocks were
  // read one iteration earlier, ahead of tile t's loads), then tile t's math — every wait is a counted vmcnt that
  // leaves the newer loads in flight; a table read placed right in front of its loads cost 20 % on paged caches.
  const int qq = c16 >> 2, pp = c16 & 3;   // transposed-read lane roles: row 4h+qq / 16+4h+qq, column group pp
  // one tile's math on the register set (kc_, vc_); the other set's loads stay in flight meanwhile
  auto compute = [&](int t, const bf16x8 (&kc_)[2][4], const bf16x8 (&vc_)[2][4]) {
  #pragma unroll
      for (int u = 0; u < 2; ++u)
  #pragma unroll
        for (int c = 0; c < 4; ++c) *reinterpret_cast<bf16x8*>(vl + voff(16 * u + c16, 4 * c + h)) = vc_[u][c];
      f32x4 s[2];
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        s[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
        for (int c = 0; c < 4; ++c) s[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kc_[u][c], qf[c], s[u], 0, 0, 0);
      }
      const int k0 = k_begin + 32 * t;
      float mt = -INFINITY;
  #pragma unroll
      for (int u = 0; u < 2; ++u)
  #pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = (k0 + 16 * u + 4 * h + e < k_end) ? s[u][e] * sl2 : -INFINITY;
          s[u][e] = v;
          mt = fmaxf(mt, v);
        }
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = exp2f(m - mn);
      m = mn;
      bf16x8 pf;
      float ps = 0.f;
  #pragma unroll
      for (int u = 0; u < 2; ++u)
  #pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = exp2f(s[u][e] - mn);
          ps += pv;
          pf[4 * u + e] = (__bf16)pv;
        }
      lsum = lsum * alpha + ps;
      float ar[4];
  #pragma unroll
      for (int e = 0; e < 4; ++e) ar[e] = __shfl(alpha, 4 * h + e, 64);   // O row g = 4h+e lives in lane column g
  #pragma unroll
      for (int tt = 0; tt < 8; ++tt)
  #pragma unroll
        for (int e = 0; e < 4; ++e) o[tt][e] *= ar[e];
  #pragma unroll
      for (int tt = 0; tt < 8; ++tt) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_char*)vl + voff(4 * h + qq, 2 * tt + (pp >> 1)) + 8 * (pp & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_char*)vl + voff(16 + 4 * h + qq, 2 * tt + (pp >> 1)) + 8 * (pp & 1)));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 vv8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vv8), o[tt], 0, 0, 0);
      }
  };
  // Two register sets in ping-pong, two tiles per trip and no exit between them: a copy at the loop end would
  // wait for the prefetch, a conditionally issued load makes the wait counting assume the worst at the join,
  // and with an exit between the halves the compiler sinks the second set's loads past it (behind the first
  // half's math).  So loads and table reads are unconditional, clamped to the wave's last tile (a re-read of
  // a tile just loaded hits L2), and an odd tile count ends with one fully masked tile (alpha = 1, p = 0).
  bf16x8 k2[2][4], v2[2][4];
  if (w < ntile) {
    const int last = w + 4 * ((ntile - 1 - w) / 4);
    int bn[2], b0[2];
    blocks(w, b0);
    blocks(min(w + 4, last), bn);
    load(w, b0, kr, vr);
    for (int t = w; t <= last; t += 8) {
      int bnn[2];
      blocks(min(t + 8, last), bnn);
      load(min(t + 4, last), bn, k2, v2);
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the math
      compute(t, kr, vr);
      blocks(min(t + 12, last), bn);
      load(min(t + 8, last), bnn, kr, vr);
      __builtin_amdgcn_sched_barrier(0);
      compute(t + 4, k2, v2);
    }
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  __syncthreads();   // every wave is done with its V image: reuse the LDS for the merge
  float* ow = reinterpret_cast<float*>(lds);                 // [4][16][HD]
  float* ml = reinterpret_cast<float*>(lds + kMfmaLds);      // [4][16][2]
  if (h == 0) {
    ml[(w * 16 + c16) * 2] = m;
    ml[(w * 16 + c16) * 2 + 1] = lsum;
  }
#pragma unroll
  for (int tt = 0; tt < 8; ++tt)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * h + e < G) ow[(w * 16 + 4 * h + e) * HD + 16 * tt + c16] = o[tt][e];
  __syncthreads();
  for (int i = tid; i < G * HD; i += 256) {
    const int g = i / HD, d = i % HD;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, ml[(ww * 16 + g) * 2]);
    float Lsum = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float wt = exp2f(ml[(ww * 16 + g) * 2] - M);
      Lsum += ml[(ww * 16 + g) * 2 + 1] * wt;
      acc += ow[(ww * 16 + g) * HD + d] * wt;
    }
    const int hq = hk * G + g;
    if (splits == 1) {
      out[(long)b * so_b + (long)hq * so_h + d].x = f2bf(Lsum > 0.f ? acc / Lsum : 0.f);
    } else {
      const long pi = (((long)b * Hq + hq) * splits + sp);
      part_o[pi * HD + d] = acc;
      if (d == 0) {
        part_ml[pi * 2] = M;
        part_ml[pi * 2 + 1] = Lsum;
      }
    }
  }
}

template <int HD>
__global__ __launch_bounds__(HD) void merge_kernel(const float* __restrict__ part_o,
                                                   const float* __restrict__ part_ml, bf16* __restrict__ out,
                                                   long so_b, long so_h, int Hq, int splits) {
  const int b = blockIdx.x, hq = blockIdx.y, d = threadIdx.x;
  const long p0 = ((long)b * Hq + hq) * splits;
  float M = -INFINITY;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, part_ml[(p0 + s) * 2]);
  float Lsum = 0.f, acc = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float ms = part_ml[(p0 + s) * 2];
    const float w = ms == -INFINITY ? 0.f : exp2f(ms - M);
    Lsum += part_ml[(p0 + s) * 2 + 1] * w;
    acc += part_o[(p0 + s) * HD + d] * w;
  }
  out[(long)b * so_b + (long)hq * so_h + d].x = f2bf(Lsum > 0.f ? acc / Lsum : 0.f);
}

// write the new tokens' k/v (rows of a [n_tok, Hk, HD] projection output) into the cache
__global__ __launch_bounds__(256) void cache_write_kernel(const bf16* __restrict__ k, const bf16* __restrict__ v,
                                                          long sk_tok, long sv_tok, bf16* __restrict__ kc,
                                                          bf16* __restrict__ vc, long s_blk, long s_tok, long s_head,
                                                          const int* __restrict__ block_table, int max_blocks,
                                                          int block_size, const int* __restrict__ tok_batch,
                                                          const int* __restrict__ tok_pos, int n_tok, int Hk, int HD) {
  const int chunks = HD / 8;
  const long total = (long)n_tok * Hk * chunks;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % chunks);
    const int h = (int)((i / chunks) % Hk);
    const int n = (int)(i / ((long)chunks * Hk));
    const int b = tok_batch[n], t = tok_pos[n];
    long blk = b;
    int off = t;
    if (block_table) {
      blk = block_table[(long)b * max_blocks + t / block_size];
      off = t % block_size;
    }
    const long dst = blk * s_blk + (long)off * s_tok + (long)h * s_head + c * 8;
    *reinterpret_cast<u16x8*>(kc + dst) = *reinterpret_cast<const u16x8*>(k + (long)n * sk_tok + h * HD + c * 8);
    *reinterpret_cast<u16x8*>(vc + dst) = *reinterpret_cast<const u16x8*>(v + (long)n * sv_tok + h * HD + c * 8);
  }
}

}  // namespace dec
}  // namespace pd

using namespace pd;

// impl: 0 = auto (MFMA for HD 128 and 2 <= G <= 16), 1 = vector path, 2 = MFMA path
extern "C" int pd_decode_attn(const void* q, long sq_b, long sq_h, const void* kc, const void* vc, long s_blk,
                              long s_tok, long s_head, const int* block_table, int max_blocks, int block_size,
                              const int* seq_lens, int max_len, float* part_o, float* part_ml, void* out, long so_b,
                              long so_h, int B, int Hq, int Hk, int HD, int splits, float scale, int impl,
                              void* stream) {
  if ((HD != 64 && HD != 128) || Hq % Hk) return -1;
  const int G = Hq / Hk;
  hipStream_t st = (hipStream_t)stream;
  if (splits < 1) splits = 1;
  const int chunk = (max_len + splits - 1) / splits;
  dim3 grid(Hk, B, splits);   // the Hk workgroups of one token row (paged: adjacent 256-B pieces) are co-resident
  const bool mfma_shape = HD == 128 && G <= 16 && ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(kc) |
                                                  reinterpret_cast<uintptr_t>(vc)) & 15) == 0 && (sq_h % 8) == 0 && (s_tok % 8) == 0 && (s_head % 8) == 0 &&
                       (s_blk % 8) == 0 && (sq_b % 8) == 0;
  int bs_shift = 0;
  while (block_table && (1 << bs_shift) < block_size) ++bs_shift;
  const bool mfma_ok = mfma_shape && (!block_table || (1 << bs_shift) == block_size);   // paged: pow-2 blocks
  if (impl == 2 && !mfma_ok) return -3;
  // auto: the MFMA kernel for grouped-query attention (2.0-2.9x the vector kernel at G = 4..16); MHA (G = 1)
  // stays on the vector kernel, which streams 256-B rows at a higher occupancy (5.37 vs 5.11 TB/s, paged
  // B64 L1088; profiles/r3_decode_attention.md)
  if (impl == 2 || (impl == 0 && mfma_ok && G >= 2)) {
#define PD_DECM2(GV, PG)                                                                                           \
  dec::decode_mfma_kernel<GV, PG><<<grid, 256, 0, st>>>((const bf16*)q, sq_b, sq_h, (const bf16*)kc,                \
                                                        (const bf16*)vc, s_blk, s_tok, s_head, block_table,           \
                                                        max_blocks, bs_shift, seq_lens, part_o, part_ml, (bf16*)out,  \
                                                        so_b, so_h, Hq, splits, chunk, scale)
#define PD_DECM(GV)          \
  if (block_table)           \
    PD_DECM2(GV, true);      \
  else                       \
    PD_DECM2(GV, false)
    switch (G) {
      case 1: PD_DECM(1); break;
      case 2: PD_DECM(2); break;
      case 4: PD_DECM(4); break;
      case 8: PD_DECM(8); break;
      case 16: PD_DECM(16); break;
      default: return -2;
    }
#undef PD_DECM
#undef PD_DECM2
    if (splits > 1) {
      dim3 mg(B, Hq);
      dec::merge_kernel<128><<<mg, 128, 0, st>>>(part_o, part_ml, (bf16*)out, so_b, so_h, Hq, splits);
    }
    return (int)hipGetLastError();
  }
#define PD_DEC(HDV, GV)                                                                                           \
  dec::decode_kernel<HDV, GV><<<grid, 256, 0, st>>>((const bf16*)q, sq_b, sq_h, (const bf16*)kc, (const bf16*)vc, \
                                                    s_blk, s_tok, s_head, block_table, max_blocks, block_size,       \
                                                    seq_lens, part_o, part_ml, (bf16*)out, so_b, so_h, Hq, Hk,       \
                                                    splits, chunk, scale)
#define PD_DEC_G(HDV)                              \
  switch (G) {                                     \
    case 1: PD_DEC(HDV, 1); break;                 \
    case 2: PD_DEC(HDV, 2); break;                 \
    case 4: PD_DEC(HDV, 4); break;                 \
    case 8: PD_DEC(HDV, 8); break;                 \
    default: return -2;                            \
  }
  if (HD == 128) { PD_DEC_G(128) } else { PD_DEC_G(64) }
#undef PD_DEC_G
#undef PD_DEC
  if (splits > 1) {
    dim3 mg(B, Hq);
    if (HD == 128) dec::merge_kernel<128><<<mg, 128, 0, st>>>(part_o, part_ml, (bf16*)out, so_b, so_h, Hq, splits);
    else dec::merge_kernel<64><<<mg, 64, 0, st>>>(part_o, part_ml, (bf16*)out, so_b, so_h, Hq, splits);
  }
  return (int)hipGetLastError();
}

extern "C" int pd_cache_write(const void* k, const void* v, long sk_tok, long sv_tok, void* kc, void* vc, long s_blk,
                              long s_tok, long s_head, const int* block_table, int max_blocks, int block_size,
                              const int* tok_batch, const int* tok_pos, int n_tok, int Hk, int HD, void* stream) {
  const long total = (long)n_tok * Hk * (HD / 8);
  long g = (total + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  dec::cache_write_kernel<<<(int)g, 256, 0, (hipStream_t)stream>>>(
      (const bf16*)k, (const bf16*)v, sk_tok, sv_tok, (bf16*)kc, (bf16*)vc, s_blk, s_tok, s_head, block_table,
      max_blocks, block_size, tok_batch, tok_pos, n_tok, Hk, HD);
  return (int)hipGetLastError();
}
