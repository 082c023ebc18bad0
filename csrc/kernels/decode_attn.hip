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
  const int b = blockIdx.x, hk = blockIdx.y, sp = blockIdx.z;
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

extern "C" int pd_decode_attn(const void* q, long sq_b, long sq_h, const void* kc, const void* vc, long s_blk,
                              long s_tok, long s_head, const int* block_table, int max_blocks, int block_size,
                              const int* seq_lens, int max_len, float* part_o, float* part_ml, void* out, long so_b,
                              long so_h, int B, int Hq, int Hk, int HD, int splits, float scale, void* stream) {
  if ((HD != 64 && HD != 128) || Hq % Hk) return -1;
  const int G = Hq / Hk;
  hipStream_t st = (hipStream_t)stream;
  if (splits < 1) splits = 1;
  const int chunk = (max_len + splits - 1) / splits;
  dim3 grid(B, Hk, splits);
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
