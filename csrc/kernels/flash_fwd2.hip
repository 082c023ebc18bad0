// The two-row-block flash forward (fwd_kernel<128, *, *, false, *, 4, 2>, see flash_attn.hip): its own translation
// unit so it can be built with the VGPR form of the MFMA instructions (-mllvm -amdgpu-mfma-vgpr-form, set for this
// file by paddle2_amd/_build.py).  The kernel pins its O accumulators to AGPRs itself; without the flag hipcc also
// homes the score accumulators in AGPRs and copies 64 of them to VGPRs for the softmax on every key tile.
#define PD_FA_DEVICE_ONLY
#include "flash_attn.hip"

namespace pd {
namespace fa {

void launch_fwd_rb2(bool f16, bool causal, int mode, dim3 grid, hipStream_t st, const void* q, const void* k,
                    const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv,
                    long so, float scale, const Ext& ex) {
#define PD_FA_RB2(FF, CC, MM)                                                                                       \
  fwd_kernel<128, CC, MM, false, FF, 4, 2><<<grid, 256, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,  \
                                                                 (bf16*)o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so,   \
                                                                 scale, ex)
#define PD_FA_RB2_M(FF, CC) \
  if (mode == 0) PD_FA_RB2(FF, CC, kDense); else PD_FA_RB2(FF, CC, kVarlen);
  if (f16) { if (causal) { PD_FA_RB2_M(true, true) } else { PD_FA_RB2_M(true, false) } }
  else { if (causal) { PD_FA_RB2_M(false, true) } else { PD_FA_RB2_M(false, false) } }
#undef PD_FA_RB2_M
#undef PD_FA_RB2
}


// =====================================================================================
// 16x16x32 forward (opt-in, PADDLE2_AMD_FA_FWD_MFMA=16): the RB = 1 structure (4 waves x 32 rows, 64-key tiles, the
// same register-staged K/V LDS images) on v_mfma_f32_16x16x32_bf16 instead of 32x32x16 — the shape the chip clocks
// higher under (profiles/r5_mfma_shape.md).  Swapped S^T = K.Q^T per (16-row query block qb, 16-key block kb):
// lane (g = lane >> 4, c = lane & 15) holds S^T[key kb*16 + 4g + i][query qb*16 + c], so a query's 64 scores of a tile
// sit in 4 lanes (c, c+16, c+32, c+48): the row max / sum take a permlane16 + permlane32 exchange.  P feeds the
// P.V MFMA as the B operand with a permuted k order — element j of lane group g is key 32ks + (j < 4 ? 4g + j :
// 16 + 4g + j - 4) — and the V^T A operand reads the same keys with two ds_read_b64_tr_b16 (rows 4g.. and 16 + 4g..).
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// max / sum over the 4 lanes that share lane & 15
__device__ __forceinline__ float quad_max(float v) {
  unsigned u = __builtin_bit_cast(unsigned, v);
  auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
  u = __builtin_bit_cast(unsigned, v);
  auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)b[0]), __builtin_bit_cast(float, (unsigned)b[1]));
}
__device__ __forceinline__ float quad_sum(float v) {
  unsigned u = __builtin_bit_cast(unsigned, v);
  auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __builtin_bit_cast(float, (unsigned)a[0]) + __builtin_bit_cast(float, (unsigned)a[1]);
  u = __builtin_bit_cast(unsigned, v);
  auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)b[0]) + __builtin_bit_cast(float, (unsigned)b[1]);
}

template <bool CAUSAL, int MODE, bool F16>
__global__ __launch_bounds__(256, 2) void fwd16_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                       const bf16* __restrict__ Vv, bf16* __restrict__ O,
                                                       float* __restrict__ LSE, int B, int SqMax, int SkMax, int Hq,
                                                       int Hk, long sq, long sk, long sv, long so, float scale, Ext ex) {
  constexpr int D = 128, BM = 128, BN = 64, NCH = D / 8, NT = 256;
  constexpr int TILE = BN * D * 2;
  constexpr int NLOAD = BN * NCH / NT;
  static_assert(MODE != kMask, "dense / varlen only");
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][K|V]

  const int nmb = (SqMax + BM - 1) / BM;
  const int total = nmb * Hq * B;
  const int w_id = xcd_remap(blockIdx.x, total);
  int mb = w_id % nmb;
  const int hq = (w_id / nmb) % Hq;
  const int b = w_id / (nmb * Hq);
  if (CAUSAL) mb = nmb - 1 - mb;
  const int hk = hq / (Hq / Hk);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int m0 = mb * BM;

  int Sq = SqMax, Sk = SkMax;
  long qt0 = (long)b * SqMax, kt0 = (long)b * SkMax;
  long lse0 = ((long)b * Hq + hq) * SqMax;
  if constexpr (MODE == kVarlen) {
    qt0 = ex.cu_q[b];
    kt0 = ex.cu_k[b];
    Sq = ex.cu_q[b + 1] - (int)qt0;
    Sk = ex.cu_k[b + 1] - (int)kt0;
    lse0 = (long)hq * ex.total_q + qt0;
    if (m0 >= Sq) return;
  }
  const int off = Sk - Sq;
  const bf16* Qb = Q + qt0 * sq + hq * D;
  const bf16* Kb = K + kt0 * sk + hk * D;
  const bf16* Vb = Vv + kt0 * sv + hk * D;

  // Q fragments (B operand): lane holds Q[q = m0 + 32 wv + 16 qb + c16][d = 32 ds + 8 g .. + 8]
  int qrow[2];
  bf16x8 qf[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    qrow[qb] = m0 + wv * 32 + qb * 16 + c16;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      if (qrow[qb] < Sq) qf[qb][ds] = *reinterpret_cast<const bf16x8*>(Qb + (long)qrow[qb] * sq + ds * 32 + 8 * g);
      else qf[qb][ds] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) asm volatile("" ::"v"(qf[qb][ds]));

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + BM + off);
  const int ntiles = n_end > 0 ? (n_end + BN - 1) / BN : 0;

  u16x8 stk[NLOAD], stv[NLOAD];
  int voff_k[NLOAD], voff_v[NLOAD];
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) {
    const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
    voff_k[i] = row * (int)sk * 2 + ch * 16;
    voff_v[i] = row * (int)sv * 2 + ch * 16;
  }
  auto gload = [&](int n0) {
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
#pragma unroll
    for (int i = 0; i < NLOAD; ++i) {
      const int c = tid + NT * i, row = c / NCH, ch = c % NCH;
      const int o = row * (D * 2) + swz(row, ch, NCH) * 16;
      *reinterpret_cast<u16x8*>(kt + o) = stk[i];
      *reinterpret_cast<u16x8*>(vt + o) = stv[i];
    }
  };

  f32x4 oacc[2][8];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int db = 0; db < 8; ++db) oacc[qb][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_i[2] = {-INFINITY, -INFINITY}, l_i[2] = {0.f, 0.f};
  const float sl2 = scale * kLog2e;

  if (0 < ntiles) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  const int wave_last_key = m0 + wv * 32 + 31 + off;

  // lane LDS bases.  K row read (key row 16 kb + c16, chunk 4 ds + g): the swizzle term of rows 16 kb + c16 is
  // mm(c16), and chunk (4 ds) ^ (g ^ mm) -> o_k ^ (ds << 6).  V^T tr read (lane c16 = 4 q + p: row 32 ks + 16 hh +
  // 4 g + q, columns 16 db + 4 p): chunk (2 db) ^ ((p >> 1) ^ mm(4 g + q)) -> o_v ^ (db << 5)
  auto mm = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
  int o_k = c16 * (D * 2) + (((g ^ mm(c16)) & (NCH - 1)) << 4);
  int o_v;
  {
    const int q = c16 >> 2, p = c16 & 3, rr = 4 * g + q;
    o_v = rr * (D * 2) + ((((p >> 1) ^ mm(rr)) & (NCH - 1)) << 4) + ((p & 1) << 3);
  }

  // one body for every tile (two compile-time bodies made the register allocator disagree on the accumulators'
  // homes at the join: ~390 B/lane of spills); the boundary / diagonal mask is a real, uniform branch
  auto tile = [&](bool masked, int BUF, int n0, bool has_next, int tn) {
    const char* kt = smem + BUF * 2 * TILE;
    const char* vt = kt + TILE;
    asm volatile("" : "+v"(o_k), "+v"(o_v));
    f32x4 s[2][4];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) s[qb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const bf16x8 a = lds_b128(kt + kb * 16 * (D * 2), o_k ^ (ds << 6));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) s[qb][kb] = mfma16<F16>(a, qf[qb][ds], s[qb][kb]);
      }
    }
    if (has_next) gload(tn * BN);
    if (masked) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        int lim = Sk - n0 - 4 * g;
        if constexpr (CAUSAL) lim = min(lim, qrow[qb] + off - n0 - 4 * g + 1);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int i = 0; i < 4; ++i) s[qb][kb][i] = (kb * 16 + i) >= lim ? -INFINITY : s[qb][kb][i];
      }
    }
    float m_cand[2];
    bool grow = false;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float mxa[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        mxa[kb] = fmaxf(fmaxf(s[qb][kb][0], s[qb][kb][1]), fmaxf(s[qb][kb][2], s[qb][kb][3]));
      const float mx = quad_max(fmaxf(fmaxf(mxa[0], mxa[1]), fmaxf(mxa[2], mxa[3])));
      m_cand[qb] = fmaxf(m_i[qb], mx * sl2);
      grow = grow || (m_cand[qb] > m_i[qb] + kDefer);
    }
    if (__builtin_expect(__any(grow), 0)) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float alpha = __builtin_amdgcn_exp2f(m_i[qb] - (m_cand[qb] == -INFINITY ? 0.f : m_cand[qb]));
        l_i[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < 8; ++db) oacc[qb][db] *= alpha;
        m_i[qb] = m_cand[qb];
      }
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const float base = m_i[qb] == -INFINITY ? 0.f : m_i[qb];
      float lsa[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(s[qb][kb][i], sl2, -base));
          s[qb][kb][i] = pv;
          lsa[kb] += pv;
        }
      l_i[qb] += (lsa[0] + lsa[1]) + (lsa[2] + lsa[3]);
    }
    // ---- O^T += V^T . P^T: k-step ks covers keys 32 ks .. 32 ks + 31 (permuted order, see above)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        if constexpr (F16) {
          f16x8 r;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            r[j] = (_Float16)s[qb][2 * ks][j];
            r[4 + j] = (_Float16)s[qb][2 * ks + 1][j];
          }
          pb[qb] = __builtin_bit_cast(bf16x8, r);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pb[qb][j] = (__bf16)s[qb][2 * ks][j];
            pb[qb][4 + j] = (__bf16)s[qb][2 * ks + 1][j];
          }
        }
      }
      const char* v0 = vt + (32 * ks) * (D * 2);
      const char* v1 = vt + (32 * ks + 16) * (D * 2);
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        const bf16x8 a = cat4(lds_tr(v0, o_v ^ (db << 5)), lds_tr(v1, o_v ^ (db << 5)));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) oacc[qb][db] = mfma16<F16>(a, pb[qb], oacc[qb][db]);
      }
    }
    if (has_next) lstore(BUF ^ 1);
    __syncthreads();
  };

  int t = 0;
  for (int buf = 0; t < ntiles; buf ^= 1) {
    const int n0 = t * BN;
    const int tn = t + 1;
    const bool has_next = tn < ntiles;
    if (CAUSAL && n0 > wave_last_key) {
      if (has_next) {
        gload(tn * BN);
        lstore(buf ^ 1);
      }
      __syncthreads();
      t = tn;
      continue;
    }
    const bool masked = (n0 + BN > Sk) || (CAUSAL && (n0 + BN - 1 > m0 + off));
    tile(masked, buf, n0, has_next, tn);
    t = tn;
  }

  // ---- epilogue: lane (g, c16) holds O^T[d = 16 db + 4 g + i][q] -> 4 consecutive d (8 B) per d block
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const float l_tot = quad_sum(l_i[qb]);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (qrow[qb] < Sq) {
      bf16* orow = O + (qt0 + qrow[qb]) * so + hq * D;
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        ushort4 v;
        v.x = cvt16<F16>(oacc[qb][db][0] * inv);
        v.y = cvt16<F16>(oacc[qb][db][1] * inv);
        v.z = cvt16<F16>(oacc[qb][db][2] * inv);
        v.w = cvt16<F16>(oacc[qb][db][3] * inv);
        *reinterpret_cast<ushort4*>(orow + 16 * db + 4 * g) = v;
      }
      if (g == 0) LSE[lse0 + qrow[qb]] = l_tot > 0.f ? (m_i[qb] + log2f(l_tot)) * kLn2 : INFINITY;
    }
  }
}

void launch_fwd_m16(bool f16, bool causal, int mode, dim3 grid, hipStream_t st, const void* q, const void* k,
                    const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv,
                    long so, float scale, const Ext& ex) {
#define PD_FA_M16(FF, CC, MM)                                                                                       \
  fwd16_kernel<CC, MM, FF><<<grid, 256, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, B,  \
                                                 Sq, Sk, Hq, Hk, sq, sk, sv, so, scale, ex)
#define PD_FA_M16_M(FF, CC) \
  if (mode == 0) PD_FA_M16(FF, CC, kDense); else PD_FA_M16(FF, CC, kVarlen);
  if (f16) { if (causal) { PD_FA_M16_M(true, true) } else { PD_FA_M16_M(true, false) } }
  else { if (causal) { PD_FA_M16_M(false, true) } else { PD_FA_M16_M(false, false) } }
#undef PD_FA_M16_M
#undef PD_FA_M16
}

}  // namespace fa
}  // namespace pd
