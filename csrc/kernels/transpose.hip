// 2-D transpose of 16-bit matrices (bf16 / fp16) for gfx950: out[N, M] = in[M, N].
//
// Why it exists: hipBLASLt on MI355X runs the "both operands contiguous along the reduction dim" GEMM
// layout 15-40 % faster than the layouts with an MN-major operand (measured on the Llama-2-7B training
// GEMMs, profiles/r1_gemm_layouts.md).  Paddle's Linear stores W as [in, out], so the forward GEMM and
// the weight-gradient GEMM (reduction over tokens) both have an MN-major operand; transposing W (fwd) or
// X / dY (dW) at HBM speed first turns them into the fast layout (paddle2_amd.ops.torch_ops.linear).
//
// Design: one workgroup (256 lanes) moves a 128 x 64 tile.  Every global access is 16 B per lane and
// every wave-instruction covers whole runs (8 x 128-B input rows, 4 x 256-B output rows); the tile is
// staged through an XOR-swizzled LDS image; the grid is a 1-D tile walk (gridDim capped, grid-stride) so
// the launch is >> 256 workgroups on the big activations and still bounded for small weights.
#include "common.h"

namespace pd {

constexpr int TR_TM = 128;  // input rows per tile
constexpr int TR_TN = 64;   // input cols per tile

__global__ __launch_bounds__(256) void transpose16_kernel(const unsigned short* __restrict__ in,
                                                          unsigned short* __restrict__ out, long M, long N,
                                                          long ld_in, long ld_out, long tiles_n, long ntiles) {
  // [128 rows][64 cols] image, 16-B chunks XOR-swizzled by row group: element (r, c) lives at chunk
  // (c / 8) ^ ((r / 8) & 7) of row r, so the column gathers of the store phase (16 row groups x 4 columns
  // per wave) spread over 8 chunk positions (<= 2-way bank conflicts) while every row stays a 128-B run.
  __shared__ __attribute__((aligned(16))) unsigned short tile[TR_TM][TR_TN];
  const int tid = threadIdx.x;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long r0 = (t / tiles_n) * TR_TM;
    const long c0 = (t % tiles_n) * TR_TN;
    // load: 128 rows x 8 chunks of 8 elements = 1024 chunks, 4 per lane (8 lanes = one 128-B row run)
    u16x8 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = tid + 256 * i;
      const int r = ch >> 3, c = (ch & 7) * 8;
      const long gr = r0 + r, gc = c0 + c;
      v[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (gr < M && gc + 8 <= N) {
        v[i] = *reinterpret_cast<const u16x8*>(in + gr * ld_in + gc);
      } else if (gr < M) {
        for (int j = 0; j < 8; ++j) v[i][j] = gc + j < N ? in[gr * ld_in + gc + j] : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = tid + 256 * i;
      const int r = ch >> 3, c8 = ch & 7;
      *reinterpret_cast<u16x8*>(&tile[r][(c8 ^ ((r >> 3) & 7)) * 8]) = v[i];
    }
    __syncthreads();
    // store: 64 out rows (input cols) x 16 chunks of 8 input rows; a wave writes 4 out rows x 256 B runs
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = tid + 256 * i;
      const int oc = ch >> 4, g = ch & 15;  // out row = input col oc; out cols = input rows 8g..8g+8
      const long gor = c0 + oc, goc = r0 + 8 * g;
      const int col = (((oc >> 3) ^ (g & 7)) << 3) | (oc & 7);
      u16x8 w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = tile[8 * g + j][col];
      if (gor < N) {
        if (goc + 8 <= M) {
          *reinterpret_cast<u16x8*>(out + gor * ld_out + goc) = w;
        } else {
          for (int j = 0; j < 8; ++j)
            if (goc + j < M) out[gor * ld_out + goc + j] = w[j];
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace pd

using namespace pd;

// in: [M, N] with row stride ld_in (elements, multiple of 8 for the vector path), out: [N, M] row stride ld_out.
extern "C" int pd_transpose16(const void* in, void* out, long M, long N, long ld_in, long ld_out, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if ((ld_in % 8) || (ld_out % 8) || ((uintptr_t)in % 16) || ((uintptr_t)out % 16)) return -1;
  const long tiles_n = (N + TR_TN - 1) / TR_TN;
  const long ntiles = ((M + TR_TM - 1) / TR_TM) * tiles_n;
  long grid = ntiles < 256L * 16 ? ntiles : 256L * 16;
  transpose16_kernel<<<(int)grid, 256, 0, (hipStream_t)stream>>>((const unsigned short*)in, (unsigned short*)out, M,
                                                                   N, ld_in, ld_out, tiles_n, ntiles);
  return (int)hipGetLastError();
}
