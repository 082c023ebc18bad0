// MFMA shape study for the bf16 GEMM wave tile (round 5): v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 on
// the GEMM's 128 x 128 wave tile, one wave per SIMD (256-thread workgroups, one per CU), every operand re-read from
// LDS by ds_read_b128 each k32 step (the GEMM's LDS read volume: 16 reads per k32 step), random bf16 operands.
// Both forms do the same FLOPs with the same LDS bytes: 64 x 16x16x32 or 32 x 32x32x16 MFMAs per k32 step.
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_shape scripts/mfma_shape.hip
// Output: one JSON line per shape (TF/s over ~1 s of back-to-back launches, effective in-kernel clock).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;   // k32 steps per launch

// LDS image: 16 KiB of random bf16 per wave (A 128 x 32, B 128 x 32 rows of 64 B)
template <int SHAPE>
__global__ __launch_bounds__(256, 1) void mfma_loop(const uint4* __restrict__ src, float* __restrict__ out,
                                                    long long* __restrict__ clk) {
  __shared__ uint4 lds[4 * 1024];   // 64 KiB: 16 KiB per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * 1024; i += 256) lds[i] = src[(blockIdx.x * 4096 + i) & 0xffff];
  __syncthreads();
  const char* base = (const char*)lds + wave * 16384;
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (SHAPE == 16) {
    f32x4 acc[8][8];
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one contiguous 1-KiB fragment per read (conflict-free for both shapes; the operand values are random either way)
    const int off = lane * 16;
    for (int it = 0; it < ITERS; ++it) {
      bf16x8 a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = *(const bf16x8*)(base + ((u * 1024 + off + it * 16) & 8191));
        b[u] = *(const bf16x8*)(base + 8192 + ((u * 1024 + off + it * 16) & 8191));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    f32x16 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
    const int off = lane * 16;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = *(const bf16x8*)(base + ((u * 2048 + s * 1024 + off + it * 16) & 8191));
          b[u] = *(const bf16x8*)(base + 8192 + ((u * 2048 + s * 1024 + off + it * 16) & 8191));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j)
        for (int e = 0; e < 16; ++e) s += acc[i][j][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int SHAPE>
void run(int cus, const uint4* src, float* out, long long* clk) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 250; ++w) mfma_loop<SHAPE><<<cus, 256>>>(src, out, clk);   // ~0.5 s warm (DVFS settles)
  hipEventRecord(e0);
  const int reps = 250;
  for (int r = 0; r < reps; ++r) mfma_loop<SHAPE><<<cus, 256>>>(src, out, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(2 * cus);
  hipMemcpy(h.data(), clk, 2 * cus * sizeof(long long), hipMemcpyDeviceToHost);
  double ghz = 0.0;
  for (int i = 0; i < cus; ++i) ghz += (double)h[2 * i] / ((double)h[2 * i + 1] * 10.0);   // realtime = 100 MHz
  ghz /= cus;
  const double flops = (double)reps * cus * 4.0 * ITERS * 128.0 * 128.0 * 32.0 * 2.0;
  printf("{\"mfma\": \"%s\", \"wave_tile\": \"128x128\", \"ms\": %.3f, \"TFs\": %.1f, \"clock_GHz\": %.3f, "
         "\"cyc_per_k32_step\": %.1f}\n",
         SHAPE == 16 ? "16x16x32_bf16" : "32x32x16_bf16", ms, flops / (ms * 1e-3) / 1e12, ghz,
         (double)h[0] / ITERS);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  std::vector<unsigned short> host(65536 * 8);
  unsigned x = 12345u;
  for (auto& v : host) {
    x = x * 1664525u + 1013904223u;
    // random bf16 in about [-2, 2]: sign, exponent 126..128, random mantissa
    v = (unsigned short)(((x >> 31) << 15) | ((126u + (x >> 8) % 3u) << 7) | ((x >> 12) & 0x7f));
  }
  uint4* src;
  float* out;
  long long* clk;
  hipMalloc(&src, host.size() * 2);
  hipMalloc(&out, cus * 256 * sizeof(float));
  hipMalloc(&clk, 2 * cus * sizeof(long long));
  hipMemcpy(src, host.data(), host.size() * 2, hipMemcpyHostToDevice);
  for (int round = 0; round < 2; ++round) {
    run<16>(cus, src, out, clk);
    run<32>(cus, src, out, clk);
  }
  hipFree(src);
  hipFree(out);
  hipFree(clk);
  return 0;
}
