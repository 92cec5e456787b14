// v_mfma_f32_32x32x2f32 throughput on RANDOM operands (8 distinct random A/B values per lane,
// cycled, so the multiplier inputs toggle like a real GEMM's) vs constant operands, with the
// in-kernel shader clock (s_memtime / s_memrealtime at 100 MHz) -- the practical fp32 MFMA ceiling
// under the chip's DVFS (MI355X_MICROARCH.md, 'DVFS give-back').
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_peak_rand tools/mfma_peak_rand.hip && /tmp/mfma_peak_rand
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>   // 0: one constant A/B register pair (as tools/mfma_peak.hip), 1: 8 constant pairs cycled, 2: 8 random pairs cycled
__global__ __launch_bounds__(256) void peak(const float* __restrict__ src, float* out, long long* clk, int iters) {
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a[8], b[8];
  for (int s = 0; s < 8; ++s) {
    a[s] = MODE == 2 ? src[(blockIdx.x * 256 + threadIdx.x) * 16 + s] : 0.5f + threadIdx.x * 1e-3f + (MODE ? s * 1e-2f : 0.f);
    b[s] = MODE == 2 ? src[(blockIdx.x * 256 + threadIdx.x) * 16 + 8 + s] : 0.25f - threadIdx.x * 1e-3f + (MODE ? s * 1e-2f : 0.f);
  }
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = MODE == 0 ? __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], b[0], acc[i], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[(s + i) & 7], acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float v = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) v += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = v;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024, iters = 4000;
  float *out, *src;
  long long* clk;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&src, blocks * 256 * 16 * 4);
  hipMalloc(&clk, blocks * 2 * 8);
  float* h = (float*)malloc(blocks * 256 * 16 * 4);
  srand(1);
  for (long i = 0; i < blocks * 256L * 16; ++i) h[i] = (float)rand() / RAND_MAX * 2.f - 1.f;
  hipMemcpy(src, h, blocks * 256 * 16 * 4, hipMemcpyHostToDevice);
  long long* hc = (long long*)malloc(blocks * 2 * 8);
  for (int mode = 0; mode < 3; ++mode) {
    auto k = mode == 0 ? peak<0> : mode == 1 ? peak<1> : peak<2>;
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, src, out, clk, iters);  // >= 2 s warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, src, out, clk, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(hc, clk, blocks * 2 * 8, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int b = 0; b < blocks; ++b) ghz += (double)hc[2 * b] / hc[2 * b + 1] * 0.1;
    ghz /= blocks;
    const double flop = 5.0 * blocks * 4 * (double)iters * 8 * 4 * 32 * 32 * 2 * 2;
    printf("blocks %5d  %-22s %.1f TF/s  in-kernel clock %.2f GHz  (=> %.1f TF/s at 2.4 GHz)\n", blocks,
           mode == 0 ? "1 constant pair" : mode == 1 ? "8 constant pairs" : "8 random pairs",
           flop / (ms * 1e-3) / 1e12, ghz, flop / (ms * 1e-3) / 1e12 * 2.4 / ghz);
  }
  return 0;
}
