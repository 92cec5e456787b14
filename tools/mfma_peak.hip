// Bare v_mfma_f32_32x32x2f32 throughput (operands in registers, 4 independent accumulators per
// wave): the ceiling the conv GEMM kernels are measured against.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_peak tools/mfma_peak.hip && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void peak(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a = a0 + threadIdx.x * 1e-3f, b = b0 - threadIdx.x * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float v = 0.f;
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) v += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 256 * 4);
  const int iters = 2000;
  for (int blocks : {256, 512, 1024}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(peak<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f, 0.25f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(peak<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f, 0.25f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 5.0 * blocks * 4 /*waves*/ * (double)iters * 8 * 4 * 32 * 32 * 2 * 2;
    printf("blocks %5d: %.1f TF/s\n", blocks, flop / (ms * 1e-3) / 1e12);
  }
  return 0;
}
