// The practical ceiling of the split6 pipe: bare bf16 MFMA loops (v_mfma_f32_32x32x16_bf16 and
// v_mfma_f32_16x16x32_bf16) on RANDOM operands (4 distinct random bf16x8 A/B registers per lane,
// cycled so the multiplier inputs toggle like a GEMM's) vs all-zero operands, at 1..4 waves per SIMD
// (1..4 resident 256-thread blocks per CU), with the in-kernel shader clock (s_memtime against
// s_memrealtime at 100 MHz) -- what the chip sustains under its DVFS (MI355X_MICROARCH.md "DVFS
// give-back") against the 2.5 PF spec.  Each configuration: 20 warm-up launches, then 10 timed.
// Prints TF/s of bf16 MFMA work and the split6 fp32-equivalent (/ 6).
//   hipcc -O3 --offload-arch=gfx950 -o tools/variants/mfma_peak_bf16 tools/mfma_peak_bf16.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <bool M32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void peak(const unsigned short* __restrict__ src, float* out, long long* clk,
                                            int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  bf16x8 a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = *reinterpret_cast<const bf16x8*>(src + (gid * 16 + s) * 8);
    b[s] = *reinterpret_cast<const bf16x8*>(src + (gid * 16 + 8 + s) * 8);
  }
  f32x16 acc[4] = {};
  f32x4 acc4[4] = {};
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  // six products per accumulator per step (the split6 pattern), register indices static
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (M32)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s & 3], b[(s + i) & 3], acc[i], 0, 0, 0);
        else
          acc4[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s & 3], b[(s + i) & 3], acc4[i], 0, 0, 0);
      }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (M32) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v += acc[i][r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) v += acc4[i][r];
    }
  }
  out[gid] = v;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <bool M32>
void run(int per_cu, bool random, int cus) {
  const int blocks = per_cu * cus, iters = M32 ? 24000 : 48000;   // ~10 ms per launch per wave/SIMD
  unsigned short* src;
  float* out;
  long long* clk;
  const size_t n = (size_t)blocks * 256 * 16 * 8;
  hipMalloc(&src, n * 2);
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&clk, (size_t)blocks * 16);
  std::vector<unsigned short> h(n);
  srand(7);
  for (size_t i = 0; i < n; ++i) {
    const float f = random ? (float)rand() / RAND_MAX * 2.f - 1.f : 0.f;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  hipMemcpy(src, h.data(), n * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(peak<M32>, dim3(blocks), dim3(256), 0, 0, src, out, clk, iters);
  const int reps = 10;
  hipEventRecord(e0);
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(peak<M32>, dim3(blocks), dim3(256), 0, 0, src, out, clk, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(2 * blocks);
  hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> ghz;
  for (int b = 0; b < blocks; ++b)
    if (c[2 * b + 1] > 0) ghz.push_back((double)c[2 * b] / c[2 * b + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  const double flop_per_mfma = M32 ? 32.0 * 32 * 16 * 2 : 16.0 * 16 * 32 * 2;
  const double flop = (double)blocks * 4 /*waves*/ * iters * 24 * flop_per_mfma * reps;
  const double tf = flop / (ms * 1e-3) / 1e12;
  printf("%s %d waves/SIMD %-6s  %8.1f TF/s bf16  = split6 %6.1f TF/s  in-kernel clock %.2f GHz (median)\n",
         M32 ? "32x32x16" : "16x16x32", per_cu, random ? "random" : "zero", tf, tf / 6, ghz[ghz.size() / 2]);
  hipFree(src);
  hipFree(out);
  hipFree(clk);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  for (int r = 1; r >= 0; --r)
    for (int w = 1; w <= 4; ++w) {
      run<true>(w, r, cus);
      run<false>(w, r, cus);
    }
  return 0;
}
