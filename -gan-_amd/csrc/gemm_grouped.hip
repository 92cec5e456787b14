// Grouped small GEMMs for the generator's style bank (gfx950, fp32 MFMA).
//
// G13_5 has 519 weight-modulated convs; each owns a style MLP and a demodulation product
// (generator_13_5.py:223-227,239-242).  Their per-conv matrices differ in shape, so instead of
// 519 launches per stage the bank runs ONE launch over a static list of 64x64 output tiles, each
// tile described by (operand offsets, leading dims, K, rows, cols, per-tile scale).  A tile never
// straddles two groups, so every tile is a plain small GEMM on MFMA 32x32x2.
//
//   C[r][n] (=|+=) epi( sum_k A(r,k) * B(k,n) )
//   A(r,k) = A_T ? A[a_off + k*lda + r] : A[a_off + r*lda + k]
//   B(k,n) = B_T ? B[b_off + n*ldb + k] : B[b_off + k*ldb + n]     (optionally squared)
//   epi:  0 store | 1 + bias[r] | 2 demod rsqrt(scale^2 * acc + 1e-8) | 3 accumulate (C += acc)
//         | 4 scale * acc

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ganamd.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int kThreads = 256;
constexpr int TB = 64;       // tile rows = tile cols
constexpr int BK = 16;
constexpr int LDK = BK + 2;  // [row][k] LDS images, conflict-free ds_read_b64

__device__ __forceinline__ void read_frag(const float* __restrict__ base, float (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 t = *reinterpret_cast<const f32x2*>(base + 2 * q);
    v[2 * q] = t[0];
    v[2 * q + 1] = t[1];
  }
}

template <bool A_T, bool B_T>
__global__ __launch_bounds__(kThreads) void grouped_gemm_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                                float* __restrict__ C, const float* __restrict__ bias,
                                                                const ganamd_gtile* __restrict__ tiles, int b_square) {
  __shared__ __attribute__((aligned(16))) float As[TB * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[TB * LDK];
  const ganamd_gtile t = tiles[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;   // 2 x 2 waves of 32 x 32
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  for (int k0 = 0; k0 < t.K; k0 += BK) {
    // A tile: TB rows x BK k
#pragma unroll
    for (int e = 0; e < TB * BK / kThreads; ++e) {
      int r, k;
      if (A_T) {   // r contiguous in memory
        r = tid % TB;
        k = tid / TB + e * (kThreads / TB);
      } else {     // k contiguous
        k = tid % BK;
        r = tid / BK + e * (kThreads / BK);
      }
      const bool ok = r < t.rows && k0 + k < t.K;
      const long off = A_T ? (long)t.a_off + (long)(k0 + k) * t.lda + r : (long)t.a_off + (long)r * t.lda + k0 + k;
      As[r * LDK + k] = ok ? A[off] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < TB * BK / kThreads; ++e) {
      int n, k;
      if (B_T) {   // k contiguous
        k = tid % BK;
        n = tid / BK + e * (kThreads / BK);
      } else {     // n contiguous
        n = tid % TB;
        k = tid / TB + e * (kThreads / TB);
      }
      const bool ok = n < t.cols && k0 + k < t.K;
      const long off = B_T ? (long)t.b_off + (long)n * t.ldb + k0 + k : (long)t.b_off + (long)(k0 + k) * t.ldb + n;
      float v = ok ? Bm[off] : 0.f;
      if (b_square) v *= v;
      Bs[n * LDK + k] = v;
    }
    __syncthreads();
    const int r = lane & 31, h = lane >> 5;
    float a[8], b[8];
    read_frag(As + (wm * 32 + r) * LDK + 8 * h, a);
    read_frag(Bs + (wn * 32 + r) * LDK + 8 * h, b);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    __syncthreads();
  }

  const int n = wn * 32 + (lane & 31);
  if (n >= t.cols) return;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
    if (r >= t.rows) continue;
    float v = acc[q];
    float* dst = C + (long)t.c_off + (long)r * t.ldc + n;
    switch (t.epi) {
      case GANAMD_EPI_BIAS: *dst = t.scale * v + bias[t.bias_off + r]; break;
      case GANAMD_EPI_DEMOD: *dst = 1.0f / sqrtf(t.scale * t.scale * v + 1e-8f); break;
      case GANAMD_EPI_ACCUM: *dst += t.scale * v; break;
      case GANAMD_EPI_SCALE: *dst = t.scale * v; break;
      default: *dst = v;
    }
  }
}

}  // namespace

extern "C" int ganamd_grouped_gemm(const float* A, const float* B, float* C, const float* bias,
                                   const ganamd_gtile* tiles, int n_tiles, int a_trans, int b_trans, int b_square,
                                   hipStream_t stream) {
  if (!A || !B || !C || !tiles || n_tiles <= 0) return GANAMD_EINVAL;
  const dim3 g(n_tiles), bl(kThreads);
  if (a_trans && b_trans)
    hipLaunchKernelGGL((grouped_gemm_kernel<true, true>), g, bl, 0, stream, A, B, C, bias, tiles, b_square);
  else if (a_trans)
    hipLaunchKernelGGL((grouped_gemm_kernel<true, false>), g, bl, 0, stream, A, B, C, bias, tiles, b_square);
  else if (b_trans)
    hipLaunchKernelGGL((grouped_gemm_kernel<false, true>), g, bl, 0, stream, A, B, C, bias, tiles, b_square);
  else
    hipLaunchKernelGGL((grouped_gemm_kernel<false, false>), g, bl, 0, stream, A, B, C, bias, tiles, b_square);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}
