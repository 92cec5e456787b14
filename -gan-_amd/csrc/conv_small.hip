// Direct convolution for convs with at most four output channels: ToRGB's 5x5 conv to RGB
// (generator_13_5.py:470-493, Cout = 3, Cin 108..396, maps 4..64) -- on the vector ALU in exact
// fp32, not on the matrix cores.
//
// Why: as an implicit GEMM this conv has M = 3 rows.  A 16-row MFMA tile computes 13 rows of
// zeros; the gather GEMM ran it at ~10 TF/s (1.8 ms per B = 256 launch at 64x64).  Here every
// thread owns PX = 2 adjacent output pixels of one row and all M outputs: per input channel and
// kernel row it reads PX + K - 1 staged inputs from LDS and issues M * K * PX fused multiply-adds
// whose weight operand is a wave-uniform value (a scalar load: all lanes use the same weight).
// Work per pixel is M * Cin * K^2 FMAs, the algorithmic count; the accumulation order per output
// is channel, kernel row, kernel column (one fp32 accumulator, as a sequential fp32 convolution).
//
// Block: 256 threads, TH = 8 output rows x the full width W = 64 of one image (32 threads per row);
// per chunk of CC input channels the (TH + K - 1) x (W + K - 1) input patch (replication-clamped or
// zero padded, scaled by x_scale[c][b]) is staged in LDS (double-buffered), then consumed.  Epilogue in the gather
// GEMM's order: alpha, * y_scale[m][b], + bias[m], PReLU(act[m]).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "patch.h"

namespace ganamd_small {
namespace {

constexpr int kNT = 256, PX = 2, CC = 8, WMAP = 64;

// (W = 64: 32 threads per output row, TH = 8 rows per block; the block's patch per chunk is
// CC x (TH + K - 1) x (W + K - 1) floats, double-buffered: chunk c + 1 is fetched into registers
// while chunk c is consumed, and stored after it)
template <int M, int K>
__global__ __launch_bounds__(kNT) void conv_small_kernel(Args p) {
  constexpr int W = WMAP, TPR = W / PX, TH = kNT / TPR, PWD = W + K - 1, PHT = TH + K - 1;
  constexpr int NPOS = PHT * PWD, NE = CC * NPOS, EPT = (NE + kNT - 1) / kNT;
  __shared__ float patch[2][NE];
  const int H = p.H, HW = H * W;
  const int tiles = H / TH;
  const int b = blockIdx.x / tiles, oh0 = (blockIdx.x - b * tiles) * TH;
  const int tid = threadIdx.x;
  const int r = tid / TPR, c0 = (tid - r * TPR) * PX;
  const long L = (long)p.B * HW;
  const int pad = p.pad, nch = (p.C + CC - 1) / CC;

  float acc[M][PX];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int q = 0; q < PX; ++q) acc[m][q] = 0.f;

  // staging element e = (cl, pr, pc), pc fastest: its source offset is fixed up to the chunk's
  // channel base, so it is computed once (zero padding and elements past the patch: an
  // out-of-range buffer offset, which the hardware returns as 0; channels past C fall off the end of
  // the buffer the same way)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0,
                                                                      (int)(4 * p.C * L), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x_scale ? p.x_scale : p.x), (short)0, p.x_scale ? 4 * p.C * p.B : 0, 0x00020000);
  constexpr int kOOB = (int)0x80000000;
  int off[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + i * kNT;
    const int cl = e / NPOS, pos = e - cl * NPOS, pr = pos / PWD, pc = pos - pr * PWD;
    int ih = oh0 - pad + pr, iw = pc - pad;
    bool in = e < NE;
    if (p.replicate) {
      ih = min(max(ih, 0), H - 1);
      iw = min(max(iw, 0), W - 1);
    } else {
      in = in && ih >= 0 && ih < H && iw >= 0 && iw < W;
    }
    off[i] = in ? 4 * (int)(cl * L + (long)b * HW + ih * W + iw) : kOOB;
  }
  const int cstep = 4 * (int)L;                  // bytes per input channel
  auto fetch = [&](int cb, float (&v)[EPT]) {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      int o = off[i] == kOOB ? kOOB : off[i] + cb * cstep;
      asm("" : "+v"(o));
      v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, o, 0, 0));
    }
    if (p.x_scale) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int cl = (tid + i * kNT) / NPOS;
        int o = 4 * ((cb + cl) * p.B + b);
        asm("" : "+v"(o));
        v[i] *= __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
      }
    }
  };
  auto put = [&](float* P, const float (&v)[EPT]) {
#pragma unroll
    for (int i = 0; i < EPT; ++i)
      if (tid + i * kNT < NE) P[tid + i * kNT] = v[i];
  };

  {
    float v[EPT];
    fetch(0, v);
    put(patch[0], v);
  }
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cb = ch * CC;
    const bool more = ch + 1 < nch;
    float v[EPT];
    if (more) fetch(cb + CC, v);                 // the next chunk, in flight during this one
    const float* P = patch[ch & 1];
    const int nc = min(CC, p.C - cb);
    for (int cl = 0; cl < nc; ++cl) {
      const float* wc = p.w + (long)(cb + cl) * K * K;          // + m * C * K * K
      const float* prow = P + cl * NPOS + r * PWD + c0;
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        float xv[PX + K - 1];
#pragma unroll
        for (int e = 0; e < PX + K - 1; ++e) xv[e] = prow[kh * PWD + e];
#pragma unroll
        for (int m = 0; m < M; ++m) {
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            const float wv = wc[(long)m * p.C * K * K + kh * K + kw];     // wave-uniform
#pragma unroll
            for (int q = 0; q < PX; ++q) acc[m][q] = __builtin_fmaf(xv[q + kw], wv, acc[m][q]);
          }
        }
      }
    }
    if (more) put(patch[(ch + 1) & 1], v);      // the idle buffer (last read in chunk ch - 1)
    __syncthreads();
  }
  const long n0 = (long)b * HW + (long)(oh0 + r) * W + c0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float osc = p.y_scale ? p.y_scale[m * p.B + b] : 1.f;
    const float bm = p.bias ? p.bias[m] : 0.f, am = p.act ? p.act[m] : 1.f;
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      float v = p.alpha * acc[m][q];
      if (p.y_scale) v *= osc;
      v += bm;
      if (p.act) v = v > 0.f ? v : am * v;
      p.y[(long)m * L + n0 + q] = v;
    }
  }
}

template <int K>
hipError_t go_k(const Args& a, hipStream_t st, dim3 grid) {
  switch (a.M) {
    case 1: hipLaunchKernelGGL((conv_small_kernel<1, K>), grid, dim3(kNT), 0, st, a); break;
    case 2: hipLaunchKernelGGL((conv_small_kernel<2, K>), grid, dim3(kNT), 0, st, a); break;
    case 3: hipLaunchKernelGGL((conv_small_kernel<3, K>), grid, dim3(kNT), 0, st, a); break;
    default: hipLaunchKernelGGL((conv_small_kernel<4, K>), grid, dim3(kNT), 0, st, a); break;
  }
  return hipGetLastError();
}

}  // namespace

// 64-wide maps only: on smaller maps the gather GEMM's split-K spreads the channel sum over the
// chip, which one block per (image, 8 rows) cannot (measured at B = 64: 32x32 117 -> 184 us,
// 8x8 45 -> 282 us with this kernel; 64x64 434 -> 253 us before its staging was double-buffered)
bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW, int transposed) {
  return !transposed && M >= 1 && M <= 4 && stride == 1 && (K == 1 || K == 3 || K == 5) && OH == H && OW == W &&
         pad == (K - 1) / 2 && W == WMAP && H % (kNT / (WMAP / PX)) == 0;
}

hipError_t launch(const Args& a, hipStream_t st) {
  if (!domain(a.M, a.H, a.W, a.K, 1, a.pad, a.H, a.W, 0) || !a.x || !a.w || !a.y || a.B <= 0 || a.C <= 0)
    return hipErrorInvalidValue;
  // 32-bit buffer offsets, including a chunk's channels past C
  if (4L * (a.C + CC) * a.B * a.H * a.W >= (1L << 31)) return hipErrorInvalidValue;
  const long blocks = (long)a.B * (a.H / (kNT / (WMAP / PX)));
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 grid((unsigned)blocks);
  switch (a.K) {
    case 1: return go_k<1>(a, st, grid);
    case 3: return go_k<3>(a, st, grid);
    default: return go_k<5>(a, st, grid);
  }
}

}  // namespace ganamd_small
