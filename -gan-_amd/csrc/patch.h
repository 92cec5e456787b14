// Internal interface between conv_gemm.hip (the conv entry points, packing, the gather GEMM) and
// conv_patch.hip (the split6 LDS-patch convolution).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

namespace ganamd_patch {

// One launch of the patch convolution: a stride-1 "same" K x K conv (K = 3 / 5) over the full map
// width W (32 or 64) of CNHW x [C][B][H][W], fp32 result
//   y[m][b,oh,ow] = alpha * sum_{t,c} A(m, t, c) * P(c, b, oh + kh - pad, ow + kw - pad)   (* epilogue)
// with the replication-padded (fwd) or zero-padded, tap-reversed (dgrad interior) patch P of
// src * scale[c][b].  A is the packed weight operand split into three bf16 planes (h, m, l):
// plane p element ((m * nct + cc) * T + t) * 16 + c16 at w + p * wplane (nct = Ckp / 16).
struct Args {
  const unsigned short* w;
  int wplane, w_bytes;        // elements per plane; bytes of all three planes
  int M, Ckp, KK;
  const float* src;
  const float* scale;         // [C][B] or null
  int C, B, H, W;
  float* y;
  long ldy;
  const float* bias;          // [M] or null (epilogue, in this order: *oscale, +bias, +noise, PReLU)
  const float* oscale;        // [M][B] or null
  const float* noise;         // [M][ldy] or null
  const float* noise_scale;
  const float* act;           // PReLU slopes [M] or null
  float alpha;
  int dgrad;                  // zero padding, taps reversed
};

// The row tile for M rows (48 or 96), 0 when the patch kernel does not take M.
int row_tile(int M);
// Pixels per block for map width W (the block covers whole rows of one image; W = 32: 16 rows on
// grids of B * H / 16 >= 512 blocks, else 8).
int block_pixels(int W, int B, int H);
// The kernel's domain (the packing and the dispatch agree through it): stride 1, same padding,
// K = 3 / 5, square, W = 32 / 64, H a multiple of the block's rows, M <= 96.
bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW);
// Blocks of one launch.
long blocks(const Args& a);
// Resident blocks per CU of the instance a launch would use (occupancy query).
int occupancy(const Args& a);
hipError_t launch(const Args& a, hipStream_t st);

}  // namespace ganamd_patch

namespace ganamd_wrow {

// One launch of the row-blocked weight gradient of a stride-1 "same" K x K conv (K = 3 / 5) on
// maps 32 / 64 wide (conv_wgrad_row.hip):
//   out[m][j][kh][kw] (+)= alpha * sum_seg sum_n a_seg[m][n] * ascale[m][b(n)]
//                                  * x_seg[j][b(n), oh(n) + kh - pad, ow(n) + kw - pad] * xscale[j][b(n)]
// (replication-clamped or zero-padded source); a block owns one kernel row kh and all K taps kw
// of it.  With splits > 1 the partial sums go to slab[split][M * J * K * K] (the caller reduces).
struct Args {
  const float* a;          // [M][B*H*W]
  const float* ascale;     // [M][B] or null (both scales or neither; one segment only)
  const float* x;          // [J][B*H*W]
  const float* xscale;     // [J][B] or null
  const float* a2;         // second segment (ganamd_conv_wgrad2) or null
  const float* x2;
  int M, J, B, H, W, KK, replicate;
  float alpha;
  float* out;
  int accumulate;
  float* slab;
  int splits, ks_per_split;   // 32-pixel K-steps per split
};

// The kernel's domain: stride 1, same padding, K = 3 / 5, W = 32 / 64, M <= 128, not transposed.
bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW, int transposed);
// Split-K of a launch: splits and K-steps per split (a function of the geometry alone).
void plan(int M, int J, int B, int H, int W, int K, int segs, int cus, int* splits, int* ks_per_split);
hipError_t launch(const Args& a, hipStream_t st);

}  // namespace ganamd_wrow

namespace ganamd_small {

// One launch of the direct (vector-ALU, exact fp32) convolution for at most four output channels
// (conv_small.hip): stride 1, "same" K x K (K = 1 / 3 / 5), CNHW x [C][B][H][W] -> y [M][B*H*W]
//   y[m][b,oh,ow] = act(alpha * sum_{c,kh,kw} w[m][c][kh][kw] * xs(c, b, oh + kh - pad, ow + kw - pad)
//                       * y_scale[m][b] + bias[m])      (xs = x * x_scale[c][b], padded)
struct Args {
  const float* x;
  const float* x_scale;    // [C][B] or null
  const float* w;          // [M][C][K][K], as stored (no packing)
  const float* bias;       // [M] or null
  const float* y_scale;    // [M][B] or null
  const float* act;        // PReLU slopes [M] or null
  float alpha;
  float* y;
  int B, C, H, W, M, K, pad, replicate;
};

bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW, int transposed);
hipError_t launch(const Args& a, hipStream_t st);

}  // namespace ganamd_small
