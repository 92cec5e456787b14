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
// Pixels per block for map width W (the block covers whole rows of one image).
int block_pixels(int W);
// The kernel's domain (the packing and the dispatch agree through it): stride 1, same padding,
// K = 3 / 5, square, W = 32 / 64, H a multiple of the block's rows, M <= 96.
bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW);
// Blocks of one launch.
long blocks(const Args& a);
// Resident blocks per CU of the instance a launch would use (occupancy query).
int occupancy(const Args& a);
hipError_t launch(const Args& a, hipStream_t st);

}  // namespace ganamd_patch
