// Real-data input pipeline on the GPU: the per-image transform chain of units/dataloader.py:5-14
//   ToTensor (u8 HWC -> f32 CHW / 255) -> RandomHorizontalFlip -> Resize((S, S), BICUBIC,
//   antialias) -> Normalize(mean, std)
// for a batch of decoded images of one size, as two separable passes over ELL tap tables built
// on the host (tables.bicubic_aa_1d, the antialiased bicubic of torch.nn.functional.interpolate
// that torchvision's Resize calls on tensors).
//
//   pass 1 (rows):  t[b][c][h][ow]  = sum_k wx[ow][k] * u8[b][h][col(ow, k)][c] / 255
//                   col = ix[ow][k], mirrored (W-1-col) when flip[b]
//   pass 2 (cols):  y[b][c][oh][ow] = (sum_k wy[oh][k] * t[b][c][iy[oh][k]][ow] - mean[c]) / std[c]
//
// Both passes are HBM-bound byte/float streaming: pass 1 reads each input byte once per tap row
// that covers it (consecutive threads take consecutive ow, so a wave reads a contiguous span of
// the image row), pass 2 reads the small intermediate through L2.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ganamd.h"

namespace {

__global__ void img_rows_kernel(const uint8_t* __restrict__ src, int B, int H, int W, const uint8_t* __restrict__ flip,
                                const int32_t* __restrict__ ix, const float* __restrict__ wx, int KX, int OW,
                                float* __restrict__ tmp) {
  const long total = (long)B * 3 * H * OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW);
    const long r = i / OW;              // (b, c, h)
    const int h = (int)(r % H);
    const int c = (int)((r / H) % 3);
    const int b = (int)(r / (3L * H));
    const bool fl = flip != nullptr && flip[b];
    const uint8_t* row = src + ((long)b * H + h) * W * 3;
    float acc = 0.f;
    for (int k = 0; k < KX; ++k) {
      int col = ix[ow * KX + k];
      if (fl) col = W - 1 - col;
      acc += wx[ow * KX + k] * ((float)row[col * 3 + c] / 255.f);
    }
    tmp[i] = acc;
  }
}

__global__ void img_cols_kernel(const float* __restrict__ tmp, int B, int H, int OW, const int32_t* __restrict__ iy,
                                const float* __restrict__ wy, int KY, int OH, const float* __restrict__ mean,
                                const float* __restrict__ stdv, float* __restrict__ y) {
  const long total = (long)B * 3 * OH * OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW);
    const int oh = (int)((i / OW) % OH);
    const long bc = i / ((long)OW * OH);
    const int c = (int)(bc % 3);
    const float* plane = tmp + bc * H * OW;
    float acc = 0.f;
    for (int k = 0; k < KY; ++k) acc += wy[oh * KY + k] * plane[(long)iy[oh * KY + k] * OW + ow];
    y[i] = (acc - mean[c]) / stdv[c];
  }
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" size_t ganamd_image_batch_workspace(int B, int H, int OW) { return (size_t)B * 3 * H * OW * sizeof(float); }

extern "C" int ganamd_image_batch(const uint8_t* src, int B, int H, int W, const uint8_t* flip, const int32_t* ix,
                                  const float* wx, int KX, int OW, const int32_t* iy, const float* wy, int KY, int OH,
                                  const float* mean, const float* stdv, float* y, float* ws, size_t ws_bytes,
                                  hipStream_t stream) {
  if (!src || !ix || !wx || !iy || !wy || !mean || !stdv || !y || !ws) return GANAMD_EINVAL;
  if (B <= 0 || H <= 0 || W <= 0 || KX <= 0 || KY <= 0 || OW <= 0 || OH <= 0) return GANAMD_EINVAL;
  if (ws_bytes < ganamd_image_batch_workspace(B, H, OW)) return GANAMD_EINVAL;
  const long n1 = (long)B * 3 * H * OW, n2 = (long)B * 3 * OH * OW;
  img_rows_kernel<<<grid_for(n1), 256, 0, stream>>>(src, B, H, W, flip, ix, wx, KX, OW, ws);
  img_cols_kernel<<<grid_for(n2), 256, 0, stream>>>(ws, B, H, OW, iy, wy, KY, OH, mean, stdv, y);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}
