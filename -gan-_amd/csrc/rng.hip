// Counter-based random numbers on the device: Philox4x32-10 (Salmon et al., SC'11), the generator
// family PyTorch's CUDA/HIP backend draws z, eps and the StyleConv noise from.  Each 128-bit
// counter {group index lo, hi, stream offset lo, hi} under the 64-bit key {seed lo, hi} yields four
// 32-bit words; element 4*g + i of a draw is word i of group g.
//   uniform  u = (word >> 8) * 2^-24                       in [0, 1)   (torch.rand's 24-bit grid)
//   normal   Box-Muller on word pairs: r = sqrt(-2 ln u1), u1 = ((w0 >> 8) + 1) * 2^-24 in (0, 1],
//            z0 = r cos(2 pi u2), z1 = r sin(2 pi u2), u2 = (w1 >> 8) * 2^-24
// The stream offset lives in device memory and is advanced by one per call (a one-thread launch
// after the draw), so a captured graph draws fresh numbers on every replay.  The key may live in
// device memory too (ganamd_philox_draw_keyed): a graph captured before a re-key (a checkpoint
// resume) then draws with the new key on its next replay.
//
// Concurrent consumers never share a counter:
//   * each consumer owns its offset word (rng.py DeviceRNG.fork gives stream s the offsets
//     s * 2^40 + k), and only the stream that owns a word ever advances it;
//   * draws that run concurrently on ONE offset (a generator forward's per-draw noise inside
//     parallel branch streams) read it without advancing and put a distinct draw index `sub` into
//     counter word 1 (group index < 2^32 there); the owner advances once after joining them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ganamd.h"

namespace {

constexpr int kNT = 256;

__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c[0] = hi1 ^ c[1] ^ k0;
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k1;
  c[3] = lo0;
}

__device__ __forceinline__ void philox10(uint32_t (&c)[4], uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

template <bool NORMAL>
__global__ __launch_bounds__(kNT) void philox_kernel(float* __restrict__ out, long n, uint64_t seed,
                                                     const uint64_t* __restrict__ key,
                                                     const uint64_t* __restrict__ offset, uint32_t sub) {
  const uint64_t off = *offset;
  if (key) seed = *key;
  const long groups = (n + 3) / 4;
  const bool aligned = ((uintptr_t)out & 15) == 0;
  for (long g = blockIdx.x * (long)kNT + threadIdx.x; g < groups; g += (long)gridDim.x * kNT) {
    uint32_t c[4] = {(uint32_t)g, (uint32_t)((uint64_t)g >> 32) + sub, (uint32_t)off, (uint32_t)(off >> 32)};
    philox10(c, seed);
    float v[4];
    if (NORMAL) {
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        const float u1 = ((c[q] >> 8) + 1u) * 5.9604644775390625e-08f;   // (0, 1]
        const float u2 = (c[q + 1] >> 8) * 5.9604644775390625e-08f;       // [0, 1)
        // hardware transcendentals: v_log_f32 is log2, v_sin/cos_f32 take revolutions (x / 2 pi),
        // so the angle 2 pi u2 needs no range reduction; ~1e-6 abs against float64 (test bar 1e-5)
        const float r = sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(u1));
        const float s = __builtin_amdgcn_sinf(u2), co = __builtin_amdgcn_cosf(u2);
        v[q] = r * co;
        v[q + 1] = r * s;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = (c[q] >> 8) * 5.9604644775390625e-08f;
    }
    const long base = 4 * g;
    if (aligned && base + 3 < n) {   // one 16-byte store per lane (four 4-byte stores fill a quarter of each line they touch)
      *reinterpret_cast<float4*>(out + base) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (base + q < n) out[base + q] = v[q];
    }
  }
}

__global__ void offset_advance_kernel(uint64_t* offset) { *offset += 1; }

int launch(bool normal, float* out, long n, uint64_t seed, const uint64_t* key, uint64_t* offset, uint32_t sub,
           bool advance, hipStream_t st) {
  if (!out || !offset || n <= 0) return GANAMD_EINVAL;
  const long groups = (n + 3) / 4;
  if (sub != 0 && groups > (1L << 32)) return GANAMD_EINVAL;    // word 1 must hold the index alone
  const unsigned blocks = (unsigned)std::min<long>((groups + kNT - 1) / kNT, 2048L * 8);
  if (normal)
    hipLaunchKernelGGL(philox_kernel<true>, dim3(blocks), dim3(kNT), 0, st, out, n, seed, key, offset, sub);
  else
    hipLaunchKernelGGL(philox_kernel<false>, dim3(blocks), dim3(kNT), 0, st, out, n, seed, key, offset, sub);
  if (advance) hipLaunchKernelGGL(offset_advance_kernel, dim3(1), dim3(1), 0, st, offset);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

}  // namespace

extern "C" {

int ganamd_philox_uniform(float* out, long n, uint64_t seed, uint64_t* offset, hipStream_t stream) {
  return launch(false, out, n, seed, nullptr, offset, 0, true, stream);
}

int ganamd_philox_normal(float* out, long n, uint64_t seed, uint64_t* offset, hipStream_t stream) {
  return launch(true, out, n, seed, nullptr, offset, 0, true, stream);
}

int ganamd_philox_draw(float* out, long n, uint64_t seed, uint64_t* offset, uint32_t sub, int normal, int advance,
                       hipStream_t stream) {
  return launch(normal != 0, out, n, seed, nullptr, offset, sub, advance != 0, stream);
}

int ganamd_philox_draw_keyed(float* out, long n, const uint64_t* key, uint64_t* offset, uint32_t sub, int normal,
                             int advance, hipStream_t stream) {
  if (!key) return GANAMD_EINVAL;
  return launch(normal != 0, out, n, 0, key, offset, sub, advance != 0, stream);
}

int ganamd_philox_advance(uint64_t* offset, hipStream_t stream) {
  if (!offset) return GANAMD_EINVAL;
  hipLaunchKernelGGL(offset_advance_kernel, dim3(1), dim3(1), 0, stream, offset);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

}  // extern "C"
