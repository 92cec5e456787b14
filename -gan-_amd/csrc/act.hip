// Pointwise activations, the BCE loss, the SK softmax and MiniBatchStdDev (gfx950).
//
//   act        sigmoid / tanh / leaky-ReLU (constant slope) and their derivatives
//              (SEBlock gates generator_13_5.py:357,376, discriminator_9_4.py:109,128; the vanilla
//              pair's Tanh / Sigmoid / LeakyReLU(0.2), generator_1.py:18-23, discriminator_1.py:15-20)
//   bce        torch.nn.BCELoss (mean reduction, log clamped at -100) and its gradient
//              (train/gan.py:21,32,48,50)
//   softmax_m  softmax over the M branches of a [M][P] attention tensor (dim=1 of the reference's
//              [B, M, C, 1, 1], generator_13_5.py:88,131) and its backward
//   mbstd      MiniBatchStdDev (discriminator_9_4.py:42-54): the forward, the backward, and the
//              two second-order sweeps of the critic's gradient penalty (tangent / adjoint, see
//              critic.py) -- std couples the samples of a segment, so its double backward has
//              cross-sample terms.
// All HBM-bound elementwise / reduction passes.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ganamd.h"

namespace {

constexpr int kNT = 256;

inline int grid_for(long n) { return (int)std::max<long>(1, std::min<long>((n + kNT - 1) / kNT, 16384)); }
inline int ok(hipError_t e) { return e == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH; }

__device__ __forceinline__ float act_f(int kind, float x, float slope) {
  switch (kind) {
    case GANAMD_ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case GANAMD_ACT_TANH: return tanhf(x);
    default: return x > 0.f ? x : slope * x;
  }
}

// derivative dy/dx written in terms of the saved OUTPUT y (sigmoid, tanh) or INPUT x (leaky)
__device__ __forceinline__ float act_d(int kind, float v, float slope) {
  switch (kind) {
    case GANAMD_ACT_SIGMOID: return v * (1.f - v);
    case GANAMD_ACT_TANH: return 1.f - v * v;
    default: return v > 0.f ? 1.f : slope;
  }
}

__global__ __launch_bounds__(kNT) void act_fwd_kernel(int kind, const float* __restrict__ x, long n, float slope,
                                                      float* __restrict__ y) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) y[i] = act_f(kind, x[i], slope);
}

__global__ __launch_bounds__(kNT) void act_bwd_kernel(int kind, const float* __restrict__ v, const float* __restrict__ gy,
                                                      long n, float slope, float* __restrict__ gx) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT)
    gx[i] = gy[i] * act_d(kind, v[i], slope);
}

// second derivative in terms of the saved output (0 for the piecewise-linear leaky ReLU)
__device__ __forceinline__ float act_dd(int kind, float v) {
  switch (kind) {
    case GANAMD_ACT_SIGMOID: return v * (1.f - v) * (1.f - 2.f * v);
    case GANAMD_ACT_TANH: return -2.f * v * (1.f - v * v);
    default: return 0.f;
  }
}

// ax = ay * f'(.) + gy * xd * f''(.)   (adjoint sweep of the GP double backward)
__global__ __launch_bounds__(kNT) void act_adjoint_kernel(int kind, const float* __restrict__ v,
                                                          const float* __restrict__ ay, const float* __restrict__ gy,
                                                          const float* __restrict__ xd, long n, float slope,
                                                          float* __restrict__ ax) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const float w = v[i];
    ax[i] = ay[i] * act_d(kind, w, slope) + gy[i] * xd[i] * act_dd(kind, w);
  }
}

// y = x1 * s1[plane] + (x2 ? x2 * s2[plane] : 0) + (r ? r : 0)
__global__ __launch_bounds__(kNT) void scale_add2_kernel(const float* __restrict__ x1, const float* __restrict__ s1,
                                                         const float* __restrict__ x2, const float* __restrict__ s2,
                                                         const float* __restrict__ r, long planes, long HW,
                                                         float* __restrict__ y) {
  const long n = planes * HW;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const long p = i / HW;
    float v = x1[i] * s1[p];
    if (x2) v += x2[i] * s2[p];
    if (r) v += r[i];
    y[i] = v;
  }
}

// out[p] = sum_hw a1*b1 (+ a2*b2), one wave per plane
__global__ __launch_bounds__(kNT) void plane_dot2_kernel(const float* __restrict__ a1, const float* __restrict__ b1,
                                                         const float* __restrict__ a2, const float* __restrict__ b2,
                                                         long planes, long HW, float* __restrict__ out) {
  const long wave = (blockIdx.x * (long)kNT + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * kNT) >> 6;
  const int lane = threadIdx.x & 63;
  for (long p = wave; p < planes; p += nwaves) {
    float acc = 0.f;
    for (long i = lane; i < HW; i += 64) {
      acc += a1[p * HW + i] * b1[p * HW + i];
      if (a2) acc += a2[p * HW + i] * b2[p * HW + i];
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) out[p] = acc;
  }
}

__global__ __launch_bounds__(kNT) void axpy_kernel(long n, float a, const float* __restrict__ x, float* __restrict__ y) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) y[i] += a * x[i];
}

// ---------------------------------------------------------------- BCE
// loss = -1/n sum t*max(log p, -100) + (1-t)*max(log(1-p), -100)           (torch BCELoss, mean)
// dp   = gout * (p - t) / max(p (1-p), 1e-12) / n                          (aten's backward)
__global__ __launch_bounds__(kNT) void bce_fwd_kernel(const float* __restrict__ p, const float* __restrict__ t, int n,
                                                      float* __restrict__ out) {
  __shared__ float sh[kNT / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += kNT) {
    const float lp = fmaxf(logf(p[i]), -100.f), lq = fmaxf(logf(1.f - p[i]), -100.f);
    acc += t[i] * lp + (1.f - t[i]) * lq;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < kNT / 64; ++w) s += sh[w];
    out[0] = -s / (float)n;
  }
}

__global__ __launch_bounds__(kNT) void bce_bwd_kernel(const float* __restrict__ p, const float* __restrict__ t, int n,
                                                      const float* __restrict__ gout, float* __restrict__ gp) {
  const float g = gout[0] / (float)n;
  for (int i = blockIdx.x * kNT + threadIdx.x; i < n; i += gridDim.x * kNT)
    gp[i] = g * (p[i] - t[i]) / fmaxf(p[i] * (1.f - p[i]), 1e-12f);
}

// ---------------------------------------------------------------- softmax over M branches
template <int M>
__global__ __launch_bounds__(kNT) void softmax_m_kernel(const float* __restrict__ x, long P, float* __restrict__ y) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < P; i += (long)gridDim.x * kNT) {
    float v[M], mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      v[m] = x[m * P + i];
      mx = fmaxf(mx, v[m]);
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      v[m] = __expf(v[m] - mx);
      s += v[m];
    }
    const float r = 1.f / s;
#pragma unroll
    for (int m = 0; m < M; ++m) y[m * P + i] = v[m] * r;
  }
}

template <int M>
__global__ __launch_bounds__(kNT) void softmax_m_bwd_kernel(const float* __restrict__ y, const float* __restrict__ gy,
                                                            long P, float* __restrict__ gx) {
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < P; i += (long)gridDim.x * kNT) {
    float d = 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m) d += y[m * P + i] * gy[m * P + i];
#pragma unroll
    for (int m = 0; m < M; ++m) gx[m * P + i] = y[m * P + i] * (gy[m * P + i] - d);
  }
}

// ---------------------------------------------------------------- MiniBatchStdDev
// CNHW x: row c (row stride ldx floats) holds the samples of S segments of Bs = B/S samples, each
// sample HW floats.  The reference groups the NCHW segment as x.view(G, -1): sample b of segment
// s sits in group g = b / (Bs/G) at column (b % (Bs/G), c, hw), so a column is the G values
// x[c][s*Bs + g*Q + q][hw], Q = Bs/G.  Per column: mean mu, unbiased variance, sigma = sqrt(var +
// 1e-8); std_s = mean over the n = Q*C*HW columns of the segment.
//
// Work split: grid (chunks, S); a thread owns columns (c, q, hw) with the G values in registers.
// Pass 1 writes per-block partial sums (double) of the column terms; pass 2 (one block per
// segment) reduces them and writes the segment's scalar outputs and the broadcast row.
struct MbGeo {
  int C, B, HW, S, G;
  long ldx;          // row stride of x / gx / xd / ax (floats)
  long ldy;          // row stride of y / gy / ay / yd (floats; y has C + 1 rows)
};

constexpr int kMbBlocks = 64;   // partial-sum blocks per segment

__device__ __forceinline__ void mb_col(const MbGeo& g, long col, int s, int* c, long* o0, long* stride) {
  // col in [0, Q*C*HW): (c, q, hw) -> offset of the group-0 value within row c, group stride
  const int Bs = g.B / g.S, Q = Bs / g.G;
  const long per_c = (long)Q * g.HW;
  *c = (int)(col / per_c);
  const long r = col - *c * per_c;
  const int q = (int)(r / g.HW), hw = (int)(r - (long)q * g.HW);
  *o0 = (long)(s * Bs + q) * g.HW + hw;
  *stride = (long)Q * g.HW;
}

template <int G>
__device__ __forceinline__ void mb_stats(const float* __restrict__ row, long o0, long st, float (&v)[G], float* mu,
                                         float* sig) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    v[k] = row[o0 + k * st];
    m += v[k];
  }
  m /= (float)G;
  float var = 0.f;
#pragma unroll
  for (int k = 0; k < G; ++k) var += (v[k] - m) * (v[k] - m);
  var /= (float)(G - 1);
  *mu = m;
  *sig = sqrtf(var + 1e-8f);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < kNT / 64; ++w) t += sh[w];
  return t;
}

// mode 0 (forward): part = sum sigma; copy x -> y rows [0, C)
// mode 1 (tangent): part = sum u / sigma, u = sum_g (x_g - mu) xd_g; copy xd -> yd rows [0, C)
template <int G>
__global__ __launch_bounds__(kNT) void mbstd_partial_kernel(MbGeo g, int mode, const float* __restrict__ x,
                                                            const float* __restrict__ xd, float* __restrict__ y,
                                                            double* __restrict__ part) {
  __shared__ double sh[kNT / 64];
  const int s = blockIdx.y;
  const int Bs = g.B / g.S, Q = Bs / G;
  const long n = (long)Q * g.C * g.HW;
  double acc = 0.0;
  for (long col = blockIdx.x * (long)kNT + threadIdx.x; col < n; col += (long)gridDim.x * kNT) {
    int c;
    long o0, st;
    mb_col(g, col, s, &c, &o0, &st);
    const float* row = x + c * g.ldx;
    float v[G], mu, sig;
    mb_stats<G>(row, o0, st, v, &mu, &sig);
    if (mode == 0) {
      acc += sig;
#pragma unroll
      for (int k = 0; k < G; ++k) y[c * g.ldy + o0 + k * st] = v[k];
    } else {
      const float* drow = xd + c * g.ldx;
      float u = 0.f;
#pragma unroll
      for (int k = 0; k < G; ++k) {
        const float d = drow[o0 + k * st];
        u += (v[k] - mu) * d;
        y[c * g.ldy + o0 + k * st] = d;
      }
      acc += u / sig;
    }
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) part[s * gridDim.x + blockIdx.x] = t;
}

// one block per segment: value = scale * sum(part) -> out[s] and the broadcast row C of y
__global__ __launch_bounds__(kNT) void mbstd_finalize_kernel(MbGeo g, const double* __restrict__ part, int nparts,
                                                             double scale, float* __restrict__ out,
                                                             float* __restrict__ y) {
  __shared__ double sh[kNT / 64];
  const int s = blockIdx.x;
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += kNT) acc += part[s * nparts + i];
  const float v = (float)(block_sum(acc, sh) * scale);
  if (threadIdx.x == 0 && out) out[s] = v;
  const int Bs = g.B / g.S;
  const long len = (long)Bs * g.HW;
  float* row = y + (long)g.C * g.ldy + (long)s * len;
  for (long i = threadIdx.x; i < len; i += kNT) row[i] = v;
}

// Sum of row C of gy (and of ay) over each segment: sums[s] (and sums[S + s]).
__global__ __launch_bounds__(kNT) void mbstd_rowsum_kernel(MbGeo g, const float* __restrict__ gy,
                                                           const float* __restrict__ ay, double* __restrict__ sums) {
  __shared__ double sh[kNT / 64];
  const int s = blockIdx.x;
  const int Bs = g.B / g.S;
  const long len = (long)Bs * g.HW;
  const float* rg = gy + (long)g.C * g.ldy + (long)s * len;
  double a = 0.0;
  for (long i = threadIdx.x; i < len; i += kNT) a += rg[i];
  a = block_sum(a, sh);
  if (threadIdx.x == 0) sums[s] = a;
  if (ay) {
    const float* ra = ay + (long)g.C * g.ldy + (long)s * len;
    double b = 0.0;
    for (long i = threadIdx.x; i < len; i += kNT) b += ra[i];
    b = block_sum(b, sh);
    if (threadIdx.x == 0) sums[g.S + s] = b;
  }
}

// First-order backward (xd == null):     gx = gy[rows < C] + Gs * (x_g - mu) / ((G-1) n sigma)
// Second-order adjoint (xd != null):     ax = ay[rows < C] + As * (x_g - mu) / ((G-1) n sigma)
//     + Gs / ((G-1) n) * [ (xd_g - mean xd) / sigma - u (x_g - mu) / ((G-1) sigma^3) ]
// with Gs = segment sum of gy's row C (sums[s]), As = the same of ay (sums[S + s]),
// u = sum_g (x_g - mu) xd_g.  `top` is gy (first order) or ay (adjoint).
template <int G>
__global__ __launch_bounds__(kNT) void mbstd_back_kernel(MbGeo g, const float* __restrict__ x,
                                                         const float* __restrict__ xd, const float* __restrict__ top,
                                                         const double* __restrict__ sums, float* __restrict__ gx) {
  const int s = blockIdx.y;
  const int Bs = g.B / g.S, Q = Bs / G;
  const long n = (long)Q * g.C * g.HW;
  const float k1 = 1.f / ((float)(G - 1) * (float)n);
  const float Gs = (float)sums[s];
  const float As = xd ? (float)sums[g.S + s] : 0.f;
  for (long col = blockIdx.x * (long)kNT + threadIdx.x; col < n; col += (long)gridDim.x * kNT) {
    int c;
    long o0, st;
    mb_col(g, col, s, &c, &o0, &st);
    float v[G], mu, sig;
    mb_stats<G>(x + c * g.ldx, o0, st, v, &mu, &sig);
    const float* trow = top + c * g.ldy;
    float* orow = gx + c * g.ldx;
    if (!xd) {
      const float k = Gs * k1 / sig;
#pragma unroll
      for (int j = 0; j < G; ++j) orow[o0 + j * st] = trow[o0 + j * st] + k * (v[j] - mu);
    } else {
      const float* drow = xd + c * g.ldx;
      float d[G], dm = 0.f, u = 0.f;
#pragma unroll
      for (int j = 0; j < G; ++j) {
        d[j] = drow[o0 + j * st];
        dm += d[j];
        u += (v[j] - mu) * d[j];
      }
      dm /= (float)G;
      const float is = 1.f / sig;
      const float ka = As * k1 * is;
      const float kb = Gs * k1;
      const float kc = u * is * is * is / (float)(G - 1);
#pragma unroll
      for (int j = 0; j < G; ++j)
        orow[o0 + j * st] = trow[o0 + j * st] + ka * (v[j] - mu) + kb * ((d[j] - dm) * is - kc * (v[j] - mu));
    }
  }
}

bool mb_ok(const MbGeo& g) {
  return g.C > 0 && g.B > 0 && g.HW > 0 && g.S > 0 && g.G == 4 && g.B % g.S == 0 && (g.B / g.S) % g.G == 0 &&
         g.ldx >= (long)g.B * g.HW && g.ldy >= (long)g.B * g.HW;
}

int mb_chunks(const MbGeo& g) {
  const long n = (long)(g.B / g.S / g.G) * g.C * g.HW;
  return (int)std::max<long>(1, std::min<long>(kMbBlocks, (n + kNT - 1) / kNT));
}

}  // namespace

extern "C" {

int ganamd_act_fwd(int kind, const float* x, long n, float slope, float* y, hipStream_t st) {
  if (!x || !y || n <= 0 || kind < 0 || kind > GANAMD_ACT_LEAKY) return GANAMD_EINVAL;
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, kind, x, n, slope, y);
  return ok(hipGetLastError());
}

int ganamd_act_bwd(int kind, const float* v, const float* gy, long n, float slope, float* gx, hipStream_t st) {
  if (!v || !gy || !gx || n <= 0 || kind < 0 || kind > GANAMD_ACT_LEAKY) return GANAMD_EINVAL;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, kind, v, gy, n, slope, gx);
  return ok(hipGetLastError());
}

int ganamd_act_adjoint(int kind, const float* v, const float* ay, const float* gy, const float* xd, long n, float slope,
                       float* ax, hipStream_t st) {
  if (!v || !ay || !gy || !xd || !ax || n <= 0 || kind < 0 || kind > GANAMD_ACT_LEAKY) return GANAMD_EINVAL;
  hipLaunchKernelGGL(act_adjoint_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, kind, v, ay, gy, xd, n, slope, ax);
  return ok(hipGetLastError());
}

int ganamd_scale_add2(const float* x1, const float* s1, const float* x2, const float* s2, const float* r, long planes,
                      long HW, float* y, hipStream_t st) {
  if (!x1 || !s1 || (x2 && !s2) || !y || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(scale_add2_kernel, dim3(grid_for(planes * HW)), dim3(kNT), 0, st, x1, s1, x2, s2, r, planes, HW,
                     y);
  return ok(hipGetLastError());
}

int ganamd_plane_dot2(const float* a1, const float* b1, const float* a2, const float* b2, long planes, long HW,
                      float* out, hipStream_t st) {
  if (!a1 || !b1 || (a2 && !b2) || !out || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  const int blocks = (int)std::min<long>((planes + 3) / 4, 16384);
  hipLaunchKernelGGL(plane_dot2_kernel, dim3(blocks), dim3(kNT), 0, st, a1, b1, a2, b2, planes, HW, out);
  return ok(hipGetLastError());
}

int ganamd_axpy(long n, float a, const float* x, float* y, hipStream_t st) {
  if (!x || !y || n <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, n, a, x, y);
  return ok(hipGetLastError());
}

int ganamd_bce_fwd(const float* p, const float* target, int n, float* out, hipStream_t st) {
  if (!p || !target || !out || n <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(1), dim3(kNT), 0, st, p, target, n, out);
  return ok(hipGetLastError());
}

int ganamd_bce_bwd(const float* p, const float* target, int n, const float* gout, float* gp, hipStream_t st) {
  if (!p || !target || !gout || !gp || n <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, p, target, n, gout, gp);
  return ok(hipGetLastError());
}

int ganamd_softmax_m(int M, const float* x, long P, float* y, hipStream_t st) {
  if (!x || !y || P <= 0) return GANAMD_EINVAL;
  switch (M) {
    case 2: hipLaunchKernelGGL(softmax_m_kernel<2>, dim3(grid_for(P)), dim3(kNT), 0, st, x, P, y); break;
    case 3: hipLaunchKernelGGL(softmax_m_kernel<3>, dim3(grid_for(P)), dim3(kNT), 0, st, x, P, y); break;
    case 4: hipLaunchKernelGGL(softmax_m_kernel<4>, dim3(grid_for(P)), dim3(kNT), 0, st, x, P, y); break;
    default: return GANAMD_EINVAL;
  }
  return ok(hipGetLastError());
}

int ganamd_softmax_m_bwd(int M, const float* y, const float* gy, long P, float* gx, hipStream_t st) {
  if (!y || !gy || !gx || P <= 0) return GANAMD_EINVAL;
  switch (M) {
    case 2: hipLaunchKernelGGL(softmax_m_bwd_kernel<2>, dim3(grid_for(P)), dim3(kNT), 0, st, y, gy, P, gx); break;
    case 3: hipLaunchKernelGGL(softmax_m_bwd_kernel<3>, dim3(grid_for(P)), dim3(kNT), 0, st, y, gy, P, gx); break;
    case 4: hipLaunchKernelGGL(softmax_m_bwd_kernel<4>, dim3(grid_for(P)), dim3(kNT), 0, st, y, gy, P, gx); break;
    default: return GANAMD_EINVAL;
  }
  return ok(hipGetLastError());
}

size_t ganamd_mbstd_workspace(int S) { return sizeof(double) * (size_t)std::max(1, S) * (kMbBlocks + 2); }

int ganamd_mbstd_fwd(const float* x, long ldx, int C, int B, int HW, int S, int G, float* y, long ldy, float* std_out,
                     void* ws, size_t ws_bytes, hipStream_t st) {
  const MbGeo g{C, B, HW, S, G, ldx, ldy};
  if (!x || !y || !ws || !mb_ok(g) || ws_bytes < ganamd_mbstd_workspace(S)) return GANAMD_EINVAL;
  const int nb = mb_chunks(g);
  const long n = (long)(B / S / G) * C * HW;
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(mbstd_partial_kernel<4>, dim3(nb, S), dim3(kNT), 0, st, g, 0, x, nullptr, y, part);
  hipLaunchKernelGGL(mbstd_finalize_kernel, dim3(S), dim3(kNT), 0, st, g, part, nb, 1.0 / (double)n, std_out, y);
  return ok(hipGetLastError());
}

int ganamd_mbstd_bwd(const float* x, long ldx, const float* gy, long ldy, int C, int B, int HW, int S, int G,
                     float* gx, void* ws, size_t ws_bytes, hipStream_t st) {
  const MbGeo g{C, B, HW, S, G, ldx, ldy};
  if (!x || !gy || !gx || !ws || !mb_ok(g) || ws_bytes < ganamd_mbstd_workspace(S)) return GANAMD_EINVAL;
  double* sums = static_cast<double*>(ws);
  hipLaunchKernelGGL(mbstd_rowsum_kernel, dim3(S), dim3(kNT), 0, st, g, gy, nullptr, sums);
  hipLaunchKernelGGL(mbstd_back_kernel<4>, dim3(mb_chunks(g), S), dim3(kNT), 0, st, g, x, nullptr, gy, sums, gx);
  return ok(hipGetLastError());
}

int ganamd_mbstd_tangent(const float* x, const float* xd, long ldx, int C, int B, int HW, int S, int G, float* yd,
                         long ldy, void* ws, size_t ws_bytes, hipStream_t st) {
  const MbGeo g{C, B, HW, S, G, ldx, ldy};
  if (!x || !xd || !yd || !ws || !mb_ok(g) || ws_bytes < ganamd_mbstd_workspace(S)) return GANAMD_EINVAL;
  const int nb = mb_chunks(g);
  const long n = (long)(B / S / G) * C * HW;
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(mbstd_partial_kernel<4>, dim3(nb, S), dim3(kNT), 0, st, g, 1, x, xd, yd, part);
  hipLaunchKernelGGL(mbstd_finalize_kernel, dim3(S), dim3(kNT), 0, st, g, part, nb,
                     1.0 / ((double)(G - 1) * (double)n), nullptr, yd);
  return ok(hipGetLastError());
}

int ganamd_mbstd_adjoint(const float* x, const float* xd, long ldx, const float* gy, const float* ay, long ldy, int C,
                         int B, int HW, int S, int G, float* ax, void* ws, size_t ws_bytes, hipStream_t st) {
  const MbGeo g{C, B, HW, S, G, ldx, ldy};
  if (!x || !xd || !gy || !ay || !ax || !ws || !mb_ok(g) || ws_bytes < ganamd_mbstd_workspace(S))
    return GANAMD_EINVAL;
  double* sums = static_cast<double*>(ws);
  hipLaunchKernelGGL(mbstd_rowsum_kernel, dim3(S), dim3(kNT), 0, st, g, gy, ay, sums);
  hipLaunchKernelGGL(mbstd_back_kernel<4>, dim3(mb_chunks(g), S), dim3(kNT), 0, st, g, x, xd, ay, sums, ax);
  return ok(hipGetLastError());
}

}  // extern "C"
