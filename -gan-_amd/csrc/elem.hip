// Memory-bound kernels of the WGAN-GP hot path for gfx950: train-mode BatchNorm fused with
// PReLU, PReLU with its first and second derivatives, separable resampling (Smooth, bicubic,
// adaptive average pooling and their adjoints), per-plane / per-row reductions and the fused
// flat-buffer AdamW.  All activations are CNHW: a channel is one contiguous row of L = B*H*W.
//
// Reductions over a row are split over S blocks per channel so that a 64x64 feature map with
// ~100 channels still launches thousands of workgroups; per-block partials go to caller-provided
// workspace and a second tiny kernel merges them (no atomics: bitwise reproducible).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ganamd.h"

namespace {

constexpr int kNT = 256;
constexpr long kChunk = 4096;  // elements of a row per reduction block
constexpr int kMaxSplit = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over a 256-thread block; result valid in every thread.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

// Per-(row, split) partial of a row reduction.  acc_mode 0: a partial slot (reduce1_kernel folds
// them); with a single split the partial IS the result and the kernel writes it directly --
// 1: store, 2: accumulate -- saving the fold launch.
__device__ __forceinline__ void put_part(float* part, long idx, float v, int acc_mode) {
  part[idx] = acc_mode == 2 ? part[idx] + v : v;
}

inline int splits_for(long L) {
  long s = (L + kChunk - 1) / kChunk;
  if (s < 1) s = 1;
  if (s > kMaxSplit) s = kMaxSplit;
  return (int)s;
}

inline int grid_for(long n) {
  long b = (n + kNT - 1) / kNT;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

// ---------------------------------------------------------------- BatchNorm statistics
// Statistics and the backward's row sums accumulate in double, as torch's CPU BatchNorm does
// (acc_type<float> on CPU is double): with B = 4..64 samples per BatchNorm1d channel the
// normalisation is ill-conditioned and float accumulation measurably moves the result.
//
// block (s, c): chunk mean and M2 of row c (two passes over an L2-resident 16 KB chunk)
__global__ __launch_bounds__(kNT) void bn_partial_kernel(const float* __restrict__ x, long L, int S,
                                                         double* __restrict__ part) {
  __shared__ double sh[4];
  const int c = blockIdx.y, s = blockIdx.x;
  const long per = (L + S - 1) / S;
  const long lo = s * per, hi = min(L, lo + per);
  const float* row = x + (long)c * L;
  double acc = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) acc += row[i];
  const double n = (double)max(0L, hi - lo);
  const double mean = n > 0 ? block_sum_d(acc, sh) / n : 0.0;
  double m2 = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    const double d = row[i] - mean;
    m2 += d * d;
  }
  m2 = block_sum_d(m2, sh);
  if (threadIdx.x == 0) {
    double* o = part + ((long)c * S + s) * 3;
    o[0] = n;
    o[1] = mean;
    o[2] = m2;
  }
}

// running-statistic update r <- (1 - m) r + m v, rounded the same way wherever it is applied (the
// segmented forward's sequential update must equal the per-call one bit for bit)
__device__ __forceinline__ float bn_ema(float r, float m, float v) { return __fmaf_rn(1.f - m, r, __fmul_rn(m, v)); }

__device__ __forceinline__ void bn_store_stats(int c, double mean, double m2, long L, float* running_mean,
                                               float* running_var, float momentum, float eps, float* save_mean,
                                               float* save_invstd, float* seg_uvar = nullptr) {
  const double var = m2 / (double)L;
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (seg_uvar) seg_uvar[c] = (float)(L > 1 ? m2 / (double)(L - 1) : var);   // segmented: running stats later
  if (running_mean) running_mean[c] = bn_ema(running_mean[c], momentum, (float)mean);
  if (running_var) running_var[c] = bn_ema(running_var[c], momentum, (float)(L > 1 ? m2 / (double)(L - 1) : var));
}

// Chan merge of the S partials, running-stat update, invstd.
__global__ void bn_finalize_kernel(const double* __restrict__ part, int C, int S, long L, float* running_mean,
                                   float* running_var, float momentum, float eps, float* save_mean,
                                   float* save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double* p = part + (long)c * S * 3;
  double n = 0, mean = 0, m2 = 0;
  for (int s = 0; s < S; ++s) {
    const double nb = p[3 * s], mb = p[3 * s + 1], m2b = p[3 * s + 2];
    if (nb <= 0) continue;
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
  }
  bn_store_stats(c, mean, m2, L, running_mean, running_var, momentum, eps, save_mean, save_invstd);
}

// Short rows (BatchNorm1d: L = batch): one wave per row, the row held in registers; statistics,
// running stats and the normalised + PReLU output in ONE launch.
constexpr int kSmallL = 512;
constexpr int kSmallPer = kSmallL / 64;

__global__ __launch_bounds__(kNT) void bn_small_fwd_kernel(const float* __restrict__ x, int C, int L,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ alpha, float* running_mean,
                                                           float* running_var, float momentum, float eps,
                                                           float* __restrict__ y, float* __restrict__ save_mean,
                                                           float* __restrict__ save_invstd, int seg,
                                                           float* __restrict__ seg_uvar) {
  const int c = blockIdx.x * (kNT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const int pc = c / seg;   // segmented BatchNorm: row c = (channel pc, segment c % seg)
  const float* row = x + (long)c * L;
  float v[kSmallPer];
  double sum = 0.0;
#pragma unroll
  for (int j = 0; j < kSmallPer; ++j) {
    const int i = lane + 64 * j;
    v[j] = i < L ? row[i] : 0.f;
    sum += v[j];
  }
  const double mean = wave_sum_d(sum) / L;
  double m2 = 0.0;
#pragma unroll
  for (int j = 0; j < kSmallPer; ++j) {
    const double d = v[j] - mean;
    if (lane + 64 * j < L) m2 += d * d;
  }
  m2 = wave_sum_d(m2);
  const float mu = (float)mean, is = (float)(1.0 / sqrt(m2 / L + (double)eps));
  if (lane == 0)
    bn_store_stats(c, mean, m2, L, running_mean, running_var, momentum, eps, save_mean, save_invstd, seg_uvar);
  const float ga = gamma[pc], be = beta[pc], al = alpha ? alpha[pc] : 1.f;
  float* yr = y + (long)c * L;
#pragma unroll
  for (int j = 0; j < kSmallPer; ++j) {
    const int i = lane + 64 * j;
    if (i < L) {
      float z = (v[j] - mu) * is * ga + be;
      if (alpha) z = z > 0.f ? z : al * z;
      yr[i] = z;
    }
  }
}

// Backward of the short-row form: row sums in double, gx and the parameter gradients in one launch.
__global__ __launch_bounds__(kNT) void bn_small_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                           int C, int L, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ alpha, float* __restrict__ gx,
                                                           float* __restrict__ ggamma, float* __restrict__ gbeta,
                                                           float* __restrict__ galpha, int accumulate) {
  const int c = blockIdx.x * (kNT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c], al = alpha ? alpha[c] : 1.f;
  const float* xr = x + (long)c * L;
  const float* gr = gy + (long)c * L;
  float xh[kSmallPer], g[kSmallPer];
  double sg = 0.0, sgx = 0.0, sa = 0.0;
#pragma unroll
  for (int j = 0; j < kSmallPer; ++j) {
    const int i = lane + 64 * j;
    xh[j] = 0.f;
    g[j] = 0.f;
    if (i < L) {
      xh[j] = (xr[i] - mu) * is;
      const float gv = gr[i];
      g[j] = gv;
      if (alpha) {
        const float z = xh[j] * ga + be;
        if (!(z > 0.f)) {
          g[j] = gv * al;
          sa += (double)gv * z;
        }
      }
      sg += g[j];
      sgx += (double)g[j] * xh[j];
    }
  }
  sg = wave_sum_d(sg);
  sgx = wave_sum_d(sgx);
  if (alpha) sa = wave_sum_d(sa);
  if (lane == 0) {
    gbeta[c] = accumulate ? gbeta[c] + (float)sg : (float)sg;
    ggamma[c] = accumulate ? ggamma[c] + (float)sgx : (float)sgx;
    if (alpha && galpha) galpha[c] = accumulate ? galpha[c] + (float)sa : (float)sa;
  }
  const float mg = (float)(sg / L), mgx = (float)(sgx / L), k = ga * is;
  float* gxr = gx + (long)c * L;
#pragma unroll
  for (int j = 0; j < kSmallPer; ++j) {
    const int i = lane + 64 * j;
    if (i < L) gxr[i] = k * (g[j] - mg - xh[j] * mgx);
  }
}

// Medium rows (the 4x4 .. 8x8 and 5x5-pool maps of the SK-attention / SE convs: 512 < L <= 8192):
// one block per row, the row held in registers (32 values per thread), double block sums --
// statistics + normalisation + PReLU (and the backward) in ONE launch instead of partial + apply.
constexpr int kMidL = 8192;
constexpr int kMidPer = kMidL / kNT;

__global__ __launch_bounds__(kNT) void bn_mid_fwd_kernel(const float* __restrict__ x, int L,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ alpha, float* running_mean,
                                                         float* running_var, float momentum, float eps,
                                                         float* __restrict__ y, float* __restrict__ save_mean,
                                                         float* __restrict__ save_invstd, int seg,
                                                         float* __restrict__ seg_uvar) {
  __shared__ double sh[kNT / 64];
  const int c = blockIdx.x, tid = threadIdx.x, pc = c / seg;
  const float* row = x + (long)c * L;
  float v[kMidPer];
  double sum = 0.0;
#pragma unroll
  for (int j = 0; j < kMidPer; ++j) {
    const int i = tid + kNT * j;
    v[j] = i < L ? row[i] : 0.f;
    sum += v[j];
  }
  const double mean = block_sum_d(sum, sh) / L;
  double m2 = 0.0;
#pragma unroll
  for (int j = 0; j < kMidPer; ++j) {
    const double d = v[j] - mean;
    if (tid + kNT * j < L) m2 += d * d;
  }
  m2 = block_sum_d(m2, sh);
  const float mu = (float)mean, is = (float)(1.0 / sqrt(m2 / L + (double)eps));
  if (tid == 0)
    bn_store_stats(c, mean, m2, L, running_mean, running_var, momentum, eps, save_mean, save_invstd, seg_uvar);
  const float ga = gamma[pc], be = beta[pc], al = alpha ? alpha[pc] : 1.f;
  float* yr = y + (long)c * L;
#pragma unroll
  for (int j = 0; j < kMidPer; ++j) {
    const int i = tid + kNT * j;
    if (i < L) {
      float z = (v[j] - mu) * is * ga + be;
      if (alpha) z = z > 0.f ? z : al * z;
      yr[i] = z;
    }
  }
}

__global__ __launch_bounds__(kNT) void bn_mid_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                         int L, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ alpha, float* __restrict__ gx,
                                                         float* __restrict__ ggamma, float* __restrict__ gbeta,
                                                         float* __restrict__ galpha, int accumulate) {
  __shared__ double sh[kNT / 64];
  const int c = blockIdx.x, tid = threadIdx.x;
  const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c], al = alpha ? alpha[c] : 1.f;
  const float* xr = x + (long)c * L;
  const float* gr = gy + (long)c * L;
  float xh[kMidPer], g[kMidPer];
  double sg = 0.0, sgx = 0.0, sa = 0.0;
#pragma unroll
  for (int j = 0; j < kMidPer; ++j) {
    const int i = tid + kNT * j;
    xh[j] = 0.f;
    g[j] = 0.f;
    if (i < L) {
      xh[j] = (xr[i] - mu) * is;
      const float gv = gr[i];
      g[j] = gv;
      if (alpha) {
        const float z = xh[j] * ga + be;
        if (!(z > 0.f)) {
          g[j] = gv * al;
          sa += (double)gv * z;
        }
      }
      sg += g[j];
      sgx += (double)g[j] * xh[j];
    }
  }
  sg = block_sum_d(sg, sh);
  sgx = block_sum_d(sgx, sh);
  if (alpha) sa = block_sum_d(sa, sh);
  if (tid == 0) {
    gbeta[c] = accumulate ? gbeta[c] + (float)sg : (float)sg;
    ggamma[c] = accumulate ? ggamma[c] + (float)sgx : (float)sgx;
    if (alpha && galpha) galpha[c] = accumulate ? galpha[c] + (float)sa : (float)sa;
  }
  const float mg = (float)(sg / L), mgx = (float)(sgx / L), k = ga * is;
  float* gxr = gx + (long)c * L;
#pragma unroll
  for (int j = 0; j < kMidPer; ++j) {
    const int i = tid + kNT * j;
    if (i < L) gxr[i] = k * (g[j] - mg - xh[j] * mgx);
  }
}

__global__ __launch_bounds__(kNT) void bn_act_apply_kernel(const float* __restrict__ x, int C, long L,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ alpha, float* __restrict__ y) {
  const long total = (long)C * L;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < total; i += (long)gridDim.x * kNT) {
    const int c = (int)(i / L);
    float z = (x[i] - mean[c]) * invstd[c] * gamma[c] + beta[c];
    if (alpha) z = z > 0.f ? z : alpha[c] * z;
    y[i] = z;
  }
}

// partial sums of g = gy*prelu'(z), g*xhat and gy*min(z,0)  (double, see above)
__global__ __launch_bounds__(kNT) void bn_act_bwd_partial_kernel(
    const float* __restrict__ gy, const float* __restrict__ x, long L, int S, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ alpha, double* __restrict__ part) {
  __shared__ double sh[4];
  const int c = blockIdx.y, s = blockIdx.x;
  const long per = (L + S - 1) / S;
  const long lo = s * per, hi = min(L, lo + per);
  const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
  const float al = alpha ? alpha[c] : 1.f;
  const float* xr = x + (long)c * L;
  const float* gr = gy + (long)c * L;
  double sg = 0.0, sgx = 0.0, sa = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    const float xh = (xr[i] - mu) * is;
    const float gv = gr[i];
    float g = gv;
    if (alpha) {
      const float z = xh * ga + be;
      if (!(z > 0.f)) {
        g = gv * al;
        sa += (double)gv * z;
      }
    }
    sg += g;
    sgx += (double)g * xh;
  }
  sg = block_sum_d(sg, sh);
  sgx = block_sum_d(sgx, sh);
  sa = block_sum_d(sa, sh);
  if (threadIdx.x == 0) {
    double* o = part + ((long)blockIdx.y * S + s) * 3;
    o[0] = sg;
    o[1] = sgx;
    o[2] = sa;
  }
}

// o0..o2 (=|+=) the row sums; s0/s1 (optional) always receive the plain sums of rows 0/1
__global__ void reduce3_kernel(const double* __restrict__ part, int C, int S, float* o0, float* o1, float* o2,
                               int accumulate, float* s0, float* s1) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double* p = part + (long)c * S * 3;
  double a = 0.0, b = 0.0, d = 0.0;
  for (int s = 0; s < S; ++s) {
    a += p[3 * s];
    b += p[3 * s + 1];
    d += p[3 * s + 2];
  }
  if (s0) s0[c] = (float)a;
  if (s1) s1[c] = (float)b;
  if (o0) o0[c] = accumulate ? o0[c] + (float)a : (float)a;
  if (o1) o1[c] = accumulate ? o1[c] + (float)b : (float)b;
  if (o2) o2[c] = accumulate ? o2[c] + (float)d : (float)d;
}

// Fused second stage of the long-row BatchNorm (one launch instead of finalize + apply): block
// (s, c) merges channel c's S partials itself -- the same Chan merge in the same order as
// bn_finalize_kernel, so the statistics are bitwise those of the two-launch form -- and
// normalises its chunk of the row; block (0, c) also stores mean / invstd and the running stats.
__global__ __launch_bounds__(kNT) void bn_act_apply_stats_kernel(
    const float* __restrict__ x, long L, int S, const double* __restrict__ part, float* running_mean,
    float* running_var, float momentum, float eps, float* save_mean, float* save_invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ alpha,
    float* __restrict__ y, int seg, float* __restrict__ seg_uvar) {
  const int c = blockIdx.y, pc = c / seg;
  const double* p = part + (long)c * S * 3;
  double n = 0, mean = 0, m2 = 0;
  for (int s = 0; s < S; ++s) {
    const double nb = p[3 * s], mb = p[3 * s + 1], m2b = p[3 * s + 2];
    if (nb <= 0) continue;
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
  }
  const float mu = (float)mean;
  const float is = (float)(1.0 / sqrt(m2 / (double)L + (double)eps));
  if (blockIdx.x == 0 && threadIdx.x == 0)
    bn_store_stats(c, mean, m2, L, running_mean, running_var, momentum, eps, save_mean, save_invstd, seg_uvar);
  const float ga = gamma[pc], be = beta[pc], al = alpha ? alpha[pc] : 1.f;
  const long per = (L + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = min(L, lo + per);
  const float* xr = x + (long)c * L;
  float* yr = y + (long)c * L;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    float z = (xr[i] - mu) * is * ga + be;
    if (alpha) z = z > 0.f ? z : al * z;
    yr[i] = z;
  }
}

// Segmented BatchNorm (one forward over `seg` independent mini-batches stacked along the batch,
// each normalised by its own statistics): the running statistics take the segments' updates in
// order, exactly as `seg` separate forwards would (momentum m per update).
__global__ void bn_running_seq_kernel(int C, int seg, const float* __restrict__ mean, const float* __restrict__ uvar,
                                      float* running_mean, float* running_var, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float rm = running_mean ? running_mean[c] : 0.f, rv = running_var ? running_var[c] : 0.f;
  for (int s = 0; s < seg; ++s) {
    rm = bn_ema(rm, momentum, mean[c * seg + s]);
    rv = bn_ema(rv, momentum, uvar[c * seg + s]);
  }
  if (running_mean) running_mean[c] = rm;
  if (running_var) running_var[c] = rv;
}

// Fused second stage of the long-row BatchNorm backward (replaces reduce3 + apply): block (s, c)
// sums channel c's partials in the order reduce3_kernel does, block (0, c) writes the parameter
// gradients, and every block forms its chunk of gx.
__global__ __launch_bounds__(kNT) void bn_act_bwd_apply_sums_kernel(
    const float* __restrict__ gy, const float* __restrict__ x, long L, int S, const double* __restrict__ part,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ alpha, float* gbeta, float* ggamma, float* galpha,
    int accumulate, float* __restrict__ gx) {
  const int c = blockIdx.y;
  const double* p = part + (long)c * S * 3;
  double a = 0.0, b = 0.0, d = 0.0;
  for (int s = 0; s < S; ++s) {
    a += p[3 * s];
    b += p[3 * s + 1];
    d += p[3 * s + 2];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    gbeta[c] = accumulate ? gbeta[c] + (float)a : (float)a;
    ggamma[c] = accumulate ? ggamma[c] + (float)b : (float)b;
    if (alpha && galpha) galpha[c] = accumulate ? galpha[c] + (float)d : (float)d;
  }
  const float invL = 1.f / (float)L;
  const float sg = (float)a, sgx = (float)b;   // the float sums bn_act_bwd_apply_kernel reads
  const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c], al = alpha ? alpha[c] : 1.f;
  const long per = (L + gridDim.x - 1) / gridDim.x;
  const long lo = blockIdx.x * per, hi = min(L, lo + per);
  const float* xr = x + (long)c * L;
  const float* gr = gy + (long)c * L;
  float* gxr = gx + (long)c * L;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    const float xh = (xr[i] - mu) * is;
    float g = gr[i];
    if (alpha) {
      const float z = xh * ga + be;
      if (!(z > 0.f)) g *= al;
    }
    gxr[i] = ga * is * (g - sg * invL - xh * sgx * invL);
  }
}

// gx = gamma*invstd*(g - sum(g)/L - xhat*sum(g*xhat)/L); the partial sums were reduced into
// gbeta (= sum g) and ggamma (= sum g*xhat)
__global__ __launch_bounds__(kNT) void bn_act_bwd_apply_kernel(
    const float* __restrict__ gy, const float* __restrict__ x, int C, long L, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ alpha, const float* __restrict__ sum_g, const float* __restrict__ sum_gx,
    float* __restrict__ gx) {
  const long total = (long)C * L;
  const float invL = 1.f / (float)L;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < total; i += (long)gridDim.x * kNT) {
    const int c = (int)(i / L);
    const float is = invstd[c];
    const float xh = (x[i] - mean[c]) * is;
    float g = gy[i];
    if (alpha) {
      const float z = xh * gamma[c] + beta[c];
      if (!(z > 0.f)) g *= alpha[c];
    }
    gx[i] = gamma[c] * is * (g - sum_g[c] * invL - xh * sum_gx[c] * invL);
  }
}

// ---------------------------------------------------------------- PReLU
__global__ __launch_bounds__(kNT) void prelu_fwd_kernel(const float* __restrict__ x, const float* __restrict__ a,
                                                        int C, long L, float* __restrict__ y) {
  const long total = (long)C * L;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < total; i += (long)gridDim.x * kNT) {
    const float v = x[i];
    y[i] = v > 0.f ? v : a[i / L] * v;
  }
}

// Rows of a multiple of 4 elements: 16-byte accesses, 32-bit index arithmetic (n4 < 2^29).
__global__ __launch_bounds__(kNT) void prelu_fwd_vec_kernel(const float* __restrict__ x, const float* __restrict__ a,
                                                            unsigned n4, unsigned L4, float* __restrict__ y) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* x4 = reinterpret_cast<const f4*>(x);
  f4* y4 = reinterpret_cast<f4*>(y);
  for (unsigned i = blockIdx.x * kNT + threadIdx.x; i < n4; i += gridDim.x * kNT) {
    const float al = a[i / L4];
    f4 v = x4[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.f ? v[j] : al * v[j];
    y4[i] = v;
  }
}

// gx (optional) and per-block partials of galpha = sum gy*x over x<=0
__global__ __launch_bounds__(kNT) void prelu_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                        const float* __restrict__ a, long L, int S,
                                                        float* __restrict__ gx, float* __restrict__ part,
                                                        int acc_mode) {
  __shared__ float sh[4];
  const int c = blockIdx.y, s = blockIdx.x;
  const long per = (L + S - 1) / S;
  const long lo = s * per, hi = min(L, lo + per);
  const float al = a[c];
  const long base = (long)c * L;
  float acc = 0.f;
  const bool vec = (L & 3) == 0 && ((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(x) |
                                     reinterpret_cast<uintptr_t>(gx)) & 15) == 0;
  if (vec) {   // 16-byte accesses; the block's range in whole float4s
    typedef float f4 __attribute__((ext_vector_type(4)));
    const long L4 = L / 4, per4 = (L4 + S - 1) / S;
    const long lo4 = s * per4, hi4 = min(L4, lo4 + per4);
    const f4* x4 = reinterpret_cast<const f4*>(x + base);
    const f4* g4 = reinterpret_cast<const f4*>(gy + base);
    f4* o4 = gx ? reinterpret_cast<f4*>(gx + base) : nullptr;
    for (long i = lo4 + threadIdx.x; i < hi4; i += kNT) {
      const f4 v = x4[i], g = g4[i];
      f4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (v[j] > 0.f) {
          o[j] = g[j];
        } else {
          o[j] = al * g[j];
          acc += g[j] * v[j];
        }
      }
      if (o4) o4[i] = o;
    }
  } else {
    for (long i = lo + threadIdx.x; i < hi; i += kNT) {
      const float v = x[base + i], g = gy[base + i];
      if (v > 0.f) {
        if (gx) gx[base + i] = g;
      } else {
        if (gx) gx[base + i] = al * g;
        acc += g * v;
      }
    }
  }
  if (part) {
    acc = block_sum(acc, sh);
    if (threadIdx.x == 0) put_part(part, (long)c * S + s, acc, acc_mode);
  }
}

__global__ __launch_bounds__(kNT) void prelu_bwd_bwd_kernel(const float* __restrict__ ggx,
                                                            const float* __restrict__ gga,
                                                            const float* __restrict__ gy, const float* __restrict__ x,
                                                            const float* __restrict__ a, long L, int S,
                                                            float* __restrict__ ggy, float* __restrict__ gx,
                                                            float* __restrict__ part, int acc_mode) {
  __shared__ float sh[4];
  const int c = blockIdx.y, s = blockIdx.x;
  const long per = (L + S - 1) / S;
  const long lo = s * per, hi = min(L, lo + per);
  const float al = a[c];
  const float ga = gga ? gga[c] : 0.f;
  const long base = (long)c * L;
  float acc = 0.f;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    const float v = x[base + i];
    const float gg = ggx ? ggx[base + i] : 0.f;
    if (v > 0.f) {
      if (ggy) ggy[base + i] = gg;
      if (gx) gx[base + i] = 0.f;
    } else {
      const float g = gy[base + i];
      if (ggy) ggy[base + i] = gg * al + ga * v;
      if (gx) gx[base + i] = ga * g;
      acc += gg * g;
    }
  }
  if (part) {
    acc = block_sum(acc, sh);
    if (threadIdx.x == 0) put_part(part, (long)c * S + s, acc, acc_mode);
  }
}

__global__ void reduce1_kernel(const float* __restrict__ part, int C, int S, float* out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f;
  for (int s = 0; s < S; ++s) a += part[(long)c * S + s];
  out[c] = accumulate ? out[c] + a : a;
}

// ---------------------------------------------------------------- row / plane reductions
__global__ __launch_bounds__(kNT) void row_dot_kernel(const float* __restrict__ a, const float* __restrict__ b, long L,
                                                      int S, float* __restrict__ part, int acc_mode) {
  __shared__ float sh[4];
  const int c = blockIdx.y, s = blockIdx.x;
  const long per = (L + S - 1) / S;
  const long lo = s * per, hi = min(L, lo + per);
  const long base = (long)c * L;
  float acc = 0.f;
  if (b) {
    for (long i = lo + threadIdx.x; i < hi; i += kNT) acc += a[base + i] * b[base + i];
  } else {
    for (long i = lo + threadIdx.x; i < hi; i += kNT) acc += a[base + i];
  }
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) put_part(part, (long)c * S + s, acc, acc_mode);
}

// Plane reductions accumulate in double: they feed the modulated conv's style / demodulation
// gradients, whose two paths nearly cancel (the output is invariant to a common scale of s), so
// their rounding is amplified downstream (tests/test_headline_gpu.py::test_g_step_b16).
// one wave per plane
__global__ __launch_bounds__(kNT) void plane_dot_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                        long planes, long HW, float scale, float* __restrict__ out) {
  const long wave = (blockIdx.x * (long)kNT + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * kNT) >> 6;
  const int lane = threadIdx.x & 63;
  for (long p = wave; p < planes; p += nwaves) {
    const float* ap = a + p * HW;
    double acc = 0.0;
    if (b) {
      const float* bp = b + p * HW;
      for (long i = lane; i < HW; i += 64) acc += (double)ap[i] * bp[i];
    } else {
      for (long i = lane; i < HW; i += 64) acc += ap[i];
    }
    acc = wave_sum_d(acc);
    if (lane == 0) out[p] = (float)(scale * acc);
  }
}

// planes of >= 1024 floats: a 256-thread block per plane, 16-byte loads
__global__ __launch_bounds__(kNT) void plane_dot_big_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                            long HW, float scale, float* __restrict__ out) {
  __shared__ double sh[4];
  typedef float f4 __attribute__((ext_vector_type(4)));
  const long p = blockIdx.x;
  const f4* a4 = reinterpret_cast<const f4*>(a + p * HW);
  const f4* b4 = b ? reinterpret_cast<const f4*>(b + p * HW) : nullptr;
  double acc = 0.0;
  for (long i = threadIdx.x; i < HW / 4; i += kNT) {
    const f4 u = a4[i];
    if (b4) {
      const f4 v = b4[i];
      acc += (double)u[0] * v[0] + (double)u[1] * v[1] + (double)u[2] * v[2] + (double)u[3] * v[3];
    } else {
      acc += (double)u[0] + u[1] + u[2] + u[3];
    }
  }
  acc = block_sum_d(acc, sh);
  if (threadIdx.x == 0) out[p] = (float)(scale * acc);
}

// Two plane dots sharing a: out1[p] = sum a*b1, out2[p] = sum a*b2 -- the modulated conv's
// backward needs <gy, y> and <gy, noise> per (channel, sample); one pass reads gy once.
__global__ __launch_bounds__(kNT) void plane_dot_pair_kernel(const float* __restrict__ a, const float* __restrict__ b1,
                                                             const float* __restrict__ b2, long HW,
                                                             float* __restrict__ out1, float* __restrict__ out2) {
  __shared__ double sh[4];
  typedef float f4 __attribute__((ext_vector_type(4)));
  const long p = blockIdx.x;
  const f4* a4 = reinterpret_cast<const f4*>(a + p * HW);
  const f4* c4 = reinterpret_cast<const f4*>(b1 + p * HW);
  const f4* d4 = reinterpret_cast<const f4*>(b2 + p * HW);
  double s1 = 0.0, s2 = 0.0;
  for (long i = threadIdx.x; i < HW / 4; i += kNT) {
    const f4 u = a4[i], v = c4[i], w = d4[i];
    s1 += (double)u[0] * v[0] + (double)u[1] * v[1] + (double)u[2] * v[2] + (double)u[3] * v[3];
    s2 += (double)u[0] * w[0] + (double)u[1] * w[1] + (double)u[2] * w[2] + (double)u[3] * w[3];
  }
  s1 = block_sum_d(s1, sh);
  s2 = block_sum_d(s2, sh);
  if (threadIdx.x == 0) {
    out1[p] = (float)s1;
    out2[p] = (float)s2;
  }
}

// The modulated conv's style-side gradients from its saved output y = d * conv + ns * noise
// (generator_13_5.py:243-247, 263-265), one block per plane p = (c, b):
//   gd[p]  = dL/dd = <gy, conv> = (<gy, y> - ns[c] <gy, noise>) / d[p]
//   pdn[p] = <gy, noise>              (noise may be null: gd = <gy, y> / d, no pdn)
// Both dots and the combination in double (the two terms nearly cancel when the noise dominates a
// plane); one pass over gy, y and noise instead of a plane-dot launch plus three elementwise ones.
__global__ __launch_bounds__(kNT) void modconv_sd_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                             const float* __restrict__ noise, const float* __restrict__ d,
                                                             const float* __restrict__ ns, int B, long HW,
                                                             float* __restrict__ gd, float* __restrict__ pdn) {
  __shared__ double sh[4];
  typedef float f4 __attribute__((ext_vector_type(4)));
  const long p = blockIdx.x;
  const f4* a4 = reinterpret_cast<const f4*>(gy + p * HW);
  const f4* c4 = reinterpret_cast<const f4*>(y + p * HW);
  double s1 = 0.0, s2 = 0.0;
  if (noise) {
    const f4* d4 = reinterpret_cast<const f4*>(noise + p * HW);
    for (long i = threadIdx.x; i < HW / 4; i += kNT) {
      const f4 u = a4[i], v = c4[i], w = d4[i];
      s1 += (double)u[0] * v[0] + (double)u[1] * v[1] + (double)u[2] * v[2] + (double)u[3] * v[3];
      s2 += (double)u[0] * w[0] + (double)u[1] * w[1] + (double)u[2] * w[2] + (double)u[3] * w[3];
    }
    s2 = block_sum_d(s2, sh);
  } else {
    for (long i = threadIdx.x; i < HW / 4; i += kNT) {
      const f4 u = a4[i], v = c4[i];
      s1 += (double)u[0] * v[0] + (double)u[1] * v[1] + (double)u[2] * v[2] + (double)u[3] * v[3];
    }
  }
  s1 = block_sum_d(s1, sh);
  if (threadIdx.x == 0) {
    const int c = (int)(p / B);
    gd[p] = (float)((noise ? s1 - (double)ns[c] * s2 : s1) / (double)d[p]);
    if (noise) pdn[p] = (float)s2;
  }
}

__global__ void segment_sumsq_kernel(const float* __restrict__ w, long rows, int T, float* __restrict__ out) {
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows; r += (long)gridDim.x * blockDim.x) {
    const float* p = w + r * T;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc += p[t] * p[t];
    out[r] = acc;
  }
}

// ---------------------------------------------------------------- separable resampling
// Separable resampling through LDS: a workgroup stages `ppb` whole input planes (16-byte loads)
// and the two ELL tap tables (KR/KC taps per output row/column, zero-weight padding), applies the
// column table along rows into an LDS intermediate [IH][OW], then the row table along columns
// straight to global memory.  HBM traffic = one read of x + one write of y.  Each thread owns V
// consecutive output columns (V = 4 when OW % 4 == 0: 16-byte LDS/global stores) and walks rows
// with a fixed stride, so there is no per-element index division.
inline __host__ __device__ int align4(int n) { return (n + 3) & ~3; }

template <int V>
__global__ __launch_bounds__(kNT) void resample2d_kernel(const float* __restrict__ x, const float* __restrict__ x2,
                                                         long planes, int IH, int IW, float* __restrict__ y, int OH,
                                                         int OW,
                                                         const int32_t* __restrict__ ri, const float* __restrict__ rw,
                                                         int KR, const int32_t* __restrict__ ci,
                                                         const float* __restrict__ cw, int KC, int ppb,
                                                         const float* __restrict__ r, float* __restrict__ y2,
                                                         const float* __restrict__ r2) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  extern __shared__ float lds[];
  const long p0 = (long)blockIdx.x * ppb;
  const int np = (int)min((long)ppb, planes - p0);
  float* xs = lds;                                  // [ppb][IH][IW]
  float* ts = xs + align4(ppb * IH * IW);           // [ppb][IH][OW]
  float* cws = ts + align4(ppb * IH * OW);          // [OW][KC]
  int* cis = reinterpret_cast<int*>(cws + OW * KC);
  float* rws = reinterpret_cast<float*>(cis + OW * KC);   // [OH][KR]
  int* ris = reinterpret_cast<int*>(rws + OH * KR);
  const int tid = threadIdx.x;
  const int nin = np * IH * IW;
  const float* xg = x + p0 * IH * IW;
  const float* x2g = x2 ? x2 + p0 * IH * IW : nullptr;   // resample of a sum: summed while staging
  if (((IH * IW) & 3) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(x2)) & 15) == 0) {
    for (int i = tid; i < nin / 4; i += kNT) {
      f4 t = reinterpret_cast<const f4*>(xg)[i];
      if (x2g) t += reinterpret_cast<const f4*>(x2g)[i];
      reinterpret_cast<f4*>(xs)[i] = t;
    }
  } else {
    for (int i = tid; i < nin; i += kNT) xs[i] = x2g ? xg[i] + x2g[i] : xg[i];
  }
  for (int i = tid; i < OW * KC; i += kNT) {
    cws[i] = cw[i];
    cis[i] = ci[i];
  }
  for (int i = tid; i < OH * KR; i += kNT) {
    rws[i] = rw[i];
    ris[i] = ri[i];
  }
  __syncthreads();
  const int QW = OW / V;                  // column groups per row (host: QW <= kNT)
  const int q = tid % QW, r0 = tid / QW, rstep = kNT / QW;
  const bool active = r0 < rstep;         // threads past rstep*QW sit out
  if (active) {
    for (int r = r0; r < np * IH; r += rstep) {
      const float* xr = xs + r * IW;
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int o = (q * V + v) * KC;
        float s = 0.f;
        for (int b = 0; b < KC; ++b) s += cws[o + b] * xr[cis[o + b]];
        acc[v] = s;
      }
      float* t = ts + r * OW + q * V;
      if constexpr (V == 4)
        *reinterpret_cast<f4*>(t) = f4{acc[0], acc[1], acc[2], acc[3]};
      else
        t[0] = acc[0];
    }
  }
  __syncthreads();
  if (!active) return;
  for (int rr = r0; rr < np * OH; rr += rstep) {
    const int pl = rr / OH, oh = rr - pl * OH;
    const float* tp = ts + pl * IH * OW + q * V;
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    for (int a = 0; a < KR; ++a) {
      const float w = rws[oh * KR + a];
      const float* t = tp + ris[oh * KR + a] * OW;
      if constexpr (V == 4) {
        const f4 u = *reinterpret_cast<const f4*>(t);
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[v] += w * u[v];
      } else {
        acc[0] += w * t[0];
      }
    }
    // y = R(x) (+ r); y2 = R(x) (+ r2): the residual / fan-out outputs of ganamd_resample2d_add
    const long oi = (p0 * OH + rr) * (long)OW + q * V;
    if constexpr (V == 4) {
      const f4 a = f4{acc[0], acc[1], acc[2], acc[3]};
      *reinterpret_cast<f4*>(y + oi) = r ? a + *reinterpret_cast<const f4*>(r + oi) : a;
      if (y2) *reinterpret_cast<f4*>(y2 + oi) = r2 ? a + *reinterpret_cast<const f4*>(r2 + oi) : a;
    } else {
      y[oi] = r ? acc[0] + r[oi] : acc[0];
      if (y2) y2[oi] = r2 ? acc[0] + r2[oi] : acc[0];
    }
  }
}

// ---------------------------------------------------------------- AdamW
__global__ void step_increment_kernel(int32_t* step) { *step += 1; }

__global__ __launch_bounds__(kNT) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long n,
                                                    const int32_t* __restrict__ step, float lr, float beta1,
                                                    float beta2, float eps, float wd) {
  const double t = (double)*step;
  const float step_size = (float)((double)lr / (1.0 - pow((double)beta1, t)));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, t));
  const float decay = (float)(1.0 - (double)lr * (double)wd);
  const float w = 1.f - beta1;  // lerp weight
  const float omb2 = 1.f - beta2;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const float gi = g[i];
    float pi = p[i] * decay;
    float mi = m[i];
    mi = w < 0.5f ? mi + w * (gi - mi) : gi - (gi - mi) * (1.f - w);
    float vi = v[i] * beta2 + omb2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + (-step_size) * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

inline int ok(hipError_t e) { return e == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH; }

}  // namespace

static int resample_launch(const float* x, const float* x2, long planes, int IH, int IW, float* y, int OH, int OW,
                           const int32_t* ri, const float* rw, int KR, const int32_t* ci, const float* cw, int KC,
                           const float* r, float* y2, const float* r2, hipStream_t st) {
  if (!x || !y || !ri || !rw || !ci || !cw || planes <= 0 || KR <= 0 || KC <= 0) return GANAMD_EINVAL;
  // planes per workgroup: ~2K staged inputs but <= ~8K outputs (an upsampling adjoint such as
  // pool5's 5x5 -> 64x64 would otherwise pack 81 planes, 330K outputs, into each of a few dozen
  // workgroups), LDS <= 48 KB (3 workgroups per CU)
  const int V = (OW % 4 == 0 && ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(r) |
                                  reinterpret_cast<uintptr_t>(y2) | reinterpret_cast<uintptr_t>(r2)) & 15) == 0) ? 4 : 1;
  if (OW / V > kNT || IH <= 0 || IW <= 0 || OH <= 0 || OW <= 0) return GANAMD_EINVAL;
  const long per_plane = (long)IH * IW + (long)IH * OW;
  const long tab = 2L * ((long)OW * KC + (long)OH * KR) + 8;   // tables + alignment slack (floats)
  if ((per_plane + tab) * 4 > 48 * 1024) return GANAMD_EINVAL;
  int ppb = (int)std::max<long>(1, std::min<long>(2048 / ((long)IH * IW), 8192 / ((long)OH * OW)));
  ppb = (int)std::min<long>(ppb, (48 * 1024 / 4 - tab) / per_plane);
  const long blocks = (planes + ppb - 1) / ppb;
  const size_t bytes = 4 * (size_t)(align4(ppb * IH * IW) + align4(ppb * IH * OW) + 2 * (OW * KC + OH * KR));
  if (V == 4)
    hipLaunchKernelGGL(resample2d_kernel<4>, dim3((unsigned)blocks), dim3(kNT), bytes, st, x, x2, planes, IH, IW, y,
                       OH, OW, ri, rw, KR, ci, cw, KC, ppb, r, y2, r2);
  else
    hipLaunchKernelGGL(resample2d_kernel<1>, dim3((unsigned)blocks), dim3(kNT), bytes, st, x, x2, planes, IH, IW, y,
                       OH, OW, ri, rw, KR, ci, cw, KC, ppb, r, y2, r2);
  return ok(hipGetLastError());
}

extern "C" {

// GANAMD_SRC_HASH: hash of the sources this library was compiled from (set by
// __graft_entry__.build(), which rebuilds whenever it differs from the tree's).
#ifndef GANAMD_SRC_HASH
#define GANAMD_SRC_HASH "unknown"
#endif
const char* ganamd_version(void) { return "ganamd 0.2 gfx950 src:" GANAMD_SRC_HASH; }

int ganamd_stream_capture_id(hipStream_t stream, unsigned long long* capture_id) {
  if (!capture_id) return GANAMD_EINVAL;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (hipStreamGetCaptureInfo(stream, &st, &id) != hipSuccess) return GANAMD_ELAUNCH;
  *capture_id = st == hipStreamCaptureStatusActive ? id + 1 : 0;   // ids may start at 0
  return GANAMD_OK;
}

size_t ganamd_rowreduce_workspace(int C, long L) {
  return sizeof(double) * 3 * (size_t)C * splits_for(L) + 2 * sizeof(float) * (size_t)C;
}

int ganamd_bn_act_fwd_seg(const float* x, int C, long L, int seg, const float* gamma, const float* beta,
                          const float* alpha, float* running_mean, float* running_var, float momentum, float eps,
                          float* y, float* save_mean, float* save_invstd, float* seg_uvar, void* workspace,
                          size_t workspace_bytes, hipStream_t st) {
  if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || !workspace || C <= 0 || L <= 0 || seg < 1 ||
      L % seg || (seg > 1 && !seg_uvar) || workspace_bytes < ganamd_rowreduce_workspace(C * seg, L / seg))
    return GANAMD_EINVAL;
  // rows of the segmented problem: (channel, segment), each L / seg long; the parameters of row r
  // are channel r / seg's, the running statistics are updated per segment in order afterwards
  const int R = C * seg;
  const long Lr = L / seg;
  float* rm = seg > 1 ? nullptr : running_mean;
  float* rv = seg > 1 ? nullptr : running_var;
  float* su = seg > 1 ? seg_uvar : nullptr;
  if (Lr <= kSmallL) {
    hipLaunchKernelGGL(bn_small_fwd_kernel, dim3((R + 3) / 4), dim3(kNT), 0, st, x, R, (int)Lr, gamma, beta, alpha,
                       rm, rv, momentum, eps, y, save_mean, save_invstd, seg, su);
  } else if (Lr <= kMidL) {
    hipLaunchKernelGGL(bn_mid_fwd_kernel, dim3(R), dim3(kNT), 0, st, x, (int)Lr, gamma, beta, alpha, rm, rv,
                       momentum, eps, y, save_mean, save_invstd, seg, su);
  } else {
    const int S = splits_for(Lr);
    double* part = static_cast<double*>(workspace);
    hipLaunchKernelGGL(bn_partial_kernel, dim3(S, R), dim3(kNT), 0, st, x, Lr, S, part);
    hipLaunchKernelGGL(bn_act_apply_stats_kernel, dim3(S, R), dim3(kNT), 0, st, x, Lr, S, part, rm, rv, momentum, eps,
                       save_mean, save_invstd, gamma, beta, alpha, y, seg, su);
  }
  if (seg > 1 && (running_mean || running_var))
    hipLaunchKernelGGL(bn_running_seq_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, seg, save_mean, seg_uvar,
                       running_mean, running_var, momentum);
  return ok(hipGetLastError());
}

int ganamd_bn_act_fwd(const float* x, int C, long L, const float* gamma, const float* beta, const float* alpha,
                      float* running_mean, float* running_var, float momentum, float eps, float* y,
                      float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes, hipStream_t st) {
  return ganamd_bn_act_fwd_seg(x, C, L, 1, gamma, beta, alpha, running_mean, running_var, momentum, eps, y, save_mean,
                               save_invstd, nullptr, workspace, workspace_bytes, st);
}

int ganamd_bn_act_bwd(const float* gy, const float* x, int C, long L, const float* gamma, const float* beta,
                      const float* alpha, const float* save_mean, const float* save_invstd, float* gx, float* ggamma,
                      float* gbeta, float* galpha, int accumulate, void* workspace, size_t workspace_bytes,
                      hipStream_t st) {
  if (!gy || !x || !gamma || !beta || !save_mean || !save_invstd || !gx || !ggamma || !gbeta || !workspace ||
      C <= 0 || L <= 0 || workspace_bytes < ganamd_rowreduce_workspace(C, L))
    return GANAMD_EINVAL;
  if (L <= kSmallL) {
    hipLaunchKernelGGL(bn_small_bwd_kernel, dim3((C + 3) / 4), dim3(kNT), 0, st, gy, x, C, (int)L, save_mean,
                       save_invstd, gamma, beta, alpha, gx, ggamma, gbeta, galpha, accumulate);
    return ok(hipGetLastError());
  }
  if (L <= kMidL) {
    hipLaunchKernelGGL(bn_mid_bwd_kernel, dim3(C), dim3(kNT), 0, st, gy, x, (int)L, save_mean, save_invstd, gamma,
                       beta, alpha, gx, ggamma, gbeta, galpha, accumulate);
    return ok(hipGetLastError());
  }
  const int S = splits_for(L);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(bn_act_bwd_partial_kernel, dim3(S, C), dim3(kNT), 0, st, gy, x, L, S, save_mean, save_invstd,
                     gamma, beta, alpha, part);
  hipLaunchKernelGGL(bn_act_bwd_apply_sums_kernel, dim3(S, C), dim3(kNT), 0, st, gy, x, L, S, part, save_mean,
                     save_invstd, gamma, beta, alpha, gbeta, ggamma, galpha, accumulate, gx);
  return ok(hipGetLastError());
}

int ganamd_prelu_fwd(const float* x, const float* alpha, int C, long L, float* y, hipStream_t st) {
  if (!x || !alpha || !y || C <= 0 || L <= 0) return GANAMD_EINVAL;
  const long n = (long)C * L;
  if ((L & 3) == 0 && n < (1L << 31) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0)
    hipLaunchKernelGGL(prelu_fwd_vec_kernel, dim3(grid_for(n / 4)), dim3(kNT), 0, st, x, alpha, (unsigned)(n / 4),
                       (unsigned)(L / 4), y);
  else
    hipLaunchKernelGGL(prelu_fwd_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, x, alpha, C, L, y);
  return ok(hipGetLastError());
}

int ganamd_prelu_bwd(const float* gy, const float* x, const float* alpha, int C, long L, float* gx, float* galpha,
                     int accumulate, void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (!gy || !x || !alpha || C <= 0 || L <= 0 ||
      (galpha && (!workspace || workspace_bytes < ganamd_rowreduce_workspace(C, L))))
    return GANAMD_EINVAL;
  const int S = splits_for(L);
  float* part = galpha ? (S == 1 ? galpha : static_cast<float*>(workspace)) : nullptr;
  hipLaunchKernelGGL(prelu_bwd_kernel, dim3(S, C), dim3(kNT), 0, st, gy, x, alpha, L, S, gx, part,
                     S == 1 ? 1 + (accumulate != 0) : 0);
  if (galpha && S > 1)
    hipLaunchKernelGGL(reduce1_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, C, S, galpha, accumulate);
  return ok(hipGetLastError());
}

int ganamd_prelu_bwd_bwd(const float* ggx, const float* ggalpha, const float* gy, const float* x, const float* alpha,
                         int C, long L, float* ggy, float* gx, float* galpha, void* workspace,
                         size_t workspace_bytes, hipStream_t st) {
  if (!gy || !x || !alpha || C <= 0 || L <= 0 ||
      (galpha && (!workspace || workspace_bytes < ganamd_rowreduce_workspace(C, L))))
    return GANAMD_EINVAL;
  const int S = splits_for(L);
  float* part = galpha ? (S == 1 ? galpha : static_cast<float*>(workspace)) : nullptr;
  hipLaunchKernelGGL(prelu_bwd_bwd_kernel, dim3(S, C), dim3(kNT), 0, st, ggx, ggalpha, gy, x, alpha, L, S, ggy, gx,
                     part, S == 1 ? 1 : 0);
  if (galpha && S > 1)
    hipLaunchKernelGGL(reduce1_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, C, S, galpha, 0);
  return ok(hipGetLastError());
}

int ganamd_prelu_tangent(const float* xd, const float* gy, const float* x, const float* alpha, int C, long L, float* yd,
                         float* galpha, int accumulate, void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (!xd || !gy || !x || !alpha || !yd || C <= 0 || L <= 0 ||
      (galpha && (!workspace || workspace_bytes < ganamd_rowreduce_workspace(C, L))))
    return GANAMD_EINVAL;
  const int S = splits_for(L);
  float* part = galpha ? (S == 1 ? galpha : static_cast<float*>(workspace)) : nullptr;
  hipLaunchKernelGGL(prelu_bwd_bwd_kernel, dim3(S, C), dim3(kNT), 0, st, xd, nullptr, gy, x, alpha, L, S, yd, nullptr,
                     part, S == 1 ? 1 + (accumulate != 0) : 0);
  if (galpha && S > 1)
    hipLaunchKernelGGL(reduce1_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, C, S, galpha, accumulate);
  return ok(hipGetLastError());
}

int ganamd_resample2d(const float* x, long planes, int IH, int IW, float* y, int OH, int OW, const int32_t* ri,
                      const float* rw, int KR, const int32_t* ci, const float* cw, int KC, hipStream_t st) {
  return ganamd_resample2d_sum(x, nullptr, planes, IH, IW, y, OH, OW, ri, rw, KR, ci, cw, KC, st);
}

int ganamd_resample2d_sum(const float* x, const float* x2, long planes, int IH, int IW, float* y, int OH, int OW,
                          const int32_t* ri, const float* rw, int KR, const int32_t* ci, const float* cw, int KC,
                          hipStream_t st) {
  return resample_launch(x, x2, planes, IH, IW, y, OH, OW, ri, rw, KR, ci, cw, KC, nullptr, nullptr, nullptr, st);
}

int ganamd_resample2d_add(const float* x, long planes, int IH, int IW, float* y, int OH, int OW, const int32_t* ri,
                          const float* rw, int KR, const int32_t* ci, const float* cw, int KC, const float* r,
                          float* y2, const float* r2, hipStream_t st) {
  return resample_launch(x, nullptr, planes, IH, IW, y, OH, OW, ri, rw, KR, ci, cw, KC, r, y2, r2, st);
}


int ganamd_plane_dot(const float* a, const float* b, long planes, long HW, float scale, float* out, hipStream_t st) {
  if (!a || !out || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  const long waves = planes;
  int blocks = (int)std::min<long>((waves + 3) / 4, 16384);
  const bool big = HW >= 1024 && (HW % 4) == 0 && (reinterpret_cast<uintptr_t>(a) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(b) & 15) == 0;
  if (big) {
    hipLaunchKernelGGL(plane_dot_big_kernel, dim3((unsigned)planes), dim3(kNT), 0, st, a, b, HW, scale, out);
    return ok(hipGetLastError());
  }
  hipLaunchKernelGGL(plane_dot_kernel, dim3(blocks), dim3(kNT), 0, st, a, b, planes, HW, scale, out);
  return ok(hipGetLastError());
}

int ganamd_plane_dot_pair(const float* a, const float* b1, const float* b2, long planes, long HW, float* out1,
                          float* out2, hipStream_t st) {
  if (!a || !b1 || !b2 || !out1 || !out2 || planes <= 0 || HW <= 0 || HW % 4 ||
      ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b1) | reinterpret_cast<uintptr_t>(b2)) & 15))
    return GANAMD_EINVAL;
  hipLaunchKernelGGL(plane_dot_pair_kernel, dim3((unsigned)planes), dim3(kNT), 0, st, a, b1, b2, HW, out1, out2);
  return ok(hipGetLastError());
}

int ganamd_modconv_sd_bwd(const float* gy, const float* y, const float* noise, const float* d, const float* ns,
                          int C, int B, long HW, float* gd, float* pdn, float* gns, hipStream_t st) {
  if (!gy || !y || !d || !gd || C <= 0 || B <= 0 || HW <= 0 || HW % 4 || (noise && (!ns || !pdn)) ||
      ((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(noise)) & 15))
    return GANAMD_EINVAL;
  hipLaunchKernelGGL(modconv_sd_bwd_kernel, dim3((unsigned)((long)C * B)), dim3(kNT), 0, st, gy, y, noise, d, ns, B, HW,
                     gd, pdn);
  if (noise && gns)   // gns[c] += sum_b pdn[c][b]  (the noise scale's gradient, into the flat buffer)
    hipLaunchKernelGGL(reduce1_kernel, dim3((C + 255) / 256), dim3(256), 0, st, pdn, C, B, gns, 1);
  return ok(hipGetLastError());
}

int ganamd_row_dot(const float* a, const float* b, int C, long L, float* out, int accumulate, void* workspace,
                   size_t workspace_bytes, hipStream_t st) {
  if (!a || !out || !workspace || C <= 0 || L <= 0 || workspace_bytes < ganamd_rowreduce_workspace(C, L))
    return GANAMD_EINVAL;
  const int S = splits_for(L);
  if (S == 1) {
    hipLaunchKernelGGL(row_dot_kernel, dim3(S, C), dim3(kNT), 0, st, a, b, L, S, out, 1 + (accumulate != 0));
    return ok(hipGetLastError());
  }
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(row_dot_kernel, dim3(S, C), dim3(kNT), 0, st, a, b, L, S, part, 0);
  hipLaunchKernelGGL(reduce1_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, C, S, out, accumulate);
  return ok(hipGetLastError());
}

int ganamd_segment_sumsq(const float* w, long rows, int T, float* out, hipStream_t st) {
  if (!w || !out || rows <= 0 || T <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(segment_sumsq_kernel, dim3(grid_for(rows)), dim3(kNT), 0, st, w, rows, T, out);
  return ok(hipGetLastError());
}

int ganamd_adamw(float* p, const float* g, float* m, float* v, long n, int32_t* step, float lr, float beta1,
                 float beta2, float eps, float weight_decay, hipStream_t st) {
  if (!p || !g || !m || !v || !step || n <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(step_increment_kernel, dim3(1), dim3(1), 0, st, step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(kNT), 0, st, p, g, m, v, n, step, lr, beta1, beta2, eps,
                     weight_decay);
  return ok(hipGetLastError());
}

}  // extern "C"
