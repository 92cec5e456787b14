// Fused per-plane elementwise kernels of the generator / critic blocks (gfx950).
//
// Tensors are CNHW, i.e. `planes` = C*B contiguous planes of HW floats; a per-(channel, sample)
// coefficient vector [C][B] is indexed by the plane number.  These kernels replace chains of
// 3-6 torch elementwise launches (and their full-tensor round trips through HBM):
//   mix        y = sum_m att[m] * f_m                 SK mixing (generator_13_5.py:80-89,165-170,196-202)
//   mix_bwd    gf_m = g * att[m],  gatt[m] = <g, f_m>_plane   (one pass over g and the f_m)
//   add_prelu  y = PReLU(a + b)                       ResnetInit outputs (generator_13_5.py:343-349)
//   scale_add  y = r + x * s                          SE gating + residual (generator_13_5.py:455-466,
//                                                     discriminator_9_4.py:158-161); r may be null
// All HBM-bound: one read of each input and one write of each output.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ganamd.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kNT = 256;
constexpr int kRouteMax = GANAMD_ROUTE_MAX;

inline int grid_for(long n) { return (int)std::max<long>(1, std::min<long>((n + kNT - 1) / kNT, 16384)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct Ptr4 {
  const float* p[4];
};
struct MPtr4 {
  float* p[4];
};

// y = sum_m att[m][plane] * f_m ; 4 elements per thread when HW % 4 == 0
template <int M, bool VEC>
__global__ __launch_bounds__(kNT) void mix_fwd_kernel(Ptr4 f, const float* __restrict__ att, long planes, long HW,
                                                      float* __restrict__ y) {
  const long n = planes * HW / (VEC ? 4 : 1);
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const long p = (VEC ? 4 * i : i) / HW;
    if (VEC) {
      f32x4 acc = reinterpret_cast<const f32x4*>(f.p[0])[i] * att[p];
#pragma unroll
      for (int m = 1; m < M; ++m) acc += reinterpret_cast<const f32x4*>(f.p[m])[i] * att[m * planes + p];
      reinterpret_cast<f32x4*>(y)[i] = acc;
    } else {
      float acc = f.p[0][i] * att[p];
#pragma unroll
      for (int m = 1; m < M; ++m) acc += f.p[m][i] * att[m * planes + p];
      y[i] = acc;
    }
  }
}

// gf_m = g * att[m], gatt[m] = sum g * f_m.  Small planes: one wave per plane.  Planes of >= 1024
// floats: one 256-thread block per plane with 16-byte accesses.
template <int M>
__global__ __launch_bounds__(kNT) void mix_bwd_kernel(Ptr4 f, const float* __restrict__ att, long planes, long HW,
                                                      const float* __restrict__ g, MPtr4 gf, float* __restrict__ gatt) {
  const long wave = (blockIdx.x * (long)kNT + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * kNT) >> 6;
  const int lane = threadIdx.x & 63;
  for (long p = wave; p < planes; p += nwaves) {
    const long base = p * HW;
    float a[M];
    double dot[M];   // plane dots in double: the style gradient <g, x*...> cancels against the
                     // demodulation path, so its rounding is amplified (tests/test_headline_gpu.py)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      a[m] = att[m * planes + p];
      dot[m] = 0.0;
    }
    for (long i = lane; i < HW; i += 64) {
      const float gv = g[base + i];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (gf.p[m]) gf.p[m][base + i] = gv * a[m];
        dot[m] += (double)gv * f.p[m][base + i];
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double d = wave_sum_d(dot[m]);
      if (lane == 0 && gatt) gatt[m * planes + p] = (float)d;
    }
  }
}

template <int M>
__global__ __launch_bounds__(kNT) void mix_bwd_plane_kernel(Ptr4 f, const float* __restrict__ att, long planes,
                                                            long HW, const float* __restrict__ g, MPtr4 gf,
                                                            float* __restrict__ gatt) {
  __shared__ double sh[M][4];
  const long p = blockIdx.x;
  const long base4 = p * HW / 4, n4 = HW / 4;
  float a[M];
  double dot[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = att[m * planes + p];
    dot[m] = 0.0;
  }
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g) + base4;
  for (long i = threadIdx.x; i < n4; i += kNT) {
    const f32x4 gv = g4[i];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (gf.p[m]) reinterpret_cast<f32x4*>(gf.p[m])[base4 + i] = gv * a[m];
      const f32x4 fv = reinterpret_cast<const f32x4*>(f.p[m])[base4 + i];
      dot[m] += (double)gv[0] * fv[0] + (double)gv[1] * fv[1] + (double)gv[2] * fv[2] + (double)gv[3] * fv[3];
    }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const double d = wave_sum_d(dot[m]);
    if (lane == 0) sh[m][w] = d;
  }
  __syncthreads();
  if (threadIdx.x < M && gatt) {
    const int m = threadIdx.x;
    gatt[m * planes + p] = (float)(sh[m][0] + sh[m][1] + sh[m][2] + sh[m][3]);
  }
}

__global__ __launch_bounds__(kNT) void add_prelu_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                        const float* __restrict__ alpha, int C, long L,
                                                        float* __restrict__ y) {
  const long n = (long)C * L;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const float z = a[i] + b[i];
    y[i] = z > 0.f ? z : alpha[i / L] * z;
  }
}

template <bool VEC>
__global__ __launch_bounds__(kNT) void scale_add_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                        const float* __restrict__ r, long planes, long HW,
                                                        float* __restrict__ y) {
  const long n = planes * HW / (VEC ? 4 : 1);
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const float sv = s[(VEC ? 4 * i : i) / HW];
    if (VEC) {
      f32x4 v = reinterpret_cast<const f32x4*>(x)[i] * sv;
      if (r) v += reinterpret_cast<const f32x4*>(r)[i];
      reinterpret_cast<f32x4*>(y)[i] = v;
    } else {
      float v = x[i] * sv;
      if (r) v += r[i];
      y[i] = v;
    }
  }
}

inline int ok(hipError_t e) { return e == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH; }

bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int M>
void launch_mix_fwd(const Ptr4& f, const float* att, long planes, long HW, float* y, hipStream_t st) {
  bool vec = (HW % 4) == 0 && aligned16(y);
  for (int m = 0; m < M; ++m) vec = vec && aligned16(f.p[m]);
  const long n = planes * HW / (vec ? 4 : 1);
  if (vec)
    hipLaunchKernelGGL((mix_fwd_kernel<M, true>), dim3(grid_for(n)), dim3(kNT), 0, st, f, att, planes, HW, y);
  else
    hipLaunchKernelGGL((mix_fwd_kernel<M, false>), dim3(grid_for(n)), dim3(kNT), 0, st, f, att, planes, HW, y);
}

template <int M>
void launch_mix_bwd(const Ptr4& f, const float* att, long planes, long HW, const float* g, const MPtr4& gf,
                    float* gatt, hipStream_t st) {
  bool vec = HW >= 1024 && (HW % 4) == 0 && aligned16(g);
  for (int m = 0; m < M; ++m) vec = vec && aligned16(f.p[m]) && aligned16(gf.p[m]);
  if (vec) {
    hipLaunchKernelGGL((mix_bwd_plane_kernel<M>), dim3((unsigned)planes), dim3(kNT), 0, st, f, att, planes, HW, g,
                       gf, gatt);
    return;
  }
  const int blocks = (int)std::min<long>((planes + 3) / 4, 16384);
  hipLaunchKernelGGL((mix_bwd_kernel<M>), dim3(blocks), dim3(kNT), 0, st, f, att, planes, HW, g, gf, gatt);
}

// ---------------------------------------------------------------- gradient penalty
// GP = lambda * mean_b (||g_b|| - center)^2 over g = grad_x D(x_hat) [B][n]
// (train/wgangp.py:34-54, lambda 10 at :68; R1/R2 of wganlazygpR2.py use the squared norm
// without the root: mode 1).  Pass 1: per-(sample, chunk) double partial sums of g^2; pass 2
// (one block): the norms and the penalty.  The backward is one elementwise pass:
//   dGP/dg = gout * lambda * 2 (||g_b|| - center) / (B ||g_b||) * g      (mode 0)
//   dR/dg  = gout * lambda * 2 / B * g                                   (mode 1)
constexpr long kGpChunk = 4096;

__global__ __launch_bounds__(kNT) void gp_partial_kernel(const float* __restrict__ g, long n, int S,
                                                         double* __restrict__ part) {
  __shared__ double sh[4];
  const int b = blockIdx.y, s = blockIdx.x;
  const long per = (n + S - 1) / S;
  const long lo = s * per, hi = min(n, lo + per);
  const float* row = g + (long)b * n;
  double acc = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += kNT) {
    const double v = row[i];
    acc += v * v;
  }
  // block sum (4 waves)
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long)b * S + s] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(kNT) void gp_finalize_kernel(const double* __restrict__ part, int B, int S, float center,
                                                          float lambda, int mode, float* __restrict__ norms,
                                                          float* __restrict__ out) {
  __shared__ double sh[kNT];
  double acc = 0.0;
  for (int b = threadIdx.x; b < B; b += kNT) {
    double sq = 0.0;
    for (int s = 0; s < S; ++s) sq += part[(long)b * S + s];
    const double nb = mode == 0 ? sqrt(sq) : sq;
    norms[b] = (float)nb;
    acc += mode == 0 ? (nb - center) * (nb - center) : nb;
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < kNT; ++i) t += sh[i];
    out[0] = (float)(lambda * t / B);
  }
}

__global__ __launch_bounds__(kNT) void gp_backward_kernel(const float* __restrict__ g, const float* __restrict__ norms,
                                                          const float* __restrict__ gout, long n, int B, float center,
                                                          float lambda, int mode, float* __restrict__ dg) {
  const long total = (long)B * n;
  const float go = gout[0];
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < total; i += (long)gridDim.x * kNT) {
    const int b = (int)(i / n);
    float k;
    if (mode == 0) {
      const float nb = norms[b];
      k = nb > 0.f ? go * lambda * 2.f * (nb - center) / ((float)B * nb) : 0.f;
    } else {
      k = go * lambda * 2.f / (float)B;
    }
    dg[i] = k * g[i];
  }
}

// route backward: gx[c][:] = sum over the parts i with lo_i <= c < hi_i of g_i[c - lo_i][:] (part
// order), 0 where no part covers c.  The gradient of several channel-range views of one CNHW tensor
// (the dual-path blocks' x[:d] / x[d:] / x[2d:] splits, generator_13_5.py:448-467, 496-564) in one
// pass -- instead of one zero-filled full-size tensor per slice plus the adds that sum them.
struct RouteParts {
  const float* g[kRouteMax];
  int lo[kRouteMax], hi[kRouteMax];
  int n;
};
template <bool VEC>
__global__ __launch_bounds__(kNT) void route_bwd_kernel(RouteParts r, int C, long L, float* __restrict__ gx) {
  const long Lv = VEC ? L / 4 : L;
  const long n = (long)C * Lv;
  for (long i = blockIdx.x * (long)kNT + threadIdx.x; i < n; i += (long)gridDim.x * kNT) {
    const int c = (int)(i / Lv);
    const long e = i - (long)c * Lv;
    if (VEC) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < r.n; ++k)
        if (c >= r.lo[k] && c < r.hi[k]) acc += reinterpret_cast<const f32x4*>(r.g[k])[(long)(c - r.lo[k]) * Lv + e];
      reinterpret_cast<f32x4*>(gx)[i] = acc;
    } else {
      float acc = 0.f;
      for (int k = 0; k < r.n; ++k)
        if (c >= r.lo[k] && c < r.hi[k]) acc += r.g[k][(long)(c - r.lo[k]) * L + e];
      gx[i] = acc;
    }
  }
}

}  // namespace

extern "C" {

size_t ganamd_gp_workspace(int B, long n) {
  const long S = std::min<long>(64, std::max<long>(1, (n + kGpChunk - 1) / kGpChunk));
  return sizeof(double) * (size_t)B * S;
}

int ganamd_gp_fwd(const float* g, int B, long n, float center, float lambda, int mode, float* norms, float* out,
                  void* workspace, size_t workspace_bytes, hipStream_t st) {
  if (!g || !norms || !out || !workspace || B <= 0 || n <= 0 || (mode != 0 && mode != 1) ||
      workspace_bytes < ganamd_gp_workspace(B, n))
    return GANAMD_EINVAL;
  const int S = (int)std::min<long>(64, std::max<long>(1, (n + kGpChunk - 1) / kGpChunk));
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(gp_partial_kernel, dim3(S, B), dim3(kNT), 0, st, g, n, S, part);
  hipLaunchKernelGGL(gp_finalize_kernel, dim3(1), dim3(kNT), 0, st, part, B, S, center, lambda, mode, norms, out);
  return ok(hipGetLastError());
}

int ganamd_gp_bwd(const float* g, const float* norms, const float* gout, int B, long n, float center, float lambda,
                  int mode, float* dg, hipStream_t st) {
  if (!g || !norms || !gout || !dg || B <= 0 || n <= 0 || (mode != 0 && mode != 1)) return GANAMD_EINVAL;
  hipLaunchKernelGGL(gp_backward_kernel, dim3(grid_for((long)B * n)), dim3(kNT), 0, st, g, norms, gout, n, B, center,
                     lambda, mode, dg);
  return ok(hipGetLastError());
}

int ganamd_mix_fwd(int M, const float* f0, const float* f1, const float* f2, const float* f3, const float* att,
                   long planes, long HW, float* y, hipStream_t st) {
  const Ptr4 f{{f0, f1, f2, f3}};
  if (M < 1 || M > 4 || !att || !y || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  for (int m = 0; m < M; ++m)
    if (!f.p[m]) return GANAMD_EINVAL;
  switch (M) {
    case 1: launch_mix_fwd<1>(f, att, planes, HW, y, st); break;
    case 2: launch_mix_fwd<2>(f, att, planes, HW, y, st); break;
    case 3: launch_mix_fwd<3>(f, att, planes, HW, y, st); break;
    default: launch_mix_fwd<4>(f, att, planes, HW, y, st); break;
  }
  return ok(hipGetLastError());
}

int ganamd_mix_bwd(int M, const float* f0, const float* f1, const float* f2, const float* f3, const float* att,
                   long planes, long HW, const float* gy, float* gf0, float* gf1, float* gf2, float* gf3, float* gatt,
                   hipStream_t st) {
  const Ptr4 f{{f0, f1, f2, f3}};
  const MPtr4 gf{{gf0, gf1, gf2, gf3}};
  if (M < 1 || M > 4 || !att || !gy || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  for (int m = 0; m < M; ++m)
    if (!f.p[m]) return GANAMD_EINVAL;
  switch (M) {
    case 1: launch_mix_bwd<1>(f, att, planes, HW, gy, gf, gatt, st); break;
    case 2: launch_mix_bwd<2>(f, att, planes, HW, gy, gf, gatt, st); break;
    case 3: launch_mix_bwd<3>(f, att, planes, HW, gy, gf, gatt, st); break;
    default: launch_mix_bwd<4>(f, att, planes, HW, gy, gf, gatt, st); break;
  }
  return ok(hipGetLastError());
}

int ganamd_add_prelu(const float* a, const float* b, const float* alpha, int C, long L, float* y, hipStream_t st) {
  if (!a || !b || !alpha || !y || C <= 0 || L <= 0) return GANAMD_EINVAL;
  hipLaunchKernelGGL(add_prelu_kernel, dim3(grid_for((long)C * L)), dim3(kNT), 0, st, a, b, alpha, C, L, y);
  return ok(hipGetLastError());
}

int ganamd_scale_add(const float* x, const float* s, const float* r, long planes, long HW, float* y, hipStream_t st) {
  if (!x || !s || !y || planes <= 0 || HW <= 0) return GANAMD_EINVAL;
  const bool vec = (HW % 4) == 0 && aligned16(x) && aligned16(r) && aligned16(y);
  const long n = planes * HW / (vec ? 4 : 1);
  if (vec)
    hipLaunchKernelGGL((scale_add_kernel<true>), dim3(grid_for(n)), dim3(kNT), 0, st, x, s, r, planes, HW, y);
  else
    hipLaunchKernelGGL((scale_add_kernel<false>), dim3(grid_for(n)), dim3(kNT), 0, st, x, s, r, planes, HW, y);
  return ok(hipGetLastError());
}

int ganamd_route_bwd(int n, const float* const* g, const int32_t* lo, const int32_t* hi, int C, long L, float* gx,
                     hipStream_t st) {
  if (n < 0 || n > kRouteMax || !gx || C <= 0 || L <= 0 || (n && (!g || !lo || !hi))) return GANAMD_EINVAL;
  RouteParts r{};
  r.n = n;
  bool vec = (L % 4) == 0 && aligned16(gx);
  for (int k = 0; k < n; ++k) {
    if (!g[k] || lo[k] < 0 || hi[k] > C || lo[k] >= hi[k]) return GANAMD_EINVAL;
    r.g[k] = g[k];
    r.lo[k] = lo[k];
    r.hi[k] = hi[k];
    vec = vec && aligned16(g[k]);
  }
  const long m = (long)C * L / (vec ? 4 : 1);
  if (vec)
    hipLaunchKernelGGL((route_bwd_kernel<true>), dim3(grid_for(m)), dim3(kNT), 0, st, r, C, L, gx);
  else
    hipLaunchKernelGGL((route_bwd_kernel<false>), dim3(grid_for(m)), dim3(kNT), 0, st, r, C, L, gx);
  return ok(hipGetLastError());
}

}  // extern "C"
