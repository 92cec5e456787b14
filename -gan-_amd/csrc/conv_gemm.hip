// Implicit-GEMM convolution family for gfx950 (CDNA4), fp32 in / fp32 accumulate on MFMA.
//
// Activations live in CNHW ("channel rows") layout: x[c][b][h][w].  With that layout every
// convolution the WGAN-GP hot path issues is one GEMM whose output is already row-major:
//
//   forward   Y[co][n]      = alpha * sum_{t,ci} W(co,t,ci) * G_x(t,ci,n) (* out_scale[co][b]) + bias[co]
//   dgrad     dXp[ci][n']   = alpha * sum_{t,co} W(co,t,ci) * T_gy(t,co,n')  then fold padding
//   wgrad     dW(co,ci,t)  += alpha * sum_n gy[co][n] * G_x(t,ci,n)
//
// n = (b, oh, ow).  G_x is the im2col gather of x (replication- or zero-padded, any stride) and
// T_gy the transposed-conv gather; neither is ever materialised.  Per-(channel, sample) scales
// on either operand carry the StyleGAN2 weight modulation (x*s) and demodulation (d) so the
// modulated conv of generator_13_5.py:219-248 runs as a batch-shared GEMM.
//
// Reference semantics replaced: F.conv2d over ReplicationPad2d (generator_13_5.py:36-38,
// discriminator_9_4.py:38-40), the grouped per-sample conv (generator_13_5.py:243-247),
// nn.ConvTranspose2d (generator_13_5.py:156,594), and their autograd backward.
//
// Tiling: 256 threads = 4 waves; block tile BM x BN, K-step BK; each wave owns a
// (32*TM) x (32*TN) sub-tile built from v_mfma_f32_32x32x2f32.  LDS holds both operand tiles
// k-major ([k][m], [k][n]) so a lane's A/B fragment element is one conflict-free ds_read_b32;
// tiles are double buffered (one barrier per K-step) and the next tile's global gather is
// issued into registers before the MFMAs of the current one.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ganamd.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int kThreads = 256;

// Gather of a CNHW source tensor as a GEMM operand indexed by (tap, channel, n).
struct Gather {
  const float* src;
  const float* scale;  // optional [C][B] per-(channel, sample) multiplier
  int C, B, H, W;      // source extents
  int OH, OW;          // GEMM spatial extents (n = (b, oh, ow))
  int KW, stride, pad;
  int mode;            // 0: conv, zero pad; 1: conv, replication pad; 2: transposed conv
};

// Offset of source pixel feeding output (oh, ow) through tap (kh, kw), or -1 if it is padding.
__device__ __forceinline__ int tap_offset(const Gather& g, int oh, int ow, int kh, int kw) {
  int ih, iw;
  if (g.mode == 2) {
    int th = oh + g.pad - kh, tw = ow + g.pad - kw;
    if (th < 0 || tw < 0) return -1;
    if (g.stride > 1) {
      if ((th % g.stride) | (tw % g.stride)) return -1;
      th /= g.stride;
      tw /= g.stride;
    }
    if (th >= g.H || tw >= g.W) return -1;
    ih = th;
    iw = tw;
  } else {
    ih = oh * g.stride - g.pad + kh;
    iw = ow * g.stride - g.pad + kw;
    if (g.mode == 1) {
      ih = min(max(ih, 0), g.H - 1);
      iw = min(max(iw, 0), g.W - 1);
    } else if (ih < 0 || iw < 0 || ih >= g.H || iw >= g.W) {
      return -1;
    }
  }
  return ih * g.W + iw;
}

struct ConvArgs {
  const float* w;      // A(m, t, c) = w[m*sm + c*sc + t*st]
  long sm, sc, st;
  int M, Ck, T;        // GEMM rows, channels per tap, taps
  Gather g;
  float* y;            // Y[m][n]
  const float* bias;   // [M] or null
  const float* oscale; // [M][B] or null
  float alpha;
  int N, ohw;          // N = B*OH*OW
  int kt_per_split, atomic;
};

struct WgradArgs {
  const float* a;      // A(m, n) = a[m*lda + n] (* ascale[m][b])
  const float* ascale;
  long lda;
  int M, J, K, ohw;    // rows, gathered channels, K = B*OH*OW
  Gather g;            // B(n, j): channel j of the gather at tap t
  float* out;          // out[m*om + j*oj + t*ot]
  long om, oj, ot;
  float alpha;
  int kt_per_split, splits, atomic;
};

template <int BM, int BN, int BK, int WGM, int WGN>
struct TileCfg {
  static constexpr int TM = BM / (32 * WGM);
  static constexpr int TN = BN / (32 * WGN);
  static constexpr int PA = BM + 2;  // +2 floats: the k-strided LDS stores hit distinct banks
  static constexpr int PB = BN + 2;
  static_assert(WGM * WGN == 4, "4 waves per block");
  static_assert(TM * 32 * WGM == BM && TN * 32 * WGN == BN, "tile must split into 32x32 MFMAs");
  static_assert(kThreads % BK == 0, "k index must be thread-invariant");
};

// One K-step of MFMAs from LDS.  lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31].
template <class C, int BK>
__device__ __forceinline__ void mfma_step(const float* __restrict__ As, const float* __restrict__ Bs,
                                          f32x16 (&acc)[C::TM][C::TN], int lane, int wm, int wn) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < BK / 2; ++s) {
    const int kk = 2 * s + h;
    float a[C::TM], b[C::TN];
#pragma unroll
    for (int i = 0; i < C::TM; ++i) a[i] = As[kk * C::PA + (wm * C::TM + i) * 32 + r];
#pragma unroll
    for (int j = 0; j < C::TN; ++j) b[j] = Bs[kk * C::PB + (wn * C::TN + j) * 32 + r];
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------
// forward / dgrad / transposed: K = (tap, channel), N = output pixels
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int WGM, int WGN>
__global__ __launch_bounds__(kThreads) void conv_gemm_kernel(ConvArgs p) {
  using C = TileCfg<BM, BN, BK, WGM, WGN>;
  constexpr int EA = BK * BM / kThreads;
  constexpr int EB = BK * BN / kThreads;
  static_assert(kThreads % BN == 0 || BN % kThreads == 0, "B mapping");
  __shared__ float As[2][BK * C::PA];
  __shared__ float Bs[2][BK * C::PB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int nct = (p.Ck + BK - 1) / BK;
  const int kt_total = nct * p.T;
  const int kt0 = blockIdx.z * p.kt_per_split;
  const int kt1 = min(kt_total, kt0 + p.kt_per_split);
  if (kt0 >= kt1) return;

  // A mapping: k fixed per thread, m strided
  const int a_k = tid % BK;
  const int a_m = tid / BK;
  constexpr int A_MSTEP = kThreads / BK;
  // B mapping: n fixed per thread, k strided
  const int b_n = tid % BN;
  const int b_k = tid / BN;
  constexpr int B_KSTEP = kThreads / BN;

  const Gather& g = p.g;
  const int gn = n0 + b_n;
  const bool n_ok = gn < p.N;
  int bb = 0, oh = 0, ow = 0;
  if (n_ok) {
    bb = gn / p.ohw;
    const int rr = gn - bb * p.ohw;
    oh = rr / g.OW;
    ow = rr - oh * g.OW;
  }
  const long cstride = (long)g.B * g.H * g.W;
  const float* src_b = g.src + (long)bb * g.H * g.W;

  float ra[EA], rb[EB];
  int cur_t = -1, sp = -1;

  auto gload = [&](int kt) {
    const int t = kt / nct;
    const int c0 = (kt - t * nct) * BK;
    if (t != cur_t) {
      cur_t = t;
      sp = n_ok ? tap_offset(g, oh, ow, t / g.KW, t - (t / g.KW) * g.KW) : -1;
    }
    {
      const int c = c0 + a_k;
      const bool cok = c < p.Ck;
      const float* wp = p.w + (long)c * p.sc + (long)t * p.st;
#pragma unroll
      for (int e = 0; e < EA; ++e) {
        const int m = m0 + a_m + e * A_MSTEP;
        ra[e] = (cok && m < p.M) ? wp[(long)m * p.sm] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int c = c0 + b_k + e * B_KSTEP;
      float v = 0.f;
      if (sp >= 0 && c < p.Ck) {
        v = src_b[(long)c * cstride + sp];
        if (g.scale) v *= g.scale[(long)c * g.B + bb];
      }
      rb[e] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EA; ++e) As[buf][a_k * C::PA + a_m + e * A_MSTEP] = ra[e];
#pragma unroll
    for (int e = 0; e < EB; ++e) Bs[buf][(b_k + e * B_KSTEP) * C::PB + b_n] = rb[e];
  };

  f32x16 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(kt0);
  sstore(0);
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) gload(kt + 1);
    mfma_step<C, BK>(As[buf], Bs[buf], acc, lane, wm, wn);
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool add_bias = p.bias && blockIdx.z == 0;
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int n = n0 + (wn * C::TN + j) * 32 + (lane & 31);
    if (n >= p.N) continue;
    const int b = p.oscale ? n / p.ohw : 0;
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * C::TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        float v = p.alpha * acc[i][j][r];
        if (p.oscale) v *= p.oscale[(long)m * g.B + b];
        if (add_bias) v += p.bias[m];
        float* dst = p.y + (long)m * p.N + n;
        if (p.atomic)
          atomicAdd(dst, v);
        else
          *dst = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// wgrad: K = output pixels n, M = output channels of the conv, N = gathered channels at tap t
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int WGM, int WGN>
__global__ __launch_bounds__(kThreads) void wgrad_gemm_kernel(WgradArgs p) {
  using C = TileCfg<BM, BN, BK, WGM, WGN>;
  constexpr int EA = BK * BM / kThreads;
  constexpr int EB = BK * BN / kThreads;
  constexpr int MSTEP = kThreads / BK;
  __shared__ float As[2][BK * C::PA];
  __shared__ float Bs[2][BK * C::PB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int j0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int t = blockIdx.z / p.splits;
  const int split = blockIdx.z - t * p.splits;
  const int kt_total = (p.K + BK - 1) / BK;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(kt_total, kt0 + p.kt_per_split);
  if (kt0 >= kt1) return;

  const Gather& g = p.g;
  const int kh = t / g.KW, kw = t - kh * g.KW;
  const long cstride = (long)g.B * g.H * g.W;
  const int tk = tid % BK;   // k fixed per thread for both operands
  const int tr = tid / BK;   // row (m or j) base

  float ra[EA], rb[EB];
  auto gload = [&](int kt) {
    const int n = kt * BK + tk;
    const bool nok = n < p.K;
    int b = 0, sp = -1;
    if (nok) {
      b = n / p.ohw;
      const int rr = n - b * p.ohw;
      const int oh = rr / g.OW;
      sp = tap_offset(g, oh, rr - oh * g.OW, kh, kw);
    }
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int m = m0 + tr + e * MSTEP;
      float v = 0.f;
      if (nok && m < p.M) {
        v = p.a[(long)m * p.lda + n];
        if (p.ascale) v *= p.ascale[(long)m * g.B + b];
      }
      ra[e] = v;
    }
    const float* src_b = g.src + (long)b * g.H * g.W + sp;
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int jj = j0 + tr + e * MSTEP;
      float v = 0.f;
      if (sp >= 0 && jj < p.J) {
        v = src_b[(long)jj * cstride];
        if (g.scale) v *= g.scale[(long)jj * g.B + b];
      }
      rb[e] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EA; ++e) As[buf][tk * C::PA + tr + e * MSTEP] = ra[e];
#pragma unroll
    for (int e = 0; e < EB; ++e) Bs[buf][tk * C::PB + tr + e * MSTEP] = rb[e];
  };

  f32x16 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(kt0);
  sstore(0);
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) gload(kt + 1);
    mfma_step<C, BK>(As[buf], Bs[buf], acc, lane, wm, wn);
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int jj = j0 + (wn * C::TN + j) * 32 + (lane & 31);
    if (jj >= p.J) continue;
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * C::TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        float* dst = p.out + (long)m * p.om + (long)jj * p.oj + (long)t * p.ot;
        const float v = p.alpha * acc[i][j][r];
        if (p.atomic)
          atomicAdd(dst, v);
        else
          *dst = v;
      }
    }
  }
}

// Sum the replication-padded dgrad image back onto the edge pixels (ReplicationPad2d backward),
// or crop it for zero padding.  xp: [C*B][Hp][Wp] -> x: [C*B][H][W].
__global__ void fold_pad_kernel(const float* __restrict__ xp, float* __restrict__ x, long planes, int H, int W,
                                int pad, int replicate) {
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const long total = planes * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = i % W;
    const int h = (i / W) % H;
    const long pl = i / ((long)H * W);
    const float* s = xp + pl * Hp * Wp;
    if (!replicate) {
      x[i] = s[(h + pad) * Wp + (w + pad)];
      continue;
    }
    const int h0 = h == 0 ? 0 : h + pad, h1 = h == H - 1 ? Hp - 1 : h + pad;
    const int w0 = w == 0 ? 0 : w + pad, w1 = w == W - 1 ? Wp - 1 : w + pad;
    float acc = 0.f;
    for (int a = h0; a <= h1; ++a)
      for (int c = w0; c <= w1; ++c) acc += s[a * Wp + c];
    x[i] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int WGM, int WGN>
hipError_t launch_conv(ConvArgs p, hipStream_t st) {
  const int gx = (p.N + BN - 1) / BN, gy = (p.M + BM - 1) / BM;
  const int nct = (p.Ck + BK - 1) / BK;
  const int kt_total = nct * p.T;
  int splits = 1;
  const int blocks = gx * gy;
  if (blocks < 1024 && kt_total >= 8) {
    splits = (1024 + blocks - 1) / blocks;
    splits = min(splits, max(1, kt_total / 4));
  }
  p.kt_per_split = (kt_total + splits - 1) / splits;
  splits = (kt_total + p.kt_per_split - 1) / p.kt_per_split;
  p.atomic = splits > 1;
  if (p.atomic) {
    hipError_t e = hipMemsetAsync(p.y, 0, sizeof(float) * (size_t)p.M * p.N, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WGM, WGN>), dim3(gx, gy, splits), dim3(kThreads), 0, st, p);
  return hipGetLastError();
}

hipError_t dispatch_conv(const ConvArgs& p, hipStream_t st) {
  if (p.M <= 32) return launch_conv<32, 256, 16, 1, 4>(p, st);
  if (p.M <= 64) return launch_conv<64, 128, 16, 2, 2>(p, st);
  if (p.M <= 96) return launch_conv<96, 128, 16, 1, 4>(p, st);
  return launch_conv<128, 128, 16, 2, 2>(p, st);
}

template <int BM, int BN, int BK, int WGM, int WGN>
hipError_t launch_wgrad(WgradArgs p, int T, int accumulate, hipStream_t st) {
  const int gx = (p.J + BN - 1) / BN, gy = (p.M + BM - 1) / BM;
  const int kt_total = (p.K + BK - 1) / BK;
  const int blocks = gx * gy * T;
  int splits = 1;
  if (blocks < 1024) splits = min((1024 + blocks - 1) / blocks, max(1, kt_total / 4));
  p.kt_per_split = (kt_total + splits - 1) / splits;
  splits = (kt_total + p.kt_per_split - 1) / p.kt_per_split;
  p.splits = splits;
  p.atomic = splits > 1 || accumulate;
  hipLaunchKernelGGL((wgrad_gemm_kernel<BM, BN, BK, WGM, WGN>), dim3(gx, gy, T * splits), dim3(kThreads), 0, st, p);
  return hipGetLastError();
}

hipError_t dispatch_wgrad(const WgradArgs& p, int T, int accumulate, hipStream_t st) {
  if (p.M <= 32) return launch_wgrad<32, 128, 32, 1, 4>(p, T, accumulate, st);
  if (p.M <= 64) return launch_wgrad<64, 64, 32, 2, 2>(p, T, accumulate, st);
  if (p.M <= 96) return launch_wgrad<96, 128, 32, 1, 4>(p, T, accumulate, st);
  return launch_wgrad<128, 128, 32, 2, 2>(p, T, accumulate, st);
}

bool desc_ok(const ganamd_conv_desc* d) {
  return d && d->B > 0 && d->Cin > 0 && d->Cout > 0 && d->H > 0 && d->W > 0 && d->OH > 0 && d->OW > 0 &&
         d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0;
}

}  // namespace

extern "C" {

int ganamd_conv_workspace(const ganamd_conv_desc* d, int op, size_t* bytes) {
  if (!desc_ok(d) || !bytes) return GANAMD_EINVAL;
  *bytes = 0;
  if (op == GANAMD_CONV_DGRAD && !d->transposed && d->pad > 0) {
    const size_t hp = d->H + 2 * d->pad, wp = d->W + 2 * d->pad;
    *bytes = sizeof(float) * (size_t)d->Cin * d->B * hp * wp;
  }
  return GANAMD_OK;
}

int ganamd_conv_fwd(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias,
                    const float* x_scale, const float* y_scale, float alpha, float* y, hipStream_t stream) {
  if (!desc_ok(d) || !x || !w || !y) return GANAMD_EINVAL;
  ConvArgs p{};
  const int T = d->KH * d->KW;
  p.w = w;
  if (d->transposed) {  // weights [Cin][Cout][KH][KW]
    p.sm = T;
    p.sc = (long)d->Cout * T;
  } else {              // weights [Cout][Cin][KH][KW]
    p.sm = (long)d->Cin * T;
    p.sc = T;
  }
  p.st = 1;
  p.M = d->Cout;
  p.Ck = d->Cin;
  p.T = T;
  p.g = Gather{x, x_scale, d->Cin, d->B, d->H, d->W, d->OH, d->OW, d->KW, d->stride, d->pad,
               d->transposed ? 2 : (d->pad_mode == GANAMD_PAD_REPLICATE ? 1 : 0)};
  p.y = y;
  p.bias = bias;
  p.oscale = y_scale;
  p.alpha = alpha;
  p.N = d->B * d->OH * d->OW;
  p.ohw = d->OH * d->OW;
  return dispatch_conv(p, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

int ganamd_conv_dgrad(const ganamd_conv_desc* d, const float* gy, const float* w, const float* gy_scale, float alpha,
                      float* gx, void* workspace, hipStream_t stream) {
  if (!desc_ok(d) || !gy || !w || !gx) return GANAMD_EINVAL;
  const int T = d->KH * d->KW;
  ConvArgs p{};
  p.w = w;
  p.st = 1;
  p.M = d->Cin;
  p.Ck = d->Cout;
  p.T = T;
  p.bias = nullptr;
  p.oscale = nullptr;
  p.alpha = alpha;
  if (d->transposed) {
    // dX of ConvT = plain zero-padded conv of gy with W viewed [Cin][Cout][KH][KW]
    p.sm = (long)d->Cout * T;
    p.sc = T;
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->H, d->W, d->KW, d->stride, d->pad, 0};
    p.y = gx;
    p.N = d->B * d->H * d->W;
    p.ohw = d->H * d->W;
    return dispatch_conv(p, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  // dX of conv = transposed gather of gy into the padded input frame, then fold the pad
  p.sm = T;
  p.sc = (long)d->Cin * T;
  const int Hp = d->H + 2 * d->pad, Wp = d->W + 2 * d->pad;
  float* out = d->pad > 0 ? static_cast<float*>(workspace) : gx;
  if (d->pad > 0 && !workspace) return GANAMD_EINVAL;
  p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, Hp, Wp, d->KW, d->stride, 0, 2};
  p.y = out;
  p.N = d->B * Hp * Wp;
  p.ohw = Hp * Wp;
  if (dispatch_conv(p, stream) != hipSuccess) return GANAMD_ELAUNCH;
  if (d->pad > 0) {
    const long planes = (long)d->Cin * d->B;
    const long total = planes * d->H * d->W;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(fold_pad_kernel, dim3(blocks), dim3(256), 0, stream, out, gx, planes, d->H, d->W, d->pad,
                       d->pad_mode == GANAMD_PAD_REPLICATE ? 1 : 0);
    if (hipGetLastError() != hipSuccess) return GANAMD_ELAUNCH;
  }
  return GANAMD_OK;
}

int ganamd_conv_wgrad(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x_scale,
                      const float* gy_scale, float alpha, float* gw, int accumulate, hipStream_t stream) {
  if (!desc_ok(d) || !x || !gy || !gw) return GANAMD_EINVAL;
  const int T = d->KH * d->KW;
  WgradArgs p{};
  p.alpha = alpha;
  p.ot = 1;
  if (d->transposed) {
    // dW[ci][co][t] = sum_n x[ci][n] * gy[co][conv-gather_t(n)]
    p.a = x;
    p.ascale = x_scale;
    p.lda = (long)d->B * d->H * d->W;
    p.M = d->Cin;
    p.J = d->Cout;
    p.K = d->B * d->H * d->W;
    p.ohw = d->H * d->W;
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->H, d->W, d->KW, d->stride, d->pad, 0};
    p.om = (long)d->Cout * T;
    p.oj = T;
  } else {
    // dW[co][ci][t] = sum_n gy[co][n] * x[ci][gather_t(n)]
    p.a = gy;
    p.ascale = gy_scale;
    p.lda = (long)d->B * d->OH * d->OW;
    p.M = d->Cout;
    p.J = d->Cin;
    p.K = d->B * d->OH * d->OW;
    p.ohw = d->OH * d->OW;
    p.g = Gather{x, x_scale, d->Cin, d->B, d->H, d->W, d->OH, d->OW, d->KW, d->stride, d->pad,
                 d->pad_mode == GANAMD_PAD_REPLICATE ? 1 : 0};
    p.om = (long)d->Cin * T;
    p.oj = T;
  }
  p.out = gw;
  const size_t wsz = sizeof(float) * (size_t)d->Cin * d->Cout * T;
  if (!accumulate) {
    if (hipMemsetAsync(gw, 0, wsz, stream) != hipSuccess) return GANAMD_ELAUNCH;
  }
  return dispatch_wgrad(p, T, 1, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

}  // extern "C"
