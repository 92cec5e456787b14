// Row-blocked weight gradient on the split6 pipe: stride-1 "same" K x K convs (K = 3, 5) on maps
// 32 / 64 wide -- the generator's 48- / 96-channel (modulated) convs and the critic's 64- / 128-
// channel block convs, including the critic adjoint's two-segment x*a + xd*g (ganamd_conv_wgrad2).
//
//   dW[m][j][kh][kw] = alpha * sum_n a[m][n] * x[j][b, oh + kh - pad, ow + kw - pad]    (n = b, oh, ow)
//
// The gather GEMM (conv_gemm.hip wgrad_gemm_kernel) runs one tap per block: every K-step stages the
// output-gradient tile A and the tap-shifted input tile B, and splits each fp32 fragment it reads
// into three bf16 planes in registers (4x over for A in its 1 x 4 wave layout) -- at 48 channels
// that split work and the half-rate 16x16x16 products leave the matrix cores at ~0.1 of the split6
// pipe.  Here a block owns one kernel ROW kh and all K taps kw of it: per K-step (32 output pixels
// of one image row) it stages A = a[m][32 px] once (scaled, split into three planes in LDS) and the
// input row segment x[j][36 px] (the 32 pixels + the K - 1 halo columns, clamped or zero padded,
// scaled, split) once; tap kw's B operand is that segment shifted by kw columns, taken in
// registers from two aligned 16-byte LDS reads per plane (an odd shift costs four v_alignbit).
// Staging work per product drops K-fold on B and K-fold on A, and every product is full-rate:
// 32x32 blocks take six v_mfma_f32_32x32x16_bf16, 16-row blocks three paired v_mfma_f32_16x16x32_bf16.
//
// Block: NW waves stacked along M (wave w owns rows m0 + MB*w .. + MB - 1), TN column blocks of MB
// input channels, all K taps of row kh: accumulators TN * K per wave.  Grid: (J tiles, M tiles,
// K rows x splits); split-K partial sums go to a slab the caller reduces.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "patch.h"

namespace ganamd_wrow {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kOOB = (int)0x80000000;
constexpr int KS = 32;                 // output pixels per K-step (one row segment: W % 32 == 0)

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)std::min<long>(bytes, 0x7fffffff),
                                           0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, int off) {
  asm("" : "+v"(off));
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, int off) {
  asm("" : "+v"(off));
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// After each unit's LDS stores the wave waits for them to complete (lgkmcnt(0)) before the next
// unit's split rewrites its registers.  Every variant of this kernel whose schedule moved (the
// round-5 all-kernel-rows rewrite, a two-stage register prefetch, hoisted load offsets) made the
// 96 -> 96 3x3 64x64 scaled instance sum differently run to run, always in A rows that lanes 48-63
// of a unit store; with this wait the hoisted-offset variant passes 8 of 8 determinism runs
// (without it 0 of 5, with 8-byte instead of 16-byte stores 4 of 5): profiles/r06_wrow_lds_store.txt.
// The mechanism is not pinned down (the gather GEMM rewrites its store registers sooner and is
// deterministic); the wait costs ~1.5 % of this kernel's time (126.4 -> 128.1 ms on the A/B set).
#ifndef GANAMD_WROW_DRAIN
#define GANAMD_WROW_DRAIN 1
#endif
__device__ __forceinline__ void lds_store_drain() {
  if (GANAMD_WROW_DRAIN) __builtin_amdgcn_s_waitcnt(0xC07F);   // vmcnt 63, expcnt 7, lgkmcnt 0
}

// exact 3-way split x = h + m + l (RNE; both differences exact in fp32)
template <int N, class V>
__device__ __forceinline__ void split3(const float* x, V& h, V& m, V& l) {
  float r[N];
#pragma unroll
  for (int e = 0; e < N; ++e) {
    h[e] = (__bf16)x[e];
    r[e] = x[e] - (float)h[e];
  }
#pragma unroll
  for (int e = 0; e < N; ++e) {
    m[e] = (__bf16)r[e];
    r[e] -= (float)m[e];
  }
#pragma unroll
  for (int e = 0; e < N; ++e) l[e] = (__bf16)r[e];
}

// A planes: rows of 16 k (one 16-pixel substep); 32-row blocks: the two 8-k halves swapped on odd
// 8-row groups, 16-row blocks (lanes 16-31 on the other half of lanes 0-15's rows): plain -- each
// conflict-free for its ds_read_b128 lane groups (conv_patch.hip poff)
template <int MB>
__device__ __forceinline__ int aoff(int r, int half) {
  return MB == 32 ? r * 16 + 8 * (half ^ ((r >> 3) & 1)) : r * 16 + 8 * half;
}

// elements kw .. kw + 7 of a 16-element bf16 window w (8 dwords): a static shift
template <int KW>
__device__ __forceinline__ bf16x8 shifted(const u32x4& w0, const u32x4& w1) {
  const unsigned d[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
  u32x4 o;
  constexpr int q = KW / 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (KW % 2 == 0)
      o[i] = d[q + i];
    else
      o[i] = __builtin_amdgcn_alignbit(d[q + i + 1], d[q + i], 16);
  }
  return __builtin_bit_cast(bf16x8, o);
}

template <int MB>
__device__ __forceinline__ int mfma_row(int lane, int r) {
  return MB == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : 4 * (lane >> 4) + r;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int MB, int NW, int TN, int KK, bool SCALED>
__global__ __launch_bounds__(64 * NW) void wgrad_row_kernel(Args p) {
  constexpr int NT = 64 * NW, BM = NW * MB, BJ = TN * MB, PAD = (KK - 1) / 2, T = KK * KK;
  constexpr int SEG = KS + KK - 1;                 // staged input columns
  // B row stride (bf16): 112 B (7 16-byte chunks) for 32-row blocks, 96 B (6 chunks) for 16-row
  // blocks -- the row strides whose window reads are conflict-free for each fragment's lane groups
  constexpr int LDB = MB == 32 ? 56 : 48;
  constexpr int PSA = BM * 16, ABUF = 2 * 3 * PSA; // two 16-pixel substeps x three planes
  constexpr int PSB = BJ * LDB, BBUF = 3 * PSB;
  constexpr int AU = BM * 4, AUT = (AU + NT - 1) / NT;   // A units: 8 pixels of one row
  constexpr int BU = BJ * 12, BUT = (BU + NT - 1) / NT;  // B units: 4 columns of one row (48 staged)
  constexpr int NR = MB == 32 ? 16 : 4;
  using acc_t = typename std::conditional<MB == 32, f32x16, f32x4>::type;
  __shared__ __attribute__((aligned(16))) unsigned short As[2][ABUF];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BBUF];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j0 = blockIdx.x * BJ, m0 = blockIdx.y * BM;
  const int kh = blockIdx.z / p.splits, split = blockIdx.z - kh * p.splits;
  const int W = p.W, HW = p.H * W;
  const long L = (long)p.B * HW;                   // row length of a / x
  const int ks_seg = (int)(L / KS);
  const int segs = p.a2 ? 2 : 1;
  const int ks_total = segs * ks_seg;
  const int k0 = split * p.ks_per_split, k1 = min(ks_total, k0 + p.ks_per_split);

  const rsrc_t ra1 = make_rsrc(p.a, 4 * p.M * L), ra2 = make_rsrc(p.a2 ? p.a2 : p.a, 4 * p.M * L);
  const rsrc_t rx1 = make_rsrc(p.x, 4 * p.J * L), rx2 = make_rsrc(p.x2 ? p.x2 : p.x, 4 * p.J * L);
  const rsrc_t rsa = make_rsrc(SCALED ? p.ascale : p.a, SCALED ? 4 * p.M * p.B : 0);
  const rsrc_t rsx = make_rsrc(SCALED ? p.xscale : p.x, SCALED ? 4 * p.J * p.B : 0);

  struct Stage {
    f32x4 ra[AUT][2];
    f32x4 rb[BUT];
    float sa[AUT], sb[BUT];
  };
  // global -> registers for K-step ks
  auto gload = [&](int ks, Stage& S) {
    const bool s2 = ks >= ks_seg;
    const int kl = s2 ? ks - ks_seg : ks;
    const rsrc_t ra = s2 ? ra2 : ra1, rx = s2 ? rx2 : rx1;
    const long n0 = (long)kl * KS;
    const int b = (int)(n0 / HW), rem = (int)(n0 - (long)b * HW);
    const int oh = rem / W, ow0 = rem - oh * W;
#pragma unroll
    for (int e = 0; e < AUT; ++e) {
      const int u = min(tid + e * NT, AU - 1), r = u >> 2, g = u & 3;
      const int m = m0 + r;
      const int off = m < p.M ? (int)(4 * ((long)m * L + n0 + 8 * g)) : kOOB;
      S.ra[e][0] = bload4(ra, off);
      S.ra[e][1] = bload4(ra, off == kOOB ? kOOB : off + 16);
      if (SCALED) S.sa[e] = bload(rsa, m < p.M ? 4 * (m * p.B + b) : kOOB);
    }
    int ih = oh + kh - PAD;
    bool row_in = true;
    if (p.replicate)
      ih = min(max(ih, 0), p.H - 1);
    else
      row_in = ih >= 0 && ih < p.H;
#pragma unroll
    for (int e = 0; e < BUT; ++e) {
      const int u = min(tid + e * NT, BU - 1), jr = u / 12, cg = u - jr * 12;
      const int j = j0 + jr;
      const long rowbase = (long)j * L + (long)b * HW + (long)ih * W;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * cg + q;
        int iw = ow0 - PAD + c;
        bool in = row_in && j < p.J && c < SEG;
        if (p.replicate)
          iw = min(max(iw, 0), W - 1);
        else
          in = in && iw >= 0 && iw < W;
        S.rb[e][q] = bload(rx, in ? (int)(4 * (rowbase + iw)) : kOOB);
      }
      if (SCALED) S.sb[e] = bload(rsx, j < p.J ? 4 * (j * p.B + b) : kOOB);
    }
  };
  // registers -> LDS (scaled, split into the three planes)
  auto sstore = [&](int buf, const Stage& S) {
#pragma unroll
    for (int e = 0; e < AUT; ++e) {
      const int u = tid + e * NT;
      if (u < AU) {
        const int r = u >> 2, g = u & 3;
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = S.ra[e][0][q];
          v[4 + q] = S.ra[e][1][q];
        }
        if (SCALED)
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] *= S.sa[e];
        bf16x8 h, m, l;
        split3<8>(v, h, m, l);
        unsigned short* d = &As[buf][(g >> 1) * 3 * PSA + aoff<MB>(r, g & 1)];
        *reinterpret_cast<bf16x8*>(d) = h;
        *reinterpret_cast<bf16x8*>(d + PSA) = m;
        *reinterpret_cast<bf16x8*>(d + 2 * PSA) = l;
        lds_store_drain();
      }
    }
#pragma unroll
    for (int e = 0; e < BUT; ++e) {
      const int u = tid + e * NT;
      if (u < BU) {
        const int jr = u / 12, cg = u - jr * 12;
        float v[4] = {S.rb[e][0], S.rb[e][1], S.rb[e][2], S.rb[e][3]};
        if (SCALED)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] *= S.sb[e];
        bf16x4 h, m, l;
        split3<4>(v, h, m, l);
        unsigned short* d = &Bs[buf][jr * LDB + 4 * cg];
        *reinterpret_cast<bf16x4*>(d) = h;
        *reinterpret_cast<bf16x4*>(d + PSB) = m;
        *reinterpret_cast<bf16x4*>(d + 2 * PSB) = l;
        lds_store_drain();
      }
    }
  };

  acc_t acc[TN][KK];
#pragma unroll
  for (int jb = 0; jb < TN; ++jb)
#pragma unroll
    for (int t = 0; t < KK; ++t)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[jb][t][r] = 0.f;

  // lane roles: 32x32 -- (r, h): A row r, k = 8h..8h+7; B column r.  16x16 paired -- (r, q):
  // half hf = q & 1 (k = 8hf..), pair hi = q >> 1: A (h|m), (h|l), (m|h); B (h|h), (m|h), (m|l)
  const int fr = MB == 32 ? (lane & 31) : (lane & 15);
  const int fh = MB == 32 ? (lane >> 5) : ((lane >> 4) & 1);
  const int hi = MB == 32 ? 0 : (lane >> 5);
  const int arow = wv * MB + fr;
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {                      // two 16-pixel substeps
      const unsigned short* A = &As[buf][s * 3 * PSA + aoff<MB>(arow, fh)];
      bf16x8 a[3];
      if constexpr (MB == 32) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const bf16x8*>(A + pl * PSA);
      } else {
        a[0] = *reinterpret_cast<const bf16x8*>(A + (hi ? PSA : 0));
        a[1] = *reinterpret_cast<const bf16x8*>(A + (hi ? 2 * PSA : 0));
        a[2] = *reinterpret_cast<const bf16x8*>(A + (hi ? 0 : PSA));
      }
#pragma unroll
      for (int jb = 0; jb < TN; ++jb) {
        const unsigned short* Bp = &Bs[buf][(jb * MB + fr) * LDB + 16 * s + 8 * fh];
        if constexpr (MB == 32) {
          u32x4 w[3][2];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            w[pl][0] = *reinterpret_cast<const u32x4*>(Bp + pl * PSB);
            w[pl][1] = *reinterpret_cast<const u32x4*>(Bp + pl * PSB + 8);
          }
          static_for<0, KK>([&](auto KWc) {
            constexpr int kw = decltype(KWc)::value;
            const bf16x8 bh = shifted<kw>(w[0][0], w[0][1]), bm = shifted<kw>(w[1][0], w[1][1]),
                         bl = shifted<kw>(w[2][0], w[2][1]);
            acc_t& c = acc[jb][kw];
            // l*h, h*l, m*m, m*h, h*m, h*h: smallest first into the same accumulator
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bl, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bm, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bm, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bh, c, 0, 0, 0);
          });
        } else {
          // planes h and X = (hi ? l : m) of this lane's window
          u32x4 wh0 = *reinterpret_cast<const u32x4*>(Bp), wh1 = *reinterpret_cast<const u32x4*>(Bp + 8);
          const unsigned short* Xp = Bp + (hi ? 2 * PSB : PSB);
          u32x4 wx0 = *reinterpret_cast<const u32x4*>(Xp), wx1 = *reinterpret_cast<const u32x4*>(Xp + 8);
          static_for<0, KK>([&](auto KWc) {
            constexpr int kw = decltype(KWc)::value;
            const bf16x8 bh = shifted<kw>(wh0, wh1), bx = shifted<kw>(wx0, wx1);
            acc_t& c = acc[jb][kw];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], hi ? bh : bx, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bx, c, 0, 0, 0);
          });
        }
      }
    }
  };

  if (k0 < k1) {
    Stage s0;
    gload(k0, s0);
    sstore(0, s0);
    __syncthreads();
    for (int ks = k0; ks < k1; ++ks) {
      const int buf = (ks - k0) & 1;
      const bool more = ks + 1 < k1;
      if (more) gload(ks + 1, s0);
      compute(buf);
      if (more) sstore(buf ^ 1, s0);
      __syncthreads();
    }
  }

  // epilogue: every block writes its whole tile (zeros for an empty K range)
  const long numel = (long)p.M * p.J * T;
#pragma unroll
  for (int jb = 0; jb < TN; ++jb) {
    const int j = j0 + jb * MB + (lane & (MB - 1));
    if (j >= p.J) continue;
#pragma unroll
    for (int kw = 0; kw < KK; ++kw) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int m = m0 + wv * MB + mfma_row<MB>(lane, r);
        if (m >= p.M) continue;
        const long o = ((long)m * p.J + j) * T + kh * KK + kw;
        const float v = p.alpha * acc[jb][kw][r];
        if (p.slab)
          p.slab[(long)split * numel + o] = v;
        else if (p.accumulate)
          p.out[o] += v;
        else
          p.out[o] = v;
      }
    }
  }
}

// tile of M rows: 16-row blocks (paired 16x16x32) x 3 waves for M <= 48, else 32-row blocks, one wave each
struct Tile {
  int mb, nw, tn;
};
Tile tile_of(int M) {
  if (M <= 48) return {16, 3, 3};
  return {32, (M + 31) / 32, 1};
}

template <int MB, int NW, int TN, int KK, bool S>
hipError_t go(const Args& a, hipStream_t st) {
  const dim3 grid((a.J + TN * MB - 1) / (TN * MB), (a.M + NW * MB - 1) / (NW * MB), KK * a.splits);
  hipLaunchKernelGGL((wgrad_row_kernel<MB, NW, TN, KK, S>), grid, dim3(64 * NW), 0, st, a);
  return hipGetLastError();
}

template <int KK, bool S>
hipError_t go_tile(const Args& a, hipStream_t st) {
  const Tile t = tile_of(a.M);
  if (t.mb == 16) return go<16, 3, 3, KK, S>(a, st);
  switch (t.nw) {
    case 2: return go<32, 2, 1, KK, S>(a, st);
    case 3: return go<32, 3, 1, KK, S>(a, st);
    case 4: return go<32, 4, 1, KK, S>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW, int transposed) {
  return !transposed && stride == 1 && (K == 3 || K == 5) && pad == (K - 1) / 2 && OH == H && OW == W &&
         (W == 32 || W == 64) && M >= 1 && M <= 128;
}

// Split-K: enough blocks for about two rounds of the chip at the kernel's occupancy (~2 blocks per
// CU), each split at least 16 K-steps (512 pixels).
void plan(int M, int J, int B, int H, int W, int K, int segs, int cus, int* splits, int* ks_per_split) {
  const Tile t = tile_of(M);
  const long tiles = (long)((J + t.tn * t.mb - 1) / (t.tn * t.mb)) * ((M + t.nw * t.mb - 1) / (t.nw * t.mb)) * K;
  const long ks_total = (long)segs * B * H * W / KS;
  const long target = 4L * cus;
  long s = std::max<long>(1, (target + tiles - 1) / tiles);
  s = std::min<long>(s, std::max<long>(1, ks_total / 16));
  s = std::min<long>(s, 256);
  const long per = (ks_total + s - 1) / s;
  *ks_per_split = (int)per;
  *splits = (int)((ks_total + per - 1) / per);
}

hipError_t launch(const Args& a, hipStream_t st) {
  if (!domain(a.M, a.H, a.W, a.KK, 1, (a.KK - 1) / 2, a.H, a.W, 0) || !a.a || !a.x || !a.out ||
      (a.splits > 1 && !a.slab) || (a.a2 && (a.ascale || a.xscale)) || (!a.ascale != !a.xscale))
    return hipErrorInvalidValue;
  const bool s = a.ascale != nullptr;
  if (a.KK == 3) return s ? go_tile<3, true>(a, st) : go_tile<3, false>(a, st);
  return s ? go_tile<5, true>(a, st) : go_tile<5, false>(a, st);
}

}  // namespace ganamd_wrow
