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
// Tiling.  256 threads = 4 waves; block tile BM x BN, K-step BK = 16; each wave owns a
// (MB*TM) x (MB*TN) sub-tile of MB x MB MFMA blocks.  fp32 products run as six bf16 products of
// exactly split operands (split6, below): the conv fwd/dgrad body (conv_body_x3) stages the split
// planes in LDS; the wgrad body keeps fp32 tiles in LDS ("k-contiguous" [m][k] / [n][k], row
// stride BK+2 floats, four conflict-free ds_read_b64 per lane) and splits the fragments it reads.
// Global gathers are branch-free (every lane loads from a valid address, padding is a select)
// so hipcc keeps all of a tile's loads in flight; per-(channel,sample) scales are applied when
// the prefetched registers are written to LDS.  Tiles are double buffered (one barrier per
// K-step) and the next tile's gather is issued before the current tile's MFMAs.

#include <atomic>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "../../include/ganamd.h"
#include "patch.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int kThreads = 256;
#ifndef GANAMD_BK
#define GANAMD_BK 16
#endif
constexpr int BK = GANAMD_BK; // conv K-step (taps x channels)
constexpr int LDK = BK + 2;   // LDS row stride in floats: 8-byte aligned, b64 reads conflict-free
#ifndef GANAMD_BKW
#define GANAMD_BKW 32
#endif
constexpr int BKW = GANAMD_BKW; // wgrad K-step (pixels): at 32 a half-wave reads one full 128-byte line
constexpr int LDKW = BKW + 2;

// kPhase: one output phase (oh % s, ow % s) of a stride-s transposed conv as a stride-1 conv over the
// input with the (K/s)^2 taps that reach it (Gather.pch/pcw: input offsets of that phase).
enum GatherMode { kZero = 0, kReplicate = 1, kTransposed = 2, kPhase = 3 };

// Buffer loads: a 32-bit byte offset against a range-checked descriptor.  An offset past the
// end returns 0 in hardware, so padding / tails are a select of the OFFSET, never a branch
// around the load (hipcc would otherwise branch and wait vmcnt per element).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kOOB = (int)0x80000000;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ float bload(rsrc_t r, int byte_off) {
  asm("" : "+v"(byte_off));  // opaque: keeps hipcc from re-splitting the select into branches
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 bload4(rsrc_t r, int byte_off) {
  asm("" : "+v"(byte_off));
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// Gather of a CNHW source tensor as a GEMM operand indexed by (tap, channel, n).
struct Gather {
  const float* src;
  const float* scale;  // optional [C][B] per-(channel, sample) multiplier
  int C, B, H, W;      // source extents
  int OH, OW;          // GEMM spatial extents (n = (b, oh, ow))
  int KW, stride, pad;
  int mode;
  int pch, pcw;        // kPhase: ih = oh + pch - kh, iw = ow + pcw - kw

  __device__ int src_bytes() const { return 4 * C * B * H * W; }
  __device__ int scale_bytes() const { return 4 * C * B; }
};

// Offset of the source pixel feeding output (oh, ow) through tap (kh, kw), or -1 for padding.
template <int MODE>
__device__ __forceinline__ int tap_offset(const Gather& g, int oh, int ow, int kh, int kw) {
  if (MODE == kPhase) {
    const int ih = oh + g.pch - kh, iw = ow + g.pcw - kw;
    if (ih < 0 || iw < 0 || ih >= g.H || iw >= g.W) return -1;
    return ih * g.W + iw;
  }
  if (MODE == kTransposed) {
    int th = oh + g.pad - kh, tw = ow + g.pad - kw;
    if (th < 0 || tw < 0) return -1;
    if (g.stride > 1) {
      if ((th % g.stride) | (tw % g.stride)) return -1;
      th /= g.stride;
      tw /= g.stride;
    }
    if (th >= g.H || tw >= g.W) return -1;
    return th * g.W + tw;
  }
  int ih = oh * g.stride - g.pad + kh;
  int iw = ow * g.stride - g.pad + kw;
  if (MODE == kReplicate) {
    ih = min(max(ih, 0), g.H - 1);
    iw = min(max(iw, 0), g.W - 1);
    return ih * g.W + iw;
  }
  if (ih < 0 || iw < 0 || ih >= g.H || iw >= g.W) return -1;
  return ih * g.W + iw;
}

// Output column of GEMM column n: the identity, or for one phase (qh, qw) of a stride-s transposed
// conv n = (b, j, i) over the OHp x OWp phase grid -> (b, s*j + qh, s*i + qw) of the OH x OW output.
//
// s = -2 (ring only, the stride-1 dgrad next to conv_patch_kernel's interior): n = (b, ring position)
// over B x Rn; the gather reads frame point ring_coord(position) and the result goes to `ring`.
// s = -1 (frame split, the stride-1 dgrad): n = (b, a, c) over the (H+2p) x (W+2p) padded input
// frame (ohwp = its size, OWp = its width, OW = W, OHW = H*W, qh = p, qw = H); interior positions
// go straight to the input gradient, ring positions to `ring` ([row][b][Rn], Rn ring positions
// per image, row stride ldr) -- dropped for zero padding (ring = null), folded onto the edge
// pixels by ring_fold_kernel for replication padding.  No frame buffer, no full fold pass.
//
// s = -3 (phased frame split, the stride-s dgrad): n = (b, j, i) over one phase (pqa, pqc) of the
// padded frame, phase grid pgw wide and pgs = rows * pgw big; frame point (ps*j + pqa, ps*i + pqc),
// then as s = -1 (the other fields are those of s = -1).
struct OutMap {
  int s, qh, qw, OWp, ohwp, OW, OHW;
  int Rn;
  long ldr;
  float* ring;
  int ps, pqa, pqc, pgw, pgs;
};
__device__ __forceinline__ long out_col(const OutMap& r, int n) {
  if (r.s == 0) return n;
  const int b = n / r.ohwp, q = n - b * r.ohwp, j = q / r.OWp, i = q - j * r.OWp;
  return (long)b * r.OHW + (long)(r.s * j + r.qh) * r.OW + r.s * i + r.qw;
}
// ring position index of frame point (a, c) (not interior): top rows, bottom rows, then the
// 2p side columns of the H middle rows
__host__ __device__ __forceinline__ int ring_idx(int a, int c, int p, int H, int W, int Wp) {
  if (a < p) return a * Wp + c;
  if (a >= p + H) return (a - H) * Wp + c;
  return 2 * p * Wp + (a - p) * 2 * p + (c < p ? c : c - W);
}
// inverse of ring_idx: frame point (a, c) of ring position idx
__host__ __device__ __forceinline__ void ring_coord(int idx, int p, int H, int W, int Wp, int& a, int& c) {
  if (idx < 2 * p * Wp) {
    const int r = idx / Wp;
    c = idx - r * Wp;
    a = r < p ? r : r + H;
    return;
  }
  const int j = idx - 2 * p * Wp, r = j / (2 * p), q = j - r * (2 * p);
  a = p + r;
  c = q < p ? q : q + W;
}
// frame split: destination (base, row stride, column) of GEMM column n; false = not stored
__device__ __forceinline__ bool frame_target(const OutMap& r, float* y, long ldy, int n, float*& base, long& ld,
                                             long& col) {
  const int p = r.qh, H = r.qw, W = r.OW;
  int b, a, c;
  if (r.s == -3) {
    b = n / r.pgs;
    const int q = n - b * r.pgs, j = q / r.pgw, i = q - j * r.pgw;
    a = r.ps * j + r.pqa;
    c = r.ps * i + r.pqc;
  } else {
    b = n / r.ohwp;
    const int q = n - b * r.ohwp;
    a = q / r.OWp;
    c = q - a * r.OWp;
  }
  if (a >= p && a < p + H && c >= p && c < p + W) {
    base = y;
    ld = ldy;
    col = (long)b * r.OHW + (long)(a - p) * W + (c - p);
    return true;
  }
  if (!r.ring) return false;
  base = r.ring;
  ld = r.ldr;
  col = (long)b * r.Rn + ring_idx(a, c, p, H, W, r.OWp);
  return true;
}

struct ConvArgs {
  const float* w;      // packed A[Mpad][T][Ckp] (see pack_a_kernel); before packing A(m,t,c) = w[m*sm + c*sc + t*st]
  int sm, sc, st, w_bytes;
  int M, Ck, T;        // GEMM rows, channels per tap, taps
  int Ckp;             // Ck rounded up to whole K-steps
  Gather g;
  float* y;            // Y[m][n]
  const float* bias;   // [M] or null
  const float* oscale; // [M][B] or null
  const float* noise;  // [M][N] or null: + noise_scale[m] * noise[m][n]   (StyleConv noise)
  const float* noise_scale;
  const float* act;    // [M] or null: PReLU with these slopes, applied last
  float alpha;
  int N, ohw;          // N = B*OH*OW
  // Block schedule (see ConvPlan): blocks [0, full_blocks) own whole tiles of the first nfull_t
  // column tiles (m fastest); the remaining blocks split the K range of the tail tiles S ways.
  int gy, full_blocks, nfull_t, S, kt_per_split;
  int tail_n0, tail_cols;  // first tail column (pixel) and the tail width
  float* slab;         // S > 1: per-split partial tail tiles [S][M][tail_cols]
  int bf16;            // GANAMD_MATH_BF16: operands rounded to bf16, fp32 accumulation
  OutMap om;           // GEMM column -> output column (identity unless kPhase)
  long ldy;            // row length of y (N unless kPhase: the full B*OH*OW)
};

struct WgradArgs {
  const float* a;      // A(m, n) = a[m*lda + n] (* ascale[m][b])
  const float* ascale;
  int lda, a_bytes;
  int M, J, K, ohw;    // rows, gathered channels, K = B*OH*OW
  Gather g;            // B(n, j): channel j of the gather at tap t
  float* out;          // out[m*om + j*oj + t*ot]
  int om, oj, ot;
  float alpha;
  int kt_per_split, splits, accumulate;
  int T;               // taps (tap-packed launches: the GEMM's N is (tap, channel) pairs)
  float* slab;         // split-K: per-split partial weights [split][numel(out)] (null: single split)
  int out_numel;
  int bf16;
  // two K segments (ganamd_conv_wgrad2): pixels [segK, 2 segK) read a2 / src2 (unscaled only;
  // segK % BKW == 0 so no K-step straddles the boundary).  0: one segment.
  const float* a2;
  const float* src2;
  int segK;
};

template <int BM, int BN, int WGM, int WGN>
struct TileCfg {
  // MFMA block edge: 32 (v_mfma_f32_32x32x2_f32) unless a wave's sub-tile is not a multiple of
  // 32 (48-row conv tiles, 96-wide wgrad tiles: v_mfma_f32_16x16x4_f32, same FLOP rate per CU,
  // 16-granular tiles)
  static constexpr int MB = ((BM / WGM) % 32 == 0 && (BN / WGN) % 32 == 0) ? 32 : 16;
  static constexpr int TM = BM / (MB * WGM);
  static constexpr int TN = BN / (MB * WGN);
  static constexpr int NR = MB == 32 ? 16 : 4;   // accumulator registers per block and lane
  using acc_t = typename std::conditional<MB == 32, f32x16, f32x4>::type;
  static_assert(WGM * WGN == 4, "4 waves per block");
  static_assert(TM * MB * WGM == BM && TN * MB * WGN == BN, "tile must split into MFMA blocks");
};
// C/D map of the block MFMAs: lane's register r holds row mfma_row<MB>(lane, r), column lane % MB
template <int MB>
__device__ __forceinline__ int mfma_row(int lane, int r) {
  return MB == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : 4 * (lane >> 4) + r;
}

// Read this lane's 8 k-values of one 32-row fragment: rows r of the [row][k] tile, k = 8h..8h+7.
template <int LD>
__device__ __forceinline__ void read_frag(const float* __restrict__ base, float (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 t = *reinterpret_cast<const f32x2*>(base + 2 * q);
    v[2 * q] = t[0];
    v[2 * q + 1] = t[1];
  }
}

// One 16-deep K-step of MFMAs for a wave over LDS tiles of row stride LD, starting at column
// k0.  In step s lane half h supplies k = k0 + 8h + s.
//
// bf16 math (GANAMD_MATH_BF16, the bf16 configuration): the same LDS tiles and lane reads; the
// lane's 8 k-values are rounded to bf16 (RNE) and ONE v_mfma_f32_32x32x16_bf16 replaces the 8
// f32 steps -- its operand map is exactly this one (lane (r, h) holds A[r][8h + j] and
// B[8h + j][r], j = 0..7) and its C/D map that of 32x32x2 f32, so nothing else changes.
// ---- fp32 products on the bf16 matrix cores (split6) --------------------------------------------
// x = h + m + l with h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (RNE; the two differences
// are exact in fp32), so x is kept to 24 significant bits.  x * y is then the six bf16 products
// with at least one high part -- hh + (hm + mh) + (hl + lh + mm) -- exact in the MFMA; the three
// dropped ones (ml, lm, ll) are below 2^-24 |x y|, fp32's own rounding.  Six
// v_mfma_f32_32x32x16_bf16 (6 x 32 cycles) replace eight v_mfma_f32_32x32x2_f32 (8 x 64); 16-row
// blocks: six half-rate v_mfma_f32_16x16x16_bf16 here, three paired full-rate 16x16x32 in the LDS
// body (mfma_tile_x3).
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ f32x16 mfma6_32(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                           const bf16x8& bm, const bf16x8& bl, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma6_16(const bf16x4& ah, const bf16x4& am, const bf16x4& al, const bf16x4& bh,
                                          const bf16x4& bm, const bf16x4& bl, f32x4 acc) {
#define GANAMD_M16(x, y) __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, x), \
                                                                   __builtin_bit_cast(s16x4, y), acc, 0, 0, 0)
  acc = GANAMD_M16(al, bh);
  acc = GANAMD_M16(ah, bl);
  acc = GANAMD_M16(am, bm);
  acc = GANAMD_M16(am, bh);
  acc = GANAMD_M16(ah, bm);
  acc = GANAMD_M16(ah, bh);
#undef GANAMD_M16
  return acc;
}

template <class C, int LD = LDK, bool BF16 = false>
__device__ __forceinline__ void mfma_tile(const float* __restrict__ As, const float* __restrict__ Bs,
                                          typename C::acc_t (&acc)[C::TM][C::TN], int lane, int wm, int wn, int k0) {
  if constexpr (C::MB == 16) {
    // 16x16x4: lane (r, q) supplies A[r][k0 + 4q + s] and B[k0 + 4q + s][r] in step s = 0..3
    static_assert(!BF16, "16-row tiles are fp32 only");
    const int r = lane & 15, q = lane >> 4;
    float a[C::TM][4], b[C::TN][4];
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
      const float* src = As + ((wm * C::TM + i) * 16 + r) * LD + k0 + 4 * q;
      const f32x2 t0 = *reinterpret_cast<const f32x2*>(src), t1 = *reinterpret_cast<const f32x2*>(src + 2);
      a[i][0] = t0[0]; a[i][1] = t0[1]; a[i][2] = t1[0]; a[i][3] = t1[1];
    }
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const float* src = Bs + ((wn * C::TN + j) * 16 + r) * LD + k0 + 4 * q;
      const f32x2 t0 = *reinterpret_cast<const f32x2*>(src), t1 = *reinterpret_cast<const f32x2*>(src + 2);
      b[j][0] = t0[0]; b[j][1] = t0[1]; b[j][2] = t1[0]; b[j][3] = t1[1];
    }

    // 16x16x16 bf16: lane (r, q) holds A[r][4q..4q+3] -- this map.  (Pairing the products on the
    // full-rate 16x16x32 as mfma_tile_x3 does needs 8 k per lane: twice the fp32 LDS reads and
    // splits here, measured 30 % slower on the 96-wide wgrad tiles.)
    bf16x4 ah[C::TM], am[C::TM], al[C::TM], bh[C::TN], bm[C::TN], bl[C::TN];
#pragma unroll
    for (int i = 0; i < C::TM; ++i) split3<4>(a[i], ah[i], am[i], al[i]);
#pragma unroll
    for (int j = 0; j < C::TN; ++j) split3<4>(b[j], bh[j], bm[j], bl[j]);
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = mfma6_16(ah[i], am[i], al[i], bh[j], bm[j], bl[j], acc[i][j]);
    return;
  } else {
  const int r = lane & 31, h = lane >> 5;
  float a[C::TM][8], b[C::TN][8];
#pragma unroll
  for (int i = 0; i < C::TM; ++i) read_frag<LD>(As + ((wm * C::TM + i) * 32 + r) * LD + k0 + 8 * h, a[i]);
#pragma unroll
  for (int j = 0; j < C::TN; ++j) read_frag<LD>(Bs + ((wn * C::TN + j) * 32 + r) * LD + k0 + 8 * h, b[j]);
  if constexpr (BF16) {
    bf16x8 av[C::TM], bv[C::TN];
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) av[i][e] = (__bf16)a[i][e];
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[j][e] = (__bf16)b[j][e];
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    return;
  }
  bf16x8 ah[C::TM], am[C::TM], al[C::TM], bh[C::TN], bm[C::TN], bl[C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i) split3<8>(a[i], ah[i], am[i], al[i]);
#pragma unroll
  for (int j = 0; j < C::TN; ++j) split3<8>(b[j], bh[j], bm[j], bl[j]);
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = mfma6_32(ah[i], am[i], al[i], bh[j], bm[j], bl[j], acc[i][j]);
  }
}

template <class C>
__device__ __forceinline__ void zero_acc(typename C::acc_t (&acc)[C::TM][C::TN]) {
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int r = 0; r < C::NR; ++r) acc[i][j][r] = 0.f;
}

// ------------------------------------------------------------------------------------------
// forward / dgrad / transposed: K = (tap, channel), N = output pixels
// ------------------------------------------------------------------------------------------
// The A operand (weights) is first packed into GEMM order A[m][t][c] (m < Mpad, c < Ckp, zero
// padded to the tile grid and to whole K-steps) so that every K-step of a row is 64 contiguous
// bytes: one 16-byte buffer load per 4 k-values, no bounds tests.  The B operand is the
// im2col/transposed gather; a thread owns one pixel n and KPT consecutive channels of the K-step.
//
// K order: channel chunk (BK channels) outer, tap inner -- k = (cc, t, c16).  All taps of one
// chunk run back to back, so the gathered rows a block re-reads through the taps (16 channels x
// its pixels + halo, ~13 KB) stay in L1/L2; tap-outer order would cycle every channel through
// the cache between re-reads (the working set of the resident blocks of an XCD then exceeds
// its 4 MB L2 on the 64-128-channel maps).
// Element i of a job's GEMM-order output.  ps > 1: the s*s phases of a stride-s transposed conv
// one after another, phase q = (qh, qw) over its (K/s)^2 taps t' = (a, b) -> kernel tap
// (kh0 + s*a, kw0 + s*b) with kh0 = (qh + pad) % s (see kPhase).
// 32-bit index arithmetic (every job's packed size and weight extent is far below 2^31, checked at
// job creation; 64-bit divisions per element made the batched repack compute-bound).
// Taps of phase q (qa, qc) = (q / s, q % s) of a stride-s dgrad (ps = -s): the kh = qa + s*th,
// kw = qc + s*tw of the K x K kernel, th < ntaps(K, s, qa), tw < ntaps(K, s, qc).
__host__ __device__ __forceinline__ int ntaps(int K, int s, int q) { return (K - q + s - 1) / s; }

__device__ __forceinline__ float pack_elem(const ganamd_pack_job& j, unsigned i) {
  const unsigned nct = (unsigned)j.Ckp / BK;
  unsigned T = (unsigned)j.T, q = 0;
  int dq = -1, dnc = 1;     // dgrad phase (ps < -1) and its tap-column count
  if (j.ps > 1) {
    T = (unsigned)(j.T / (j.ps * j.ps));
    const unsigned per = (unsigned)j.Mpad * T * (unsigned)j.Ckp;
    q = i / per;
    i -= q * per;
  } else if (j.ps < -1) {
    // the s*s phase blocks, each Mpad x T_q x Ckp, one after another (sum of T_q = K*K)
    const int s = -j.ps;
    for (dq = 0; dq < s * s - 1; ++dq) {
      const unsigned per = (unsigned)j.Mpad * (unsigned)(ntaps(j.pk, s, dq / s) * ntaps(j.pk, s, dq % s)) *
                           (unsigned)j.Ckp;
      if (i < per) break;
      i -= per;
    }
    dnc = ntaps(j.pk, s, dq % s);
    T = (unsigned)(ntaps(j.pk, s, dq / s) * dnc);
  }
  const unsigned c16 = i % BK;
  const unsigned r = i / BK;
  unsigned t = r % T;
  const unsigned r2 = r / T;
  const unsigned cc = r2 % nct;
  const int m = (int)(r2 / nct);
  const int c = (int)(cc * BK + c16);
  if (j.ps > 1) {
    const int kk = j.pk / j.ps, qh = (int)q / j.ps, qw = (int)q - qh * j.ps;
    const int kh = (qh + j.ppad) % j.ps + j.ps * ((int)t / kk), kw = (qw + j.ppad) % j.ps + j.ps * ((int)t % kk);
    t = (unsigned)(kh * j.pk + kw);
  } else if (dq >= 0) {
    const int s = -j.ps;
    const int kh = dq / s + s * ((int)t / dnc), kw = dq % s + s * ((int)t % dnc);
    t = (unsigned)(kh * j.pk + kw);
  }
  return (m < j.M && c < j.Ck) ? j.w[(unsigned)(m * j.sm + c * j.sc) + t * (unsigned)j.st] : 0.f;
}

// Element i of a packed copy: the fp32 value, and with x3 also its three bf16 planes after the
// copy (plane p element i at ((ushort*)(out + total))[p * total + i]; x = h + m + l exactly)
__device__ __forceinline__ void pack_store(const ganamd_pack_job& j, unsigned total, unsigned i, float v) {
  j.out[i] = v;
  if (j.x3) {
    unsigned short* pl = reinterpret_cast<unsigned short*>(j.out + total);
    const __bf16 h = (__bf16)v;
    const float r = v - (float)h;
    const __bf16 m = (__bf16)r;
    const __bf16 l = (__bf16)(r - (float)m);
    pl[i] = __builtin_bit_cast(unsigned short, h);
    pl[total + i] = __builtin_bit_cast(unsigned short, m);
    pl[2 * total + i] = __builtin_bit_cast(unsigned short, l);
  }
}

__global__ void pack_a_kernel(ganamd_pack_job j) {
  const unsigned total = (unsigned)j.Mpad * j.T * j.Ckp;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x)
    pack_store(j, total, i, pack_elem(j, i));
}


// ---- bf16 operands in LDS (GANAMD_MATH_BF16, config 4) --------------------------------------
// The same GEMM with both operand tiles staged in LDS as bf16 (RNE from the fp32 packed weights
// and the fp32 gather, scales applied first): a K-step of 32 = two of the fp32 path's 16-wide
// steps (consecutive (channel chunk, tap) pairs of the packed K order), 80-byte LDS rows read
// with one ds_read_b128 per lane per fragment, one v_mfma_f32_32x32x16_bf16 per 16 k.  Half the
// LDS bytes of the fp32 tile per k, a quarter of the LDS read instructions; fp32 accumulation and
// epilogue as in the fp32 kernel.
constexpr int BKB = 32;        // bf16 K-step
constexpr int LDB = BKB + 8;   // LDS row stride (bf16 elements): 80 B, 16-B aligned, ds_read_b128 conflict-free

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// One 16-deep K-step of bf16 MFMAs for a wave over bf16 LDS tiles (rows of LDB elements):
// lane (r, h) reads the 8 k of its row with one ds_read_b128.
template <class C>
__device__ __forceinline__ void mfma_tile_lds_bf16(const unsigned short* __restrict__ As,
                                                   const unsigned short* __restrict__ Bs,
                                                   f32x16 (&acc)[C::TM][C::TN], int lane, int wm, int wn, int k0) {
  const int r = lane & 31, h = lane >> 5;
  bf16x8 av[C::TM], bv[C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
    av[i] = *reinterpret_cast<const bf16x8*>(&As[((wm * C::TM + i) * 32 + r) * LDB + k0 + 8 * h]);
#pragma unroll
  for (int j = 0; j < C::TN; ++j)
    bv[j] = *reinterpret_cast<const bf16x8*>(&Bs[((wn * C::TN + j) * 32 + r) * LDB + k0 + 8 * h]);
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
}

__device__ __forceinline__ u16x8 to_bf16x8(const float* v) {
  bf16x8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (__bf16)v[e];
  return __builtin_bit_cast(u16x8, b);
}

template <int BM, int BN, int WGM, int WGN, int MODE, bool BSCALE>
__device__ __forceinline__ void conv_body_bf16(const ConvArgs& p) {
  using C = TileCfg<BM, BN, WGM, WGN>;
  constexpr int SA = BM * 4;                          // A slots: 8 consecutive k of one row
  constexpr int EA = (SA + kThreads - 1) / kThreads;
  constexpr int H2 = 2 * BN / kThreads;               // 16-k halves per thread (1: BN = 128, 2: BN = 256)
  static_assert(H2 == 1 || H2 == 2, "B mapping");
  __shared__ __attribute__((aligned(16))) unsigned short As[2][BM * LDB];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BN * LDB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nct = p.Ckp / BK;
  const int kf_total = nct * p.T;                     // fp32-packed 16-wide K-steps
  const int kt_total = (kf_total + 1) / 2;            // bf16 K-steps
  int tx, ty, kt0, kt1, split = -1;
  {
    const int bid = blockIdx.x;
    if (bid < p.full_blocks) {
      ty = bid % p.gy;
      tx = bid / p.gy;
      kt0 = 0;
      kt1 = kt_total;
    } else {
      const int t = bid - p.full_blocks;
      const int r = t / p.S;
      split = t - r * p.S;
      ty = r % p.gy;
      tx = p.nfull_t + r / p.gy;
      kt0 = split * p.kt_per_split;
      kt1 = min(kt_total, kt0 + p.kt_per_split);
    }
  }
  const int n0 = tx * BN, m0 = ty * BM;
  const int Krow = p.T * p.Ckp;
  const rsrc_t rw = make_rsrc(p.w, p.w_bytes);
  const Gather& g = p.g;
  const unsigned cs4 = 4u * (unsigned)(g.B * g.H * g.W);
  const rsrc_t rx = make_rsrc(g.src, g.src_bytes());
  const rsrc_t rsc = make_rsrc(BSCALE ? g.scale : g.src, BSCALE ? g.scale_bytes() : 0);
  const int KH = p.T / g.KW;

  // B: pixel n0 + b_n; this thread fills the 16-k halves hb0 .. hb0 + H2 - 1 of every K-step
  const int b_n = tid % BN, hb0 = (tid / BN) * H2;
  const int gn = n0 + b_n;
  const bool n_ok = gn < p.N;
  int bb = 0, oh = 0, ow = 0;
  if (n_ok) {
    bb = gn / p.ohw;
    const int rr = gn - bb * p.ohw;
    if (MODE == kTransposed && p.om.s == -2) {
      ring_coord(rr, p.om.qh, p.om.qw, p.om.OW, p.om.OWp, oh, ow);
    } else {
      oh = rr / g.OW;
      ow = rr - oh * g.OW;
    }
  }
  const int img = bb * g.H * g.W;
  // per half: (channel chunk, tap) of its fp32 step f = 2*kt + half, advanced by 2 steps per K-step
  int hcc[H2], hkh[H2], hkw[H2];
#pragma unroll
  for (int h = 0; h < H2; ++h) {
    const int f = 2 * kt0 + hb0 + h;
    hcc[h] = f / p.T;
    const int t = f - hcc[h] * p.T;
    hkh[h] = t / g.KW;
    hkw[h] = t - hkh[h] * g.KW;
  }

  struct Stage {
    f32x4 ra[EA][2];
    float rb[H2][16], rs[H2][16];
  };
  auto gload = [&](int kt, Stage& S) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int slot = tid + e * kThreads;
      const int row = slot >> 2, q = slot & 3;          // k = 8q .. 8q+7 of the step
      const bool ok = slot < SA && 2 * kt + (q >> 1) < kf_total;
      const int off = ok ? 4 * ((m0 + row) * Krow + kt * BKB + 8 * q) : kOOB;
      S.ra[e][0] = bload4(rw, off);
      S.ra[e][1] = bload4(rw, ok ? off + 16 : kOOB);
    }
#pragma unroll
    for (int h = 0; h < H2; ++h) {
      const int f = 2 * kt + hb0 + h;
      const int sp = (n_ok && f < kf_total) ? tap_offset<MODE>(g, oh, ow, hkh[h], hkw[h]) : -1;
      const int c = hcc[h] * BK;
      const unsigned base = sp >= 0 ? 4u * (unsigned)(img + sp) + (unsigned)c * cs4 : (unsigned)kOOB;
      const unsigned sbase = sp >= 0 ? 4u * (unsigned)(c * g.B + bb) : (unsigned)kOOB;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        S.rb[h][e] = bload(rx, (int)(base + (unsigned)e * cs4));
        if (BSCALE) S.rs[h][e] = bload(rsc, (int)(sbase + 4u * (unsigned)(e * g.B)));
      }
      // next K-step: two fp32 steps on
      hkw[h] += 2;
      while (hkw[h] >= g.KW) {
        hkw[h] -= g.KW;
        if (++hkh[h] >= KH) {
          hkh[h] = 0;
          ++hcc[h];
        }
      }
    }
  };
  auto sstore = [&](int buf, const Stage& S) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int slot = tid + e * kThreads;
      if (slot < SA) {
        const float v[8] = {S.ra[e][0][0], S.ra[e][0][1], S.ra[e][0][2], S.ra[e][0][3],
                            S.ra[e][1][0], S.ra[e][1][1], S.ra[e][1][2], S.ra[e][1][3]};
        *reinterpret_cast<u16x8*>(&As[buf][(slot >> 2) * LDB + 8 * (slot & 3)]) = to_bf16x8(v);
      }
    }
#pragma unroll
    for (int h = 0; h < H2; ++h) {
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = BSCALE ? S.rb[h][e] * S.rs[h][e] : S.rb[h][e];
      unsigned short* d = &Bs[buf][b_n * LDB + 16 * (hb0 + h)];
      *reinterpret_cast<u16x8*>(d) = to_bf16x8(v);
      *reinterpret_cast<u16x8*>(d + 8) = to_bf16x8(v + 8);
    }
  };
  f32x16 acc[C::TM][C::TN];
  zero_acc<C>(acc);
  const int r = lane & 31, hh = lane >> 5;
  auto mfma_step = [&](int buf) {
#pragma unroll
    for (int k0 = 0; k0 < BKB; k0 += 16) {
      bf16x8 av[C::TM], bv[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
        av[i] = *reinterpret_cast<const bf16x8*>(&As[buf][((wm * C::TM + i) * 32 + r) * LDB + k0 + 8 * hh]);
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        bv[j] = *reinterpret_cast<const bf16x8*>(&Bs[buf][((wn * C::TN + j) * 32 + r) * LDB + k0 + 8 * hh]);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };

  Stage s0, s1;
  gload(kt0, s0);
  sstore(0, s0);
  if (kt0 + 1 < kt1) gload(kt0 + 1, s1);
  __syncthreads();
  int kt = kt0;
  for (; kt + 1 < kt1; kt += 2) {
    gload(kt + 2, s0);              // unconditional (past the range: zeros), see conv_body_x3
    mfma_step(0);
    sstore(1, s1);
    __syncthreads();
    gload(kt + 3, s1);
    mfma_step(1);
    if (kt + 2 < kt1) sstore(0, s0);
    __syncthreads();
  }
  if (kt < kt1) mfma_step(0);

  const bool finish = split < 0 || p.S == 1;
  float* out = finish ? p.y : p.slab + (long)split * p.M * p.tail_cols - p.tail_n0;
  const long ldo = finish ? p.ldy : p.tail_cols;
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int n = n0 + (wn * C::TN + j) * 32 + (lane & 31);
    if (n >= p.N) continue;
    const int b = (finish && p.oscale) ? n / p.ohw : 0;
    float* obase = out;
    long old = ldo, col = n;
    if (finish) {
      if constexpr (MODE == kPhase) {
        if (p.om.s == -3) {
          if (!frame_target(p.om, p.y, p.ldy, n, obase, old, col)) continue;
        } else {
          col = out_col(p.om, n);
        }
      }
      if constexpr (MODE == kTransposed) {
        if (p.om.s == -2) {
          obase = p.om.ring;
          old = p.om.ldr;
        } else if (p.om.s < 0 && !frame_target(p.om, p.y, p.ldy, n, obase, old, col)) {
          continue;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int m = m0 + (wm * C::TM + i) * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        float v = p.alpha * acc[i][j][rr];
        if (finish) {
          if (p.oscale) v *= p.oscale[m * g.B + b];
          if (p.bias) v += p.bias[m];
          if (p.noise) v += p.noise_scale[m] * p.noise[(long)m * p.ldy + col];
          if (p.act) v = v > 0.f ? v : p.act[m] * v;
        }
        obase[(long)m * old + col] = v;
      }
    }
  }
}

// Epilogue of the conv GEMM bodies: C/D map of the block MFMA (mfma_row).  Split-K blocks store
// raw partial tiles to their slab; the reduce kernel applies the rest.
template <class C, int MODE>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& p, const typename C::acc_t (&acc)[C::TM][C::TN], int n0,
                                              int m0, int split, int lane, int wm, int wn) {
  const Gather& g = p.g;
  const bool finish = split < 0 || p.S == 1;
  float* out = finish ? p.y : p.slab + (long)split * p.M * p.tail_cols - p.tail_n0;
  const long ldo = finish ? p.ldy : p.tail_cols;
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int n = n0 + (wn * C::TN + j) * C::MB + (lane & (C::MB - 1));
    if (n >= p.N) continue;
    const int b = (finish && p.oscale) ? n / p.ohw : 0;
    float* obase = out;
    long old = ldo, col = n;
    if (finish) {
      if constexpr (MODE == kPhase) {
        if (p.om.s == -3) {
          if (!frame_target(p.om, p.y, p.ldy, n, obase, old, col)) continue;
        } else {
          col = out_col(p.om, n);
        }
      }
      if constexpr (MODE == kTransposed) {
        if (p.om.s == -2) {
          obase = p.om.ring;
          old = p.om.ldr;
        } else if (p.om.s < 0 && !frame_target(p.om, p.y, p.ldy, n, obase, old, col)) {
          continue;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int r = 0; r < C::NR; ++r) {
        const int m = m0 + (wm * C::TM + i) * C::MB + mfma_row<C::MB>(lane, r);
        if (m >= p.M) continue;
        float v = p.alpha * acc[i][j][r];
        if (finish) {
          if (p.oscale) v *= p.oscale[m * g.B + b];
          if (p.bias) v += p.bias[m];
          if (p.noise) v += p.noise_scale[m] * p.noise[(long)m * p.ldy + col];
          if (p.act) v = v > 0.f ? v : p.act[m] * v;
        }
        obase[(long)m * old + col] = v;
      }
    }
  }
}

#ifndef GANAMD_CONV_WPE
#define GANAMD_CONV_WPE 3   // split6 LDS body: 3 waves/SIMD fit (<= 168 VGPRs, 3 x 49 KB LDS per CU)
#endif
#ifndef GANAMD_WGRAD_WPE
#define GANAMD_WGRAD_WPE 1
#endif

// ---- fp32 GEMM body with split operands in LDS ----------------------------------------------
// The conv block schedule (ConvPlan) and gather; each operand element is split ONCE -- by the
// thread that stores it to LDS -- into three bf16 planes (h, m, l: split3); the waves read bf16
// fragments and issue the six split products per 16 k on the bf16 matrix cores (mfma6_32 /
// mfma6_16) instead of splitting every fragment they read.  K-step 16; 48-byte plane rows (16 k
// + 8 pad): the fragment reads (ds_read_b128 / _b64) and the 8-k slot stores (ds_write_b128) are
// conflict-free (MI355X_MICROARCH.md "LDS" lane groups).
// plane row stride (bf16 elements): 32-byte rows (no pad) with the two 16-byte halves of row r
// swapped when bit 3 of r is set -- conflict-free fragment reads in two thirds of a padded layout's LDS
constexpr int LDH = BK;
// element offset of k-group `half` (8 k) of plane row r.  32x32 fragments (a ds_read_b128 lane
// group on one half) need the halves swapped on odd 8-row groups; 16x16 fragments (lanes 16-31 on
// the other half of lanes 0-15's rows) the plain layout (2-way conflicts otherwise; conv_patch.hip poff)
template <int MB>
__device__ __forceinline__ int x3_off(int r, int half) {
  return MB == 32 ? r * LDH + 8 * (half ^ ((r >> 3) & 1)) : r * LDH + 8 * half;
}

template <class C, int PSA, int PSB>
__device__ __forceinline__ void mfma_tile_x3(const unsigned short* __restrict__ As, const unsigned short* __restrict__ Bs,
                                             typename C::acc_t (&acc)[C::TM][C::TN], int lane, int wm, int wn) {
  if constexpr (C::MB == 16) {
    // full-rate v_mfma_f32_16x16x32_bf16 on PAIRS of split products: its 32 k are two 16-k halves
    // (lane (r, q) holds k = 8q .. 8q+7: q < 2 the first half, q >= 2 the second), so
    // (h|m)x(h|h) = hh + mh, (h|l)x(m|h) = hm + lh, (m|h)x(m|l) = mm + hl -- three instructions
    // for the six products where 16x16x16 would need six at half the rate
    const int r = lane & 15, q = lane >> 4, hf = q & 1, hi = q >> 1;
    const int a0 = hi ? PSA : 0, a1 = hi ? 2 * PSA : 0, a2 = hi ? 0 : PSA;   // plane offsets of this
    const int b0 = 0, b1 = hi ? 0 : PSB, b2 = hi ? 2 * PSB : PSB;           // lane's k-half
    bf16x8 a[C::TM][3], b[C::TN][3];
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
      const int o = x3_off<16>((wm * C::TM + i) * 16 + r, hf);
      a[i][0] = *reinterpret_cast<const bf16x8*>(&As[a0 + o]);   // (h | m)
      a[i][1] = *reinterpret_cast<const bf16x8*>(&As[a1 + o]);   // (h | l)
      a[i][2] = *reinterpret_cast<const bf16x8*>(&As[a2 + o]);   // (m | h)
    }
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int o = x3_off<16>((wn * C::TN + j) * 16 + r, hf);
      b[j][0] = *reinterpret_cast<const bf16x8*>(&Bs[b0 + o]);   // (h | h)
      b[j][1] = *reinterpret_cast<const bf16x8*>(&Bs[b1 + o]);   // (m | h)
      b[j][2] = *reinterpret_cast<const bf16x8*>(&Bs[b2 + o]);   // (m | l)
    }
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
  } else {                       // 32x32x16 bf16: lane (r, h) holds k = 8h .. 8h+7 of row r
    const int r = lane & 31, h = lane >> 5;
    bf16x8 a[C::TM][3], b[C::TN][3];
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = *reinterpret_cast<const bf16x8*>(&As[pl * PSA + x3_off<32>((wm * C::TM + i) * 32 + r, h)]);
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[j][pl] = *reinterpret_cast<const bf16x8*>(&Bs[pl * PSB + x3_off<32>((wn * C::TN + j) * 32 + r, h)]);
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        acc[i][j] = mfma6_32(a[i][0], a[i][1], a[i][2], b[j][0], b[j][1], b[j][2], acc[i][j]);
  }
}

// the three bf16 planes of 8 consecutive fp32 values to plane rows at `d` (plane stride PS)
template <int PS>
__device__ __forceinline__ void store_split8(unsigned short* d, const float* v) {
  bf16x8 h, m, l;
  split3<8>(v, h, m, l);
  *reinterpret_cast<bf16x8*>(d) = h;
  *reinterpret_cast<bf16x8*>(d + PS) = m;
  *reinterpret_cast<bf16x8*>(d + 2 * PS) = l;
}

template <int BM, int BN, int WGM, int WGN, int MODE, bool BSCALE>
__device__ __forceinline__ void conv_body_x3(const ConvArgs& p) {
  using C = TileCfg<BM, BN, WGM, WGN>;
  constexpr int SPR = BK / 8;                          // 8-k A slots per row and K-step
  constexpr int SA = BM * SPR;
  constexpr int EA = (SA + kThreads - 1) / kThreads;   // slots per thread
  constexpr int KPT = BK * BN / kThreads;              // B k-values per thread
  static_assert(KPT % 8 == 0 && BK % KPT == 0, "B mapping");
  constexpr int PSA = BM * LDH, PSB = BN * LDH;
  __shared__ __attribute__((aligned(16))) unsigned short As[2][3 * PSA];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][3 * PSB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nct = p.Ckp / BK;
  const int kt_total = nct * p.T;
  int tx, ty, kt0, kt1, split = -1;
  {
    const int bid = blockIdx.x;
    if (bid < p.full_blocks) {
      ty = bid % p.gy;
      tx = bid / p.gy;
      kt0 = 0;
      kt1 = kt_total;
    } else {
      const int t = bid - p.full_blocks;
      const int r = t / p.S;
      split = t - r * p.S;
      ty = r % p.gy;
      tx = p.nfull_t + r / p.gy;
      kt0 = split * p.kt_per_split;
      kt1 = min(kt_total, kt0 + p.kt_per_split);
    }
  }
  const int n0 = tx * BN, m0 = ty * BM;

  const int Krow = p.T * p.Ckp;
  const rsrc_t rw = make_rsrc(p.w, p.w_bytes);
  int a_off[EA];
#pragma unroll
  for (int e = 0; e < EA; ++e) {
    const int slot = min(tid + e * kThreads, SA - 1);
    a_off[e] = 4 * ((m0 + slot / SPR) * Krow + 8 * (slot % SPR));
  }

  const int b_n = tid % BN, b_kg = tid / BN;
  const Gather& g = p.g;
  const int gn = n0 + b_n;
  const bool n_ok = gn < p.N;
  int bb = 0, oh = 0, ow = 0;
  if (n_ok) {
    bb = gn / p.ohw;
    const int rr = gn - bb * p.ohw;
    if (MODE == kTransposed && p.om.s == -2) {
      ring_coord(rr, p.om.qh, p.om.qw, p.om.OW, p.om.OWp, oh, ow);
    } else {
      oh = rr / g.OW;
      ow = rr - oh * g.OW;
    }
  }
  const unsigned cs4 = 4u * (unsigned)(g.B * g.H * g.W);
  const int img = bb * g.H * g.W;
  const rsrc_t rx = make_rsrc(g.src, g.src_bytes());
  const rsrc_t rsc = make_rsrc(BSCALE ? g.scale : g.src, BSCALE ? g.scale_bytes() : 0);

  struct Stage {
    f32x4 ra[EA][2];
    float rb[KPT], rs[KPT];
  };
  int cc = kt0 / p.T;
  int kh, kw;
  {
    const int t = kt0 - cc * p.T;
    kh = t / g.KW;
    kw = t - kh * g.KW;
  }
  auto tap = [&]() { return n_ok ? tap_offset<MODE>(g, oh, ow, kh, kw) : -1; };
  int sp = tap();

  // Every load is unconditional (a slot past the tile re-reads a valid one, a K-step past the
  // range reads zeros or ignored rows within the buffer bounds): the compiler then knows how many
  // loads are in flight and the wait for step kt+1's operands leaves step kt+2's gather in flight
  // (after a conditional load it drains them all -- vmcnt counts in order).
  auto gload = [&](int kt, Stage& S) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int o = a_off[e] + kt * (BK * 4);
      S.ra[e][0] = bload4(rw, o);
      S.ra[e][1] = bload4(rw, o + 16);
    }
    const int c = cc * BK + b_kg * KPT;
    const unsigned base = sp >= 0 ? 4u * (unsigned)(img + sp) + (unsigned)c * cs4 : (unsigned)kOOB;
    const unsigned sbase = sp >= 0 ? 4u * (unsigned)(c * g.B + bb) : (unsigned)kOOB;
#pragma unroll
    for (int e = 0; e < KPT; ++e) {
      S.rb[e] = bload(rx, (int)(base + (unsigned)e * cs4));
      if (BSCALE) S.rs[e] = bload(rsc, (int)(sbase + 4u * (unsigned)(e * g.B)));
    }
    if (++kw == g.KW) {
      kw = 0;
      if (++kh * g.KW >= p.T) {
        kh = 0;
        ++cc;
      }
    }
    sp = tap();
  };
  auto sstore = [&](int buf, const Stage& S) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int slot = tid + e * kThreads;
      if (slot < SA) {
        const float v[8] = {S.ra[e][0][0], S.ra[e][0][1], S.ra[e][0][2], S.ra[e][0][3],
                            S.ra[e][1][0], S.ra[e][1][1], S.ra[e][1][2], S.ra[e][1][3]};
        store_split8<PSA>(&As[buf][x3_off<C::MB>(slot / SPR, slot % SPR)], v);
      }
    }
#pragma unroll
    for (int e = 0; e < KPT; e += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = BSCALE ? S.rb[e + q] * S.rs[e + q] : S.rb[e + q];
      store_split8<PSB>(&Bs[buf][x3_off<C::MB>(b_n, (b_kg * KPT + e) / 8)], v);
    }
  };

  typename C::acc_t acc[C::TM][C::TN];
  zero_acc<C>(acc);

  Stage s0, s1;
  gload(kt0, s0);
  sstore(0, s0);
  if (kt0 + 1 < kt1) gload(kt0 + 1, s1);
  __syncthreads();
  int kt = kt0;
  for (; kt + 1 < kt1; kt += 2) {
    gload(kt + 2, s0);
    mfma_tile_x3<C, PSA, PSB>(As[0], Bs[0], acc, lane, wm, wn);
    sstore(1, s1);
    __syncthreads();
    gload(kt + 3, s1);
    mfma_tile_x3<C, PSA, PSB>(As[1], Bs[1], acc, lane, wm, wn);
    if (kt + 2 < kt1) sstore(0, s0);
    __syncthreads();
  }
  if (kt < kt1) mfma_tile_x3<C, PSA, PSB>(As[0], Bs[0], acc, lane, wm, wn);
  conv_epilogue<C, MODE>(p, acc, n0, m0, split, lane, wm, wn);
}

template <int BM, int BN, int WGM, int WGN, int MODE, bool BSCALE, bool BF16>
// (the bf16 body with per-(channel, sample) scales needs more than 3 waves/SIMD's registers: it spilled
// 12-101 VGPRs there; 2 waves/SIMD -- except the 128x256 tile, which spills at 2 and not at 3)
// (the fp32 128x256 tile runs at 2 waves/SIMD: 250 VGPRs, no spill)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(
    (BF16 && BSCALE && BM * BN < 128 * 256) || (!BF16 && BM == 128 && BN == 256) ? 2 : GANAMD_CONV_WPE)))
void conv_gemm_kernel(ConvArgs p) {
  if constexpr (BF16) {
    conv_body_bf16<BM, BN, WGM, WGN, MODE, BSCALE>(p);
  } else {
    conv_body_x3<BM, BN, WGM, WGN, MODE, BSCALE>(p);
  }
}

// Batched repack: block b finds its job by binary search over the jobs' chunk offsets and packs
// kPackChunk consecutive elements of that job's GEMM-order output.
constexpr int kPackChunk = 4096;

// Jobs whose channel stride is the large one (the dgrad-order, scatter-dgrad and ConvT copies:
// A(m, t, c) = S[c][m*T + t], rows r = m*T + t contiguous) pack as tiled transposes: a block reads
// 16 channel rows x (kPackRows(T) * T) contiguous floats into LDS and writes kPackRows(T) output
// rows of T*16 contiguous floats -- coalesced on both sides (the element-wise map reads them with a
// stride of Cin*T floats).
__host__ __device__ inline bool pack_transposed(const ganamd_pack_job& j) {
  return (j.ps == 0 || j.ps == 1) && j.st == 1 && j.sm == j.T && j.sc > j.sm;
}
__host__ __device__ inline int pack_rows(int T) { return T >= 256 ? 1 : 256 / T; }

__device__ void pack_tile(const ganamd_pack_job& j, long tile, float* lds) {
  const int T = j.T, R = pack_rows(T), nct = j.Ckp / BK;
  const int cc = (int)(tile % nct), m0 = (int)(tile / nct) * R;
  const int rows = min(R, j.Mpad - m0);
  const int span = rows * T;                                  // contiguous floats per channel row
  for (int idx = threadIdx.x; idx < BK * span; idx += blockDim.x) {
    const int c16 = idx / span, r = idx - c16 * span;
    const int c = cc * BK + c16, m = m0 + r / T;
    lds[c16 * (R * T + 1) + r] = (c < j.Ck && m < j.M) ? j.w[(long)c * j.sc + (long)m0 * T + r] : 0.f;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < span * BK; idx += blockDim.x) {
    const int mr = idx / (T * BK), rem = idx - mr * T * BK, t = rem / BK, c16 = rem - t * BK;
    pack_store(j, (unsigned)j.Mpad * T * j.Ckp, (unsigned)((((long)(m0 + mr) * nct + cc) * T + t) * BK + c16),
               lds[c16 * (R * T + 1) + mr * T + t]);
  }
}

__global__ __launch_bounds__(256) void pack_batch_kernel(const ganamd_pack_job* __restrict__ jobs, int n_jobs) {
  const long b = blockIdx.x;
  int lo = 0, hi = n_jobs - 1;
  while (lo < hi) {   // last job with chunk0 <= b
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].chunk0 <= b) lo = mid; else hi = mid - 1;
  }
  const ganamd_pack_job j = jobs[lo];
  if (pack_transposed(j)) {
    __shared__ float lds[BK * (256 + 1)];
    pack_tile(j, b - j.chunk0, lds);
    return;
  }
  const unsigned total = (unsigned)j.Mpad * j.T * j.Ckp;
  const unsigned i0 = (unsigned)(b - j.chunk0) * kPackChunk;
  const unsigned i1 = min(total, i0 + kPackChunk);
  for (unsigned i = i0 + threadIdx.x; i < i1; i += 256) pack_store(j, total, i, pack_elem(j, i));
}

// ------------------------------------------------------------------------------------------
// wgrad: K = output pixels n, M = output channels of the conv, N = gathered channels at tap t
// ------------------------------------------------------------------------------------------
// TP (tap-packed): the N dimension runs over (tap, channel) pairs, n = t*J + j, so narrow gathered
// sides (J = 3, 48, 96 against 64/128-wide tiles) fill their tiles across taps instead of padding
// every tap's tile; each B row then has its own tap.
template <int BM, int BN, int WGM, int WGN, int MODE, bool SCALED, bool BF16, bool TP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(GANAMD_WGRAD_WPE)))
void wgrad_gemm_kernel(WgradArgs p) {
  using C = TileCfg<BM, BN, WGM, WGN>;
  constexpr int A4 = BM * BKW / 4;                     // 16-byte slots of the A tile (4 pixels of a row)
  constexpr int EA = (A4 + kThreads - 1) / kThreads;
  constexpr int EB = BKW * BN / kThreads;
  constexpr int RSTEP = kThreads / BKW;
  // bf16 math stages the tiles in LDS as bf16 (80-byte rows, one ds_read_b128 per fragment);
  // fp32 keeps fp32 rows of LDKW floats
  using LT = typename std::conditional<BF16, unsigned short, float>::type;
  constexpr int LDW = BF16 ? LDB : LDKW;
  __shared__ __attribute__((aligned(16))) LT As[2][BM * LDW];
  __shared__ __attribute__((aligned(16))) LT Bs[2][BN * LDW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  // Block order: consecutive blocks are consecutive K-slices of one tap (they stream adjacent
  // pixel ranges of gy and x).  A tap-fastest order with an XCD-contiguous remap, meant to share
  // the taps' overlapping source rows through one XCD's L2, measured 5-15 % slower.
  const int j0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int t = TP ? 0 : blockIdx.z / p.splits;
  const int split = blockIdx.z - t * p.splits;
  const int kt_total = (p.K + BKW - 1) / BKW;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(kt_total, kt0 + p.kt_per_split);
  if (kt0 >= kt1) return;

  const Gather& g = p.g;
  const int kh = t / g.KW, kw = t - kh * g.KW;
  const unsigned cs4 = 4u * (unsigned)(g.B * g.H * g.W);
  const int tk = tid % BKW;   // B: pixel fixed per thread
  const int tr = tid / BKW;   // B: channel base
  // TP: (tap, channel, kh, kw) of this thread's first B row, stepped by RSTEP rows per e
  int tp_t = 0, tp_j = 0, tp_kh = 0, tp_kw = 0;
  if (TP) {
    tp_t = (j0 + tr) / p.J;
    tp_j = j0 + tr - tp_t * p.J;
    tp_kh = tp_t / g.KW;
    tp_kw = tp_t - tp_kh * g.KW;
  }

  const rsrc_t ra_r1 = make_rsrc(p.a, p.a_bytes);
  const rsrc_t rx1 = make_rsrc(g.src, g.src_bytes());
  const rsrc_t ra_r2 = make_rsrc(p.segK ? p.a2 : p.a, p.a_bytes);
  const rsrc_t rx2 = make_rsrc(p.segK ? p.src2 : g.src, g.src_bytes());
  const rsrc_t rsa_r = make_rsrc(SCALED ? p.ascale : p.a, SCALED ? 4 * p.M * g.B : 0);
  const rsrc_t rsb_r = make_rsrc(SCALED ? g.scale : g.src, SCALED ? g.scale_bytes() : 0);
  // 16-byte A loads need 16-byte aligned rows; a quad of pixels shares its sample when ohw % 4 == 0
  const bool vec_ok = (p.lda & 3) == 0;
  const bool quad_b = (p.ohw & 3) == 0;

  f32x4 ra[EA], rsa[EA];
  float rb[EB], rsb[EB];
  int sb_b = -1;   // sample whose B-side scales rsb holds (SCALED, not TP)
  // pixel of this thread's B column for the next K-step, advanced by BKW pixels per step
  const int d_b = BKW / p.ohw, d_rem = BKW - d_b * p.ohw, d_oh = d_rem / g.OW, d_ow = d_rem - d_oh * g.OW;
  int pb, poh, pow_;
  {
    const int n = kt0 * BKW + tk;
    pb = n / p.ohw;
    const int rr = n - pb * p.ohw;
    poh = rr / g.OW;
    pow_ = rr - poh * g.OW;
  }
  auto gload = [&](int kt) {
    // segment of this K-step (uniform): the second one reads a2 / src2 at pixel n - segK
    const bool s2 = p.segK > 0 && kt * BKW >= p.segK;
    const rsrc_t ra_r = s2 ? ra_r2 : ra_r1;
    const rsrc_t rx = s2 ? rx2 : rx1;
    const int noff = s2 ? p.segK : 0, boff = s2 ? g.B : 0;
    // ---- A: rows m of gy (or x), 4 consecutive pixels per slot
    const bool full = vec_ok && (kt + 1) * BKW <= p.K;
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int slot = tid + e * kThreads;
      if (slot < A4) {
        const int m = m0 + slot / (BKW / 4), n = kt * BKW + 4 * (slot % (BKW / 4));
        const bool mok = m < p.M;
        if (full) {
          ra[e] = bload4(ra_r, mok ? 4 * (m * p.lda + n - noff) : kOOB);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            ra[e][i] = bload(ra_r, (mok && n + i < p.K) ? 4 * (m * p.lda + n - noff + i) : kOOB);
        }
        if (SCALED) {
          if (quad_b) {
            const float sv = bload(rsa_r, mok ? 4 * (m * g.B + min(n, p.K - 1) / p.ohw) : kOOB);
            rsa[e] = f32x4{sv, sv, sv, sv};
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              rsa[e][i] = bload(rsa_r, (mok && n + i < p.K) ? 4 * (m * g.B + (n + i) / p.ohw) : kOOB);
          }
        }
      }
    }
    // ---- B: the gathered source at tap t, pixel n = kt*BKW + tk (tracked incrementally as
    // (pb, poh, pow)), channels j0 + tr + e*RSTEP
    const int n = kt * BKW + tk;
    const int b = pb - boff;
    const int poh_cur = poh, pow_cur = pow_;
    const int sp = (!TP && n < p.K) ? tap_offset<MODE>(g, poh, pow_, kh, kw) : -1;
    pow_ += d_ow;
    if (pow_ >= g.OW) {
      pow_ -= g.OW;
      ++poh;
    }
    poh += d_oh;
    if (poh >= g.OH) {
      poh -= g.OH;
      ++pb;
    }
    pb += d_b;
    // channels past the source's end fall outside the buffer: the hardware returns 0
    if constexpr (TP) {
      int te = tp_t, je = tp_j, khe = tp_kh, kwe = tp_kw;
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        const int spe = (n < p.K && te < p.T) ? tap_offset<MODE>(g, poh_cur, pow_cur, khe, kwe) : -1;
        rb[e] = bload(rx, spe >= 0 ? (int)(4u * (unsigned)(b * g.H * g.W + spe) + (unsigned)je * cs4) : kOOB);
        if (SCALED) rsb[e] = bload(rsb_r, spe >= 0 ? 4 * (je * g.B + b) : kOOB);
        je += RSTEP;
        while (je >= p.J) {
          je -= p.J;
          ++te;
          if (++kwe == g.KW) {
            kwe = 0;
            ++khe;
          }
        }
      }
      return;
    }
    const unsigned base = sp >= 0 ? 4u * (unsigned)(b * g.H * g.W + sp) + (unsigned)(j0 + tr) * cs4 : (unsigned)kOOB;
#pragma unroll
    for (int e = 0; e < EB; ++e) rb[e] = bload(rx, (int)(base + (unsigned)(e * RSTEP) * cs4));
    // the B-side scales s[j][b] change only when this thread's pixel enters the next sample
    // (every ohw / BKW K-steps): reload them then, not per step.  Where the gather is out of
    // range rb is 0, so a stale or out-of-range scale there multiplies 0.
    if (SCALED && b != sb_b) {
      sb_b = b;
      const unsigned sbase = 4u * (unsigned)((j0 + tr) * g.B + b);
#pragma unroll
      for (int e = 0; e < EB; ++e) rsb[e] = bload(rsb_r, (int)(sbase + 4u * (unsigned)(e * RSTEP * g.B)));
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int slot = tid + e * kThreads;
      if (slot < A4) {
        f32x4 v = ra[e];
        if (SCALED) v *= rsa[e];
        LT* d = &As[buf][(slot / (BKW / 4)) * LDW + 4 * (slot % (BKW / 4))];
        if constexpr (BF16) {
          bf16x4 b;
#pragma unroll
          for (int q = 0; q < 4; ++q) b[q] = (__bf16)v[q];
          *reinterpret_cast<bf16x4*>(d) = b;
        } else {
          *reinterpret_cast<f32x2*>(d) = f32x2{v[0], v[1]};
          *reinterpret_cast<f32x2*>(d + 2) = f32x2{v[2], v[3]};
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const float v = SCALED ? rb[e] * rsb[e] : rb[e];
      if constexpr (BF16)
        Bs[buf][(tr + e * RSTEP) * LDW + tk] = __builtin_bit_cast(unsigned short, (__bf16)v);
      else
        Bs[buf][(tr + e * RSTEP) * LDW + tk] = v;
    }
  };

  typename C::acc_t acc[C::TM][C::TN];
  zero_acc<C>(acc);

  gload(kt0);
  sstore(0);
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) gload(kt + 1);
#pragma unroll
    for (int k0 = 0; k0 < BKW; k0 += 16) {
      if constexpr (BF16)
        mfma_tile_lds_bf16<C>(As[buf], Bs[buf], acc, lane, wm, wn, k0);
      else
        mfma_tile<C, LDKW, false>(As[buf], Bs[buf], acc, lane, wm, wn, k0);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    int jj = j0 + (wn * C::TN + j) * C::MB + (lane & (C::MB - 1));
    int tt = t;
    if (TP) {
      if (jj >= p.T * p.J) continue;
      tt = jj / p.J;
      jj -= tt * p.J;
    } else if (jj >= p.J) {
      continue;
    }
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int r = 0; r < C::NR; ++r) {
        const int m = m0 + (wm * C::TM + i) * C::MB + mfma_row<C::MB>(lane, r);
        if (m >= p.M) continue;
        const int o = m * p.om + jj * p.oj + tt * p.ot;
        const float v = p.alpha * acc[i][j][r];
        if (p.slab)
          p.slab[(long)split * p.out_numel + o] = v;
        else if (p.accumulate)
          p.out[o] += v;   // single split: this block is the element's only writer
        else
          p.out[o] = v;
      }
    }
  }
}

// Replication padding's adjoint on the ring of the frame-split dgrad (OutMap s = -1): every edge
// pixel of the input gradient adds the ring positions of the padded frame that clamp onto it
// (its interior position went to gx directly).  One thread per (plane, edge pixel): top row,
// bottom row, then the left and right columns of the middle rows.
__global__ void ring_fold_kernel(const float* __restrict__ ring, float* __restrict__ gx, int planes, int H, int W,
                                 int p) {
  const int Hp = H + 2 * p, Wp = W + 2 * p, Rn = Hp * Wp - H * W;
  const int mid = H > 2 ? H - 2 : 0;
  const int e_top = W, e_bot = H > 1 ? W : 0, e_right = W > 1 ? mid : 0;
  const int E = e_top + e_bot + mid + e_right;
  const long total = (long)planes * E;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int pl = (int)(idx / E), e = (int)(idx - (long)pl * E);
    int i, j;
    if (e < e_top) {
      i = 0;
      j = e;
    } else if (e < e_top + e_bot) {
      i = H - 1;
      j = e - e_top;
    } else if (e < e_top + e_bot + mid) {
      i = 1 + (e - e_top - e_bot);
      j = 0;
    } else {
      i = 1 + (e - e_top - e_bot - mid);
      j = W - 1;
    }
    const int h0 = i == 0 ? 0 : i + p, h1 = i == H - 1 ? Hp - 1 : i + p;
    const int w0 = j == 0 ? 0 : j + p, w1 = j == W - 1 ? Wp - 1 : j + p;
    const float* r = ring + (long)pl * Rn;
    float acc = 0.f;
    for (int a = h0; a <= h1; ++a)
      for (int c = w0; c <= w1; ++c)
        if (a != i + p || c != j + p) acc += r[ring_idx(a, c, p, H, W, Wp)];
    gx[(long)pl * H * W + (long)i * W + j] += acc;
  }
}

// Input gradient of a conv from the per-tap products Z[(ci,t)][b,oh,ow] (the "scatter" form of
// dgrad, see ganamd_conv_dgrad): every input pixel sums, per tap, the outputs whose (padded)
// receptive field reads it through that tap -- one output per tap in the interior (none for a
// stride-2 tap of the wrong parity), a run of outputs at a replication-padded edge.  Input row i
// is read by output row oh through tap kh iff clamp(oh*s - pad + kh) lies in [lo, hi], where
// lo = hi = i, except that a replicated edge row also takes every position beyond the edge.
//
// SK, KK != 0: stride and (square) kernel size as compile-time constants -- the tap bounds' divisions
// by the stride become shifts and the tap loops unroll (the generic form spends most of its time in
// four runtime integer divisions per tap, not in its loads).  Same loop and summation order.
// The 32-bit instance (every index < 2^31) splits the element index with multiply-high divisions.
struct Div31 {   // x / d for 0 <= x < 2^31: m = ceil(2^(31+l) / d), l = ceil(log2 d) (m < 2^32), q = mulhi(x, m) >> (l-1)
  unsigned m = 0;
  int s = 0;     // m == 0: d == 1
  static Div31 of(unsigned d) {
    Div31 r;
    if (d <= 1) return r;
    int l = 0;
    while ((1ull << l) < d) ++l;
    r.m = (unsigned)(((1ull << (31 + l)) + d - 1) / d);
    r.s = l - 1;
    return r;
  }
  __device__ __forceinline__ unsigned operator()(unsigned x) const { return m ? __umulhi(x, m) >> s : x; }
};
struct FoldDivs {
  Div31 w, h, b;
};

template <typename I, int SK = 0, int KK = 0>
__global__ void dgrad_fold_kernel(const float* __restrict__ Z, float* __restrict__ gx, int C, int B, int H, int W,
                                  int OH, int OW, int KH_, int KW_, int stride_, int pad, int replicate, FoldDivs dv) {
  const int stride = SK ? SK : stride_, KH = KK ? KK : KH_, KW = KK ? KK : KW_;
  const I total = (I)C * B * H * W;
  const int T = KH * KW;
  constexpr int kFar = 1 << 20;
  auto div = [](I x, I d, const Div31& f) -> I {
    if constexpr (sizeof(I) == 4) return f(x);
    return x / d;
  };
  for (I idx = blockIdx.x * (I)blockDim.x + threadIdx.x; idx < total; idx += (I)gridDim.x * blockDim.x) {
    const I r1 = div(idx, (I)W, dv.w);
    const int j = (int)(idx - r1 * (I)W);
    const I r2 = div(r1, (I)H, dv.h);
    const int i = (int)(r1 - r2 * (I)H);
    const I c_ = div(r2, (I)B, dv.b);
    const int b = (int)(r2 - c_ * (I)B);
    const int c = (int)c_;
    const int ilo = (replicate && i == 0) ? -kFar : i, ihi = (replicate && i == H - 1) ? kFar : i;
    const int jlo = (replicate && j == 0) ? -kFar : j, jhi = (replicate && j == W - 1) ? kFar : j;
    float acc = 0.f;
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      // oh*s in [ilo + pad - kh, ihi + pad - kh]
      const int a0 = ilo + pad - kh, a1 = ihi + pad - kh;
      const int h0 = max(0, a0 <= 0 ? 0 : (a0 + stride - 1) / stride);
      const int h1 = min(OH - 1, a1 < 0 ? -1 : a1 / stride);
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        const int b0 = jlo + pad - kw, b1 = jhi + pad - kw;
        const int w0 = max(0, b0 <= 0 ? 0 : (b0 + stride - 1) / stride);
        const int w1 = min(OW - 1, b1 < 0 ? -1 : b1 / stride);
        const float* z = Z + ((long)(c * T + kh * KW + kw) * B + b) * OH * OW;
        for (int oh = h0; oh <= h1; ++oh)
          for (int ow = w0; ow <= w1; ++ow) acc += z[oh * OW + ow];
      }
    }
    gx[idx] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------------
// Tuning knobs (read once): target number of workgroups the split-K heuristics aim for.
// Tuning switches of the GEMM planners (the A/B experiments behind them are in profiles/r01-r03;
// the library reads no environment): tap-packed wgrad columns, the skinny-GEMM linears, split-K,
// no LDS padding (occupancy).
constexpr bool wgrad_tp_enabled() { return true; }
constexpr bool linear_enabled() { return true; }
constexpr bool splitk_enabled() { return true; }
constexpr int conv_lds_pad() { return 0; }
constexpr int wgrad_lds_pad() { return 0; }

struct Plan {
  int bm, bn, splits, kt_per_split;
  int tp = 0;          // wgrad: taps packed into N (see wgrad_gemm_kernel TP)
};

// Row tile: the least padded rows per unit of tile efficiency (measured: 96-row tiles ~0.95 and
// 64-row ~0.9 of the 128-row rate) -- e.g. M = 192 takes two 96-row tiles, not two 128-row ones
// (256 rows, 25 % empty); a smaller tile has to beat the 128-row one by 5 %.
constexpr bool tile48() { return true; }
int conv_bm(int M) {
  if (M <= 16 && tile48()) return 16;   // ToRGB (M = 3): 16x16x4 blocks halve the empty rows
  if (M <= 32) return 32;
  if (M <= 48 && tile48()) return 48;   // 16x16x4 MFMA blocks: 48 rows without 64-row padding
  if (M <= 64) return 64;
  if (M <= 96) return 96;
  const double c128 = (M + 127) / 128 * 128.0, c96 = (M + 95) / 96 * 96.0 / 0.95, c64 = (M + 63) / 64 * 64.0 / 0.9;
  const double bar = 0.95 * c128;   // a smaller tile only for a clear win
  return (c96 < bar && c96 <= c64) ? 96 : (c64 < bar ? 64 : 128);
}
#ifndef GANAMD_WIDE
#define GANAMD_WIDE 1   // 128x256 tiles (2 waves/SIMD) for the unscaled fp32 GEMMs with 128-row tiles
#endif
constexpr bool wide_tiles() { return GANAMD_WIDE != 0; }
// The 128x256 split6 tile at 2 waves/SIMD: the critic's 128- to 1025-channel convs (measured vs the
// 128x128 tile at 3 waves/SIMD: 128->128 3x3 at 32x32 fwd 160 -> 183 TF/s, dgrad 107 -> 118;
// 256->256 at 16x16 fwd 148 -> 159, dgrad 92 -> 100; profiles/r05_ab_wide.txt).  Not for scaled
// (modulated) GEMMs -- their per-(channel, sample) scale loads spill it -- nor bf16 math.
int conv_bn(int bm, bool bscale, bool bf16) {
  return bm <= 32 ? 256 : (bm == 128 && wide_tiles() && !bscale && !bf16) ? 256 : 128;
}
constexpr bool tile96() { return true; }
constexpr bool big96() { return true; }
int wgrad_bm(int M, bool scaled) { return M <= 32 ? 32 : M <= 64 ? 64 : (M <= 96 || scaled) ? (M <= 96 ? 96 : 64) : 128; }

// Split-K: pure functions of the geometry (the workspace query and the launch agree).
constexpr int kCUs = 256;

int num_cus();
double list_makespan(long F, double L, long R, double d, long slots);

// Price of the extra reduce launch of a split GEMM (its own ~5 us run time on tiny data plus the
// dependent-launch boundary).
#ifndef GANAMD_REDUCE_US
#define GANAMD_REDUCE_US 3.0
#endif
constexpr double reduce_launch_us() { return GANAMD_REDUCE_US; }

// wgrad split-K by a small cost model: a GEMM of `tiles` output tiles, each `kt_total` K-steps of
// `kflop` FLOPs, runs in ceil(tiles*s / slots) rounds of blocks (slots = resident blocks per CU
// x CUs) of ceil(kt_total/s) K-steps; splitting adds the slab round trip and a reduce launch.
// (A CU-level "fluid" model -- one block alone runs at the CU's full rate -- was measured to
// under-split the big-K wgrads 1.4-2x: a lone block of 4 waves does not fill its CU.)
constexpr double kBlockTflops = 130.0;   // measured sustained fp32 rate of the GEMM kernels (split6 products)
Plan split_plan(int bm, int bn, int tiles, int kt_total, double kflop, long out_elems, int occ, int max_splits,
                int min_k) {
  const int slots = occ * kCUs;
  const double t_k = kflop / (kBlockTflops * 1e12 / slots) * 1e6;   // us per K-step of one block
  auto cost = [&](int s) {
    const long per = (kt_total + s - 1) / s;
    const long waves = ((long)tiles * s + slots - 1) / slots;
    double c = (double)waves * per * t_k;
    if (s > 1) c += reduce_launch_us() + (2.0 * s + 1.0) * out_elems * 4.0 / 4e12 * 1e6;
    return c;
  };
  int best = 1;
  double bc = cost(1);
  if (splitk_enabled())
    for (int s = 2; s <= max_splits && kt_total / s >= min_k; ++s) {
      const double c = cost(s);
      if (c < bc * 0.97) {   // split only for a clear win
        bc = c;
        best = s;
      }
    }
  const int per = (kt_total + best - 1) / best;
  return Plan{bm, bn, (kt_total + per - 1) / per, per};
}

// (bn: the unscaled fp32 tile; conv_plan picks the launch's own with conv_bn -- the packed operand
// depends on bm alone)
void conv_tile(int M, int* bm, int* bn) {
  *bm = conv_bm(M);
  *bn = conv_bn(*bm, false, false);
}

// Resident blocks per CU of a kernel instance (the runtime's occupancy calculator; without a
// device -- CPU-only builds and ABI tests -- a conservative 2) and the CU count.
int num_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = kCUs;
    return n;
  }();
  return v;
}

template <int BM, int BN, int WGM, int WGN, int MODE, bool BSCALE, bool BF16>
int conv_occ() {
  static const int v = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv_gemm_kernel<BM, BN, WGM, WGN, MODE, BSCALE, BF16>, kThreads,
                                                     conv_lds_pad()) != hipSuccess || n <= 0)
      n = 2;
    return n;
  }();
  return v;
}

template <int MODE, bool BSCALE, bool BF16>
int conv_occ_tile(int bm, int bn) {
  switch (bm) {
    case 16:
      if constexpr (!BF16) return conv_occ<16, 256, 1, 4, MODE, BSCALE, BF16>();
      return conv_occ<32, 256, 1, 4, MODE, BSCALE, BF16>();
    case 32: return conv_occ<32, 256, 1, 4, MODE, BSCALE, BF16>();
    case 48:
      if constexpr (!BF16) return conv_occ<48, 128, 1, 4, MODE, BSCALE, BF16>();
      return conv_occ<64, 128, 2, 2, MODE, BSCALE, BF16>();
    case 64: return conv_occ<64, 128, 2, 2, MODE, BSCALE, BF16>();
    case 96: return conv_occ<96, 128, 1, 4, MODE, BSCALE, BF16>();
    default:
      if constexpr (!BSCALE && !BF16)
        if (bn == 256) return conv_occ<128, 256, 2, 2, MODE, BSCALE, BF16>();
      return conv_occ<128, 128, 2, 2, MODE, BSCALE, BF16>();
  }
}

template <bool BF16>
int conv_occupancy_t(int bm, int bn, int mode, bool bscale) {
  switch (mode) {
    case kZero: return bscale ? conv_occ_tile<kZero, true, BF16>(bm, bn) : conv_occ_tile<kZero, false, BF16>(bm, bn);
    case kReplicate:
      return bscale ? conv_occ_tile<kReplicate, true, BF16>(bm, bn) : conv_occ_tile<kReplicate, false, BF16>(bm, bn);
    default:
      return bscale ? conv_occ_tile<kTransposed, true, BF16>(bm, bn) : conv_occ_tile<kTransposed, false, BF16>(bm, bn);
  }
}

int conv_occupancy(int bm, int bn, int mode, bool bscale, bool bf16) {
  return bf16 ? conv_occupancy_t<true>(bm, bn, mode, bscale) : conv_occupancy_t<false>(bm, bn, mode, bscale);
}

// Conv GEMM block schedule.  The plan keeps whole tiles for the first nfull_t column tiles and
// splits the K range of the remaining "tail" tiles S ways into extra blocks; their partial sums
// go to slabs that conv_split_reduce_kernel folds (deterministic, no atomics).  nfull_t = 0 is
// plain split-K (small GEMMs), S = 1 no splitting.  The choice minimises the makespan of greedy
// list scheduling of the blocks (in dispatch order, onto CUs) plus the reduce's cost.  A pure
// function of the geometry (workspace query == launch).
struct ConvPlan {
  int bm, bn, gx, gy, nfull_t, S, kt_per_split;
  long slab_elems;   // S > 1: S * M * tail_cols
};

// Makespan (in K-steps of one block) of F equal blocks of length L followed by R equal blocks of
// length d, list-scheduled in order on `slots` identical slots.
double list_makespan(long F, double L, long R, double d, long slots) {
  const long q = F / slots, r = F % slots;
  const double a = q * L, b = (q + (r ? 1 : 0)) * L;   // (slots - r) slots free at a, r slots at b
  if (R == 0) return b;
  const long n1 = slots - r, n2 = r;
  // smallest T (a breakpoint a + k d or b + k d) with n1 floor((T-a)/d) + n2 floor((T-b)/d) >= R
  for (long k = 1;; ++k) {
    const double T1 = a + k * d;
    const long c1 = n1 * k + (T1 >= b + d ? n2 * (long)((T1 - b) / d + 1e-9) : 0);
    if (c1 >= R) {
      // the b-aligned breakpoint just below T1 may already suffice
      const long kb = (long)((T1 - b) / d + 1e-9);
      if (n2 && kb >= 1) {
        const double T2 = b + kb * d;
        if (T2 < T1 && n1 * (long)((T2 - a) / d + 1e-9) + n2 * kb >= R) return std::max(b, T2);
      }
      return std::max(b, T1);
    }
  }
}

#ifndef GANAMD_SUSTAINED_TFLOPS
#define GANAMD_SUSTAINED_TFLOPS 150.0
#endif
constexpr double kSustainedTflops = GANAMD_SUSTAINED_TFLOPS;   // chip-wide fp32 rate of the GEMM body (split6), all slots busy
constexpr double kSustainedTflopsBf16 = 300.0;   // the bf16-LDS body (conv_body_bf16), gather-bound

// The plan of one tile shape (bm x bn) and its modelled makespan in microseconds.
static ConvPlan conv_plan_tile(int M, int N, int Ck, int T, int mode, bool bscale, bool bf16, int bm, int bn,
                               double rate, double* cost_us) {
  ConvPlan pl{};
  pl.bm = bm;
  pl.bn = bn;
  pl.gx = (N + pl.bn - 1) / pl.bn;
  pl.gy = (M + pl.bm - 1) / pl.bm;
  // bf16 kernels take K-steps of BKB = two fp32 steps (conv_body_bf16)
  const int kt_total = bf16 ? (((Ck + BK - 1) / BK) * T + 1) / 2 : ((Ck + BK - 1) / BK) * T;
  const int bk = bf16 ? BKB : BK;
  const long tiles = (long)pl.gx * pl.gy;
  // slot-level model (blocks run in rounds of occupancy x CUs); the CU-level "fluid" model was
  // measured 7 % slower over the iteration (it under-splits: a lone block does not fill its CU)
  const long slots = (long)conv_occupancy(pl.bm, pl.bn, mode, bscale, bf16) * num_cus();
  const double t_k = 2.0 * pl.bm * pl.bn * bk / (rate * 1e12 / slots) * 1e6;   // us per K-step
  const double ovh = 1.0 / t_k;           // ~1 us per block of prologue / epilogue, in K-steps
  auto cost = [&](int nf, int S, int* per_out) {
    const int per = (kt_total + S - 1) / S;
    const int Sx = (kt_total + per - 1) / per;   // no empty splits
    const long F = (long)nf * pl.gy, R = (tiles - F) * Sx;
    double c = list_makespan(F, kt_total + ovh, R, per + ovh, slots);
    if (Sx > 1 && R > 0) {
      const long tail_cols = N - (long)nf * pl.bn;
      c += (reduce_launch_us() + (2.0 * Sx + 1.0) * (double)M * tail_cols * 4.0 / 4e12 * 1e6) / t_k;
    }
    *per_out = per;
    return c;
  };
  int best_nf = pl.gx, best_S = 1, per = kt_total;
  double best = cost(pl.gx, 1, &per);
  if (splitk_enabled()) {
    const long q = tiles / slots;
    int cand[4] = {0, (int)std::min<long>(pl.gx, q * slots / pl.gy), (int)std::min<long>(pl.gx, (q > 0 ? q - 1 : 0) * slots / pl.gy),
                   pl.gx};
    for (int nf : cand)
      for (int S = 1; S <= 16 && kt_total / S >= 4; ++S) {
        if (nf == pl.gx && S > 1) break;
        int pp;
        const double c = cost(nf, S, &pp);
        if (c < best * 0.97) {   // deviate from whole tiles only for a clear win
          best = c;
          best_nf = nf;
          best_S = S;
        }
      }
  }
  pl.nfull_t = best_nf;
  const int pp = (kt_total + best_S - 1) / best_S;
  pl.kt_per_split = pp;
  pl.S = (kt_total + pp - 1) / pp;
  const long tail_cols = std::max<long>(0, N - (long)pl.nfull_t * pl.bn);
  pl.slab_elems = (pl.S > 1 && tail_cols > 0) ? (long)pl.S * M * tail_cols : 0;
  *cost_us = best * t_k;
  return pl;
}

// 128x256 tiles (2 waves/SIMD) over 128x128 (3 waves/SIMD): per FLOP the wide tile is faster
// when the chip is full (128 -> 128 3x3 32x32 at B = 128: 246 -> 213 us), but it halves the tile
// count, so a grid that fills the narrow tile's slots in whole rounds leaves the wide tile's
// slots a round and a half (B = 96: 179 -> 203 us).  Both plans are costed; the wide one carries
// this measured per-FLOP gain (profiles/r05_ab_wide.txt).
constexpr double kWideGain = 1.14;

ConvPlan conv_plan(int M, int N, int Ck, int T, int mode, bool bscale, bool bf16) {
  int bm, bn;
  conv_tile(M, &bm, &bn);
  bn = (bm <= 32) ? 256 : 128;
  // the bf16 body has 32x32 blocks only: its 48-row GEMMs run on the 64-row tile over the same
  // 48-row packed operand (rows past it read as 0 through the buffer bound, are not stored)
  if (bf16 && bm == 48) bm = 64;
  if (bf16 && bm == 16) bm = 32;
  const double rate = bf16 ? kSustainedTflopsBf16 : kSustainedTflops;
  double c0 = 0.0;
  ConvPlan pl = conv_plan_tile(M, N, Ck, T, mode, bscale, bf16, bm, bn, rate, &c0);
  if (conv_bn(bm, bscale, bf16) == 256 && bn != 256) {
    double c1 = 0.0;
    const ConvPlan w = conv_plan_tile(M, N, Ck, T, mode, bscale, bf16, bm, 256, rate * kWideGain, &c1);
    if (c1 < c0) pl = w;
  }
  return pl;
}

// bytes of the packed A operand of a conv GEMM (rows padded to the tile, K to whole K-steps); x3:
// plus its three bf16 planes (the patch conv's operand)
size_t pack_bytes(int M, int Ck, int T, bool x3 = false) {
  int bm, bn;
  conv_tile(M, &bm, &bn);
  const size_t mpad = (size_t)((M + bm - 1) / bm) * bm;
  return (x3 ? 10 : 4) * mpad * T * (size_t)((Ck + BK - 1) / BK * BK);
}

template <int BM, int BN, int WGM, int WGN, bool SCALED>
int wgrad_occ() {
  static const int v = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wgrad_gemm_kernel<BM, BN, WGM, WGN, kReplicate, SCALED, false, false>,
                                                     kThreads, wgrad_lds_pad()) != hipSuccess || n <= 0)
      n = 2;
    return n;
  }();
  return v;
}

template <bool SCALED>
int wgrad_occ_tile(int bm, int bn) {
  if (bn == 64) return bm == 48 ? wgrad_occ<48, 64, 1, 4, SCALED>() : wgrad_occ<64, 64, 2, 2, SCALED>();
  if (bn == 96) return bm == 96 ? wgrad_occ<96, 96, 2, 2, SCALED>() : wgrad_occ<64, 96, 2, 2, SCALED>();
  switch (bm) {
    case 32: return wgrad_occ<32, 128, 1, 4, SCALED>();
    case 64: return wgrad_occ<64, 128, 2, 2, SCALED>();
    case 96: return wgrad_occ<96, 128, 1, 4, SCALED>();
    default: return wgrad_occ<128, 128, 2, 2, SCALED>();
  }
}

Plan wgrad_plan(int M, int J, int K, int T, bool scaled, bool bf16) {
  int bm = wgrad_bm(M, scaled), bn = 128;
  if (J <= 64 && bm >= 64) {  // narrow gathered side: a 64x64 tile wastes nothing on J = 48..64
    bm = (M <= 48 && !bf16 && tile48()) ? 48 : 64;   // 48x64: 16x16x4 blocks, no empty rows at M = 48
    bn = 64;
  } else if (bm == 128 && !bf16 && tile96() && big96() &&
             (double)M / ((M + 95) / 96 * 96) * J / ((J + 95) / 96 * 96) >
                 (double)M / ((M + 127) / 128 * 128) * J / ((J + 127) / 128 * 128) / 0.9) {
    bm = 96;   // M, J = 1025: 96x96 tiles fill 94 % against 79 % for 128x128
    bn = 96;
  } else if ((bm == 64 || bm == 96) && !bf16 && tile96() && (J + 95) / 96 * 96 / 0.97 < 0.95 * ((J + 127) / 128 * 128)) {
    bn = 96;   // J = 96, 192, ...: 96-wide tiles (16x16x4 blocks) instead of 25 % empty 128-wide ones
  }
  int tiles = ((J + bn - 1) / bn) * ((M + bm - 1) / bm) * T;
  // tap-packed N = (tap, channel) for very narrow gathered sides (the critic's 3-channel input
  // conv: 27 of 576 tile columns used per tap otherwise; 1.85x measured).  For J = 48..192 the
  // per-row tap offsets cost more than the padding they remove (3-13 % slower, tools/ab_shapes.py)
  const int tiles_tp = ((T * J + bn - 1) / bn) * ((M + bm - 1) / bm);
  const bool tp = T > 1 && J < 32 && tiles_tp <= 0.5 * tiles && wgrad_tp_enabled();
  if (tp) tiles = tiles_tp;
  const int occ = scaled ? wgrad_occ_tile<true>(bm, bn) : wgrad_occ_tile<false>(bm, bn);
  Plan pl = split_plan(bm, bn, tiles, (K + BKW - 1) / BKW, 2.0 * bm * bn * BKW, (long)M * J * T, occ, 256, 4);
  pl.tp = tp;
  return pl;
}

// Folds the S partial slabs of the tail columns [n0, n0 + cols) and applies the epilogue.
// Memory-bound: (S + 1) x M x cols floats.  32-bit element indices (M * cols < 2^31 is checked by
// the launcher) and, when every row segment is a whole number of 16-byte vectors landing on
// 16-byte aligned output addresses (VEC), four columns per thread with one row division.
template <bool VEC>
__global__ __launch_bounds__(256) void conv_split_reduce_kernel(
    const float* __restrict__ slab, int S, int M, int cols, int n0, long ldy, int ohw, int B,
    const float* __restrict__ oscale, const float* __restrict__ bias, const float* __restrict__ noise,
    const float* __restrict__ noise_scale, const float* __restrict__ act, float* __restrict__ y, OutMap om) {
  constexpr int V = VEC ? 4 : 1;
  const unsigned total = (unsigned)M * (unsigned)cols, cv = (unsigned)cols / V, units = total / V;
  for (unsigned u = blockIdx.x * 256u + threadIdx.x; u < units; u += gridDim.x * 256u) {
    const unsigned m = u / cv, c = (u - m * cv) * V;
    const unsigned e = m * (unsigned)cols + c;
    float v[V];
    if constexpr (VEC) {
      f32x4 a = *reinterpret_cast<const f32x4*>(slab + e);
#pragma unroll 8   // the slab loads of 8 splits in flight at once (same summation order)
      for (int s = 1; s < S; ++s) a += *reinterpret_cast<const f32x4*>(slab + (long)s * total + e);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    } else {
      float a = slab[e];
#pragma unroll 8   // the slab loads of 8 splits in flight at once (same summation order)
      for (int s = 1; s < S; ++s) a += slab[(long)s * total + e];
      v[0] = a;
    }
    const int n = n0 + (int)c;
    float* yb = y;
    long o;
    if (!VEC && om.s == -2) {   // ring only: column n is the ring position
      yb = om.ring;
      o = (long)m * om.ldr + n;
    } else if (!VEC && om.s < 0) {   // frame split (stride-1 dgrad): interior -> y, ring -> om.ring
      long ld, col;
      if (!frame_target(om, y, ldy, n, yb, ld, col)) continue;
      o = (long)m * ld + col;
    } else {
      o = (long)m * ldy + out_col(om, n);   // VEC: om is the identity, o .. o + 3 contiguous
    }
    const float bm = bias ? bias[m] : 0.f, ns = noise ? noise_scale[m] : 0.f, am = act ? act[m] : 1.f;
    float nz[V];
    if (noise) {
      if constexpr (VEC) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(noise + o);
        nz[0] = t[0]; nz[1] = t[1]; nz[2] = t[2]; nz[3] = t[3];
      } else {
        nz[0] = noise[o];
      }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      float r = v[q];
      if (oscale) r *= oscale[m * B + (unsigned)(n + q) / (unsigned)ohw];
      r += bm;
      if (noise) r += ns * nz[q];
      if (act) r = r > 0.f ? r : am * r;
      v[q] = r;
    }
    if constexpr (VEC) {
      *reinterpret_cast<f32x4*>(yb + o) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
      yb[o] = v[0];
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void wgrad_split_reduce_kernel(const float* __restrict__ slab, int S, int total,
                                                                 float* __restrict__ out, int accumulate) {
  constexpr int V = VEC ? 4 : 1;
  const unsigned units = (unsigned)total / V;
  for (unsigned u = blockIdx.x * 256u + threadIdx.x; u < units; u += gridDim.x * 256u) {
    const unsigned e = u * V;
    if constexpr (VEC) {
      f32x4 a = *reinterpret_cast<const f32x4*>(slab + e);
#pragma unroll 8   // the slab loads of 8 splits in flight at once (same summation order)
      for (int s = 1; s < S; ++s) a += *reinterpret_cast<const f32x4*>(slab + (long)s * total + e);
      if (accumulate) a += *reinterpret_cast<const f32x4*>(out + e);
      *reinterpret_cast<f32x4*>(out + e) = a;
    } else {
      float a = slab[e];
#pragma unroll 8   // the slab loads of 8 splits in flight at once (same summation order)
      for (int s = 1; s < S; ++s) a += slab[(long)s * total + e];
      out[e] = accumulate ? out[e] + a : a;
    }
  }
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int grid1d(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

template <int BM, int BN, int WGM, int WGN, int MODE, bool BSCALE, bool BF16>
hipError_t launch_conv(ConvArgs p, const ConvPlan& pl, float* slab, hipStream_t st) {
  p.gy = pl.gy;
  p.nfull_t = pl.nfull_t;
  p.full_blocks = pl.nfull_t * pl.gy;
  p.S = pl.S;
  p.kt_per_split = pl.kt_per_split;
  p.tail_n0 = pl.nfull_t * BN;
  p.tail_cols = std::max(0, p.N - p.tail_n0);
  p.slab = pl.slab_elems ? slab : nullptr;
  const long blocks = (long)p.full_blocks + (long)(pl.gx - pl.nfull_t) * pl.gy * pl.S;
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WGM, WGN, MODE, BSCALE, BF16>), dim3((unsigned)blocks), dim3(kThreads),
                     conv_lds_pad(), st, p);
  if (pl.slab_elems) {
    const long total = (long)p.M * p.tail_cols;
    if (total >= (1L << 31)) return hipErrorInvalidValue;
    const bool vec = p.om.s == 0 && p.tail_cols % 4 == 0 && p.tail_n0 % 4 == 0 && p.ldy % 4 == 0 && aligned16(slab) &&
                     aligned16(p.y) && (!p.noise || aligned16(p.noise));
    if (vec)
      hipLaunchKernelGGL(conv_split_reduce_kernel<true>, dim3(grid1d(total / 4)), dim3(256), 0, st, slab, pl.S, p.M,
                         p.tail_cols, p.tail_n0, p.ldy, p.ohw, p.g.B, p.oscale, p.bias, p.noise, p.noise_scale, p.act,
                         p.y, p.om);
    else
      hipLaunchKernelGGL(conv_split_reduce_kernel<false>, dim3(grid1d(total)), dim3(256), 0, st, slab, pl.S, p.M,
                         p.tail_cols, p.tail_n0, p.ldy, p.ohw, p.g.B, p.oscale, p.bias, p.noise, p.noise_scale, p.act,
                         p.y, p.om);
  }
  return hipGetLastError();
}

template <int MODE, bool BSCALE, bool BF16>
hipError_t dispatch_conv_tile(const ConvArgs& p, const ConvPlan& pl, float* slab, hipStream_t st) {
  switch (pl.bm) {
    case 16:
      if constexpr (!BF16) return launch_conv<16, 256, 1, 4, MODE, BSCALE, BF16>(p, pl, slab, st);
      return hipErrorInvalidValue;   // conv_plan moves bf16 to the 32-row tile
    case 32: return launch_conv<32, 256, 1, 4, MODE, BSCALE, BF16>(p, pl, slab, st);
    case 48:
      if constexpr (!BF16) return launch_conv<48, 128, 1, 4, MODE, BSCALE, BF16>(p, pl, slab, st);
      return hipErrorInvalidValue;   // conv_plan moves bf16 to the 64-row tile
    case 64: return launch_conv<64, 128, 2, 2, MODE, BSCALE, BF16>(p, pl, slab, st);
    case 96: return launch_conv<96, 128, 1, 4, MODE, BSCALE, BF16>(p, pl, slab, st);
    default:
      if constexpr (!BSCALE && !BF16)   // (conv_bn: the wide tile is for unscaled fp32 GEMMs only)
        if (pl.bn == 256) return launch_conv<128, 256, 2, 2, MODE, BSCALE, BF16>(p, pl, slab, st);
      return launch_conv<128, 128, 2, 2, MODE, BSCALE, BF16>(p, pl, slab, st);
  }
}

void launch_pack(const ganamd_pack_job& j, hipStream_t st) {
  hipLaunchKernelGGL(pack_a_kernel, dim3(grid1d((long)j.Mpad * j.T * j.Ckp)), dim3(256), 0, st, j);
}

template <bool BF16>
hipError_t dispatch_conv_mode(const ConvArgs& p, const ConvPlan& pl, float* slab, hipStream_t st, bool s) {
  switch (p.g.mode) {
    case kZero:
      return s ? dispatch_conv_tile<kZero, true, BF16>(p, pl, slab, st)
               : dispatch_conv_tile<kZero, false, BF16>(p, pl, slab, st);
    case kReplicate:
      return s ? dispatch_conv_tile<kReplicate, true, BF16>(p, pl, slab, st)
               : dispatch_conv_tile<kReplicate, false, BF16>(p, pl, slab, st);
    case kPhase:   // unmodulated only (ConvTranspose2d)
      return s ? hipErrorInvalidValue : dispatch_conv_tile<kPhase, false, BF16>(p, pl, slab, st);
    default:
      return s ? dispatch_conv_tile<kTransposed, true, BF16>(p, pl, slab, st)
               : dispatch_conv_tile<kTransposed, false, BF16>(p, pl, slab, st);
  }
}


// ---- skinny GEMM for the linears ------------------------------------------------------------
// EqualizedLinear / nn.Linear on [features][batch] (a 1x1 conv at H = W = 1): M = out features,
// N = batch (64 .. 384), K = in features.  The tiled conv GEMM spends most of such a launch on one
// block's serial K loop (or on split-K slabs and a reduce launch): ~16-40 us for a few MFLOP.
// Here a block owns 32 rows x 128 columns; its 4 waves split K four ways, each streams its quarter
// straight from global memory into registers (packed A rows: 8 consecutive k per lane; X: one
// 128-byte line per half-wave per k) two 16-k chunks ahead, and the partial tiles are summed
// through LDS before the conv epilogue (alpha, scale, bias, PReLU).  No slab, no second launch.
constexpr int LBM = 32;

// Train-mode BatchNorm1d (+ PReLU) fused into the linear's epilogue (ganamd_linear_bn_act): the
// block owns whole rows (N <= 64 columns = one wave), so the batch statistics are wave sums.
struct BNArgs {
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float momentum, eps;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// JT: 32-column MFMA tiles per block (2: N <= 64, 4: 128 columns); NW waves split K; chunks of 16 k
// are loaded four at a time (four in flight per wave) before their MFMAs.
template <int JT, int NW, bool BN = false>
__global__ __launch_bounds__(64 * NW) void linear_gemm_kernel(ConvArgs p, BNArgs bn) {
  constexpr int LBN = 32 * JT;
  __shared__ __attribute__((aligned(16))) float red[NW][LBM * LBN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * LBM, n0 = blockIdx.y * LBN;
  const int nch = p.Ckp / 16;                                    // 16-k chunks
  const int c0 = wave * nch / NW, c1 = (wave + 1) * nch / NW;    // this wave's share of K
  const rsrc_t ra = make_rsrc(p.w, p.w_bytes);
  const rsrc_t rx = make_rsrc(p.g.src, p.g.src_bytes());
  const int N = p.N;
  const bool row_ok = m0 + r < p.M;
  struct Chunk {
    f32x4 a0, a1;
    float b[8][JT];
  };
  auto load = [&](int c, Chunk& C) {
    const bool ok = c < c1;
    const int ka = c * 16 + 8 * h;
    const int aoff = (row_ok && ok) ? 4 * ((m0 + r) * p.Ckp + ka) : kOOB;
    C.a0 = bload4(ra, aoff);
    C.a1 = bload4(ra, aoff == kOOB ? kOOB : aoff + 16);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = ka + s;
#pragma unroll
      for (int j = 0; j < JT; ++j) {
        const int n = n0 + 32 * j + r;
        C.b[s][j] = bload(rx, (ok && k < p.Ck && n < N) ? 4 * (k * N + n) : kOOB);
      }
    }
  };
  f32x16 acc[JT];
#pragma unroll
  for (int j = 0; j < JT; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  auto mma = [&](const Chunk& C) {
    const float a[8] = {C.a0[0], C.a0[1], C.a0[2], C.a0[3], C.a1[0], C.a1[1], C.a1[2], C.a1[3]};
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < JT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], C.b[s][j], acc[j], 0, 0, 0);
  };
  for (int c = c0; c < c1; c += 4) {     // chunks past c1 load zeros (OOB), their MFMAs add 0
    Chunk x0, x1, x2, x3;
    load(c, x0);
    load(c + 1, x1);
    load(c + 2, x2);
    load(c + 3, x3);
    mma(x0);
    if (c + 1 < c1) mma(x1);
    if (c + 2 < c1) mma(x2);
    if (c + 3 < c1) mma(x3);
  }
  // partial tiles of the NW waves -> LDS -> summed, epilogue, coalesced stores
#pragma unroll
  for (int j = 0; j < JT; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) red[wave][((e & 3) + 8 * (e >> 2) + 4 * h) * LBN + 32 * j + r] = acc[j][e];
  __syncthreads();
  if constexpr (BN) {
    // rows wave + NW*q, one column per lane: y = act(gamma (v - mean) / sqrt(var + eps) + beta)
    // with the batch mean / biased variance of the row; running stats take the unbiased variance
    static_assert(LBN == 64 && LBM % NW == 0, "BN epilogue: one wave per 64-column row");
    const float inv_n = 1.f / (float)N;
    constexpr int RW = LBM / NW;                   // rows per wave
    // the rows' constants are fetched together up front (one memory round trip, not one per row)
    float cb[RW], cg[RW], cbt[RW], ca[RW], rm[RW], rv[RW];
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int m = min(m0 + wave + NW * q, p.M - 1);
      rm[q] = bn.running_mean[m];
      rv[q] = bn.running_var[m];
      cb[q] = p.bias ? p.bias[m] : 0.f;
      cg[q] = bn.gamma[m];
      cbt[q] = bn.beta[m];
      ca[q] = p.act ? p.act[m] : 1.f;
    }
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int row = wave + NW * q;
      const int m = m0 + row;
      if (m >= p.M) break;                         // wave-uniform
      const bool ok = lane < N;
      float v = 0.f;
      if (ok) {
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[w][row * LBN + lane];
        v = v * p.alpha + cb[q];
      }
      const float mean = wave_sum(v) * inv_n;
      const float d = ok ? v - mean : 0.f;
      const float var = wave_sum(d * d) * inv_n;
      float yv = d * (1.f / sqrtf(var + bn.eps)) * cg[q] + cbt[q];
      yv = yv > 0.f ? yv : ca[q] * yv;
      if (ok) p.y[(long)m * p.ldy + lane] = yv;
      if (lane == 0) {
        const float mo = bn.momentum;
        bn.running_mean[m] = (1.f - mo) * rm[q] + mo * mean;
        bn.running_var[m] = (1.f - mo) * rv[q] + mo * var * ((float)N / (float)(N - 1));
      }
    }
    return;
  }
  // each thread owns EI elements (rows tid / LBN + q * (64 NW / LBN), one column); their per-row
  // constants are loaded together (clamped indices, no per-element branches) before the stores
  constexpr int EI = LBM * LBN / (64 * NW);
  const int col = tid % LBN, n = n0 + col, nc = min(n, N - 1);
  float osc[EI], cb[EI], cn[EI], ca[EI];
#pragma unroll
  for (int q = 0; q < EI; ++q) {
    const int m = min(m0 + (tid + q * 64 * NW) / LBN, p.M - 1);
    osc[q] = p.oscale ? p.oscale[m * p.g.B + nc / p.ohw] : 1.f;
    cb[q] = p.bias ? p.bias[m] : 0.f;
    cn[q] = p.noise ? p.noise_scale[m] * p.noise[(long)m * p.ldy + nc] : 0.f;
    ca[q] = p.act ? p.act[m] : 1.f;
  }
#pragma unroll
  for (int q = 0; q < EI; ++q) {
    const int idx = tid + q * 64 * NW;
    const int m = m0 + idx / LBN;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][idx];
    v = (v * p.alpha) * osc[q] + cb[q] + cn[q];
    v = v > 0.f ? v : ca[q] * v;
    if (m < p.M && n < N) p.y[(long)m * p.ldy + n] = v;
  }
}

// The linear path: 1x1, 1x1 maps, unmodulated, fp32, and small enough that the K loop of one
// block does not dominate (above ~4 M weights the tiled GEMM's split-K wins).
bool linear_ok(const ConvArgs& p) {
  const Gather& g = p.g;
  return p.T == 1 && g.H == 1 && g.W == 1 && g.OH == 1 && g.OW == 1 && !g.scale && !p.bf16 && p.ldy == p.N &&
         (long)p.M * p.Ck <= (4L << 20) && linear_enabled();
}

hipError_t launch_linear(const ConvArgs& p, hipStream_t st) {
  if (p.N <= 64)
    hipLaunchKernelGGL((linear_gemm_kernel<2, 8>), dim3((p.M + LBM - 1) / LBM, 1), dim3(512), 0, st, p, BNArgs{});
  else
    hipLaunchKernelGGL((linear_gemm_kernel<4, 4>), dim3((p.M + LBM - 1) / LBM, (p.N + 127) / 128), dim3(256), 0, st, p,
                       BNArgs{});
  return hipGetLastError();
}

// ---- the split6 LDS-patch conv (conv_patch.hip) and row-blocked wgrad (conv_wgrad_row.hip) ------
// Which of them a call may use is the descriptor's kernel_off (GANAMD_KERNEL_*: per call, no library
// state; 0 = all allowed where their domains and grids fit).
constexpr int kMaxPatchScaleChannels = 1024;   // conv_patch.hip kMaxScale: scales staged in LDS

// The packed operand carries the three bf16 planes the patch conv reads (after the fp32 copy the
// gather GEMM reads) whenever the GEMM's geometry is in the patch kernel's domain -- a function of
// the geometry alone, so every copy of one weight has the same layout whatever math or mask is on.
bool patch_packed(int M, int H, int W, int K, int stride, int pad, int OH, int OW) {
  return ganamd_patch::domain(M, H, W, K, stride, pad, OH, OW);
}
long patch_blocks(int M, int B, int H, int W) {
  ganamd_patch::Args a{};
  a.M = M;
  a.B = B;
  a.H = H;
  a.W = W;
  return ganamd_patch::blocks(a);
}
// ... and where it runs: fp32 math, allowed by the descriptor, at most kMaxPatchScaleChannels input
// channels (the modulation scales the block stages in LDS: past that the gather GEMM takes the conv
// instead of the launch failing), and a grid of at least one block per CU whose last round is full or
// follows another (these long one-per-CU blocks leave a half-empty last round idle)
bool patch_geometry(int M, int Ck, int B, int H, int W, int K, int stride, int pad, int OH, int OW, int math,
                    int kernel_off, bool dgrad) {
  if ((kernel_off & (dgrad ? GANAMD_KERNEL_PATCH_DGRAD : GANAMD_KERNEL_PATCH_FWD)) || math != GANAMD_MATH_F32 ||
      Ck > kMaxPatchScaleChannels || !patch_packed(M, H, W, K, stride, pad, OH, OW))
    return false;
  const long blocks = patch_blocks(M, B, H, W), cus = num_cus();
  return blocks >= cus && (blocks % cus == 0 || blocks >= 2 * cus);
}

// p.w/sm/sc/st describe the weights as stored, unless `prepacked` (then p.w is already the
// GEMM-order operand); otherwise `packed` (pack_bytes) receives the GEMM-order copy first.
hipError_t dispatch_conv(ConvArgs p, bool prepacked, float* packed, float* slab, hipStream_t st) {
  const ConvPlan pl = conv_plan(p.M, p.N, p.Ck, p.T, p.g.mode, p.g.scale != nullptr, p.bf16 != 0);
  if ((pl.slab_elems && !slab) || (!prepacked && !packed)) return hipErrorInvalidValue;
  const int bmp = conv_bm(p.M);   // packing granularity (pl.bm may be wider: bf16 48 -> 64)
  const int mpad = (p.M + bmp - 1) / bmp * bmp;
  p.Ckp = (p.Ck + BK - 1) / BK * BK;
  if (p.ldy == 0) p.ldy = p.N;   // output rows are the GEMM rows unless a phase remap says otherwise
  if (!prepacked) {
    launch_pack(ganamd_pack_job{p.w, packed, p.sm, p.sc, p.st, p.M, p.Ck, p.T, mpad, p.Ckp, 1, 0, 0, 0, 0}, st);
    p.w = packed;
  }
  p.w_bytes = 4 * mpad * p.T * p.Ckp;
  if (linear_ok(p)) return launch_linear(p, st);
  const bool s = p.g.scale != nullptr;
  return p.bf16 ? dispatch_conv_mode<true>(p, pl, slab, st, s) : dispatch_conv_mode<false>(p, pl, slab, st, s);
}

template <int BM, int BN, int WGM, int WGN, int MODE, bool SCALED, bool BF16>
hipError_t launch_wgrad(WgradArgs p, int T, const Plan& pl, float* slab, hipStream_t st) {
  const int gy = (p.M + BM - 1) / BM;
  p.kt_per_split = pl.kt_per_split;
  p.splits = pl.splits;
  p.slab = pl.splits > 1 ? slab : nullptr;
  p.T = T;
  if (pl.tp)
    hipLaunchKernelGGL((wgrad_gemm_kernel<BM, BN, WGM, WGN, MODE, SCALED, BF16, true>),
                       dim3((T * p.J + BN - 1) / BN, gy, pl.splits), dim3(kThreads), wgrad_lds_pad(), st, p);
  else
    hipLaunchKernelGGL((wgrad_gemm_kernel<BM, BN, WGM, WGN, MODE, SCALED, BF16, false>),
                       dim3((p.J + BN - 1) / BN, gy, T * pl.splits), dim3(kThreads), wgrad_lds_pad(), st, p);
  if (pl.splits > 1) {
    if (p.out_numel % 4 == 0 && aligned16(slab) && aligned16(p.out))
      hipLaunchKernelGGL(wgrad_split_reduce_kernel<true>, dim3(grid1d(p.out_numel / 4)), dim3(256), 0, st, slab,
                         pl.splits, p.out_numel, p.out, p.accumulate);
    else
      hipLaunchKernelGGL(wgrad_split_reduce_kernel<false>, dim3(grid1d(p.out_numel)), dim3(256), 0, st, slab,
                         pl.splits, p.out_numel, p.out, p.accumulate);
  }
  return hipGetLastError();
}

template <int MODE, bool SCALED, bool BF16>
hipError_t dispatch_wgrad_tile(const WgradArgs& p, int T, const Plan& pl, float* slab, hipStream_t st) {
  if (pl.bn == 64) {
    if constexpr (!BF16)
      if (pl.bm == 48) return launch_wgrad<48, 64, 1, 4, MODE, SCALED, BF16>(p, T, pl, slab, st);
    return launch_wgrad<64, 64, 2, 2, MODE, SCALED, BF16>(p, T, pl, slab, st);
  }
  if (pl.bn == 96) {   // 16x16x4 blocks: fp32 only (wgrad_plan gives bf16 128-wide tiles)
    if constexpr (!BF16)
      return pl.bm == 96 ? launch_wgrad<96, 96, 2, 2, MODE, SCALED, BF16>(p, T, pl, slab, st)
                         : launch_wgrad<64, 96, 2, 2, MODE, SCALED, BF16>(p, T, pl, slab, st);
    return hipErrorInvalidValue;
  }
  switch (pl.bm) {
    case 32: return launch_wgrad<32, 128, 1, 4, MODE, SCALED, BF16>(p, T, pl, slab, st);
    case 64: return launch_wgrad<64, 128, 2, 2, MODE, SCALED, BF16>(p, T, pl, slab, st);
    case 96: return launch_wgrad<96, 128, 1, 4, MODE, SCALED, BF16>(p, T, pl, slab, st);
    default: return launch_wgrad<128, 128, 2, 2, MODE, SCALED, BF16>(p, T, pl, slab, st);
  }
}

hipError_t dispatch_wgrad(const WgradArgs& p, int T, float* slab, hipStream_t st) {
  const bool s = p.ascale != nullptr || p.g.scale != nullptr;
  if (s && !(p.ascale && p.g.scale)) return hipErrorInvalidValue;  // both scales or none
  const Plan pl = wgrad_plan(p.M, p.J, p.K, T, s, p.bf16 != 0);
  if (pl.splits > 1 && !slab) return hipErrorInvalidValue;
  if (p.bf16) {
    if (p.g.mode == kReplicate)
      return s ? dispatch_wgrad_tile<kReplicate, true, true>(p, T, pl, slab, st)
               : dispatch_wgrad_tile<kReplicate, false, true>(p, T, pl, slab, st);
    return s ? dispatch_wgrad_tile<kZero, true, true>(p, T, pl, slab, st)
             : dispatch_wgrad_tile<kZero, false, true>(p, T, pl, slab, st);
  }
  if (p.g.mode == kReplicate)
    return s ? dispatch_wgrad_tile<kReplicate, true, false>(p, T, pl, slab, st)
             : dispatch_wgrad_tile<kReplicate, false, false>(p, T, pl, slab, st);
  return s ? dispatch_wgrad_tile<kZero, true, false>(p, T, pl, slab, st)
           : dispatch_wgrad_tile<kZero, false, false>(p, T, pl, slab, st);
}

// Every tensor a conv call touches is addressed through a buffer descriptor with a 32-bit byte
// range (and offsets at or past 2^31 are the out-of-range sentinel): reject geometries whose
// largest operand -- input, output, the padded dgrad frame, the scatter-dgrad tap products, the
// packed weights -- reaches 2^31 bytes instead of letting an offset wrap.
bool extents_ok(const ganamd_conv_desc* d) {
  const long lim = (1L << 31) - 1;
  const long T = (long)d->KH * d->KW;
  const long x = 4L * d->Cin * d->B * d->H * d->W;
  const long y = 4L * d->Cout * d->B * d->OH * d->OW;
  const long frame = 4L * d->Cin * d->B * (d->H + 2L * d->KH) * (d->W + 2L * d->KW);
  const long frame_t = 4L * d->Cout * d->B * (d->OH + 2L * d->KH) * (d->OW + 2L * d->KW);
  const bool scatter = !d->transposed && T > 1 && (d->stride > 1 || (long)d->H * d->W <= 100);   // dgrad_scatter
  const long taps = scatter ? 4L * d->Cin * T * d->B * d->OH * d->OW : 0;
  const long wpk = 4L * (d->Cout + 256L) * T * (d->Cin + 64L);
  return x <= lim && y <= lim && frame <= lim && frame_t <= lim && taps <= lim && wpk <= lim;
}

bool desc_ok(const ganamd_conv_desc* d) {
  return d && d->B > 0 && d->Cin > 0 && d->Cout > 0 && d->H > 0 && d->W > 0 && d->OH > 0 && d->OW > 0 &&
         d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0 &&
         (d->math == GANAMD_MATH_F32 || d->math == GANAMD_MATH_BF16) &&
         (d->kernel_off & ~(GANAMD_KERNEL_PATCH_FWD | GANAMD_KERNEL_PATCH_DGRAD | GANAMD_KERNEL_WGRAD_ROW |
                            GANAMD_KERNEL_SMALL)) == 0 &&
         extents_ok(d);
}

// The workspace query's answer per (device, descriptor, op), so the size check of every conv call
// does not re-plan (the query runs two or three planner evaluations): an open-addressed table of
// whole-descriptor keys under a lock (calls may come from several threads); a full table is cleared.
struct WsKey {
  ganamd_conv_desc d;
  int op, dev;
};
struct WsSlot {
  WsKey k;
  size_t need;
  bool used;
};
constexpr int kWsSlots = 4096;
WsSlot g_ws_cache[kWsSlots];
int g_ws_count = 0;
std::mutex g_ws_mu;

uint64_t ws_hash(const WsKey& k) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(&k);
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < sizeof(WsKey); ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

// the call's workspace against the query for its descriptor (GANAMD_EINVAL when short or missing)
int ws_check(const ganamd_conv_desc* d, int op, const void* workspace, size_t workspace_bytes) {
  WsKey k;
  memset(&k, 0, sizeof(k));
  k.d = *d;
  k.op = op;
  if (hipGetDevice(&k.dev) != hipSuccess) k.dev = -1;
  const uint64_t h = ws_hash(k);
  size_t need = 0;
  bool hit = false;
  {
    std::lock_guard<std::mutex> lock(g_ws_mu);
    for (int i = 0; i < kWsSlots; ++i) {
      WsSlot& sl = g_ws_cache[(h + i) % kWsSlots];
      if (!sl.used) break;
      if (memcmp(&sl.k, &k, sizeof(k)) == 0) {
        need = sl.need;
        hit = true;
        break;
      }
    }
  }
  if (!hit) {
    if (ganamd_conv_workspace(d, op, &need) != GANAMD_OK) return GANAMD_EINVAL;
    std::lock_guard<std::mutex> lock(g_ws_mu);
    if (2 * (g_ws_count + 1) > kWsSlots) {        // keep probes short: start over when half full
      for (auto& sl : g_ws_cache) sl.used = false;
      g_ws_count = 0;
    }
    for (int i = 0; i < kWsSlots; ++i) {
      WsSlot& sl = g_ws_cache[(h + i) % kWsSlots];
      if (!sl.used) {
        sl.k = k;
        sl.need = need;
        sl.used = true;
        ++g_ws_count;
        break;
      }
      if (memcmp(&sl.k, &k, sizeof(k)) == 0) break;
    }
  }
  return need && (!workspace || workspace_bytes < need) ? GANAMD_EINVAL : GANAMD_OK;
}

}  // namespace

extern "C" {

// Geometry of each GEMM the three entry points issue (shared by the workspace query and launch).
static bool fwd_phased(const ganamd_conv_desc* d);
// (phased: the GEMM of ONE output phase; there are stride^2 of them)
static void fwd_gemm(const ganamd_conv_desc* d, int* M, int* N, int* Ck, int* T) {
  const int s2 = fwd_phased(d) ? d->stride * d->stride : 1;
  *M = d->Cout;
  *N = d->B * d->OH * d->OW / s2;
  *Ck = d->Cin;
  *T = d->KH * d->KW / s2;
}

// Small maps (<= 10x10) and strided convs: dgrad as a plain GEMM over the conv's OUTPUT pixels,
// Z[(ci,t)][n] = sum_co W[co][ci][t] * gy[co][n], then dgrad_fold_kernel.  The transposed
// gather into the padded frame would feed the MFMAs mostly zero taps there (a 4x4 map's 6x6
// frame: 2.25x the work; a valid 3x3 conv on 5x5: 2.8x; stride 2: 4x, three taps in four
// have the wrong parity).  The Z round trip costs (KH*KW / stride^2) x the input gradient's bytes.
//
// Strided convs on larger maps: dgrad as s*s phase GEMMs over the padded input frame (kPhase
// gather of gy, OutMap s = -3).  Frame point (s*j + qa, s*i + qc) takes only the taps
// kh = qa + s*th, kw = qc + s*tw -- ntaps(K, s, qa) x ntaps(K, s, qc) of them (3x3, s = 2: 4, 2, 2, 1),
// summed over gy(j - th, i - tw): the algorithmic work (plus the frame ring), no tap-product buffer,
// no fold pass; interior points are stored straight into gx, the ring folded like the stride-1
// frame split.  Needs every phase grid the same size ((H + 2p) % s == 0) and no gy scale.
static bool dgrad_phased(const ganamd_conv_desc* d) {
  const int s = d->stride;
  return !d->transposed && s > 1 && d->KH == d->KW && d->KH > 1 && d->H * d->W > 100 &&
         (d->H + 2 * d->pad) % s == 0 && (d->W + 2 * d->pad) % s == 0 &&
         d->OH == (d->H + 2 * d->pad - d->KH) / s + 1 && d->OW == (d->W + 2 * d->pad - d->KW) / s + 1;
}

static bool dgrad_scatter(const ganamd_conv_desc* d) {
  return !d->transposed && d->KH * d->KW > 1 && ((d->stride > 1 && !dgrad_phased(d)) || d->H * d->W <= 100);
}

// taps and grid of dgrad phase q of a phased dgrad
static void dgrad_phase(const ganamd_conv_desc* d, int q, int* T, int* KWq, int* Hq, int* Wq) {
  const int s = d->stride, qa = q / s, qc = q % s;
  *KWq = ntaps(d->KW, s, qc);
  *T = ntaps(d->KH, s, qa) * *KWq;
  *Hq = (d->H + 2 * d->pad) / s;
  *Wq = (d->W + 2 * d->pad) / s;
}

static void dgrad_gemm(const ganamd_conv_desc* d, int* M, int* N, int* Ck, int* T) {
  *Ck = d->Cout;
  if (dgrad_phased(d)) {   // the largest phase (q = 0)
    int kw, hq, wq;
    dgrad_phase(d, 0, T, &kw, &hq, &wq);
    *M = d->Cin;
    *N = d->B * hq * wq;
    return;
  }
  if (dgrad_scatter(d)) {
    *M = d->Cin * d->KH * d->KW;
    *T = 1;
    *N = d->B * d->OH * d->OW;
    return;
  }
  *M = d->Cin;
  *T = d->KH * d->KW;
  const int hp = d->transposed ? d->H : d->H + 2 * d->pad, wp = d->transposed ? d->W : d->W + 2 * d->pad;
  *N = d->B * hp * wp;
}

static size_t dgrad_scatter_bytes(const ganamd_conv_desc* d) {
  return dgrad_scatter(d) ? sizeof(float) * (size_t)d->Cin * d->KH * d->KW * d->B * d->OH * d->OW : 0;
}

// The A operand (weights) of the fwd / dgrad GEMM as stored: A(m, t, c) = w[m*sm + c*sc + t*st].
static void a_operand(const ganamd_conv_desc* d, int op, int* M, int* Ck, int* T, int* sm, int* sc) {
  *T = d->KH * d->KW;
  if (op == GANAMD_CONV_FWD) {
    *M = d->Cout;
    *Ck = d->Cin;
    if (d->transposed) {  // weights [Cin][Cout][KH][KW], transposed gather
      *sm = *T;
      *sc = d->Cout * *T;
    } else {              // weights [Cout][Cin][KH][KW]
      *sm = d->Cin * *T;
      *sc = *T;
    }
  } else if (dgrad_scatter(d)) {  // Z GEMM: A((ci,t), co) = W[co][ci][t]
    *M = d->Cin * *T;
    *Ck = d->Cout;
    *sm = 1;
    *sc = d->Cin * *T;
    *T = 1;
  } else {
    *M = d->Cin;
    *Ck = d->Cout;
    if (d->transposed) {  // dX of ConvT: plain conv of gy with W viewed [Cin][Cout][KH][KW]
      *sm = d->Cout * *T;
      *sc = *T;
    } else {              // dX of conv: transposed gather, W[co][ci][t] as A(ci, t, co)
      *sm = *T;
      *sc = d->Cin * *T;
    }
  }
}

// Forward of a stride-s transposed conv as s*s phase GEMMs (kPhase): each output phase
// (oh % s, ow % s) sees only (K/s)^2 of the K^2 taps, so the transposed gather's zero taps
// (3 in 4 at s = 2) never reach the MFMAs.
static bool fwd_phased(const ganamd_conv_desc* d) {
  return d->transposed && d->stride > 1 && d->KH == d->KW && d->KH % d->stride == 0 && d->OH % d->stride == 0 &&
         d->OW % d->stride == 0;
}

// Whether op's packed copy also carries the bf16 planes of the patch conv (patch_packed): the
// replicate-padded forward and the (frame-split) dgrad of a stride-1 same conv in its domain.
static bool pack_x3(const ganamd_conv_desc* d, int op) {
  if (d->transposed || d->KH != d->KW) return false;
  if (op == GANAMD_CONV_FWD)
    return d->pad_mode == GANAMD_PAD_REPLICATE &&
           patch_packed(d->Cout, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW);
  return op == GANAMD_CONV_DGRAD && !dgrad_scatter(d) &&
         patch_packed(d->Cin, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW);
}

static ganamd_pack_job pack_job(const ganamd_conv_desc* d, int op, const float* w, float* packed) {
  int M, Ck, T, sm, sc, bm, bn;
  a_operand(d, op, &M, &Ck, &T, &sm, &sc);
  conv_tile(M, &bm, &bn);
  const bool ph = op == GANAMD_CONV_FWD && fwd_phased(d);
  const bool dph = op == GANAMD_CONV_DGRAD && dgrad_phased(d);
  return ganamd_pack_job{w, packed, sm, sc, 1, M, Ck, T, (M + bm - 1) / bm * bm, (Ck + BK - 1) / BK * BK,
                         ph ? d->stride : dph ? -d->stride : 1, (ph || dph) ? d->KH : 0, ph ? d->pad : 0,
                         pack_x3(d, op) ? 1 : 0, 0};
}

// the direct conv of Cout <= 4 forwards (conv_small.hip): raw weights only (packed_w = 0)
static bool small_fwd(const ganamd_conv_desc* d) {
  return !(d->kernel_off & GANAMD_KERNEL_SMALL) && !d->packed_w && d->math == GANAMD_MATH_F32 && d->KH == d->KW &&
         ganamd_small::domain(d->Cout, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->transposed);
}
// The row-blocked split6 weight gradient (conv_wgrad_row.hip) where its domain fits: fp32 math,
// stride-1 same convs on 32 / 64-wide maps; the split-K partial sums reduced here.
static bool wrow_ok(const ganamd_conv_desc* d) {
  return !(d->kernel_off & GANAMD_KERNEL_WGRAD_ROW) && d->math == GANAMD_MATH_F32 && d->KH == d->KW &&
         ganamd_wrow::domain(d->Cout, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->transposed);
}
static int wrow_splits(const ganamd_conv_desc* d, int segs) {
  int s = 1, per = 0;
  ganamd_wrow::plan(d->Cout, d->Cin, d->B, d->H, d->W, d->KH, segs, num_cus(), &s, &per);
  return s;
}
// the patch conv's arguments from the GEMM's (p: its A rows / K layout, gather source and epilogue)
static ganamd_patch::Args patch_args(const ConvArgs& p, const float* packed, int mpad, int K, bool dgrad) {
  ganamd_patch::Args a{};
  const int wplane = mpad * p.T * p.Ckp;
  a.w = reinterpret_cast<const unsigned short*>(packed + wplane);
  a.wplane = wplane;
  a.w_bytes = 6 * wplane;
  a.M = p.M;
  a.Ckp = p.Ckp;
  a.KK = K;
  a.src = p.g.src;
  a.scale = p.g.scale;
  a.C = p.g.C;
  a.B = p.g.B;
  a.H = p.g.H;
  a.W = p.g.W;
  a.y = p.y;
  a.ldy = p.ldy;
  a.bias = p.bias;
  a.oscale = p.oscale;
  a.noise = p.noise;
  a.noise_scale = p.noise_scale;
  a.act = p.act;
  a.alpha = p.alpha;
  a.dgrad = dgrad ? 1 : 0;
  return a;
}

// The frame-split dgrad's ring buffer (replication padding only: zero padding drops the ring)
static size_t dgrad_pad_bytes(const ganamd_conv_desc* d) {
  if (d->transposed || d->pad == 0 || dgrad_scatter(d) || d->pad_mode != GANAMD_PAD_REPLICATE) return 0;
  // (also the phased strided dgrad's ring)
  const size_t Hp = d->H + 2 * d->pad, Wp = d->W + 2 * d->pad;
  return sizeof(float) * (size_t)d->Cin * d->B * (Hp * Wp - (size_t)d->H * d->W);
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Gather mode of the fwd / dgrad GEMM; the split slabs the plan needs, for either scale variant
// (the query does not know whether a scale will be passed; the launch plans with the actual one).
static int fwd_mode(const ganamd_conv_desc* d) {
  if (fwd_phased(d)) return kPhase;
  return d->transposed ? kTransposed : (d->pad_mode == GANAMD_PAD_REPLICATE ? kReplicate : kZero);
}
static int dgrad_mode(const ganamd_conv_desc* d) {
  if (dgrad_phased(d)) return kPhase;
  return (dgrad_scatter(d) || d->transposed) ? kZero : kTransposed;
}
static size_t slab_bytes(int M, int N, int Ck, int T, int mode, bool bf16) {
  const long a = conv_plan(M, N, Ck, T, mode, false, bf16).slab_elems, b = conv_plan(M, N, Ck, T, mode, true, bf16).slab_elems;
  return sizeof(float) * (size_t)std::max(a, b);
}

int ganamd_conv_pack_bytes(const ganamd_conv_desc* d, int op, size_t* bytes) {
  if (!desc_ok(d) || !bytes || (op != GANAMD_CONV_FWD && op != GANAMD_CONV_DGRAD)) return GANAMD_EINVAL;
  int M, Ck, T, sm, sc;
  a_operand(d, op, &M, &Ck, &T, &sm, &sc);
  *bytes = pack_bytes(M, Ck, T, pack_x3(d, op));
  return GANAMD_OK;
}

int ganamd_conv_plan_info(const ganamd_conv_desc* d, int op, int scaled, int* info) {
  if (!desc_ok(d) || !info || (op != GANAMD_CONV_FWD && op != GANAMD_CONV_DGRAD)) return GANAMD_EINVAL;
  int M, N, Ck, T;
  if (op == GANAMD_CONV_FWD)
    fwd_gemm(d, &M, &N, &Ck, &T);
  else
    dgrad_gemm(d, &M, &N, &Ck, &T);
  const int mode = op == GANAMD_CONV_FWD ? fwd_mode(d) : dgrad_mode(d);
  const int Mp = op == GANAMD_CONV_FWD ? d->Cout : d->Cin;
  if (op == GANAMD_CONV_FWD && small_fwd(d)) {
    // kernel 2: the direct conv -- {M, pixels per block, blocks, 1, blocks, 1, input channels, blocks, -, CUs, 2}
    const int th = 8, blocks = d->B * (d->H / th);
    const int v[11] = {d->Cout, th * d->W, blocks, 1, blocks, 1, d->Cin, blocks, 1, num_cus(), 2};
    for (int i = 0; i < 11; ++i) info[i] = v[i];
    return GANAMD_OK;
  }
  if (pack_x3(d, op) && patch_geometry(Mp, Ck, d->B, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->math,
                                       d->kernel_off, op == GANAMD_CONV_DGRAD)) {
    ganamd_patch::Args a{};
    a.M = Mp;
    a.B = d->B;
    a.H = d->H;
    a.W = d->W;
    a.KK = d->KH;
    a.dgrad = op == GANAMD_CONV_DGRAD;
    a.scale = scaled ? reinterpret_cast<const float*>(info) : nullptr;   // selects the instance only
    const int bm = ganamd_patch::row_tile(Mp), gy = (Mp + bm - 1) / bm;
    const int blocks = (int)ganamd_patch::blocks(a), gx = blocks / gy;
    const int v[11] = {bm, ganamd_patch::block_pixels(d->W, d->B, d->H), gx, gy, gx, 1, ((Ck + BK - 1) / BK) * T, blocks,
                       ganamd_patch::occupancy(a), num_cus(), 1};
    for (int i = 0; i < 11; ++i) info[i] = v[i];
    return GANAMD_OK;
  }
  const ConvPlan pl = conv_plan(M, N, Ck, T, mode, scaled != 0, d->math == GANAMD_MATH_BF16);
  const int v[11] = {pl.bm, pl.bn, pl.gx, pl.gy, pl.nfull_t, pl.S, pl.kt_per_split,
                     pl.nfull_t * pl.gy + (pl.gx - pl.nfull_t) * pl.gy * pl.S,
                     conv_occupancy(pl.bm, pl.bn, mode, scaled, d->math == GANAMD_MATH_BF16),
                     num_cus(), 0};
  for (int i = 0; i < 11; ++i) info[i] = v[i];
  return GANAMD_OK;
}

int ganamd_conv_pack_job(const ganamd_conv_desc* d, int op, const float* w, float* packed, ganamd_pack_job* job) {
  if (!desc_ok(d) || !w || !packed || !job || (op != GANAMD_CONV_FWD && op != GANAMD_CONV_DGRAD)) return GANAMD_EINVAL;
  *job = pack_job(d, op, w, packed);
  return GANAMD_OK;
}

int64_t ganamd_pack_job_chunks(const ganamd_pack_job* job) {
  if (!job) return 0;
  if (pack_transposed(*job))   // one tile = kPackRows(T) output rows of one channel chunk
    return (long)(job->Ckp / BK) * ((job->Mpad + pack_rows(job->T) - 1) / pack_rows(job->T));
  const long total = (long)job->Mpad * job->T * job->Ckp;
  return (total + kPackChunk - 1) / kPackChunk;
}

int ganamd_conv_pack_batch(const ganamd_pack_job* jobs, int n_jobs, int64_t total_chunks, hipStream_t stream) {
  if (!jobs || n_jobs <= 0 || total_chunks <= 0 || total_chunks > 0x7fffffffL) return GANAMD_EINVAL;
  hipLaunchKernelGGL(pack_batch_kernel, dim3((unsigned)total_chunks), dim3(256), 0, stream, jobs, n_jobs);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

int ganamd_conv_pack(const ganamd_conv_desc* d, int op, const float* w, float* packed, hipStream_t stream) {
  if (!desc_ok(d) || !w || !packed || (op != GANAMD_CONV_FWD && op != GANAMD_CONV_DGRAD)) return GANAMD_EINVAL;
  launch_pack(pack_job(d, op, w, packed), stream);
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

int ganamd_conv_workspace(const ganamd_conv_desc* d, int op, size_t* bytes) {
  if (!desc_ok(d) || !bytes) return GANAMD_EINVAL;
  int M, N, Ck, T;
  *bytes = 0;
  if (op == GANAMD_CONV_FWD) {
    if (small_fwd(d)) return GANAMD_OK;     // the direct conv needs no workspace
    fwd_gemm(d, &M, &N, &Ck, &T);
    *bytes = (d->packed_w ? 0 : align256(pack_bytes(M, Ck, d->KH * d->KW, pack_x3(d, op)))) +
             slab_bytes(M, N, Ck, T, fwd_mode(d), d->math == GANAMD_MATH_BF16);
  } else if (op == GANAMD_CONV_DGRAD) {
    dgrad_gemm(d, &M, &N, &Ck, &T);
    // split slabs: the frame GEMM's, or the ring-only GEMM's next to the patch conv (B x ring columns)
    const int Hp = d->H + 2 * d->pad, Wp = d->W + 2 * d->pad;
    const int Nring = d->B * (Hp * Wp - d->H * d->W);
    size_t slabs = std::max(slab_bytes(M, N, Ck, T, dgrad_mode(d), d->math == GANAMD_MATH_BF16),
                            Nring > 0 ? slab_bytes(M, Nring, Ck, T, kTransposed, d->math == GANAMD_MATH_BF16) : 0);
    if (dgrad_phased(d))
      for (int q = 1; q < d->stride * d->stride; ++q) {
        int Tq, kw, hq, wq;
        dgrad_phase(d, q, &Tq, &kw, &hq, &wq);
        slabs = std::max(slabs, slab_bytes(M, d->B * hq * wq, Ck, Tq, kPhase, d->math == GANAMD_MATH_BF16));
      }
    // the packed copy as ganamd_conv_dgrad lays it out: a_operand's shape (the phased form packs
    // all s*s phases, KH*KW taps in all -- not phase 0's, which sized the GEMM above)
    int Ma, Cka, Ta, sma, sca;
    a_operand(d, GANAMD_CONV_DGRAD, &Ma, &Cka, &Ta, &sma, &sca);
    *bytes = (d->packed_w ? 0 : align256(pack_bytes(Ma, Cka, Ta, pack_x3(d, op)))) + align256(dgrad_pad_bytes(d)) +
             align256(dgrad_scatter_bytes(d)) + slabs;
  } else if (op == GANAMD_CONV_WGRAD) {
    const int Kpix = d->transposed ? d->B * d->H * d->W : d->B * d->OH * d->OW;
    T = d->KH * d->KW;
    const int Mw = d->transposed ? d->Cin : d->Cout, Jw = d->transposed ? d->Cout : d->Cin;
    // the modulated (scaled) variant plans the same or more splits; size for the larger
    const bool bf = d->math == GANAMD_MATH_BF16;
    const Plan a = wgrad_plan(Mw, Jw, Kpix, T, false, bf), b = wgrad_plan(Mw, Jw, Kpix, T, true, bf);
    // ... and for the two-segment GEMM of ganamd_conv_wgrad2 (K = 2 Kpix, unscaled)
    const Plan c = wgrad_plan(Mw, Jw, 2 * Kpix, T, false, bf);
    int S = std::max(std::max(a.splits, b.splits), c.splits);
    // ... and the row-blocked kernel's (one and two segments), where it can run
    if (d->math == GANAMD_MATH_F32 && d->KH == d->KW &&
        ganamd_wrow::domain(d->Cout, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->transposed))
      S = std::max(S, std::max(wrow_splits(d, 1), wrow_splits(d, 2)));
    *bytes = S > 1 ? sizeof(float) * (size_t)S * d->Cin * d->Cout * T : 0;
  } else {
    return GANAMD_EINVAL;
  }
  return GANAMD_OK;
}

int ganamd_conv_fwd(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias,
                    const float* x_scale, const float* y_scale, float alpha, float* y, void* workspace,
                    size_t workspace_bytes, hipStream_t stream) {
  return ganamd_conv_fwd_ex(d, x, w, bias, x_scale, y_scale, alpha, nullptr, nullptr, nullptr, y, workspace,
                            workspace_bytes, stream);
}

int ganamd_linear_bn_act(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias, float alpha,
                         const float* gamma, const float* beta, const float* act_alpha, float* running_mean,
                         float* running_var, float momentum, float eps, float* y, void* workspace,
                         size_t workspace_bytes, hipStream_t stream) {
  if (!desc_ok(d) || !x || !w || !y || !gamma || !beta || !running_mean || !running_var) return GANAMD_EINVAL;
  if (d->H != 1 || d->W != 1 || d->KH != 1 || d->KW != 1 || d->transposed || d->stride != 1 || d->pad != 0 ||
      d->math != GANAMD_MATH_F32 || d->B < 2 || d->B > 64)
    return GANAMD_EINVAL;
  if (!d->packed_w && ws_check(d, GANAMD_CONV_FWD, workspace, workspace_bytes) != GANAMD_OK) return GANAMD_EINVAL;
  ConvArgs p{};
  p.M = d->Cout;
  p.Ck = d->Cin;
  p.T = 1;
  p.sm = d->Cin;
  p.sc = 1;
  p.st = 1;
  p.g = Gather{x, nullptr, d->Cin, d->B, 1, 1, 1, 1, 1, 1, 0, kZero};
  p.y = y;
  p.bias = bias;
  p.act = act_alpha;
  p.alpha = alpha;
  p.N = d->B;
  p.ohw = 1;
  p.ldy = d->B;
  const int bmp = conv_bm(p.M);
  const int mpad = (p.M + bmp - 1) / bmp * bmp;
  p.Ckp = (p.Ck + BK - 1) / BK * BK;
  if (!linear_ok(p)) return GANAMD_EINVAL;     // the skinny-GEMM domain (M x K <= 4 M weights)
  p.w = w;
  if (!d->packed_w) {
    float* packed = static_cast<float*>(workspace);
    launch_pack(ganamd_pack_job{w, packed, p.sm, p.sc, p.st, p.M, p.Ck, 1, mpad, p.Ckp, 1, 0, 0, 0, 0}, stream);
    p.w = packed;
  }
  p.w_bytes = 4 * mpad * p.Ckp;
  hipLaunchKernelGGL((linear_gemm_kernel<2, 8, true>), dim3((p.M + LBM - 1) / LBM, 1), dim3(512), 0, stream, p,
                     BNArgs{gamma, beta, running_mean, running_var, momentum, eps});
  return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
}

int ganamd_conv_fwd_ex(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias,
                       const float* x_scale, const float* y_scale, float alpha, const float* noise,
                       const float* noise_scale, const float* act_alpha, float* y, void* workspace,
                       size_t workspace_bytes, hipStream_t stream) {
  if (!desc_ok(d) || !x || !w || !y || (noise && !noise_scale)) return GANAMD_EINVAL;
  if (ws_check(d, GANAMD_CONV_FWD, workspace, workspace_bytes) != GANAMD_OK) return GANAMD_EINVAL;
  if (small_fwd(d)) {
    if (noise) return GANAMD_EINVAL;        // (no noisy conv has Cout <= 4)
    const ganamd_small::Args a{x, x_scale, w, bias, y_scale, act_alpha, alpha, y, d->B, d->Cin, d->H, d->W,
                               d->Cout, d->KH, d->pad, d->pad_mode == GANAMD_PAD_REPLICATE ? 1 : 0};
    return ganamd_small::launch(a, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  ConvArgs p{};
  int M, N, Ck, T, sm, sc;
  fwd_gemm(d, &M, &N, &Ck, &T);
  const int Nph = N, Tph = T;
  a_operand(d, GANAMD_CONV_FWD, &M, &Ck, &T, &sm, &sc);
  p.w = w;
  p.sm = sm;
  p.sc = sc;
  p.st = 1;
  p.M = M;
  p.Ck = Ck;
  p.T = T;
  p.g = Gather{x, x_scale, d->Cin, d->B, d->H, d->W, d->OH, d->OW, d->KW, d->stride, d->pad,
               d->transposed ? kTransposed : (d->pad_mode == GANAMD_PAD_REPLICATE ? kReplicate : kZero)};
  p.y = y;
  p.bias = bias;
  p.oscale = y_scale;
  p.noise = noise;
  p.noise_scale = noise_scale;
  p.act = act_alpha;
  p.alpha = alpha;
  p.N = N;
  p.ohw = d->OH * d->OW;
  p.bf16 = d->math == GANAMD_MATH_BF16;
  p.ldy = N;
  char* ws = static_cast<char*>(workspace);
  float* packed = d->packed_w ? nullptr : reinterpret_cast<float*>(ws);
  float* slab = reinterpret_cast<float*>(ws + (d->packed_w ? 0 : align256(pack_bytes(M, Ck, T, pack_x3(d, GANAMD_CONV_FWD)))));
  if (pack_x3(d, GANAMD_CONV_FWD) &&
      patch_geometry(M, Ck, d->B, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->math, d->kernel_off, false)) {
    // the split6 LDS-patch conv (conv_patch.hip) on the planes of the packed operand
    const int bmp = conv_bm(M), mpad = (M + bmp - 1) / bmp * bmp;
    p.Ckp = (Ck + BK - 1) / BK * BK;
    const float* pw = w;
    if (!d->packed_w) {
      launch_pack(pack_job(d, GANAMD_CONV_FWD, w, packed), stream);
      pw = packed;
    }
    return ganamd_patch::launch(patch_args(p, pw, mpad, d->KH, false), stream) == hipSuccess ? GANAMD_OK
                                                                                              : GANAMD_ELAUNCH;
  }
  if (!fwd_phased(d))
    return dispatch_conv(p, d->packed_w != 0, packed, slab, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  if (x_scale || y_scale) return GANAMD_EINVAL;   // phased transposed convs are unmodulated
  // s*s phase GEMMs over the phase-packed weights (pack_job): phase q = (qh, qw) writes the
  // outputs (b, s*j + qh, s*i + qw) of its OHp x OWp grid
  const int s = d->stride, OHp = d->OH / s, OWp = d->OW / s;
  const float* wq = w;
  if (!d->packed_w) {
    launch_pack(pack_job(d, GANAMD_CONV_FWD, w, packed), stream);
    wq = packed;
  }
  int bm, bn;
  conv_tile(M, &bm, &bn);
  const long per = (long)((M + bm - 1) / bm * bm) * Tph * ((Ck + BK - 1) / BK * BK);
  p.T = Tph;
  p.N = Nph;
  p.ohw = OHp * OWp;
  p.ldy = (long)d->B * d->OH * d->OW;
  for (int q = 0; q < s * s; ++q) {
    const int qh = q / s, qw = q % s, kh0 = (qh + d->pad) % s, kw0 = (qw + d->pad) % s;
    p.w = wq + q * per;
    p.g = Gather{x, nullptr, d->Cin, d->B, d->H, d->W, OHp, OWp, d->KW / s, 1, 0, kPhase,
                 (qh + d->pad - kh0) / s, (qw + d->pad - kw0) / s};
    p.om = OutMap{s, qh, qw, OWp, OHp * OWp, d->OW, d->OH * d->OW};
    if (dispatch_conv(p, true, nullptr, slab, stream) != hipSuccess) return GANAMD_ELAUNCH;
  }
  return GANAMD_OK;
}

int ganamd_conv_dgrad(const ganamd_conv_desc* d, const float* gy, const float* w, const float* gy_scale, float alpha,
                      float* gx, void* workspace, size_t workspace_bytes, hipStream_t stream) {
  if (!desc_ok(d) || !gy || !w || !gx) return GANAMD_EINVAL;
  if (ws_check(d, GANAMD_CONV_DGRAD, workspace, workspace_bytes) != GANAMD_OK) return GANAMD_EINVAL;
  int M, N, Ck, T, sm, sc;
  dgrad_gemm(d, &M, &N, &Ck, &T);
  a_operand(d, GANAMD_CONV_DGRAD, &M, &Ck, &T, &sm, &sc);
  ConvArgs p{};
  p.w = w;
  p.sm = sm;
  p.sc = sc;
  p.st = 1;
  p.M = M;
  p.Ck = Ck;
  p.T = T;
  p.bias = nullptr;
  p.oscale = nullptr;
  p.alpha = alpha;
  p.N = N;
  p.bf16 = d->math == GANAMD_MATH_BF16;
  const size_t pad_bytes = dgrad_pad_bytes(d);
  char* ws = static_cast<char*>(workspace);
  float* packed = d->packed_w ? nullptr : reinterpret_cast<float*>(ws);
  if (!d->packed_w) ws += align256(pack_bytes(M, Ck, T, pack_x3(d, GANAMD_CONV_DGRAD)));
  float* slab = reinterpret_cast<float*>(ws + align256(pad_bytes) + align256(dgrad_scatter_bytes(d)));
  const bool pre = d->packed_w != 0;
  if (dgrad_phased(d)) {
    if (gy_scale) return GANAMD_EINVAL;   // strided convs are unmodulated (no kPhase x scale instance)
    // s*s phase GEMMs over the padded frame (OutMap s = -3): interior -> gx, ring -> ring buffer
    // (replication padding; dropped for zero padding), then ring_fold_kernel
    const int s = d->stride, Hp = d->H + 2 * d->pad, Wp = d->W + 2 * d->pad;
    const float* wq = w;
    if (!pre) {
      launch_pack(pack_job(d, GANAMD_CONV_DGRAD, w, packed), stream);
      wq = packed;
    }
    int bm, bn;
    conv_tile(M, &bm, &bn);
    const long mpad = (M + bm - 1) / bm * bm, ckp = (Ck + BK - 1) / BK * BK;
    float* ring = pad_bytes ? reinterpret_cast<float*>(ws) : nullptr;
    const int Rn = Hp * Wp - d->H * d->W;
    p.ldy = (long)d->B * d->H * d->W;
    p.y = gx;
    long off = 0;
    for (int q = 0; q < s * s; ++q) {
      int Tq, KWq, Hq, Wq;
      dgrad_phase(d, q, &Tq, &KWq, &Hq, &Wq);
      p.w = wq + off;
      off += mpad * Tq * ckp;
      p.T = Tq;
      p.N = d->B * Hq * Wq;
      p.ohw = Hq * Wq;
      p.g = Gather{gy, nullptr, d->Cout, d->B, d->OH, d->OW, Hq, Wq, KWq, 1, 0, kPhase, 0, 0};
      p.om = OutMap{-3, d->pad, d->H, Wp, Hp * Wp, d->W, d->H * d->W, Rn, (long)d->B * Rn, ring,
                    s, q / s, q % s, Wq, Hq * Wq};
      if (dispatch_conv(p, true, nullptr, slab, stream) != hipSuccess) return GANAMD_ELAUNCH;
    }
    if (ring) {
      const long planes = (long)d->Cin * d->B;
      const long edges = (long)2 * d->W + 2 * d->H;
      hipLaunchKernelGGL(ring_fold_kernel, dim3(grid1d(planes * edges)), dim3(256), 0, stream, ring, gx, (int)planes,
                         d->H, d->W, d->pad);
    }
    return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  if (dgrad_scatter(d)) {
    float* Z = reinterpret_cast<float*>(ws);
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->OH, d->OW, 1, 1, 0, kZero};
    p.y = Z;
    p.ohw = d->OH * d->OW;
    if (dispatch_conv(p, pre, packed, slab, stream) != hipSuccess) return GANAMD_ELAUNCH;
    const long total = (long)d->Cin * d->B * d->H * d->W;
    const int rep = d->pad_mode == GANAMD_PAD_REPLICATE ? 1 : 0;
    const bool k3 = d->KH == 3 && d->KW == 3, k5 = d->KH == 5 && d->KW == 5;
    const FoldDivs dv{Div31::of(d->W), Div31::of(d->H), Div31::of(d->B)};
    if (total < (1L << 31) - (1L << 24)) {
      auto fold = k3 && d->stride == 1   ? dgrad_fold_kernel<unsigned, 1, 3>
                  : k3 && d->stride == 2 ? dgrad_fold_kernel<unsigned, 2, 3>
                  : k5 && d->stride == 1 ? dgrad_fold_kernel<unsigned, 1, 5>
                                         : dgrad_fold_kernel<unsigned>;
      hipLaunchKernelGGL(fold, dim3(grid1d(total)), dim3(256), 0, stream, Z, gx, d->Cin, d->B, d->H, d->W, d->OH, d->OW,
                         d->KH, d->KW, d->stride, d->pad, rep, dv);
    } else
      hipLaunchKernelGGL(dgrad_fold_kernel<long>, dim3(grid1d(total)), dim3(256), 0, stream, Z, gx, d->Cin, d->B, d->H,
                         d->W, d->OH, d->OW, d->KH, d->KW, d->stride, d->pad, rep, dv);
    return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  if (d->transposed) {
    // dX of ConvT = plain zero-padded conv of gy with W viewed [Cin][Cout][KH][KW]
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->H, d->W, d->KW, d->stride, d->pad, kZero};
    p.y = gx;
    p.ohw = d->H * d->W;
    return dispatch_conv(p, pre, packed, slab, stream) == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  // dX of conv = transposed gather of gy over the padded input frame.  Padded convs split the
  // frame in the epilogue (OutMap s = -1): interior -> gx, ring -> ring buffer (replication) or
  // dropped (zero padding); ring_fold_kernel then adds the ring onto the edge pixels.
  const int Hp = d->H + 2 * d->pad, Wp = d->W + 2 * d->pad;
  if (pack_x3(d, GANAMD_CONV_DGRAD) &&
      patch_geometry(M, Ck, d->B, d->H, d->W, d->KH, d->stride, d->pad, d->OH, d->OW, d->math, d->kernel_off, true)) {
    // the frame's interior with the split6 patch conv (zero-padded, taps reversed), then -- for
    // replication padding -- the ring alone through the gather GEMM (OutMap s = -2) and its fold
    const int bmp = conv_bm(M), mpad = (M + bmp - 1) / bmp * bmp;
    p.Ckp = (Ck + BK - 1) / BK * BK;
    if (!pre) {
      launch_pack(pack_job(d, GANAMD_CONV_DGRAD, w, packed), stream);
      p.w = packed;
    }
    p.w_bytes = 4 * mpad * T * p.Ckp;
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->H, d->W, d->KW, 1, d->pad, kZero};
    p.y = gx;
    p.N = d->B * d->H * d->W;
    p.ohw = d->H * d->W;
    p.ldy = p.N;
    if (ganamd_patch::launch(patch_args(p, p.w, mpad, d->KH, true), stream) != hipSuccess) return GANAMD_ELAUNCH;
    if (!pad_bytes) return GANAMD_OK;
    float* ring = reinterpret_cast<float*>(ws);
    const int Rn = Hp * Wp - d->H * d->W;
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, Hp, Wp, d->KW, d->stride, 0, kTransposed};
    p.N = d->B * Rn;
    p.ohw = Rn;
    p.om = OutMap{-2, d->pad, d->H, Wp, Hp * Wp, d->W, d->H * d->W, Rn, (long)d->B * Rn, ring};
    p.ldy = p.N;
    p.y = ring;
    if (dispatch_conv(p, true, nullptr, slab, stream) != hipSuccess) return GANAMD_ELAUNCH;
    const long planes = (long)d->Cin * d->B;
    const long edges = (long)2 * d->W + 2 * d->H;
    hipLaunchKernelGGL(ring_fold_kernel, dim3(grid1d(planes * edges)), dim3(256), 0, stream, ring, gx, (int)planes,
                       d->H, d->W, d->pad);
    return hipGetLastError() == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH;
  }
  float* ring = pad_bytes ? reinterpret_cast<float*>(ws) : nullptr;
  const int Rn = Hp * Wp - d->H * d->W;
  p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, Hp, Wp, d->KW, d->stride, 0, kTransposed};
  p.y = gx;
  p.ohw = Hp * Wp;
  if (d->pad > 0) {
    p.om = OutMap{-1, d->pad, d->H, Wp, Hp * Wp, d->W, d->H * d->W, Rn, (long)d->B * Rn, ring};
    p.ldy = (long)d->B * d->H * d->W;
  }
  if (dispatch_conv(p, pre, packed, slab, stream) != hipSuccess) return GANAMD_ELAUNCH;
  if (ring) {
    const long planes = (long)d->Cin * d->B;
    const long edges = (long)2 * d->W + 2 * d->H;
    hipLaunchKernelGGL(ring_fold_kernel, dim3(grid1d(planes * edges)), dim3(256), 0, stream, ring, gx, (int)planes,
                       d->H, d->W, d->pad);
    if (hipGetLastError() != hipSuccess) return GANAMD_ELAUNCH;
  }
  return GANAMD_OK;
}

static WgradArgs wgrad_args(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x_scale,
                            const float* gy_scale, float alpha, float* gw, int accumulate) {
  const int T = d->KH * d->KW;
  WgradArgs p{};
  p.alpha = alpha;
  p.ot = 1;
  p.bf16 = d->math == GANAMD_MATH_BF16;
  if (d->transposed) {
    // dW[ci][co][t] = sum_n x[ci][n] * gy[co][conv-gather_t(n)]
    p.a = x;
    p.ascale = x_scale;
    p.lda = d->B * d->H * d->W;
    p.a_bytes = 4 * d->Cin * p.lda;
    p.M = d->Cin;
    p.J = d->Cout;
    p.K = d->B * d->H * d->W;
    p.ohw = d->H * d->W;
    p.g = Gather{gy, gy_scale, d->Cout, d->B, d->OH, d->OW, d->H, d->W, d->KW, d->stride, d->pad, kZero};
    p.om = d->Cout * T;
    p.oj = T;
  } else {
    // dW[co][ci][t] = sum_n gy[co][n] * x[ci][gather_t(n)]
    p.a = gy;
    p.ascale = gy_scale;
    p.lda = d->B * d->OH * d->OW;
    p.a_bytes = 4 * d->Cout * p.lda;
    p.M = d->Cout;
    p.J = d->Cin;
    p.K = d->B * d->OH * d->OW;
    p.ohw = d->OH * d->OW;
    p.g = Gather{x, x_scale, d->Cin, d->B, d->H, d->W, d->OH, d->OW, d->KW, d->stride, d->pad,
                 d->pad_mode == GANAMD_PAD_REPLICATE ? kReplicate : kZero};
    p.om = d->Cin * T;
    p.oj = T;
  }
  p.out = gw;
  p.out_numel = d->Cin * d->Cout * T;
  p.accumulate = accumulate;
  return p;
}

static int wgrad_row(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x_scale,
                     const float* gy_scale, const float* x2, const float* gy2, float alpha, float* gw, int accumulate,
                     void* workspace, hipStream_t stream) {
  ganamd_wrow::Args a{};
  a.a = gy;
  a.ascale = gy_scale;
  a.x = x;
  a.xscale = x_scale;
  a.a2 = gy2;
  a.x2 = x2;
  a.M = d->Cout;
  a.J = d->Cin;
  a.B = d->B;
  a.H = d->H;
  a.W = d->W;
  a.KK = d->KH;
  a.replicate = d->pad_mode == GANAMD_PAD_REPLICATE;
  a.alpha = alpha;
  a.out = gw;
  a.accumulate = accumulate;
  ganamd_wrow::plan(a.M, a.J, a.B, a.H, a.W, a.KK, gy2 ? 2 : 1, num_cus(), &a.splits, &a.ks_per_split);
  a.slab = a.splits > 1 ? static_cast<float*>(workspace) : nullptr;
  if (a.splits > 1 && !a.slab) return GANAMD_EINVAL;
  if (ganamd_wrow::launch(a, stream) != hipSuccess) return GANAMD_ELAUNCH;
  if (a.splits > 1) {
    const int numel = d->Cout * d->Cin * d->KH * d->KW;
    if (numel % 4 == 0 && aligned16(a.slab) && aligned16(gw))
      hipLaunchKernelGGL(wgrad_split_reduce_kernel<true>, dim3(grid1d(numel / 4)), dim3(256), 0, stream, a.slab,
                         a.splits, numel, gw, accumulate);
    else
      hipLaunchKernelGGL(wgrad_split_reduce_kernel<false>, dim3(grid1d(numel)), dim3(256), 0, stream, a.slab,
                         a.splits, numel, gw, accumulate);
    if (hipGetLastError() != hipSuccess) return GANAMD_ELAUNCH;
  }
  return GANAMD_OK;
}

int ganamd_conv_wgrad(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x_scale,
                      const float* gy_scale, float alpha, float* gw, int accumulate, void* workspace,
                      size_t workspace_bytes, hipStream_t stream) {
  if (!desc_ok(d) || !x || !gy || !gw) return GANAMD_EINVAL;
  if ((x_scale == nullptr) != (gy_scale == nullptr)) return GANAMD_EINVAL;
  if (ws_check(d, GANAMD_CONV_WGRAD, workspace, workspace_bytes) != GANAMD_OK) return GANAMD_EINVAL;
  if (wrow_ok(d))
    return wgrad_row(d, x, gy, x_scale, gy_scale, nullptr, nullptr, alpha, gw, accumulate, workspace, stream);
  const WgradArgs p = wgrad_args(d, x, gy, x_scale, gy_scale, alpha, gw, accumulate);
  return dispatch_wgrad(p, d->KH * d->KW, static_cast<float*>(workspace), stream) == hipSuccess ? GANAMD_OK
                                                                                                : GANAMD_ELAUNCH;
}

int ganamd_conv_wgrad2(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x2, const float* gy2,
                       float alpha, float* gw, int accumulate, void* workspace, size_t workspace_bytes,
                       hipStream_t stream) {
  if (!desc_ok(d) || !x || !gy || !x2 || !gy2 || !gw) return GANAMD_EINVAL;
  if (ws_check(d, GANAMD_CONV_WGRAD, workspace, workspace_bytes) != GANAMD_OK) return GANAMD_EINVAL;
  if (wrow_ok(d)) return wgrad_row(d, x, gy, nullptr, nullptr, x2, gy2, alpha, gw, accumulate, workspace, stream);
  WgradArgs p = wgrad_args(d, x, gy, nullptr, nullptr, alpha, gw, accumulate);
  if (d->transposed || p.K % BKW != 0 || (long)2 * p.K >= (1L << 31) / 4) {   // two launches instead
    int rc = ganamd_conv_wgrad(d, x, gy, nullptr, nullptr, alpha, gw, accumulate, workspace, workspace_bytes, stream);
    return rc != GANAMD_OK ? rc
                           : ganamd_conv_wgrad(d, x2, gy2, nullptr, nullptr, alpha, gw, 1, workspace, workspace_bytes,
                                               stream);
  }
  p.segK = p.K;
  p.K *= 2;
  p.a2 = gy2;
  p.src2 = x2;
  return dispatch_wgrad(p, d->KH * d->KW, static_cast<float*>(workspace), stream) == hipSuccess ? GANAMD_OK
                                                                                                : GANAMD_ELAUNCH;
}

}  // extern "C"
