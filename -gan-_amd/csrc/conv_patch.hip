// LDS-patch convolution on the split6 pipe: stride 1, "same" padding, K x K taps (K = 3, 5),
// maps 32 / 64 wide -- the generator's modulated convs at 32x32 / 64x64 (48- and 96-channel,
// generator_13_5.py:219-248 in the batch-shared form) and their input gradients.
//
// Why not the gather GEMM (conv_gemm.hip conv_body_x3) for these: the implicit GEMM gathers its B
// operand per K-step, so every input element is fetched, scaled by its modulation s[c][b], split
// into three bf16 planes (h, m, l) and written to LDS once per TAP -- 25 times for a 5x5 conv.  At
// 48 output channels that staging work per MFMA exceeds what the VALU can hide behind the matrix
// cores (each element feeds only 48 rows), and the halo is re-fetched from L2/HBM per tap (PMC:
// 2.06x the algorithmic bytes on the 96-channel 5x5).  Here a block stages its input PATCH -- the
// (TH + K - 1) x (W + K - 1) positions around its TH output rows, 16 channels, already scaled and
// split into the three planes -- once per 16-channel chunk, and runs all K*K taps on it: tap
// (kh, kw)'s B fragment of pixel (i, j) is patch position (i + kh, j + kw).  Staging work and halo
// traffic drop K*K-fold; what is left per tap is the MFMA work and LDS fragment reads.
//
// A operand: the packed weights pre-split into three bf16 planes by the pack kernels (the optimizer
// refreshes them with the fp32 copy, conv_gemm.hip pack_x3), read straight from global memory into
// each wave's registers one tap ahead (the same few hundred KB for every block: L1/L2 resident).
// No LDS stage and no barrier per tap: a block synchronises once per chunk, when its double-
// buffered patch swaps; the next chunk's patch is fetched into registers during the first tap and
// written to the idle buffer a few taps later.
//
// fp32 products on the bf16 matrix cores (split6, as conv_gemm.hip): x = h + m + l exactly, the six
// products with a high part per 16 k -- 32x32 blocks: six v_mfma_f32_32x32x16_bf16; 16-row blocks
// (48 rows): three full-rate v_mfma_f32_16x16x32_bf16 on pairs of products.
//
// Block: NW waves, NPIX pixels (whole rows) of ONE image, all BM (<= 96) output channels of a row
// tile; wave w owns pixels [w * NPIX / NW, (w + 1) * NPIX / NW) of all rows -- or, 96-row blocks at
// W = 64 (12 waves), rows 32 (w % 3) .. +31 of pixels 128 (w / 3) .. +127.  W = 64: 512 pixels, 8 waves;
// W = 32: 256 pixels, 4 waves.  LDS: 2 x 3 planes x positions x 16 channels x 2 B (W = 64, K = 5:
// 153 KiB) -- one block per CU.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "patch.h"

namespace ganamd_patch {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kOOB = (int)0x80000000;
constexpr int kMaxScale = 1024;   // input channels whose scales the block stages in LDS

// instance shapes (compile-time; tools/build_variant.sh A/B builds override them)
#ifndef GANAMD_P96_NW
#define GANAMD_P96_NW 12          // waves of a 96-row block at W = 64
#endif
#ifndef GANAMD_P96_MB
#define GANAMD_P96_MB 16          // MFMA block edge of the 96-row 5x5 blocks at W = 64 (16: paired 16x16x32)
#endif
#ifndef GANAMD_P48_NW
#define GANAMD_P48_NW 8           // waves of a 48-row block at W = 64
#endif
#ifndef GANAMD_P_UNROLL4
#define GANAMD_P_UNROLL4 1        // fully unroll the tap loop of the 4-wave 5x5 blocks (3x3: a loop of tap pairs)
#endif
#ifndef GANAMD_P16_ADUP
#define GANAMD_P16_ADUP 0         // 16x16 paths: pair-low lanes load h for X2 too (no select; +1/3 weight bytes)
#endif
#ifndef GANAMD_P64
#define GANAMD_P64 1              // a 64-row tile for 48 < M <= 64 (else the 96-row one, a third empty)
#endif
#ifndef GANAMD_P128
#define GANAMD_P128 0             // a 128-row tile for 96 < M <= 128 (else the gather GEMM takes the conv)
#endif
#ifndef GANAMD_P32_TALL
#define GANAMD_P32_TALL 1         // W = 32 on large grids: 16-row (512-pixel) blocks, the W = 64 wave layouts
#endif
#ifndef GANAMD_P64_NW
#define GANAMD_P64_NW 8           // waves of a 64-row block at W = 64 (8: 2 along M x 4 along pixels)
#endif

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
// buffer loads: an out-of-range offset returns 0 in hardware (padding / tails are a select of the
// offset, never a branch around the load)
__device__ __forceinline__ float bload(rsrc_t r, int off) {
  asm("" : "+v"(off));
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ bf16x8 bload8h(rsrc_t r, int off) {   // 8 bf16 (16 bytes)
  asm("" : "+v"(off));
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// exact 3-way split x = h + m + l (RNE; both differences are exact in fp32)
__device__ __forceinline__ void split4(const f32x4& x, bf16x4& h, bf16x4& m, bf16x4& l) {
  float r[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (__bf16)x[e];
    r[e] = x[e] - (float)h[e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    m[e] = (__bf16)r[e];
    r[e] -= (float)m[e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) l[e] = (__bf16)r[e];
}

// element offset of 8-channel half `half` of patch position `pos` in one plane: 32-byte rows.  The
// ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) see 16 consecutive positions:
// 32x32 fragments (all lanes of a group on one half) need the two 16-byte halves swapped on odd
// 8-position groups; 16x16 fragments (lanes 16-31 on the other half of lanes 0-15's positions) need
// the plain layout -- each is conflict-free at any start position, the other one 2-way.
template <int MB>
__device__ __forceinline__ int poff(int pos, int half) {
  return MB == 32 ? pos * 16 + 8 * (half ^ ((pos >> 3) & 1)) : pos * 16 + 8 * half;
}

template <int MB>
__device__ __forceinline__ int mfma_row(int lane, int r) {
  return MB == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : 4 * (lane >> 4) + r;
}

template <int BM, int NW, int NPIX, int KK, int TW, bool BSCALE, bool DGRAD>
__global__ __launch_bounds__(64 * NW) void conv_patch_x3_kernel(Args p) {
  constexpr int NT = 64 * NW;
  constexpr int MB = (BM % 32 == 0) ? ((BM == 96 && NPIX == 512 && KK == 5) ? GANAMD_P96_MB : 32) : 16;   // MFMA block edge (48 rows: 16)
  // waves along M: blocks of 4 waves per 32 rows (the 12-wave 96-row and 8-wave 64-row blocks) give
  // each wave 32 rows x 128 pixels (a third / half of the weight fragments per wave, 3 / 2 waves per
  // SIMD); the 8-wave 96-row block on 16x16 fragments gives each wave 48 rows x 128 pixels (2 waves
  // per SIMD); otherwise every wave owns all rows
  constexpr int WM = (MB == 32 && NW % 4 == 0 && BM % (32 * (NW / 4)) == 0) ? NW / 4
                     : (MB == 16 && BM == 96 && NW == 8) ? 2 : 1,
                WN = NW / WM;
  constexpr int NA = MB == 32 ? 3 : 2;                      // A fragment registers per row block
  constexpr int PW = NPIX / WN;                             // pixels per wave
  constexpr int TM = BM / (MB * WM), TN = PW / MB, NR = MB == 32 ? 16 : 4;
  using acc_t = typename std::conditional<MB == 32, f32x16, f32x4>::type;
  constexpr int TH = NPIX / TW, PAD = (KK - 1) / 2, T = KK * KK;
  constexpr int PWD = TW + KK - 1, NPOS = (TH + KK - 1) * PWD;
  constexpr int PS = NPOS * 16;                             // plane stride (bf16 elements)
  constexpr int BUF = 3 * PS;
  constexpr int NU = NPOS * 4, UPT = (NU + NT - 1) / NT;    // staging units: 4 channels at one position
  constexpr int kStoreTap = T > 4 ? 3 : T - 1;
  static_assert(TN >= 1 && TM * MB * WM == BM && TN * MB == PW && WM * WN == NW, "tile");
  __shared__ __attribute__((aligned(16))) unsigned short Ps[2 * BUF];
  // the block's modulation scales s[c][b] (one image per block: one value per input channel),
  // staged once so the patch stores read them from LDS -- a global load there would make every
  // store wait for all of the wave's loads in flight (vmcnt is in order)
  __shared__ __attribute__((aligned(16))) float Ssc[BSCALE ? kMaxScale : 4];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wrow = (wv % WM) * TM * MB, wcol = (wv / WM) * PW;   // this wave's rows / pixels
  const int H = p.H, HW = H * TW;
  const int gy = (p.M + BM - 1) / BM;
  // XCD-aware order: blocks b and b + 8 land on one XCD (round-robin dispatch), so block b takes
  // tile (b % 8) * (nb / 8) + b / 8 -- each XCD runs a contiguous range of row tiles and adjacent
  // tiles' halo rows are fetched from HBM once into that XCD's L2 (PMC: 1.33x -> see DESIGN §3)
  int bid = blockIdx.x;
  if ((gridDim.x & 7) == 0) bid = (bid & 7) * (int)(gridDim.x >> 3) + (bid >> 3);
  const int ty = bid % gy, reg = bid / gy;
  const int tiles_img = H / TH;
  const int b = reg / tiles_img, oh0 = (reg - b * tiles_img) * TH;
  const int m0 = ty * BM;
  const int nct = p.Ckp / 16;

  const rsrc_t rw = make_rsrc(p.w, p.w_bytes);
  const rsrc_t rx = make_rsrc(p.src, 4 * p.C * p.B * HW);
  const rsrc_t rsc = make_rsrc(BSCALE ? p.scale : p.src, BSCALE ? 4 * p.C * p.B : 0);
  const unsigned cs4 = 4u * (unsigned)(p.B * HW);           // one channel row of the source

  // ---- patch staging: unit u = (channel group cg of 4, position pos), pos fastest (consecutive
  // lanes read consecutive columns).  u is opaque so its index math is redone per chunk.
  auto patch_load = [&](int cc, f32x4 (&pv)[UPT]) {
#pragma unroll
    for (int e = 0; e < UPT; ++e) {
      int u = min(tid + e * NT, NU - 1);
      asm volatile("" : "+v"(u));
      const int cg = u / NPOS, pos = u - cg * NPOS;
      const int pr = pos / PWD, pc = pos - pr * PWD;
      int ih = oh0 - PAD + pr, iw = pc - PAD;
      bool in = true;
      if constexpr (DGRAD) {
        in = ih >= 0 && ih < H && iw >= 0 && iw < TW;
      } else {
        ih = min(max(ih, 0), H - 1);
        iw = min(max(iw, 0), TW - 1);
      }
      // channels past the source's end fall outside the buffer: the hardware returns 0
      const unsigned off = 4u * (unsigned)(b * HW + ih * TW + iw) + (unsigned)(cc * 16 + 4 * cg) * cs4;
#pragma unroll
      for (int q = 0; q < 4; ++q) pv[e][q] = bload(rx, in ? (int)(off + q * cs4) : kOOB);
    }
  };
  auto patch_store = [&](unsigned short* P, int cc, const f32x4 (&pv)[UPT]) {
#pragma unroll
    for (int e = 0; e < UPT; ++e) {
      int u = min(tid + e * NT, NU - 1);
      asm volatile("" : "+v"(u));
      const int cg = u / NPOS, pos = u - cg * NPOS;
      f32x4 v = pv[e];
      if constexpr (BSCALE) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(&Ssc[cc * 16 + 4 * cg]);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] *= sc[q];
      }
      bf16x4 h, m, l;
      split4(v, h, m, l);
      const int o = poff<MB>(pos, cg >> 1) + 4 * (cg & 1);
      *reinterpret_cast<bf16x4*>(&P[o]) = h;
      *reinterpret_cast<bf16x4*>(&P[PS + o]) = m;
      *reinterpret_cast<bf16x4*>(&P[2 * PS + o]) = l;
    }
  };

  // ---- A fragments of one tap from global memory (pre-split planes).  32x32: lane (r, h) holds
  // rows m0 + 32i + r, k = 8h .. 8h+7 of the three planes.  16x16 paired (lane (r, q): k-half
  // hf = q & 1 of the 16 channels, pair half hi = q >> 1): two fragments, X1 = (h|m) and X2 = (h|l)
  // -- lanes with hi = 0 hold h in both, so they load it once (load 0) and their second load is an
  // out-of-range offset (no memory traffic, hardware zero) that the product step replaces by load 0:
  // 1.5 planes of weight bytes per 16 rows, the 32x32 form's 3 planes per 32 rows.
  const int fr = MB == 32 ? (lane & 31) : (lane & 15);
  const int fhalf = MB == 32 ? (lane >> 5) : ((lane >> 4) & 1);
  const int fhi = MB == 32 ? 0 : (lane >> 5);
  int a_row[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) a_row[i] = 2 * (((m0 + wrow + i * MB + fr) * nct * T) * 16 + 8 * fhalf);   // bytes
  const int wpb = 2 * p.wplane;                             // plane stride in bytes
  auto a_load = [&](int kt, bf16x8 (&fa)[TM][NA]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int o = a_row[i] + kt * 32;
      if constexpr (MB == 32) {
        fa[i][0] = bload8h(rw, o);
        fa[i][1] = bload8h(rw, o + wpb);
        fa[i][2] = bload8h(rw, o + 2 * wpb);
      } else {
        fa[i][0] = bload8h(rw, o + (fhi ? wpb : 0));              // h | m
        if constexpr (GANAMD_P16_ADUP)
          fa[i][1] = bload8h(rw, o + (fhi ? 2 * wpb : 0));        // h | l
        else
          fa[i][1] = bload8h(rw, fhi ? o + 2 * wpb : kOOB);       // - | l
      }
    }
  };

  // patch position of each of this lane's B columns at tap (0, 0)
  int posb[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int q = wcol + j * MB + fr;
    posb[j] = (q / TW) * PWD + q % TW;
  }
  // the three B fragments of column block j at tap offset toff: the planes h, m, l (32x32); for the
  // paired 16x16 products Y1 = (h|h), Y2 = (m|m), Y3 = (l|h) -- the third read takes its plane from
  // a per-lane offset (pair-high lanes read h again), so the product step needs no select: one
  // v_cndmask per dword per column block per tap would cost more issue slots than the 16x16x32
  // MFMAs leave free (8 of their 16 cycles)
  // (16x16: the plain layout is linear in the position, so each column block's lane address is a
  // per-lane byte base plus the tap's uniform offset -- one address add per read group)
  const int pl3 = MB == 32 ? 2 * PS : (fhi ? 0 : 2 * PS);
  int pbyte[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) pbyte[j] = 2 * poff<MB>(posb[j], fhalf);
  auto b_frag = [&](const unsigned short* P, int toff, int j, bf16x8 (&f)[3]) {
    if constexpr (MB == 16) {
      const char* q = reinterpret_cast<const char*>(P) + toff * 32 + pbyte[j];
      f[0] = *reinterpret_cast<const bf16x8*>(q);
      f[1] = *reinterpret_cast<const bf16x8*>(q + 2 * PS);
      f[2] = *reinterpret_cast<const bf16x8*>(q + 2 * pl3);
    } else {
      const int o = poff<MB>(posb[j] + toff, fhalf);
      f[0] = *reinterpret_cast<const bf16x8*>(&P[o]);
      f[1] = *reinterpret_cast<const bf16x8*>(&P[PS + o]);
      f[2] = *reinterpret_cast<const bf16x8*>(&P[pl3 + o]);
    }
  };

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;

  // the products of column block j (B fragments fb) with all of the wave's row blocks
  auto mfma_j = [&](const bf16x8 (&fa)[TM][NA], const bf16x8 (&fb)[3], int j) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (MB == 32) {
        // l*h, h*l, m*m, m*h, h*m, h*h: smallest first into the same accumulator
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], acc[i][j], 0, 0, 0);
      } else {
        // X2 x Y3 = (h|l)x(l|h) = hl + lh, X1 x Y2 = (h|m)x(m|m) = hm + mm, X1 x Y1 = (h|m)x(h|h) =
        // hh + mh -- smallest first; lanes q < 2 carry the first 16-k half of the 32, q >= 2 the
        // second (the same 16 channels)
        const bf16x8 x2 = GANAMD_P16_ADUP ? fa[i][1] : fhi ? fa[i][1] : fa[i][0];
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, fb[2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[0], acc[i][j], 0, 0, 0);
      }
    }
  };

  // prologue: the block's scales, chunk 0's patch and tap 0's A fragments
  bf16x8 fa[2][TM][NA];
  {
    f32x4 pv[UPT];
    patch_load(0, pv);
    a_load(DGRAD ? T - 1 : 0, fa[0]);
    if constexpr (BSCALE) {
      for (int c = tid; c < p.Ckp; c += NT) Ssc[c] = bload(rsc, 4 * (c * p.B + b));   // Ckp <= kMaxScale (launch)
      __syncthreads();
    }
    patch_store(Ps, 0, pv);
  }
  __syncthreads();
  for (int cc = 0; cc < nct; ++cc) {
    const unsigned short* P = Ps + (cc & 1) * BUF;
    const bool more = cc + 1 < nct;
    f32x4 pv[UPT];
    int kh = 0, kw = 0;
    // B fragments rotate one column block ahead: block j + 1's (or the next tap's block 0) reads are
    // issued before block j's products, so each read has a block of products to arrive under instead
    // of exposing its latency right before the product that needs it.  After the chunk's last tap
    // the look-ahead re-reads position 0 (a dummy: the next chunk's patch is behind the barrier).
    bf16x8 cur[3];
    b_frag(P, 0, 0, cur);
    auto tap_pair = [&](int t) {
      // two taps per iteration: register double buffer fa[0] / fa[1] without dynamic indexing
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int tt = t + u;
        if (tt < T) {
          const int kt = cc * T + tt;
          const int toff = kh * PWD + kw;
          const int tnext = tt + 1 == T ? -posb[0] : (kw + 1 == KK ? toff + PWD - (KK - 1) : toff + 1);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            bf16x8 nxt[3];
            if (j + 1 < TN)
              b_frag(P, toff, j + 1, nxt);
            else
              b_frag(P, tnext, 0, nxt);
            __builtin_amdgcn_sched_barrier(0);   // keep the look-ahead reads ahead of the products
            mfma_j(fa[u], cur, j);
#pragma unroll
            for (int q = 0; q < 3; ++q) cur[q] = nxt[q];
          }
          // loads AFTER the products are issued: the wait for this tap's weights (above) then
          // never covers the loads of the next tap or chunk (vmcnt counts in order), and they
          // overlap the products all the same
          if (kt + 1 < nct * T) {                               // the next tap's weights
            const int nt = (tt + 1 == T) ? 0 : tt + 1, nc = (tt + 1 == T) ? cc + 1 : cc;
            a_load(nc * T + (DGRAD ? T - 1 - nt : nt), fa[u ^ 1]);
          }
          if (tt == 0 && more) patch_load(cc + 1, pv);          // the next chunk's patch
          // the idle buffer (last read in chunk cc - 1), a few taps after its loads were issued
          if (tt == kStoreTap && more) patch_store(Ps + ((cc + 1) & 1) * BUF, cc + 1, pv);
          if (++kw == KK) {
            kw = 0;
            ++kh;
          }
        }
      }
      if (T % 2 == 1 && t + 2 > T) {
        // odd tap count: the last tap used fa[0] and prefetched into fa[1]; realign
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < NA; ++q) fa[0][i][q] = fa[1][i][q];
      }
    };
    // the tap loop: fully unrolled where the registers allow it (48-row blocks, the 4-wave W = 32
    // 5x5 blocks: the taps' index math, weight prefetch and patch stores resolve at compile time and
    // the next tap's fragment reads can be scheduled under the current tap's products); the 12-wave
    // 96-row blocks spill when unrolled (or with the first taps peeled) and keep a loop of two taps,
    // and so do the 4-wave 3x3 blocks (measured: 96->96 3x3 at 32x32, B = 256, 117 -> 151 TF/s as a
    // loop; profiles/r05_ab_patch.txt)
    if constexpr (BM == 48 || (NW == 4 && KK == 5 && GANAMD_P_UNROLL4)) {
#pragma unroll
      for (int t = 0; t < T; t += 2) tap_pair(t);
    } else {
#pragma unroll 1
      for (int t = 0; t < T; t += 2) tap_pair(t);
    }
    if (more) __syncthreads();       // chunk cc + 1's patch is complete; chunk cc's buffer is free
  }

  // epilogue
  const long n_img = (long)b * HW + (long)oh0 * TW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int q = wcol + j * MB + (lane & (MB - 1));
    const long col = n_img + (q / TW) * TW + q % TW;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int m = m0 + wrow + i * MB + mfma_row<MB>(lane, r);
        if (m >= p.M) continue;
        float v = p.alpha * acc[i][j][r];
        if (p.oscale) v *= p.oscale[m * p.B + b];
        if (p.bias) v += p.bias[m];
        if (p.noise) v += p.noise_scale[m] * p.noise[(long)m * p.ldy + col];
        if (p.act) v = v > 0.f ? v : p.act[m] * v;
        p.y[(long)m * p.ldy + col] = v;
      }
    }
  }
}

template <int BM, int NW, int NPIX, int KK, int TW, bool BSCALE, bool DGRAD>
int occ_of() {
  static const int v = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv_patch_x3_kernel<BM, NW, NPIX, KK, TW, BSCALE, DGRAD>,
                                                     64 * NW, 0) != hipSuccess || n <= 0)
      n = 1;
    return n;
  }();
  return v;
}

// instance selection: W = 64 -> 512 pixels (8 rows) / 8-12 waves; W = 32 on large grids -> 512 pixels
// (16 rows) with the same waves; W = 32 otherwise -> 256 pixels / 4 waves
template <int BM, int KK>
constexpr int nw512() {
  return BM == 128 ? 8 : BM == 96 ? ((GANAMD_P96_MB == 16 && KK == 5) ? 8 : GANAMD_P96_NW)
                   : BM == 64 ? GANAMD_P64_NW : GANAMD_P48_NW;
}
template <int BM, int KK, bool BSCALE, bool DGRAD>
hipError_t go(const Args& a, hipStream_t st, bool dry, int* occ) {
  constexpr int NW = nw512<BM, KK>();
  if (a.W == 64) {
    if (occ) *occ = occ_of<BM, NW, 512, KK, 64, BSCALE, DGRAD>();
    if (!dry)
      hipLaunchKernelGGL((conv_patch_x3_kernel<BM, NW, 512, KK, 64, BSCALE, DGRAD>), dim3((unsigned)blocks(a)),
                         dim3(64 * NW), 0, st, a);
  } else if (block_pixels(a.W, a.B, a.H) == 512) {
    if (occ) *occ = occ_of<BM, NW, 512, KK, 32, BSCALE, DGRAD>();
    if (!dry)
      hipLaunchKernelGGL((conv_patch_x3_kernel<BM, NW, 512, KK, 32, BSCALE, DGRAD>), dim3((unsigned)blocks(a)),
                         dim3(64 * NW), 0, st, a);
  } else {
    constexpr int NW = BM == 128 ? 8 : 4;     // 128 rows: 2 waves along M x 4 along pixels
    if (occ) *occ = occ_of<BM, NW, 256, KK, 32, BSCALE, DGRAD>();
    if (!dry)
      hipLaunchKernelGGL((conv_patch_x3_kernel<BM, NW, 256, KK, 32, BSCALE, DGRAD>), dim3((unsigned)blocks(a)),
                         dim3(64 * NW), 0, st, a);
  }
  return dry ? hipSuccess : hipGetLastError();
}

template <int BM, int KK>
hipError_t go_k(const Args& a, hipStream_t st, bool dry, int* occ) {
  const bool s = a.scale != nullptr;
  if (a.dgrad) return s ? go<BM, KK, true, true>(a, st, dry, occ) : go<BM, KK, false, true>(a, st, dry, occ);
  return s ? go<BM, KK, true, false>(a, st, dry, occ) : go<BM, KK, false, false>(a, st, dry, occ);
}

hipError_t dispatch(const Args& a, hipStream_t st, bool dry, int* occ) {
  const int bm = row_tile(a.M);
  if (bm == 48) return a.KK == 3 ? go_k<48, 3>(a, st, dry, occ) : go_k<48, 5>(a, st, dry, occ);
  if (bm == 96) return a.KK == 3 ? go_k<96, 3>(a, st, dry, occ) : go_k<96, 5>(a, st, dry, occ);
#if GANAMD_P64
  if (bm == 64) return a.KK == 3 ? go_k<64, 3>(a, st, dry, occ) : go_k<64, 5>(a, st, dry, occ);
#endif
#if GANAMD_P128
  if (bm == 128) return a.KK == 3 ? go_k<128, 3>(a, st, dry, occ) : go_k<128, 5>(a, st, dry, occ);
#endif
  return hipErrorInvalidValue;
}

}  // namespace

int row_tile(int M) {
  return M <= 0 ? 0 : M <= 48 ? 48 : (GANAMD_P64 && M <= 64) ? 64 : M <= 96 ? 96 : (GANAMD_P128 && M <= 128) ? 128 : 0;
}

// W = 32: 16-row blocks when the grid still has two rounds of them (B * H / 16 >= 512: the fake
// batches' 256-sample forward), else 8-row blocks
int block_pixels(int W, int B, int H) {
  return W == 64 ? 512 : W == 32 ? ((GANAMD_P32_TALL && H % 16 == 0 && (long)B * H / 16 >= 512) ? 512 : 256) : 0;
}

bool domain(int M, int H, int W, int K, int stride, int pad, int OH, int OW) {
  if (stride != 1 || (K != 3 && K != 5) || pad != (K - 1) / 2 || OH != H || OW != W || (W != 32 && W != 64))
    return false;
  return row_tile(M) != 0 && H % (block_pixels(W, 1, H) / W) == 0;
}

long blocks(const Args& a) {
  const int bm = row_tile(a.M), th = block_pixels(a.W, a.B, a.H) / a.W;
  return (long)((a.M + bm - 1) / bm) * a.B * (a.H / th);
}

int occupancy(const Args& a) {
  int occ = 1;
  (void)dispatch(a, nullptr, true, &occ);
  return occ;
}

hipError_t launch(const Args& a, hipStream_t st) {
  if (!domain(a.M, a.H, a.W, a.KK, 1, (a.KK - 1) / 2, a.H, a.W) || !a.w || !a.src || !a.y ||
      (a.scale && a.Ckp > kMaxScale))
    return hipErrorInvalidValue;
  return dispatch(a, st, false, nullptr);
}

}  // namespace ganamd_patch
