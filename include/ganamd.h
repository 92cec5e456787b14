/*
 * ganamd.h — C ABI of the MI355X-native WGAN-GP hot path (G13_5 + D9_4), libganamd.so.
 *
 * The reference has no FFI: its hot path sits behind PyTorch's nn.Module + autograd protocol
 * (SURVEY.md §8(b)).  Each entry point below replaces the ATen kernel(s) that the reference's
 * modules reach through that protocol; the file:line of the reference call site is cited per
 * function.  The drop-in Python modules (-gan-_amd/) call these through ctypes.
 *
 * Conventions
 *   - Activations are fp32 in CNHW layout ("channel rows"): x[c][b][h][w], row length
 *     L = B*H*W.  A vector indexed by (channel, sample), e.g. a style or a demodulation
 *     coefficient, is stored [C][B].
 *   - All pointers are device pointers; every call is asynchronous on `stream` and performs no
 *     allocation and no host synchronisation (safe under hipGraph stream capture).
 *   - Scratch memory is caller-provided; query its size with the *_workspace functions.
 *   - Return 0 (GANAMD_OK) or a negative error code.  No exceptions cross the ABI.
 *   - Stateless: calls on distinct streams may run concurrently from several threads.
 */
#ifndef GANAMD_H
#define GANAMD_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GANAMD_OK 0
#define GANAMD_EINVAL (-1)
#define GANAMD_ELAUNCH (-2)

#define GANAMD_PAD_ZERO 0
#define GANAMD_PAD_REPLICATE 1

/* Arithmetic of the conv GEMMs: fp32 MFMA (exact fp32 products, the default), or operands
 * rounded to bf16 (RNE) with fp32 accumulation and fp32 storage (the bf16 configuration). */
#define GANAMD_MATH_F32 0
#define GANAMD_MATH_BF16 1

#define GANAMD_CONV_FWD 0
#define GANAMD_CONV_DGRAD 1
#define GANAMD_CONV_WGRAD 2

/* Geometry of one convolution.  For transposed=0 the weight is [Cout][Cin][KH][KW] and
 * OH = (H + 2*pad - KH)/stride + 1.  For transposed=1 (nn.ConvTranspose2d semantics, zero
 * padding) the weight is [Cin][Cout][KH][KW] and OH = (H-1)*stride - 2*pad + KH.  A linear
 * layer is the case H = W = OH = OW = KH = KW = 1. */
typedef struct ganamd_conv_desc {
  int32_t B, Cin, H, W;
  int32_t Cout, OH, OW;
  int32_t KH, KW, stride, pad;
  int32_t pad_mode;   /* GANAMD_PAD_ZERO | GANAMD_PAD_REPLICATE (ignored when transposed) */
  int32_t transposed;
  int32_t packed_w;   /* 1: the w argument of conv_fwd/conv_dgrad is already in GEMM order
                         (ganamd_conv_pack for the same op and geometry); 0: as stored */
  int32_t math;       /* GANAMD_MATH_F32 | GANAMD_MATH_BF16 */
  int32_t kernel_off; /* kernels this call must NOT use (0 = the library's choice, all allowed):
                         GANAMD_KERNEL_PATCH_FWD / _PATCH_DGRAD (the split6 LDS-patch conv of
                         stride-1 3x3 / 5x5 convs on 32- / 64-wide maps, csrc/conv_patch.hip) and
                         GANAMD_KERNEL_WGRAD_ROW (the row-blocked weight gradient,
                         csrc/conv_wgrad_row.hip) -- a per-call A/B switch, no library state */
} ganamd_conv_desc;

#define GANAMD_KERNEL_PATCH_FWD 1
#define GANAMD_KERNEL_PATCH_DGRAD 2
#define GANAMD_KERNEL_WGRAD_ROW 4
#define GANAMD_KERNEL_SMALL 8     /* the direct vector-ALU conv of Cout <= 4 forwards (ToRGB, csrc/conv_small.hip) */

/* Workspace bytes needed by op (GANAMD_CONV_FWD/DGRAD/WGRAD).  Every entry point that takes a
 * workspace also takes its size in bytes and returns GANAMD_EINVAL (launching nothing) when it is
 * smaller than this query's answer for the same descriptor. */
int ganamd_conv_workspace(const ganamd_conv_desc* d, int op, size_t* bytes);

/* The block schedule conv_fwd / conv_dgrad will launch for d (d->kernel_off included;
 * introspection for tests and tools):
 * info[11] = {BM, BN, column tiles, row tiles, whole-tile columns, tail K-splits, K-steps per
 * split, blocks launched, resident blocks per CU of the instance, CUs, kernel (0: the gather
 * GEMM, 1: the split6 LDS-patch conv -- BN is then its pixel region: 512 pixels at W = 64,
 * 256 at W = 32)}.  scaled: whether the x_scale / gy_scale operand will be passed (it selects
 * the kernel instance). */
int ganamd_conv_plan_info(const ganamd_conv_desc* d, int op, int scaled, int* info);

/* The weight operand of conv_fwd / conv_dgrad in GEMM order (rows padded to the tile grid,
 * channels to whole K-steps, zero filled).  A caller that reuses a weight across calls (the
 * same parameter in forward, backward and the gradient penalty's double backward) packs it
 * once per optimizer step and passes packed_w = 1.  op: GANAMD_CONV_FWD or GANAMD_CONV_DGRAD. */
int ganamd_conv_pack_bytes(const ganamd_conv_desc* d, int op, size_t* bytes);
int ganamd_conv_pack(const ganamd_conv_desc* d, int op, const float* w, float* packed, hipStream_t stream);

/* Batched repack.  A model keeps one GEMM-order copy per (weight, op, geometry) it convolves
 * with and refreshes ALL of them with one launch right after its optimizer step (instead of
 * one pack launch per weight per step).  ganamd_conv_pack_job fills a job on the host (no GPU
 * work); the caller sets chunk0 = the running sum of ganamd_pack_job_chunks over the preceding
 * jobs, uploads the array, and launches ganamd_conv_pack_batch with the total chunk count. */
typedef struct ganamd_pack_job {
  const float* w;
  float* out;
  int32_t sm, sc, st, M, Ck, T, Mpad, Ckp;
  int32_t ps, pk, ppad;   /* ps > 1: the s*s output phases of a stride-ps transposed conv (kernel pk,
                             padding ppad), each packed over its (pk/ps)^2 taps; T counts all pk^2 */
  int32_t x3;             /* also the three bf16 planes (h, m, l: x = h + m + l exactly) of the copy,
                             after it, for the split6 LDS-patch conv (ganamd_conv_pack_bytes counts them) */
  int64_t chunk0;
} ganamd_pack_job;
int ganamd_conv_pack_job(const ganamd_conv_desc* d, int op, const float* w, float* packed, ganamd_pack_job* job);
int64_t ganamd_pack_job_chunks(const ganamd_pack_job* job);
int ganamd_conv_pack_batch(const ganamd_pack_job* jobs, int n_jobs, int64_t total_chunks, hipStream_t stream);

/* y[co][b,oh,ow] = alpha * y_scale[co][b] * sum W * (x * x_scale[ci][b]) + bias[co]
 * Replaces: EqualizedConv2d.forward = F.conv2d(ReplicationPad2d(x), W*c, b)
 *   (generator_13_5.py:36-38, discriminator_9_4.py:38-40); Conv2dWeightModulate.forward's
 *   grouped conv with per-sample weights W*c*s*d (generator_13_5.py:234-248) via x_scale = s,
 *   y_scale = d; nn.ConvTranspose2d (generator_13_5.py:156,594) with transposed=1;
 *   EqualizedLinear = F.linear (generator_13_5.py:25-26, discriminator_9_4.py:26-27).
 * x_scale, y_scale, bias may be NULL.  Workspace: ganamd_conv_workspace(d, GANAMD_CONV_FWD)
 * (split-K partial tiles when the output grid is too small to fill the chip; may be 0). */
int ganamd_conv_fwd(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias,
                    const float* x_scale, const float* y_scale, float alpha, float* y, void* workspace,
                    size_t workspace_bytes, hipStream_t stream);

/* ganamd_conv_fwd with an extended epilogue, applied after bias in this order:
 *   y += noise_scale[co] * noise[co][b,oh,ow]      (StyleConv noise, generator_13_5.py:263-266)
 *   y  = PReLU(y; act_alpha[co])                    (the PReLU that follows a StyleConv)
 * noise / act_alpha may be NULL.  Used by the generator's no-grad forward (the critic step's
 * fake batch), where no pre-activation needs to be kept. */
int ganamd_conv_fwd_ex(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias,
                       const float* x_scale, const float* y_scale, float alpha, const float* noise,
                       const float* noise_scale, const float* act_alpha, float* y, void* workspace,
                       size_t workspace_bytes, hipStream_t stream);

/* gx = alpha * dConv/dx applied to (gy * gy_scale[co][b]), including the ReplicationPad2d
 * backward (edge folding).  Replaces aten convolution_backward (input grad) + replication_pad2d_backward.
 * Workspace: ganamd_conv_workspace(d, GANAMD_CONV_DGRAD). */
int ganamd_conv_dgrad(const ganamd_conv_desc* d, const float* gy, const float* w, const float* gy_scale,
                      float alpha, float* gx, void* workspace, size_t workspace_bytes, hipStream_t stream);

/* gw (+)= alpha * dConv/dW for inputs (x * x_scale) and (gy * gy_scale) (both scales or
 * neither).  accumulate=0 overwrites gw.  Replaces aten convolution_backward (weight grad).
 * Workspace: ganamd_conv_workspace(d, GANAMD_CONV_WGRAD).  Deterministic (no atomics). */
int ganamd_conv_wgrad(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x_scale,
                      const float* gy_scale, float alpha, float* gw, int accumulate, void* workspace,
                      size_t workspace_bytes, hipStream_t stream);

/* gw (+)= alpha * [dConv/dW(x, gy) + dConv/dW(x2, gy2)] as ONE GEMM over both pixel ranges (two
 * K segments of the same weight gradient; unscaled, not transposed, else two launches).  The critic
 * adjoint's x * a + xd * g (critic.hip; the second-order term of the gradient penalty,
 * train/wgangp.py:68-69).  Workspace: ganamd_conv_workspace(d, GANAMD_CONV_WGRAD). */
int ganamd_conv_wgrad2(const ganamd_conv_desc* d, const float* x, const float* gy, const float* x2, const float* gy2,
                       float alpha, float* gw, int accumulate, void* workspace, size_t workspace_bytes,
                       hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Train-mode BatchNorm (1d or 2d) fused with an optional per-channel PReLU.
 * Replaces nn.BatchNorm2d/1d -> nn.PReLU pairs (generator_13_5.py:166,196,211-212,48-49,...).
 * x, y: [C][L].  alpha may be NULL (no activation).  running_* may be NULL.
 * save_mean / save_invstd: [C] outputs kept for the backward.
 * Workspace: ganamd_rowreduce_workspace(C, L).
 * ------------------------------------------------------------------------------------- */
size_t ganamd_rowreduce_workspace(int C, long L);

int ganamd_bn_act_fwd(const float* x, int C, long L, const float* gamma, const float* beta, const float* alpha,
                      float* running_mean, float* running_var, float momentum, float eps, float* y,
                      float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes,
                      hipStream_t stream);
/* Segmented form: x holds `seg` independent mini-batches stacked along the batch (each row's L
 * elements are seg consecutive runs of L / seg), each normalised with its OWN statistics -- the
 * outputs of seg separate calls, in one launch (the critic steps' fake batches generated in one
 * generator forward, train/wgangp.py:58-59 x n_critic).  save_mean / save_invstd / seg_uvar:
 * [C][seg]; running statistics take the seg updates in order.  Workspace:
 * ganamd_rowreduce_workspace(C * seg, L / seg). */
int ganamd_bn_act_fwd_seg(const float* x, int C, long L, int seg, const float* gamma, const float* beta,
                          const float* alpha, float* running_mean, float* running_var, float momentum, float eps,
                          float* y, float* save_mean, float* save_invstd, float* seg_uvar, void* workspace,
                          size_t workspace_bytes, hipStream_t stream);

/* Backward of ganamd_bn_act_fwd: writes gx [C][L]; ggamma, gbeta, galpha ([C]; galpha may be
 * NULL when alpha is NULL) are overwritten, or accumulated into when accumulate = 1 (parameter
 * gradients written straight into an optimizer's flat gradient buffer). */
int ganamd_bn_act_bwd(const float* gy, const float* x, int C, long L, const float* gamma, const float* beta,
                      const float* alpha, const float* save_mean, const float* save_invstd, float* gx,
                      float* ggamma, float* gbeta, float* galpha, int accumulate, void* workspace,
                      size_t workspace_bytes, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * PReLU (per-channel slope) with first and second derivatives (nn.PReLU; the critic's
 * gradient penalty differentiates through its backward: wgangp.py:47-50,69).
 * ------------------------------------------------------------------------------------- */
int ganamd_prelu_fwd(const float* x, const float* alpha, int C, long L, float* y, hipStream_t stream);
/* gx = gy * (x>0 ? 1 : alpha); galpha[c] (=|+= with accumulate) sum gy*x over x<=0 */
int ganamd_prelu_bwd(const float* gy, const float* x, const float* alpha, int C, long L, float* gx, float* galpha,
                     int accumulate, void* workspace, size_t workspace_bytes, hipStream_t stream);
/* Backward of ganamd_prelu_bwd given ggx = dR/dgx and ggalpha = dR/dgalpha (may be NULL):
 *   ggy = ggx*(x>0?1:alpha) + ggalpha[c]*(x>0?0:x)
 *   gx  = ggalpha[c]*gy*(x>0?0:1)            (may be NULL)
 *   galpha[c] = sum ggx*gy over x<=0         (may be NULL) */
int ganamd_prelu_bwd_bwd(const float* ggx, const float* ggalpha, const float* gy, const float* x, const float* alpha,
                         int C, long L, float* ggy, float* gx, float* galpha, void* workspace,
                         size_t workspace_bytes, hipStream_t stream);
/* Tangent sweep of the critic's gradient-penalty double backward (critic.py) through a PReLU:
 *   yd = xd * (x>0 ? 1 : alpha);  galpha[c] (=|+= with accumulate) sum gy*xd over x<=0
 * (the slope's second-order term; gy = the first backward's gradient at the PReLU output). */
int ganamd_prelu_tangent(const float* xd, const float* gy, const float* x, const float* alpha, int C, long L,
                         float* yd,
                         float* galpha, int accumulate, void* workspace, size_t workspace_bytes, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Separable 2-D resampling with per-axis tap tables (ELL format, K taps per output index):
 *   y[p][oh][ow] = sum_i sum_j rw[oh][i] * cw[ow][j] * x[p][ri[oh][i]][ci[ow][j]]
 * Covers Smooth (binomial 3x3, replication pad; generator_13_5.py:134-150,
 * discriminator_9_4.py:56-72), bicubic x2 / x1/2 with A=-0.75 and clamped taps
 * (generator_13_5.py:160, discriminator_9_4.py:81), AdaptiveAvgPool2d(5)
 * (generator_13_5.py:44,355; discriminator_9_4.py:86), their compositions and, with the
 * transposed tables, their adjoints (backward).  One plane plus its row-pass intermediate
 * (IH*IW + IH*OW floats) must fit 48 KB of LDS, else GANAMD_EINVAL.
 * ------------------------------------------------------------------------------------- */
int ganamd_resample2d(const float* x, long planes, int IH, int IW, float* y, int OH, int OW, const int32_t* ri,
                      const float* rw, int KR, const int32_t* ci, const float* cw, int KC, hipStream_t stream);
/* The same resampling of (x + x2) (the sum formed while staging; SK attention's pool of the branch
 * sum u = sum_m feas_m, generator_13_5.py:82-84, without materialising u). */
int ganamd_resample2d_sum(const float* x, const float* x2, long planes, int IH, int IW, float* y, int OH, int OW,
                          const int32_t* ri, const float* rw, int KR, const int32_t* ci, const float* cw, int KC,
                          hipStream_t stream);
/* y = R(x) + r and (y2 non-NULL) y2 = R(x) + r2 (r / r2 may be NULL: no residual), R the resampling
 * above.  The backward of SK attention's pool of the branch sum (generator_13_5.py:82-84): each branch
 * receives R^T(g_t) on top of the gradient its mixing use gave it -- one pass, no R^T(g_t) tensor and
 * no adds. */
int ganamd_resample2d_add(const float* x, long planes, int IH, int IW, float* y, int OH, int OW, const int32_t* ri,
                          const float* rw, int KR, const int32_t* ci, const float* cw, int KC, const float* r,
                          float* y2, const float* r2, hipStream_t stream);

/* out[p] = scale * sum_{hw} a[p][hw] * (b ? b[p][hw] : 1)   (planes of HW elements).
 * Replaces AdaptiveAvgPool2d(1) (generator_13_5.py:52,362) and the per-(channel,sample)
 * reductions of the modulated-conv / SK / SE backward. */
int ganamd_plane_dot(const float* a, const float* b, long planes, long HW, float scale, float* out,
                     hipStream_t stream);
/* out1[p] = sum_hw a*b1, out2[p] = sum_hw a*b2 in one pass over a (HW % 4 == 0, 16-byte aligned
 * planes): the modulated conv backward's <gy, y> and <gy, noise> (generator_13_5.py:234-248, 265). */
int ganamd_plane_dot_pair(const float* a, const float* b1, const float* b2, long planes, long HW, float* out1,
                          float* out2, hipStream_t stream);
/* The modulated conv's style-side gradients from its saved output y = d * conv + ns * noise
 * (generator_13_5.py:234-248, 263-265), planes p = (c, b) of HW floats (HW % 4 == 0, 16-byte aligned):
 *   gd[p] = dL/dd = (<gy, y> - ns[c] * <gy, noise>) / d[p]    (dots and combination in double)
 *   pdn[p] = <gy, noise>,  gns[c] += sum_b pdn[c][b]           (noise may be NULL: gd = <gy, y> / d;
 *                                                               gns may be NULL)
 * Replaces the per-sample-weight backward of F.conv2d(groups=B) with respect to the demodulation. */
int ganamd_modconv_sd_bwd(const float* gy, const float* y, const float* noise, const float* d, const float* ns,
                          int C, int B, long HW, float* gd, float* pdn, float* gns, hipStream_t stream);

/* out[c] (=|+= with accumulate) sum_{l} a[c][l] * (b ? b[c][l] : 1) over rows of length L
 * (with b = NULL and accumulate = 1: a conv bias gradient added into the flat gradient buffer). */
int ganamd_row_dot(const float* a, const float* b, int C, long L, float* out, int accumulate, void* workspace,
                   size_t workspace_bytes, hipStream_t stream);

/* out[i] = sum_{t<T} w[i*T + t]^2  (row sums of squares; the demodulation norm's sum over taps) */
int ganamd_segment_sumsq(const float* w, long rows, int T, float* out, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Fused AdamW over one flat fp32 buffer (torch.optim.AdamW as configured at wgangp.py:17-18):
 *   step += 1 (device counter, so a captured graph replays correctly)
 *   p *= 1 - lr*wd; m = lerp(m, g, 1-beta1); v = beta2*v + (1-beta2)*g*g
 *   p -= lr/(1-beta1^t) * m / (sqrt(v)/sqrt(1-beta2^t) + eps)
 * ------------------------------------------------------------------------------------- */
int ganamd_adamw(float* p, const float* g, float* m, float* v, long n, int32_t* step, float lr, float beta1,
                 float beta2, float eps, float weight_decay, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Grouped small GEMMs over a static tile list (the generator's style bank: the 519 per-conv
 * style MLPs and demodulation products of generator_13_5.py:223-227,239-242 in one launch).
 *   C[c_off + r*ldc + n] (=|+=) epi( sum_k A(r,k) * B(k,n) ),  r < rows, n < cols (each <= 64)
 *   A(r,k) = a_trans ? A[a_off + k*lda + r] : A[a_off + r*lda + k]
 *   B(k,n) = b_trans ? B[b_off + n*ldb + k] : B[b_off + k*ldb + n]   (squared if b_square)
 * ------------------------------------------------------------------------------------- */
#define GANAMD_EPI_STORE 0
#define GANAMD_EPI_BIAS 1   /* scale*acc + bias[bias_off + r] */
#define GANAMD_EPI_DEMOD 2  /* rsqrt(scale^2 * acc + 1e-8) */
#define GANAMD_EPI_ACCUM 3  /* C += scale*acc */
#define GANAMD_EPI_SCALE 4  /* scale*acc */

typedef struct ganamd_gtile {
  int32_t a_off, lda, b_off, ldb, c_off, ldc;
  int32_t rows, cols, K, epi, bias_off;
  float scale;
} ganamd_gtile;

int ganamd_grouped_gemm(const float* A, const float* B, float* C, const float* bias, const ganamd_gtile* tiles,
                        int n_tiles, int a_trans, int b_trans, int b_square, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Fused per-plane elementwise ops (CNHW: planes = C*B planes of HW floats; per-(c,b)
 * coefficients [C][B] are indexed by plane).
 * ------------------------------------------------------------------------------------- */
/* y = sum_{m<M} att[m][plane] * f_m   (M <= 4; SK mixing, generator_13_5.py:80-89,165-170,196-202) */
int ganamd_mix_fwd(int M, const float* f0, const float* f1, const float* f2, const float* f3, const float* att,
                   long planes, long HW, float* y, hipStream_t stream);
/* gf_m = gy * att[m] (gf_m may be NULL), gatt[m][plane] = sum_hw gy * f_m (gatt may be NULL) */
int ganamd_mix_bwd(int M, const float* f0, const float* f1, const float* f2, const float* f3, const float* att,
                   long planes, long HW, const float* gy, float* gf0, float* gf1, float* gf2, float* gf3, float* gatt,
                   hipStream_t stream);
/* y[c][l] = PReLU(a + b; alpha[c])   (ResnetInit, generator_13_5.py:343-349) */
int ganamd_add_prelu(const float* a, const float* b, const float* alpha, int C, long L, float* y, hipStream_t stream);
/* y = r + x * s[plane]  (r may be NULL: y = x * s)   (SE gating + residual, generator_13_5.py:455-466,
 * discriminator_9_4.py:158-161) */
int ganamd_scale_add(const float* x, const float* s, const float* r, long planes, long HW, float* y,
                     hipStream_t stream);
/* gx[c][l] = sum over the parts k (in order) with lo[k] <= c < hi[k] of g[k][c - lo[k]][l], 0 where no
 * part covers row c (C rows of L floats; n <= GANAMD_ROUTE_MAX parts, each g[k] [hi-lo][L]).  The
 * backward of several channel-range views of one CNHW tensor -- the dual-path split / concat of
 * BasicBlock and Tree (generator_13_5.py:448-467, 496-564) -- in one pass.  Replaces autograd's
 * slice backward (a zero-filled full-size tensor per view) and the adds that sum them. */
#define GANAMD_ROUTE_MAX 8
int ganamd_route_bwd(int n, const float* const* g, const int32_t* lo, const int32_t* hi, int C, long L, float* gx,
                     hipStream_t stream);

/* Gradient penalty on the critic's input gradient g = grad_x D(x_hat), [B][n] (n = 3*64*64):
 *   mode 0 (WGAN-GP, train/wgangp.py:34-54,68):  out = lambda * mean_b (||g_b||_2 - center)^2
 *   mode 1 (R1 / R2, train/wganlazygpR2.py:57-70): out = lambda * mean_b ||g_b||_2^2
 * norms[b] receives ||g_b|| (mode 0) or ||g_b||^2 (mode 1).  ganamd_gp_bwd: dg = d out / d g
 * scaled by gout[0] (device scalar), from g and the saved norms -- the closed form, no autograd
 * graph of the penalty itself.  Workspace: ganamd_gp_workspace(B, n) bytes. */
size_t ganamd_gp_workspace(int B, long n);
int ganamd_gp_fwd(const float* g, int B, long n, float center, float lambda, int mode, float* norms, float* out,
                  void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_gp_bwd(const float* g, const float* norms, const float* gout, int B, long n, float center, float lambda,
                  int mode, float* dg, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Real-data input pipeline (units/dataloader.py:5-14): a batch of B
 * decoded images u8 [B][H][W][3] (one size) -> f32 NCHW [B][3][OH][OW]:
 *   ToTensor (/255) -> RandomHorizontalFlip (flip[b] != 0 mirrors image b; flip may be NULL)
 *   -> Resize((OH, OW), BICUBIC, antialias) as separable ELL tap tables (ix/wx: OW x KX over
 *   the W axis, iy/wy: OH x KY over the H axis) -> Normalize(mean[3], std[3]).
 * workspace: ganamd_image_batch_workspace(B, H, OW) bytes (the row-pass intermediate).
 * ------------------------------------------------------------------------------------- */
size_t ganamd_image_batch_workspace(int B, int H, int OW);
int ganamd_image_batch(const uint8_t* src, int B, int H, int W, const uint8_t* flip, const int32_t* ix,
                       const float* wx, int KX, int OW, const int32_t* iy, const float* wy, int KY, int OH,
                       const float* mean, const float* stdv, float* y, float* workspace, size_t workspace_bytes,
                       hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Pointwise activations (csrc/act.hip) over n contiguous floats.
 *   GANAMD_ACT_SIGMOID  SE gates (generator_13_5.py:357,376; discriminator_9_4.py:109,128),
 *                       the vanilla critic's Sigmoid (discriminator_1.py:20)
 *   GANAMD_ACT_TANH     the vanilla generator's Tanh (generator_1.py:23)
 *   GANAMD_ACT_LEAKY    LeakyReLU(slope) (generator_1.py:19,21; discriminator_1.py:16,18)
 * ganamd_act_bwd: gx = gy * f'(.) where v is the forward OUTPUT for sigmoid / tanh and the
 * forward INPUT for leaky.
 * ------------------------------------------------------------------------------------- */
#define GANAMD_ACT_SIGMOID 0
#define GANAMD_ACT_TANH 1
#define GANAMD_ACT_LEAKY 2
int ganamd_act_fwd(int kind, const float* x, long n, float slope, float* y, hipStream_t stream);
int ganamd_act_bwd(int kind, const float* v, const float* gy, long n, float slope, float* gx, hipStream_t stream);
/* Adjoint sweep of the critic's gradient-penalty double backward (critic.py) through an
 * activation: ax = ay * f'(.) + gy * xd * f''(.)  (v as for ganamd_act_bwd; f'' = 0 for leaky). */
int ganamd_act_adjoint(int kind, const float* v, const float* ay, const float* gy, const float* xd, long n,
                       float slope,
                       float* ax, hipStream_t stream);

/* y = x1 * s1[plane] + x2 * s2[plane] + r over planes of HW floats (x2/s2 and r may be NULL): the
 * tangent and adjoint of the SE-gated residual y = x * s + r (discriminator_9_4.py:158-161). */
int ganamd_scale_add2(const float* x1, const float* s1, const float* x2, const float* s2, const float* r, long planes,
                      long HW, float* y, hipStream_t stream);
/* out[plane] = sum a1*b1 + sum a2*b2 (a2/b2 may be NULL): the gate's adjoint of the same op. */
int ganamd_plane_dot2(const float* a1, const float* b1, const float* a2, const float* b2, long planes, long HW,
                      float* out, hipStream_t stream);
/* y += a * x over n floats (gradient accumulation where an activation feeds two consumers). */
int ganamd_axpy(long n, float a, const float* x, float* y, hipStream_t stream);

/* torch.nn.BCELoss (mean; logs clamped at -100) of probabilities p against targets, n values
 * (train/gan.py:21,32,48,50).  out: device scalar.  ganamd_bce_bwd: gp = d out/d p * gout[0]. */
int ganamd_bce_fwd(const float* p, const float* target, int n, float* out, hipStream_t stream);
int ganamd_bce_bwd(const float* p, const float* target, int n, const float* gout, float* gp, hipStream_t stream);

/* Softmax over M in {2,3,4} branches of x[M][P] (the SK attention heads, dim=1 of the
 * reference's [B, M, C, 1, 1]: generator_13_5.py:88,131) and its backward gx = y (gy - <y, gy>). */
int ganamd_softmax_m(int M, const float* x, long P, float* y, hipStream_t stream);
int ganamd_softmax_m_bwd(int M, const float* y, const float* gy, long P, float* gx, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * MiniBatchStdDev (discriminator_9_4.py:42-54) on CNHW x[C][B][HW] (row stride ldx floats)
 * holding S independent segments of B/S samples; group size G = 4 (x.view(G, -1) of each
 * segment's NCHW tensor, unbiased variance, + 1e-8, sqrt, mean).  y[C+1][B][HW] (row stride
 * ldy) = x with one more row holding each segment's std; std_out[S] (may be NULL).
 *   bwd      gx = d/dx <gy, y>
 *   tangent  yd = directional derivative of y along xd (the forward sweep of the critic's
 *            gradient-penalty double backward, critic.py)
 *   adjoint  ax = J^T ay + (d(J xd)/dx)^T gy (its reverse sweep: the second-order term of the
 *            batch coupling)
 * Workspace: ganamd_mbstd_workspace(S) bytes.
 * ------------------------------------------------------------------------------------- */
size_t ganamd_mbstd_workspace(int S);
int ganamd_mbstd_fwd(const float* x, long ldx, int C, int B, int HW, int S, int G, float* y, long ldy, float* std_out,
                     void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_mbstd_bwd(const float* x, long ldx, const float* gy, long ldy, int C, int B, int HW, int S, int G,
                     float* gx, void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_mbstd_tangent(const float* x, const float* xd, long ldx, int C, int B, int HW, int S, int G, float* yd,
                         long ldy, void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_mbstd_adjoint(const float* x, const float* xd, long ldx, const float* gy, const float* ay, long ldy, int C,
                         int B, int HW, int S, int G, float* ax, void* workspace, size_t workspace_bytes,
                         hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Linear + train-mode BatchNorm1d (+ PReLU) in one launch, the generator's
 * EqualizedLinear -> BatchNorm1d -> PReLU chains (SK attention fc / heads, SE fc, mapping MLPs;
 * generators/generator_13_5.py:19-26, 48-50, 71-79) on feature-major [Cin][B] activations:
 *   v = alpha * W x + bias;  y = act(gamma * (v - mean_b v) / sqrt(var_b v + eps) + beta)
 * with the batch mean and biased variance of each output row; running_mean / running_var
 * updated in place with momentum (unbiased variance), as torch.nn.BatchNorm1d in train mode.
 * The block owns whole rows: 2 <= B <= 64, Cout * Cin <= 4 M, fp32, 1x1 geometry (H = W = 1).
 * Workspace: ganamd_conv_workspace(d, GANAMD_CONV_FWD) bytes unless d->packed_w.
 * ------------------------------------------------------------------------------------- */
int ganamd_linear_bn_act(const ganamd_conv_desc* d, const float* x, const float* w, const float* bias, float alpha,
                         const float* gamma, const float* beta, const float* act_alpha, float* running_mean,
                         float* running_var, float momentum, float eps, float* y, void* workspace,
                         size_t workspace_bytes, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Device random numbers (Philox4x32-10) for z, eps and the StyleConv noise.
 * Replaces torch.randn / torch.rand on the path (train/wgangp.py:22,35,58;
 * generator_13_5.py:265; train/gan.py:21,32 label noise).  Element 4g+i of a draw is word i of
 * Philox4x32-10(counter {g lo, g hi, off lo, off hi}, key {seed lo, seed hi}) where off = *offset
 * read on the device; the call then advances *offset by one on the stream (graph-replay safe).
 *   uniform: (word >> 8) * 2^-24 in [0, 1)
 *   normal:  Box-Muller on (w0, w1) and (w2, w3): u1 = ((w >> 8) + 1) * 2^-24, u2 = (w >> 8) * 2^-24,
 *            z = sqrt(-2 ln u1) * (cos, sin)(2 pi u2)
 * offset: device pointer to one uint64.  n > 0.
 * ------------------------------------------------------------------------------------- */
int ganamd_philox_uniform(float* out, long n, uint64_t seed, uint64_t* offset, hipStream_t stream);
int ganamd_philox_normal(float* out, long n, uint64_t seed, uint64_t* offset, hipStream_t stream);
/* The general draw: counter word 1 = (g >> 32) + sub; advance != 0 advances *offset after the
 * draw.  sub != 0 (then at most 2^34 elements) with advance = 0 lets several draws that may run
 * concurrently on different streams share one offset word with distinct counters (a generator
 * forward's per-draw noise inside ResnetInit's branch streams, generator_13_5.py:265,343-349);
 * their owner calls ganamd_philox_advance once after joining them.  Consumers that run
 * concurrently with each other own separate offset words (DeviceRNG.fork: word s starts at
 * s * 2^40), so no two draws of an iteration share a counter. */
int ganamd_philox_draw(float* out, long n, uint64_t seed, uint64_t* offset, uint32_t sub, int normal, int advance,
                       hipStream_t stream);
/* The same draw with the key read on the device from *key (one uint64, non-NULL): re-keying the
 * generator (a checkpoint resume, rng.py DeviceRNG.set_seed) is then a device write that graphs
 * captured before it see on their next replay, as they see the offset. */
int ganamd_philox_draw_keyed(float* out, long n, const uint64_t* key, uint64_t* offset, uint32_t sub, int normal,
                             int advance, hipStream_t stream);
int ganamd_philox_advance(uint64_t* offset, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Critic program engine: the critic as a straight-line layer program, and the gradient
 * penalty's double backward as C-ABI sweeps over it (csrc/critic.hip).
 * Replaces the critic step's autograd protocol: train/wgangp.py:45-54 (compute_grad2:
 *   autograd.grad(d_out.sum(), x_hat, create_graph=True) then grad.pow(2)...),
 *   wgangp.py:34-43 (gradient_penalty), wgangp.py:68-69 (gp.backward() = the double backward),
 *   train/wganlazygpR2.py:48-77 (R1 / R2 / GP on stacked segments).
 * Program ops (value ids: value 0 is the NCHW input [B][C0][H0][W0]; every other value is CNHW
 * [C][B][H][W], H = W = 1 for per-sample vectors):
 *   SWAP       NCHW input -> CNHW                            in[0] = 0
 *   CONV       EqualizedConv2d (ReplicationPad2d(pad) + conv, discriminator_9_4.py:30-40) or,
 *              with H = W = 1 and k = 1, EqualizedLinear (discriminator_9_4.py:20-27):
 *              y = alpha * conv(x, w) + bias; cout, k, stride, pad; w as stored [cout][cin][k][k]
 *              (w_fwd / w_dgrad: optional GEMM-order copies, ganamd_conv_pack)
 *   PRELU      nn.PReLU(C): per-channel slope
 *   RESAMPLE   separable resampler (ganamd_resample2d tables: forward ri/rw/kr, adjoint
 *              ari/arw/akr), H -> n_out (Smooth, DownSample, AdaptiveAvgPool2d(5))
 *   PMEAN      AdaptiveAvgPool2d(1) -> [C][B]
 *   SIGMOID    the SE gate
 *   SCALE_ADD  y = x * s + r: x = in[0] [C][B][H][W], s = in[1] [C][B], r = in[2] (-1: none)
 *              (discriminator_9_4.py:158-161)
 *   MBSTD      MiniBatchStdDev(group) (discriminator_9_4.py:42-54), over `segments` equal
 *              segments of the batch (the plan's)
 *   FLATTEN    [C][B][H][W] -> [(c,h,w)][B] (the NCHW .view(B, -1), discriminator_9_4.py:197)
 * The output value must be [1][B] (the critic's score).
 *
 * Sweeps (all on `stream`, into the caller's workspace; the plan records which values are
 * live between calls, so forward -> backward -> tangent -> adjoint must run in that order on
 * the SAME workspace, and the input x (and the tangent seed v) must stay valid until the
 * adjoint has run):
 *   forward   X_v for every value; out[b] = D(x)_b (out may be NULL)
 *   backward  G_v = d <seed, D(x)> / d X_v (seed [B], NULL = ones); gx = G_0 (NCHW, may be NULL)
 *   tangent   XD_v = directional derivative of X_v along the input direction v (NCHW)
 *   adjoint   A_v  = d h / d X_v for h = <v, G_0> + <a_seed, D(x)> (a_seed may be NULL): the
 *             reverse sweep with the second-order terms (PReLU slope, sigmoid, the SE product,
 *             MiniBatchStdDev); ax = A_0 (NCHW, may be NULL)
 * Parameter gradients: with `grads` non-NULL ([n_ops] entries; NULL members skip that tensor)
 * every sweep ACCUMULATES its parameter terms into them -- backward the first-order ones,
 * tangent the PReLU slopes' second-order term, adjoint the rest -- so backward(params) +
 * tangent + adjoint(a_seed = w) leave d/dtheta [<w, D(x)> + <v, G_0>] in the gradient buffers.
 *
 * ganamd_critic_gp_step is the fused GP double-backward driver: forward, backward (seed ones),
 * the penalty P = lambda * mean_b (||G_0,b|| - center)^2 (mode 0) or lambda * mean_b
 * ||G_0,b||^2 (mode 1) into *penalty (device scalar), v = dP/dG_0, tangent and adjoint, with
 * dP/dtheta accumulated into `grads`.
 *
 * Threads and streams: a plan is driven by one thread at a time.  Distinct plans may be driven
 * concurrently from several threads on distinct streams, also while one of those streams is being
 * captured into a HIP graph: the sweeps fork their weight gradients onto a side stream that
 * belongs to the caller's stream (one per device and caller stream, never shared between two
 * caller streams) and join it before returning, so a capture only ever pulls its own stream's
 * side stream into its graph.
 * ------------------------------------------------------------------------------------- */
#define GANAMD_COP_SWAP 0
#define GANAMD_COP_CONV 1
#define GANAMD_COP_PRELU 2
#define GANAMD_COP_RESAMPLE 3
#define GANAMD_COP_PMEAN 4
#define GANAMD_COP_SIGMOID 5
#define GANAMD_COP_SCALE_ADD 6
#define GANAMD_COP_MBSTD 7
#define GANAMD_COP_FLATTEN 8

typedef struct ganamd_critic_op {
  int32_t kind;
  int32_t in[3];                   /* input value ids (unused: -1); the output is value index+1 */
  int32_t cout, k, stride, pad;    /* CONV */
  int32_t pad_mode;                /* CONV: GANAMD_PAD_REPLICATE (EqualizedConv2d) or ZERO */
  int32_t n_out;                   /* RESAMPLE: output side */
  int32_t kr, akr;                 /* RESAMPLE: taps per output index (forward / adjoint table) */
  int32_t group;                   /* MBSTD */
  float alpha;                     /* CONV: the equalized-lr constant c */
  const float* w;                  /* CONV weight as stored; PRELU slopes */
  const float* w_fwd;              /* CONV: GEMM-order copies (may be NULL) */
  const float* w_dgrad;
  const float* bias;               /* CONV */
  const int32_t* ri;               /* RESAMPLE forward table */
  const float* rw;
  const int32_t* ari;              /* RESAMPLE adjoint table */
  const float* arw;
} ganamd_critic_op;

typedef struct ganamd_critic_grads {
  float* gw;                       /* CONV weight / PRELU slope gradient */
  float* gb;                       /* CONV bias gradient */
} ganamd_critic_grads;

typedef struct ganamd_critic_plan ganamd_critic_plan;

/* Validates the program and sizes every value; NULL on an invalid program (shape mismatch,
 * unknown op, a value used before it is defined).  math: GANAMD_MATH_F32 | GANAMD_MATH_BF16;
 * kernel_off: the ganamd_conv_desc.kernel_off of every conv the plan issues (0: all kernels). */
ganamd_critic_plan* ganamd_critic_create(const ganamd_critic_op* ops, int n_ops, int B, int C0, int H0, int W0,
                                         int segments, int math, int kernel_off);
void ganamd_critic_destroy(ganamd_critic_plan* plan);
int ganamd_critic_workspace(const ganamd_critic_plan* plan, size_t* bytes);
/* The workspace in four regions, each allocated only when the sweep that fills it starts:
 * 0 = scratch + X (forward), 1 = G (backward), 2 = XD (tangent), 3 = A (adjoint).  With
 * `workspace` = NULL every sweep uses the regions bound here (binding region 0 starts a new
 * evaluation); with a non-NULL `workspace` (ganamd_critic_workspace bytes) the four regions are
 * carved from it in that order.  A first-order evaluation (the real / fake critic passes) then
 * needs regions 0-1 only.  Bound regions and the contiguous workspace carry their byte sizes
 * (region_bytes / workspace_bytes), checked against these queries: GANAMD_EINVAL when short. */
int ganamd_critic_region_bytes(const ganamd_critic_plan* plan, int which, size_t* bytes);
int ganamd_critic_bind(ganamd_critic_plan* plan, int which, void* region, size_t region_bytes);
/* Device pointer of value v in sweep `which` (0 X, 1 G, 2 XD, 3 A) as the last sweep left it
 * (NULL: no such value yet).  For callers that read saved activations / gradients. */
int ganamd_critic_value(const ganamd_critic_plan* plan, int which, int v, const float** ptr);
int ganamd_critic_forward(ganamd_critic_plan* plan, const float* x, float* out, void* workspace,
                          size_t workspace_bytes, hipStream_t stream);
int ganamd_critic_backward(ganamd_critic_plan* plan, const float* seed, const ganamd_critic_grads* grads, float* gx,
                           void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_critic_tangent(ganamd_critic_plan* plan, const float* v, const ganamd_critic_grads* grads,
                          void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_critic_adjoint(ganamd_critic_plan* plan, const float* a_seed, const ganamd_critic_grads* grads, float* ax,
                          void* workspace, size_t workspace_bytes, hipStream_t stream);
int ganamd_critic_gp_step(ganamd_critic_plan* plan, const float* x, float center, float lambda, int mode,
                          const ganamd_critic_grads* grads, float* out, float* gx, float* norms, float* penalty,
                          void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Library identification (for load checks). */
const char* ganamd_version(void);

/* Capture state of a stream: *capture_id = the id of the HIP graph capture in progress on it, or
 * 0 when the stream is not capturing.  Lets host-side caches of device buffers (packed weights)
 * tell one graph capture from another and from eager execution. */
int ganamd_stream_capture_id(hipStream_t stream, unsigned long long* capture_id);

#ifdef __cplusplus
}
#endif

#endif /* GANAMD_H */
