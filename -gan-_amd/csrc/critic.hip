// The critic program engine (include/ganamd.h, "Critic program engine"): the critic as a
// straight-line layer program and the gradient penalty's double backward as four sweeps over it,
// driven from the host side of libganamd.so -- no autograd graph, no per-layer host round trips
// above the C ABI.
//
// Reference: the critic step's penalty (train/wgangp.py:34-54, 68-69) takes the critic's input
// gradient g = grad_x sum D(x_hat) with autograd.grad(create_graph=True) and back-propagates
// (||g_b|| - 1)^2 through it.  The same derivative, by sweeps over the saved activations:
//
//   forward   X_v                                       (every value of the program, saved)
//   backward  G_v  = d <seed, D> / d X_v                 -> g = G_0
//   penalty   P(g), v = dP/dg                            (ganamd_gp_fwd / _bwd)
//   tangent   XD_v = directional derivative of X_v along v   (forward mode, seed XD_0 = v)
//   adjoint   A_v  = d h / d X_v, h(theta) = <v, G_0(theta)> (+ <a_seed, D>): the reverse sweep
//             carrying the second-order terms
//               conv      A_in += W^T A_out;  dW += wgrad(X_in, A_out) + wgrad(XD_in, G_out)
//                         (one two-segment GEMM, ganamd_conv_wgrad2)
//               PReLU     A_in  = A_out prelu'(X);  dslope: A_out*min(X,0) here, G_out*XD[X<=0]
//                         in the tangent sweep (ganamd_prelu_tangent)
//               sigmoid   A_in  = A_out s(1-s) + G_out XD s(1-s)(1-2s)      (ganamd_act_adjoint)
//               x*s + r   A_x = A_out s + G_out XD_s;  A_s = <A_out, X_x> + <G_out, XD_x>;  A_r = A_out
//               MiniBatchStdDev   ganamd_mbstd_adjoint (the cross-sample term)
//   dP/dtheta = dh/dtheta, accumulated into the caller's gradient buffers.
//
// Every arithmetic step is one of the library's kernels (conv GEMMs, PReLU, resample, act,
// mbstd, gp); this file adds only the sweep sequencing, the workspace layout and three layout
// kernels (NCHW <-> CNHW swap, flatten, plane broadcast).  Accumulation into a value that
// several consumers feed follows a written/borrowed table per sweep: the first contribution is
// produced straight into the value's buffer (or, for an identity pass-through, borrowed by
// pointer), later ones through one scratch buffer + axpy.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/ganamd.h"

namespace {

constexpr int kNT = 256;

inline int ok(hipError_t e) { return e == hipSuccess ? GANAMD_OK : GANAMD_ELAUNCH; }
inline int grid_for(long n) { return (int)std::max<long>(1, std::min<long>((n + kNT - 1) / kNT, 16384)); }

// out (contiguous [n0][n1][n2]) = in[i0*s0 + i1*s1 + i2*s2]
__global__ void permute3_kernel(const float* __restrict__ in, float* __restrict__ out, long n0, long n1, long n2,
                                long s0, long s1, long s2) {
  const long n = n0 * n1 * n2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long i2 = i % n2;
    const long t = i / n2;
    const long i1 = t % n1;
    const long i0 = t / n1;
    out[i] = in[i0 * s0 + i1 * s1 + i2 * s2];
  }
}

// out[p][hw] = g[p] * scale   (the adjoint of the plane mean)
__global__ void plane_bcast_kernel(const float* __restrict__ g, long P, long HW, float scale, float* __restrict__ out) {
  const long n = P * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = g[i / HW] * scale;
}

__global__ void fill_kernel(float* __restrict__ p, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}

int permute3(const float* in, float* out, long n0, long n1, long n2, long s0, long s1, long s2, hipStream_t s) {
  const long n = n0 * n1 * n2;
  if (n == 0) return GANAMD_OK;
  permute3_kernel<<<grid_for(n), kNT, 0, s>>>(in, out, n0, n1, n2, s0, s1, s2);
  return ok(hipGetLastError());
}

int fill(float* p, long n, float v, hipStream_t s) {
  if (n == 0) return GANAMD_OK;
  fill_kernel<<<grid_for(n), kNT, 0, s>>>(p, n, v);
  return ok(hipGetLastError());
}

// Weight gradients off the critical path: inside a backward / adjoint sweep every conv's weight
// (and bias) gradient is forked onto a side stream -- it needs only the conv's saved input and its
// output gradient, while the sweep's chain continues with the input gradient -- and the sweep joins
// it at its end.  Under graph capture the fork / join become graph edges.  The side stream belongs
// to the CALLER's stream (one per (device, caller stream), created on first use, never shared
// between two caller streams): two plans driven from two threads on two streams never serialise
// on one side stream, and a capture on one caller stream pulls only that stream's side stream into
// its graph -- an eager sweep on another stream never touches a stream being captured.  Each plan
// has its own fork / join events.  Same kernels, same per-buffer accumulation order (all weight
// gradients of a sweep run in sweep order on the side stream), so results are unchanged.
// Why this is capture-safe where round 4's penalty-on-a-second-stream path crashed capture_end: here the
// fork / join are plain hipEventRecord / hipStreamWaitEvent pairs on a library stream, nothing is
// allocated on it (all memory is the caller's workspace), and every sweep joins before it returns, so
// a capture never ends with unjoined side-stream work; the removed path ran a PyTorch autograd node's
// backward on a torch side stream inside the capture (the engine's cross-stream event syncs and
// caching-allocator blocks on a non-origin stream), which is what brought capture_end down.
// A stream that cannot be created is remembered as such (no retry per sweep: that caller's sweeps run
// serially).  Entries live as long as the process (one per caller stream).
hipStream_t side_stream(hipStream_t caller) {
  struct Entry {
    int dev;
    hipStream_t caller, side;
  };
  static std::mutex mu;
  static std::vector<Entry> table;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  for (const Entry& e : table)
    if (e.dev == dev && e.caller == caller) return e.side;
  hipStream_t side = nullptr;
  if (hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess) side = nullptr;
  table.push_back(Entry{dev, caller, side});
  return side;
}

struct Val {
  int C = 0, H = 0, W = 0;
  long n = 0;          // C * B * H * W
  long hw() const { return (long)H * W; }
};

// the value table of one sweep: current pointer (nullptr: no contribution yet), whether it is
// borrowed (points at another value's buffer: never written in place), and the own buffer
struct Sweep {
  std::vector<float*> cur, own;
  std::vector<char> borrowed;
  void reset() {
    std::fill(cur.begin(), cur.end(), nullptr);
    std::fill(borrowed.begin(), borrowed.end(), 0);
  }
};

}  // namespace

struct ganamd_critic_plan {
  std::vector<ganamd_critic_op> ops;
  std::vector<Val> val;            // value v = output of op v-1; value 0 = the NCHW input
  std::vector<char> input_only;    // value is the input or a layout copy of it (no gradient needed)
  int B = 0, S = 1, math = GANAMD_MATH_F32, kernel_off = 0, out = 0;
  long maxn = 0;
  // workspace layout (bytes), set by ganamd_critic_workspace
  bool sized = false;
  size_t total = 0, off_tmp = 0, off_conv = 0, off_rr = 0, off_mb = 0, off_gp = 0, off_ones = 0, off_v = 0,
         off_g0 = 0, off_norms = 0, off_conv2 = 0, off_rr2 = 0;   // *2: the side stream's scratch
  size_t conv_ws = 0, rr_ws = 0, mb_ws = 0, gp_ws = 0;
  std::vector<size_t> offX, offG, offXD, offA;   // X: in region 0 after the scratch; G, XD, A: regions 1-3
  size_t rsz[4] = {0, 0, 0, 0};                  // region bytes
  // state between sweeps: the regions' bases -- carved from one contiguous workspace (ws != NULL)
  // or bound one by one (ganamd_critic_bind, ws == NULL)
  char* ws = nullptr;
  char* R[4] = {nullptr, nullptr, nullptr, nullptr};
  int stage = 0;                   // 1 forward, 2 backward, 3 tangent done
  std::vector<float*> X, XD;
  Sweep G, A;
  // this plan's fork / join events to the caller stream's side stream (see side_stream); `side`
  // is the side stream of the sweep in progress
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool forked = false, has_events = false;
  ~ganamd_critic_plan() {
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
  }

  ganamd_conv_desc desc(int i, bool packed) const {
    const ganamd_critic_op& op = ops[i];
    const Val& x = val[op.in[0]];
    const Val& y = val[i + 1];
    ganamd_conv_desc d;
    d.B = B;
    d.Cin = x.C;
    d.H = x.H;
    d.W = x.W;
    d.Cout = op.cout;
    d.OH = y.H;
    d.OW = y.W;
    d.KH = d.KW = op.k;
    d.stride = op.stride;
    d.pad = op.pad;
    d.pad_mode = op.pad_mode;
    d.transposed = 0;
    d.packed_w = packed ? 1 : 0;
    d.math = math;
    d.kernel_off = kernel_off;
    return d;
  }
  float* at(size_t off) const { return reinterpret_cast<float*>(R[0] + off); }   // scratch and X
  float* atr(int r, size_t off) const { return reinterpret_cast<float*>(R[r] + off); }
};

namespace {

using Plan = ganamd_critic_plan;

// produce the next contribution to value v of sweep S (produce(dst) writes a fresh tensor)
template <class F>
int acc(Plan& p, Sweep& S, int v, F produce, hipStream_t s) {
  const long n = p.val[v].n;
  if (!S.cur[v]) {
    int rc = produce(S.own[v]);
    S.cur[v] = S.own[v];
    return rc;
  }
  if (S.borrowed[v]) {         // the borrowed one is added into a fresh own tensor
    int rc = produce(S.own[v]);
    if (rc == GANAMD_OK) rc = ganamd_axpy(n, 1.f, S.cur[v], S.own[v], s);
    S.cur[v] = S.own[v];
    S.borrowed[v] = 0;
    return rc;
  }
  float* tmp = p.at(p.off_tmp);
  int rc = produce(tmp);
  if (rc == GANAMD_OK) rc = ganamd_axpy(n, 1.f, tmp, S.cur[v], s);
  return rc;
}

// an identity pass-through: value v += src (src is another value's final tensor)
int acc_borrow(Plan& p, Sweep& S, int v, float* src, hipStream_t s) {
  const long n = p.val[v].n;
  if (!S.cur[v]) {
    S.cur[v] = src;
    S.borrowed[v] = 1;
    return GANAMD_OK;
  }
  if (S.borrowed[v]) {
    int rc = ok(hipMemcpyAsync(S.own[v], src, n * sizeof(float), hipMemcpyDeviceToDevice, s));
    if (rc == GANAMD_OK) rc = ganamd_axpy(n, 1.f, S.cur[v], S.own[v], s);
    S.cur[v] = S.own[v];
    S.borrowed[v] = 0;
    return rc;
  }
  return ganamd_axpy(n, 1.f, src, S.cur[v], s);
}

// NCHW [B][C][HW] -> CNHW [C][B][HW] and back; [C][B][HW] <-> [C][HW][B]
int swap_in(const Plan& p, const float* x, float* y, hipStream_t s) {
  const Val& v = p.val[0];
  return permute3(x, y, v.C, p.B, v.hw(), v.hw(), (long)v.C * v.hw(), 1, s);
}
int swap_out(const Plan& p, const float* g, float* gx, hipStream_t s) {
  const Val& v = p.val[0];
  return permute3(g, gx, p.B, v.C, v.hw(), v.hw(), (long)p.B * v.hw(), 1, s);
}
int flatten(const Plan& p, const Val& x, const float* in, float* out, hipStream_t s) {
  return permute3(in, out, x.C, x.hw(), p.B, (long)p.B * x.hw(), 1, x.hw(), s);
}
int unflatten(const Plan& p, const Val& x, const float* in, float* out, hipStream_t s) {
  return permute3(in, out, x.C, p.B, x.hw(), x.hw() * p.B, 1, p.B, s);
}

int resample(const Plan& p, const ganamd_critic_op& op, const Val& x, const float* in, float* out, bool adjoint,
             hipStream_t s) {
  const long planes = (long)x.C * p.B;
  if (!adjoint)
    return ganamd_resample2d(in, planes, x.H, x.W, out, op.n_out, op.n_out, op.ri, op.rw, op.kr, op.ri, op.rw,
                             op.kr, s);
  return ganamd_resample2d(in, planes, op.n_out, op.n_out, out, x.H, x.W, op.ari, op.arw, op.akr, op.ari, op.arw,
                           op.akr, s);
}

const float* wf(const ganamd_critic_op& op) { return op.w_fwd ? op.w_fwd : op.w; }
const float* wd(const ganamd_critic_op& op) { return op.w_dgrad ? op.w_dgrad : op.w; }

// need_stage: 0 forward, 1 backward, 2 tangent, 3 adjoint (the sweep that must have run before,
// and the regions the sweep touches: 0..need_stage)
int check_ws(Plan& p, void* ws, size_t ws_bytes, int need_stage) {
  if (!p.sized) return GANAMD_EINVAL;
  if (ws) {
    if (ws_bytes < p.total) return GANAMD_EINVAL;
    if (need_stage == 0) {                 // one contiguous workspace: carve the four regions
      p.ws = static_cast<char*>(ws);
      size_t o = 0;
      for (int r = 0; r < 4; ++r) {
        p.R[r] = p.ws + o;
        o += p.rsz[r];
      }
    } else if (p.ws != ws) {
      return GANAMD_EINVAL;
    }
  } else {
    if (need_stage == 0) p.ws = nullptr;
    if (p.ws) return GANAMD_EINVAL;        // started contiguous: stays contiguous
    for (int r = 0; r <= need_stage; ++r)
      if (!p.R[r]) return GANAMD_EINVAL;
  }
  if (need_stage > 0 && p.stage < need_stage) return GANAMD_EINVAL;
  return GANAMD_OK;
}

// the stream a weight gradient goes to: the side stream (after a fork from s) or s itself
// (every call forks again: the weight gradient needs the output gradient the sweep has just made)
hipStream_t wstream(Plan& p, hipStream_t s) {
  if (!p.has_events) return s;
  hipStream_t side = p.forked ? p.side : side_stream(s);
  if (!side) return s;
  if (hipEventRecord(p.ev_fork, s) != hipSuccess || hipStreamWaitEvent(side, p.ev_fork, 0) != hipSuccess) return s;
  p.side = side;
  p.forked = true;
  return side;
}
int join(Plan& p, hipStream_t s) {
  if (!p.forked) return GANAMD_OK;
  p.forked = false;
  if (hipEventRecord(p.ev_join, p.side) != hipSuccess) return GANAMD_ELAUNCH;
  return ok(hipStreamWaitEvent(s, p.ev_join, 0));
}

#define TRY(expr)                       \
  do {                                  \
    int rc_ = (expr);                   \
    if (rc_ != GANAMD_OK) return rc_;   \
  } while (0)

}  // namespace

extern "C" {

ganamd_critic_plan* ganamd_critic_create(const ganamd_critic_op* ops, int n_ops, int B, int C0, int H0, int W0,
                                         int segments, int math, int kernel_off) {
  if (!ops || n_ops <= 0 || B <= 0 || C0 <= 0 || H0 <= 0 || W0 <= 0 || segments <= 0 || B % segments) return nullptr;
  if (kernel_off & ~(GANAMD_KERNEL_PATCH_FWD | GANAMD_KERNEL_PATCH_DGRAD | GANAMD_KERNEL_WGRAD_ROW | GANAMD_KERNEL_SMALL))
    return nullptr;
  auto* p = new ganamd_critic_plan();
  p->ops.assign(ops, ops + n_ops);
  p->B = B;
  p->S = segments;
  p->math = math;
  p->kernel_off = kernel_off;
  p->val.resize(n_ops + 1);
  p->input_only.assign(n_ops + 1, 0);
  p->val[0] = Val{C0, H0, W0, (long)C0 * B * H0 * W0};
  p->input_only[0] = 1;
  bool good = true;
  for (int i = 0; i < n_ops && good; ++i) {
    const ganamd_critic_op& op = ops[i];
    auto valid_in = [&](int j) { return op.in[j] >= 0 && op.in[j] <= i; };
    if (!valid_in(0)) { good = false; break; }
    const Val& x = p->val[op.in[0]];
    Val y;
    switch (op.kind) {
      case GANAMD_COP_SWAP:
        good = op.in[0] == 0;
        y = Val{C0, H0, W0, 0};
        p->input_only[i + 1] = 1;
        break;
      case GANAMD_COP_CONV:
        good = op.in[0] != 0 && op.cout > 0 && op.k > 0 && op.stride > 0 && op.pad >= 0 && op.w &&
               x.H + 2 * op.pad >= op.k && x.W + 2 * op.pad >= op.k;
        y = Val{op.cout, (x.H + 2 * op.pad - op.k) / std::max(op.stride, 1) + 1,
                (x.W + 2 * op.pad - op.k) / std::max(op.stride, 1) + 1, 0};
        break;
      case GANAMD_COP_PRELU:
      case GANAMD_COP_SIGMOID:
        good = op.in[0] != 0 && (op.kind != GANAMD_COP_PRELU || op.w);
        y = x;
        break;
      case GANAMD_COP_RESAMPLE:
        good = op.in[0] != 0 && x.H == x.W && op.n_out > 0 && op.ri && op.rw && op.ari && op.arw && op.kr > 0 &&
               op.akr > 0;
        y = Val{x.C, op.n_out, op.n_out, 0};
        break;
      case GANAMD_COP_PMEAN:
        good = op.in[0] != 0;
        y = Val{x.C, 1, 1, 0};
        break;
      case GANAMD_COP_SCALE_ADD: {
        good = op.in[0] != 0 && valid_in(1) && op.in[1] != 0 && (op.in[2] < 0 || (valid_in(2) && op.in[2] != 0));
        if (good) {
          const Val& sv = p->val[op.in[1]];
          good = sv.C == x.C && sv.H == 1 && sv.W == 1;
          if (op.in[2] >= 0) {
            const Val& r = p->val[op.in[2]];
            good = good && r.C == x.C && r.H == x.H && r.W == x.W;
          }
        }
        y = x;
        break;
      }
      case GANAMD_COP_MBSTD:
        good = op.in[0] != 0 && op.group > 0;
        y = Val{x.C + 1, x.H, x.W, 0};
        break;
      case GANAMD_COP_FLATTEN:
        good = op.in[0] != 0;
        y = Val{(int)(x.C * x.hw()), 1, 1, 0};
        break;
      default:
        good = false;
    }
    y.n = (long)y.C * B * y.H * y.W;
    p->val[i + 1] = y;
  }
  p->out = n_ops;
  if (good) {
    const Val& o = p->val[n_ops];
    good = o.C == 1 && o.H == 1 && o.W == 1;
  }
  if (!good) {
    delete p;
    return nullptr;
  }
  for (const Val& v : p->val) p->maxn = std::max(p->maxn, v.n);
  const int nv = n_ops + 1;
  p->X.assign(nv, nullptr);
  p->XD.assign(nv, nullptr);
  for (Sweep* S : {&p->G, &p->A}) {
    S->cur.assign(nv, nullptr);
    S->own.assign(nv, nullptr);
    S->borrowed.assign(nv, 0);
  }
  p->has_events = hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) == hipSuccess;   // else: sequential
  return p;
}

void ganamd_critic_destroy(ganamd_critic_plan* plan) { delete plan; }

int ganamd_critic_workspace(const ganamd_critic_plan* cplan, size_t* bytes) {
  if (!cplan || !bytes) return GANAMD_EINVAL;
  auto* p = const_cast<ganamd_critic_plan*>(cplan);
  if (!p->sized) {
    size_t conv = 0, rr = 0;
    for (int i = 0; i < (int)p->ops.size(); ++i) {
      const ganamd_critic_op& op = p->ops[i];
      const Val& x = p->val[op.in[0]];
      if (op.kind == GANAMD_COP_CONV) {
        size_t b = 0;
        ganamd_conv_desc d = p->desc(i, op.w_fwd != nullptr);
        TRY(ganamd_conv_workspace(&d, GANAMD_CONV_FWD, &b));
        conv = std::max(conv, b);
        d = p->desc(i, op.w_dgrad != nullptr);
        TRY(ganamd_conv_workspace(&d, GANAMD_CONV_DGRAD, &b));
        conv = std::max(conv, b);
        d = p->desc(i, false);
        TRY(ganamd_conv_workspace(&d, GANAMD_CONV_WGRAD, &b));
        conv = std::max(conv, b);
        const Val& y = p->val[i + 1];
        rr = std::max(rr, ganamd_rowreduce_workspace(y.C, (long)p->B * y.hw()));
      } else if (op.kind == GANAMD_COP_PRELU) {
        rr = std::max(rr, ganamd_rowreduce_workspace(x.C, (long)p->B * x.hw()));
      }
    }
    const Val& in = p->val[0];
    const long n0 = (long)in.C * in.hw();
    p->conv_ws = conv;
    p->rr_ws = rr;
    p->mb_ws = ganamd_mbstd_workspace(p->S);
    p->gp_ws = ganamd_gp_workspace(p->B, n0);
    size_t off = 0;
    auto take = [&](size_t nbytes) {
      size_t o = off;
      off += (nbytes + 255) / 256 * 256;
      return o;
    };
    const int nv = (int)p->val.size();
    p->offX.assign(nv, 0);
    p->offG.assign(nv, 0);
    p->offXD.assign(nv, 0);
    p->offA.assign(nv, 0);
    // region 0: scratch, then X
    p->off_tmp = take(p->maxn * sizeof(float));
    p->off_conv = take(conv);
    p->off_rr = take(rr);
    p->off_conv2 = take(conv);
    p->off_rr2 = take(rr);
    p->off_mb = take(p->mb_ws);
    p->off_gp = take(p->gp_ws);
    p->off_ones = take(std::max(p->B, 1) * sizeof(float));
    p->off_v = take(p->val[0].n * sizeof(float));
    p->off_g0 = take(p->val[0].n * sizeof(float));
    p->off_norms = take(p->B * sizeof(float));
    for (int v = 1; v < nv; ++v) p->offX[v] = take(p->val[v].n * sizeof(float));
    p->rsz[0] = off;
    std::vector<size_t>* offs[3] = {&p->offG, &p->offXD, &p->offA};
    for (int r = 1; r < 4; ++r) {
      off = 0;
      for (int v = 1; v < nv; ++v) (*offs[r - 1])[v] = take(p->val[v].n * sizeof(float));
      p->rsz[r] = off;
    }
    p->total = p->rsz[0] + p->rsz[1] + p->rsz[2] + p->rsz[3];
    p->sized = true;
  }
  *bytes = p->total;
  return GANAMD_OK;
}

int ganamd_critic_region_bytes(const ganamd_critic_plan* p, int which, size_t* bytes) {
  size_t total = 0;
  if (!p || !bytes || which < 0 || which > 3) return GANAMD_EINVAL;
  TRY(ganamd_critic_workspace(p, &total));
  *bytes = p->rsz[which];
  return GANAMD_OK;
}

int ganamd_critic_bind(ganamd_critic_plan* p, int which, void* region, size_t region_bytes) {
  if (!p || !region || which < 0 || which > 3 || !p->sized || region_bytes < p->rsz[which]) return GANAMD_EINVAL;
  if (which == 0) {                         // a new evaluation in bound mode
    p->ws = nullptr;
    for (char*& r : p->R) r = nullptr;
    p->stage = 0;
  } else if (p->ws) {
    return GANAMD_EINVAL;                   // the plan runs on a contiguous workspace
  }
  p->R[which] = static_cast<char*>(region);
  return GANAMD_OK;
}

int ganamd_critic_value(const ganamd_critic_plan* p, int which, int v, const float** ptr) {
  if (!p || !ptr || v < 0 || v >= (int)p->val.size() || which < 0 || which > 3) return GANAMD_EINVAL;
  const std::vector<float*>& t = which == 0 ? p->X : which == 1 ? p->G.cur : which == 2 ? p->XD : p->A.cur;
  *ptr = t[v];
  return GANAMD_OK;
}

int ganamd_critic_forward(ganamd_critic_plan* p, const float* x, float* out, void* workspace, size_t workspace_bytes,
                          hipStream_t s) {
  if (!p || !x) return GANAMD_EINVAL;
  TRY(check_ws(*p, workspace, workspace_bytes, 0));
  p->stage = 0;
  p->X[0] = const_cast<float*>(x);
  for (int i = 0; i < (int)p->ops.size(); ++i) {
    const ganamd_critic_op& op = p->ops[i];
    const int v = i + 1;
    const Val& xv = p->val[op.in[0]];
    const float* in = p->X[op.in[0]];
    float* y = p->at(p->offX[v]);
    const long L = (long)p->B * xv.hw();
    switch (op.kind) {
      case GANAMD_COP_SWAP: TRY(swap_in(*p, in, y, s)); break;
      case GANAMD_COP_CONV: {
        ganamd_conv_desc d = p->desc(i, op.w_fwd != nullptr);
        TRY(ganamd_conv_fwd(&d, in, wf(op), op.bias, nullptr, nullptr, op.alpha, y, p->at(p->off_conv), p->conv_ws, s));
        break;
      }
      case GANAMD_COP_PRELU: TRY(ganamd_prelu_fwd(in, op.w, xv.C, L, y, s)); break;
      case GANAMD_COP_RESAMPLE: TRY(resample(*p, op, xv, in, y, false, s)); break;
      case GANAMD_COP_PMEAN:
        if (xv.hw() == 1) y = const_cast<float*>(in);          // a view (nothing to reduce)
        else TRY(ganamd_plane_dot(in, nullptr, (long)xv.C * p->B, xv.hw(), 1.f / xv.hw(), y, s));
        break;
      case GANAMD_COP_SIGMOID: TRY(ganamd_act_fwd(GANAMD_ACT_SIGMOID, in, xv.n, 0.f, y, s)); break;
      case GANAMD_COP_SCALE_ADD:
        TRY(ganamd_scale_add2(in, p->X[op.in[1]], nullptr, nullptr, op.in[2] >= 0 ? p->X[op.in[2]] : nullptr,
                              (long)xv.C * p->B, xv.hw(), y, s));
        break;
      case GANAMD_COP_MBSTD:
        TRY(ganamd_mbstd_fwd(in, L, xv.C, p->B, (int)xv.hw(), p->S, op.group, y, L, nullptr, p->at(p->off_mb), p->mb_ws, s));
        break;
      case GANAMD_COP_FLATTEN: TRY(flatten(*p, xv, in, y, s)); break;
    }
    p->X[v] = y;
  }
  if (out) TRY(ok(hipMemcpyAsync(out, p->X[p->out], p->B * sizeof(float), hipMemcpyDeviceToDevice, s)));
  p->stage = 1;
  return GANAMD_OK;
}

int ganamd_critic_backward(ganamd_critic_plan* p, const float* seed, const ganamd_critic_grads* gr, float* gx,
                           void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (!p) return GANAMD_EINVAL;
  TRY(check_ws(*p, workspace, workspace_bytes, 1));
  Sweep& G = p->G;
  G.reset();
  for (int v = 1; v < (int)p->val.size(); ++v) G.own[v] = p->atr(1, p->offG[v]);
  if (!seed) {
    float* ones = p->at(p->off_ones);
    TRY(fill(ones, p->B, 1.f, s));
    seed = ones;
  }
  G.cur[p->out] = const_cast<float*>(seed);
  G.borrowed[p->out] = 1;
  for (int i = (int)p->ops.size() - 1; i >= 0; --i) {
    const ganamd_critic_op& op = p->ops[i];
    const int v = i + 1;
    float* gy = G.cur[v];
    if (!gy) continue;
    const int u = op.in[0];
    const Val& xv = p->val[u];
    const float* x = p->X[u];
    const long L = (long)p->B * xv.hw();
    float* gw = gr ? gr[i].gw : nullptr;
    float* gb = gr ? gr[i].gb : nullptr;
    switch (op.kind) {
      case GANAMD_COP_SWAP:
        if (gx) TRY(swap_out(*p, gy, gx, s));
        break;
      case GANAMD_COP_CONV: {
        if (!p->input_only[u] || gx) {
          ganamd_conv_desc d = p->desc(i, op.w_dgrad != nullptr);
          TRY(acc(*p, G, u, [&](float* dst) {
            return ganamd_conv_dgrad(&d, gy, wd(op), nullptr, op.alpha, dst, p->at(p->off_conv), p->conv_ws, s);
          }, s));
        }
        const Val& yv = p->val[v];
        if (gw || gb) {
          const hipStream_t ws = wstream(*p, s);
          const bool sd = ws != s;
          if (gw) {
            ganamd_conv_desc d = p->desc(i, false);
            TRY(ganamd_conv_wgrad(&d, x, gy, nullptr, nullptr, op.alpha, gw, 1, p->at(sd ? p->off_conv2 : p->off_conv), p->conv_ws,
                                  ws));
          }
          if (gb) TRY(ganamd_row_dot(gy, nullptr, yv.C, (long)p->B * yv.hw(), gb, 1, p->at(sd ? p->off_rr2 : p->off_rr), p->rr_ws, ws));
        }
        break;
      }
      case GANAMD_COP_PRELU:
        TRY(acc(*p, G, u, [&](float* dst) {
          return ganamd_prelu_bwd(gy, x, op.w, xv.C, L, dst, gw, 1, p->at(p->off_rr), p->rr_ws, s);
        }, s));
        break;
      case GANAMD_COP_RESAMPLE:
        TRY(acc(*p, G, u, [&](float* dst) { return resample(*p, op, xv, gy, dst, true, s); }, s));
        break;
      case GANAMD_COP_PMEAN:
        if (xv.hw() == 1) {
          TRY(acc_borrow(*p, G, u, gy, s));
        } else {
          TRY(acc(*p, G, u, [&](float* dst) {
            plane_bcast_kernel<<<grid_for(xv.n), kNT, 0, s>>>(gy, (long)xv.C * p->B, xv.hw(), 1.f / xv.hw(), dst);
            return ok(hipGetLastError());
          }, s));
        }
        break;
      case GANAMD_COP_SIGMOID:
        TRY(acc(*p, G, u, [&](float* dst) {
          return ganamd_act_bwd(GANAMD_ACT_SIGMOID, p->X[v], gy, xv.n, 0.f, dst, s);
        }, s));
        break;
      case GANAMD_COP_SCALE_ADD: {
        const int xi = op.in[0], si = op.in[1], ri = op.in[2];
        const long P = (long)xv.C * p->B;
        TRY(acc(*p, G, xi, [&](float* dst) {
          return ganamd_scale_add2(gy, p->X[si], nullptr, nullptr, nullptr, P, xv.hw(), dst, s);
        }, s));
        TRY(acc(*p, G, si, [&](float* dst) {
          return ganamd_plane_dot2(gy, p->X[xi], nullptr, nullptr, P, xv.hw(), dst, s);
        }, s));
        if (ri >= 0) TRY(acc_borrow(*p, G, ri, gy, s));
        break;
      }
      case GANAMD_COP_MBSTD:
        TRY(acc(*p, G, u, [&](float* dst) {
          return ganamd_mbstd_bwd(x, L, gy, L, xv.C, p->B, (int)xv.hw(), p->S, op.group, dst, p->at(p->off_mb), p->mb_ws, s);
        }, s));
        break;
      case GANAMD_COP_FLATTEN:
        TRY(acc(*p, G, u, [&](float* dst) { return unflatten(*p, xv, gy, dst, s); }, s));
        break;
    }
  }
  TRY(join(*p, s));
  p->stage = 2;
  return GANAMD_OK;
}

int ganamd_critic_tangent(ganamd_critic_plan* p, const float* vdir, const ganamd_critic_grads* gr, void* workspace,
                          size_t workspace_bytes, hipStream_t s) {
  if (!p || !vdir) return GANAMD_EINVAL;
  TRY(check_ws(*p, workspace, workspace_bytes, 2));
  p->XD[0] = const_cast<float*>(vdir);
  for (int i = 0; i < (int)p->ops.size(); ++i) {
    const ganamd_critic_op& op = p->ops[i];
    const int v = i + 1;
    const Val& xv = p->val[op.in[0]];
    const float* xd = p->XD[op.in[0]];
    const float* x = p->X[op.in[0]];
    float* y = p->atr(2, p->offXD[v]);
    const long L = (long)p->B * xv.hw();
    switch (op.kind) {
      case GANAMD_COP_SWAP: TRY(swap_in(*p, xd, y, s)); break;
      case GANAMD_COP_CONV: {
        ganamd_conv_desc d = p->desc(i, op.w_fwd != nullptr);
        TRY(ganamd_conv_fwd(&d, xd, wf(op), nullptr, nullptr, nullptr, op.alpha, y, p->at(p->off_conv), p->conv_ws, s));
        break;
      }
      case GANAMD_COP_PRELU: {
        float* gy = p->G.cur[v];
        float* gw = (gr && gy) ? gr[i].gw : nullptr;
        TRY(ganamd_prelu_tangent(xd, gy ? gy : xd, x, op.w, xv.C, L, y, gw, 1, p->at(p->off_rr), p->rr_ws, s));
        break;
      }
      case GANAMD_COP_RESAMPLE: TRY(resample(*p, op, xv, xd, y, false, s)); break;
      case GANAMD_COP_PMEAN:
        if (xv.hw() == 1) y = const_cast<float*>(xd);
        else TRY(ganamd_plane_dot(xd, nullptr, (long)xv.C * p->B, xv.hw(), 1.f / xv.hw(), y, s));
        break;
      case GANAMD_COP_SIGMOID: TRY(ganamd_act_bwd(GANAMD_ACT_SIGMOID, p->X[v], xd, xv.n, 0.f, y, s)); break;
      case GANAMD_COP_SCALE_ADD: {
        const int xi = op.in[0], si = op.in[1], ri = op.in[2];
        TRY(ganamd_scale_add2(p->XD[xi], p->X[si], p->X[xi], p->XD[si], ri >= 0 ? p->XD[ri] : nullptr,
                              (long)xv.C * p->B, xv.hw(), y, s));
        break;
      }
      case GANAMD_COP_MBSTD:
        TRY(ganamd_mbstd_tangent(x, xd, L, xv.C, p->B, (int)xv.hw(), p->S, op.group, y, L, p->at(p->off_mb), p->mb_ws, s));
        break;
      case GANAMD_COP_FLATTEN: TRY(flatten(*p, xv, xd, y, s)); break;
    }
    p->XD[v] = y;
  }
  p->stage = 3;
  return GANAMD_OK;
}

int ganamd_critic_adjoint(ganamd_critic_plan* p, const float* a_seed, const ganamd_critic_grads* gr, float* ax,
                          void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (!p) return GANAMD_EINVAL;
  TRY(check_ws(*p, workspace, workspace_bytes, 3));
  Sweep& A = p->A;
  A.reset();
  for (int v = 1; v < (int)p->val.size(); ++v) A.own[v] = p->atr(3, p->offA[v]);
  if (a_seed) {
    A.cur[p->out] = const_cast<float*>(a_seed);
    A.borrowed[p->out] = 1;
  }
  for (int i = (int)p->ops.size() - 1; i >= 0; --i) {
    const ganamd_critic_op& op = p->ops[i];
    const int v = i + 1;
    float* ay = A.cur[v];
    float* gy = p->G.cur[v];
    const int u = op.in[0];
    const Val& xv = p->val[u];
    const float* x = p->X[u];
    const long L = (long)p->B * xv.hw();
    float* gw = gr ? gr[i].gw : nullptr;
    float* gb = gr ? gr[i].gb : nullptr;
    switch (op.kind) {
      case GANAMD_COP_SWAP:
        if (ax && ay) TRY(swap_out(*p, ay, ax, s));
        break;
      case GANAMD_COP_CONV: {
        if (ay && (!p->input_only[u] || ax)) {
          ganamd_conv_desc d = p->desc(i, op.w_dgrad != nullptr);
          TRY(acc(*p, A, u, [&](float* dst) {
            return ganamd_conv_dgrad(&d, ay, wd(op), nullptr, op.alpha, dst, p->at(p->off_conv), p->conv_ws, s);
          }, s));
        }
        ganamd_conv_desc d = p->desc(i, false);
        const Val& yv = p->val[v];
        // dW += wgrad(X_in, A_out) + wgrad(XD_in, G_out): one GEMM over both pixel ranges
        if ((gw && (ay || gy)) || (gb && ay)) {
          const hipStream_t ws = wstream(*p, s);
          float* cw = p->at(ws != s ? p->off_conv2 : p->off_conv);
          if (gw && ay && gy)
            TRY(ganamd_conv_wgrad2(&d, x, ay, p->XD[u], gy, op.alpha, gw, 1, cw, p->conv_ws, ws));
          else if (gw)
            TRY(ganamd_conv_wgrad(&d, ay ? x : p->XD[u], ay ? ay : gy, nullptr, nullptr, op.alpha, gw, 1, cw, p->conv_ws, ws));
          if (gb && ay)
            TRY(ganamd_row_dot(ay, nullptr, yv.C, (long)p->B * yv.hw(), gb, 1, p->at(ws != s ? p->off_rr2 : p->off_rr), p->rr_ws,
                               ws));
        }
        break;
      }
      case GANAMD_COP_PRELU:
        if (ay)
          TRY(acc(*p, A, u, [&](float* dst) {
            return ganamd_prelu_bwd(ay, x, op.w, xv.C, L, dst, gw, 1, p->at(p->off_rr), p->rr_ws, s);
          }, s));
        break;
      case GANAMD_COP_RESAMPLE:
        if (ay) TRY(acc(*p, A, u, [&](float* dst) { return resample(*p, op, xv, ay, dst, true, s); }, s));
        break;
      case GANAMD_COP_PMEAN:
        if (!ay) break;
        if (xv.hw() == 1) {
          TRY(acc_borrow(*p, A, u, ay, s));
        } else {
          TRY(acc(*p, A, u, [&](float* dst) {
            plane_bcast_kernel<<<grid_for(xv.n), kNT, 0, s>>>(ay, (long)xv.C * p->B, xv.hw(), 1.f / xv.hw(), dst);
            return ok(hipGetLastError());
          }, s));
        }
        break;
      case GANAMD_COP_SIGMOID:
        if (!gy) {
          if (ay)
            TRY(acc(*p, A, u, [&](float* dst) {
              return ganamd_act_bwd(GANAMD_ACT_SIGMOID, p->X[v], ay, xv.n, 0.f, dst, s);
            }, s));
          break;
        }
        if (!ay) {
          ay = A.own[v];
          TRY(ok(hipMemsetAsync(ay, 0, xv.n * sizeof(float), s)));
        }
        TRY(acc(*p, A, u, [&](float* dst) {
          return ganamd_act_adjoint(GANAMD_ACT_SIGMOID, p->X[v], ay, gy, p->XD[u], xv.n, 0.f, dst, s);
        }, s));
        break;
      case GANAMD_COP_SCALE_ADD: {
        const int xi = op.in[0], si = op.in[1], ri = op.in[2];
        const long P = (long)xv.C * p->B;
        if (!ay && !gy) break;
        if (!ay) {
          TRY(acc(*p, A, xi, [&](float* dst) {
            return ganamd_scale_add2(gy, p->XD[si], nullptr, nullptr, nullptr, P, xv.hw(), dst, s);
          }, s));
          TRY(acc(*p, A, si, [&](float* dst) {
            return ganamd_plane_dot2(gy, p->XD[xi], nullptr, nullptr, P, xv.hw(), dst, s);
          }, s));
        } else {
          TRY(acc(*p, A, xi, [&](float* dst) {
            return ganamd_scale_add2(ay, p->X[si], gy, gy ? p->XD[si] : nullptr, nullptr, P, xv.hw(), dst, s);
          }, s));
          TRY(acc(*p, A, si, [&](float* dst) {
            return ganamd_plane_dot2(ay, p->X[xi], gy, gy ? p->XD[xi] : nullptr, P, xv.hw(), dst, s);
          }, s));
          if (ri >= 0) TRY(acc_borrow(*p, A, ri, ay, s));
        }
        break;
      }
      case GANAMD_COP_MBSTD: {
        if (!ay && !gy) break;
        const Val& yv = p->val[v];
        if (!ay) {
          ay = A.own[v];
          TRY(ok(hipMemsetAsync(ay, 0, yv.n * sizeof(float), s)));
        }
        if (!gy) {
          TRY(acc(*p, A, u, [&](float* dst) {
            return ganamd_mbstd_bwd(x, L, ay, L, xv.C, p->B, (int)xv.hw(), p->S, op.group, dst, p->at(p->off_mb), p->mb_ws, s);
          }, s));
          break;
        }
        TRY(acc(*p, A, u, [&](float* dst) {
          return ganamd_mbstd_adjoint(x, p->XD[u], L, gy, ay, L, xv.C, p->B, (int)xv.hw(), p->S, op.group, dst,
                                      p->at(p->off_mb), p->mb_ws, s);
        }, s));
        break;
      }
      case GANAMD_COP_FLATTEN:
        if (ay) TRY(acc(*p, A, u, [&](float* dst) { return unflatten(*p, xv, ay, dst, s); }, s));
        break;
    }
  }
  return join(*p, s);
}

int ganamd_critic_gp_step(ganamd_critic_plan* p, const float* x, float center, float lambda, int mode,
                          const ganamd_critic_grads* gr, float* out, float* gx, float* norms, float* penalty,
                          void* workspace, size_t workspace_bytes, hipStream_t s) {
  if (!p || !x || !penalty || (mode != 0 && mode != 1)) return GANAMD_EINVAL;
  TRY(ganamd_critic_forward(p, x, out, workspace, workspace_bytes, s));
  float* g = gx ? gx : p->at(p->off_g0);
  TRY(ganamd_critic_backward(p, nullptr, nullptr, g, workspace, workspace_bytes, s));
  const Val& in = p->val[0];
  const long n = (long)in.C * in.hw();
  float* nrm = norms ? norms : p->at(p->off_norms);
  float* v = p->at(p->off_v);
  TRY(ganamd_gp_fwd(g, p->B, n, center, lambda, mode, nrm, penalty, p->at(p->off_gp), p->gp_ws, s));
  // gout = 1: the ones the backward's seed left at off_ones (B >= 1 of them)
  TRY(ganamd_gp_bwd(g, nrm, p->at(p->off_ones), p->B, n, center, lambda, mode, v, s));
  TRY(ganamd_critic_tangent(p, v, gr, workspace, workspace_bytes, s));
  return ganamd_critic_adjoint(p, nullptr, gr, nullptr, workspace, workspace_bytes, s);
}

}  // extern "C"
