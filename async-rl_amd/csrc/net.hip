// A3C FF / LSTM network on gfx950: batched-env forward, lockstep-window
// backward, parameter layout and workspace layout.
//
// Reference: a3c_ale.py:28-70 (A3CFF, A3CLSTM), dqn_head.py:31-52
// (NIPSDQNHead: conv 4->16 k8 s4, conv 16->32 k4 s2, Linear 2592->256, ReLU
// after each), policy.py:32-58, v_function.py:10-34, Chainer 1.8.1 L.LSTM /
// F.lstm (interleaved a,i,f,o gates), a3c.py:129-130 (backward of the window
// loss), a3c.py:144 (unchain_backward: truncated BPTT at the window edge).
//
// The window's launches in order (the kernels live in their own files):
// forward per step t: phi_ring (phi.hip) -> conv_fwd (conv_fwd.hip) -> fc_fwd
// (fc.hip) -> policy_fc (FF) or the LSTM gate kernel + policy (lstm.hip,
// policy.hip); learner: returns + heads dh (policy.hip), [LSTM BPTT + gate
// weight gradients], fc_bwd (fc_bwd.hip), conv_bwd + its slab reduce
// (conv_bwd.hip), then clip + RMSProp + the window advance (optim.hip).  The
// f32-state forward (pi_and_v) and the ARCH_STATES / Nature convolutions run on
// the generic implicit-GEMM template (gemm.hpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "arl_internal.hpp"
#include "gemm.hpp"
#include "layers.hpp"

namespace arl {

// ---------------------------------------------------------------- accessors

// (conv1 from the uint8 frame ring has dedicated kernels: conv1.hip)
struct Conv1F32A {      // same from an f32 (n,C,84,84) state tensor (dqn_phi output; C = 3 for RGB)
  const float* __restrict__ x;
  int C;
  __device__ float load(int m, int k) const {
    const int s = m / C1_P, p = m - s * C1_P;
    const int ic = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
    const int oy = p / 20, ox = p - oy * 20;
    return x[((int64_t)s * C + ic) * PLANE + (4 * oy + ky) * 84 + 4 * ox + kx];
  }
};
struct Conv2A {         // A(m, k) = a1[s][ic][2oy+ky][2ox+kx], m = s*81 + p, k = ic*16+ky*4+kx
  const float* __restrict__ a1;
  __device__ float load(int m, int k) const {
    const int s = m / C2_P, p = m - s * C2_P;
    const int oy = p / 9, ox = p - oy * 9;
    const int ic = k >> 4, ky = (k >> 2) & 3, kx = k & 3;
    return a1[(int64_t)s * A1 + ic * C1_P + (2 * oy + ky) * 20 + 2 * ox + kx];
  }
};
#define ARL_TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

// Where the LSTM step's FC split-K partials are reduced: in the gate kernel's staging (XRED) for
// launches under 512 envs, by the FC's last-arriver ticket for 512 and more (fc_fwd_big_kernel's
// tail; the gate kernel then stages hfc: every one of its 16 column-tile workgroups of a row block
// otherwise re-reads the block's 8 partial slabs -- C3 1.185 -> 1.160 ms, profiles/r03/r3aa).
// ARL_LSTM_XRED=1 / 0 forces one form (the bitwise arm of test_lstm_fc_ticket_big_tiles_identical).
static const int LSTM_XRED_ENV = [] {
  const char* e = getenv("ARL_LSTM_XRED");
  return e == nullptr ? -1 : (e[0] != '0' ? 1 : 0);
}();
static bool lstm_xred(int launch_envs) { return LSTM_XRED_ENV >= 0 ? LSTM_XRED_ENV == 1 : launch_envs < 512; }

// ---------------------------------------------------------------- elementwise
__device__ inline float sigm(float x) { return __fdiv_rn(1.f, __fadd_rn(1.f, expf(-x))); }

// F.lstm backward of element i = (m, unit) at step t: dh = dL/dh_t (heads +
// carried), dcn in: dc carried from t+1 (first: none), out: dc carried to t-1.
__device__ inline void lstm_cell_bwd_elem(const float* __restrict__ gates, const float* __restrict__ c_t,
                                          const float* __restrict__ c_prev, bool rs, float dh, float* __restrict__ dcn,
                                          float* __restrict__ dG, bool first, int64_t i) {
  const float4 g = reinterpret_cast<const float4*>(gates)[i];
  const float a = tanhf(g.x), ig = sigm(g.y), fg = sigm(g.z), og = sigm(g.w);
  const float c = c_t[i];
  const float tc = tanhf(c);
  float dc = __fmul_rn(__fmul_rn(dh, og), __fsub_rn(1.f, __fmul_rn(tc, tc)));
  if (!first) dc = __fadd_rn(dc, dcn[i]);
  const float cp = rs ? 0.f : c_prev[i];
  float4 d;
  d.x = __fmul_rn(__fmul_rn(dc, ig), __fsub_rn(1.f, __fmul_rn(a, a)));
  d.y = __fmul_rn(__fmul_rn(__fmul_rn(dc, a), ig), __fsub_rn(1.f, ig));
  d.z = __fmul_rn(__fmul_rn(__fmul_rn(dc, cp), fg), __fsub_rn(1.f, fg));
  d.w = __fmul_rn(__fmul_rn(__fmul_rn(dh, tc), og), __fsub_rn(1.f, og));
  reinterpret_cast<float4*>(dG)[i] = d;
  dcn[i] = rs ? 0.f : __fmul_rn(dc, fg);
}

// F.lstm backward for step t.  dH: dL/dh_t from the heads; dhn/dcn: carried
// from step t+1 (ignored when first); writes dG (interleaved) and dcn for t-1.
__global__ void lstm_cell_bwd_kernel(const float* __restrict__ gates, const float* __restrict__ c_t,
                                     const float* __restrict__ c_prev, const uint8_t* __restrict__ reset,
                                     const float* __restrict__ dH, const float* __restrict__ dhn,
                                     float* __restrict__ dcn, float* __restrict__ dG, int first, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t m = i / HID;
  const float dh = first ? dH[i] : __fadd_rn(dH[i], dhn[i]);
  lstm_cell_bwd_elem(gates, c_t, c_prev, reset[m] != 0, dh, dcn, dG, first != 0, i);
}

// dh[s][j] = sum_k dlogits[s][k] Wpi[k][j] + dv[s] Wv[j]; with mask: * (h > 0)
__global__ void heads_bwd_kernel(const float* __restrict__ dl, const float* __restrict__ dv,
                                 const float* __restrict__ Wpi, const float* __restrict__ Wv, int A, int H,
                                 const float* __restrict__ mask, float* __restrict__ out, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t s = i / H;
  const int j = (int)(i - s * H);
  float acc = 0.f;
  for (int k = 0; k < A; ++k) acc = __fadd_rn(acc, __fmul_rn(dl[s * A + k], Wpi[k * H + j]));
  acc = __fadd_rn(acc, __fmul_rn(dv[s], Wv[j]));
  if (mask) acc = mask[i] > 0.f ? acc : 0.f;
  out[i] = acc;
}

hipError_t launch_heads_bwd(const float* dl, const float* dv, const float* Wpi, const float* Wv, int A, int H,
                            const float* mask, float* out, int64_t S, hipStream_t s) {
  const int64_t cnt = S * H;
  hipLaunchKernelGGL(heads_bwd_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, dl, dv, Wpi, Wv, A, H,
                     mask, out, cnt);
  return hipGetLastError();
}

__global__ void advance_kernel(int64_t* ctl, int T, uint8_t* reset, int n, float* hbuf, float* cbuf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) reset[i] = reset[(int64_t)T * n + i];
  if (hbuf != nullptr && i < (int64_t)n * HID) {
    hbuf[i] = hbuf[(int64_t)T * n * HID + i];
    cbuf[i] = cbuf[(int64_t)T * n * HID + i];
  }
  if (i == 0) {
    ctl[CTL_STEP] += T;
    ctl[CTL_WINDOW] += 1;
  }
}

static int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

bool net_init(Net& net, int arch, int n_actions, int n_envs, int t_max, int env_offset, uint64_t seed,
              std::string& err) {
  const bool rgb = (arch & ARCH_RGB) != 0;
  const bool stk = (arch & ARCH_STACK) != 0;
  const bool sts = (arch & ARCH_STATES) != 0;
  arch &= ~(ARCH_RGB | ARCH_STACK | ARCH_STATES);
  if ((rgb || stk || sts) && arch == ARCH_FF_NATURE) {
    err = "ARCH_RGB / ARCH_STACK / ARCH_STATES apply to the NIPS head (FF or LSTM) only";
    return false;
  }
  if ((int)rgb + (int)stk + (int)sts > 1) { err = "ARCH_RGB, ARCH_STACK and ARCH_STATES are exclusive"; return false; }
  net.rgb = rgb;
  net.stack = stk;
  net.states = sts;
  net.layout = rgb ? FRAMES_RGB : stk ? FRAMES_STACK : sts ? FRAMES_STATES : FRAMES_RING;
  if (arch != ARCH_FF && arch != ARCH_LSTM && arch != ARCH_FF_NATURE) {
    err = "arch must be 0 (FF), 1 (LSTM) or 2 (FF, Nature head), optionally | 16 (RGB), | 32 (STACK) or | 64 (STATES)";
    return false;
  }
  if (n_actions < 1 || n_actions > MAXA) { err = "n_actions must be in [1, 32]"; return false; }
  if (n_envs < 1 || n_envs > (1 << 20)) { err = "n_envs out of range"; return false; }
  if (t_max < 1 || t_max > 64) { err = "t_max must be in [1, 64]"; return false; }
  if ((int64_t)t_max * n_envs * C1_P >= (int64_t)1 << 31) { err = "t_max * n_envs too large"; return false; }
  net.arch = arch; net.A = n_actions; net.N = n_envs; net.T = t_max; net.R = t_max + 4;
  net.env_offset = env_offset; net.seed = seed;
  const bool NAT = arch == ARCH_FF_NATURE;
  net.hid = NAT ? NHID : HID;
  // ---- parameters, Chainer link order (a3c_ale.py:35,52)
  net.params.clear();
  int64_t off = 0;
  auto add = [&](const char* name, int64_t numel) {
    ParamInfo pi; pi.name = name; pi.offset = off; pi.numel = numel;
    net.params.push_back(pi);
    off = align_up(off + numel, 64);
    return pi.offset;
  };
  net.o_luW = net.o_lub = net.o_llW = net.o_c3W = net.o_c3b = -1;
  if (NAT) {   // dqn_head.py:16-20, then FCSoftmaxPolicy(512) / FCVFunction(512)
    net.o_c1W = add("0/0/W", NC1 * 4 * 8 * 8);
    net.o_c1b = add("0/0/b", NC1);
    net.o_c2W = add("0/1/W", NC2 * NC1 * 4 * 4);
    net.o_c2b = add("0/1/b", NC2);
    net.o_c3W = add("0/2/W", NC3 * NC2 * 3 * 3);
    net.o_c3b = add("0/2/b", NC3);
    net.o_fcW = add("0/3/W", (int64_t)NHID * NA3);
    net.o_fcb = add("0/3/b", NHID);
    net.o_piW = add("1/0/W", (int64_t)n_actions * NHID);
    net.o_pib = add("1/0/b", n_actions);
    net.o_vW = add("2/0/W", NHID);
    net.o_vb = add("2/0/b", 1);
  } else {
    net.o_c1W = add("0/0/W", 16 * (rgb ? 3 : 4) * 8 * 8);
    net.o_c1b = add("0/0/b", 16);
    net.o_c2W = add("0/1/W", 32 * 16 * 4 * 4);
    net.o_c2b = add("0/1/b", 32);
    net.o_fcW = add("0/2/W", (int64_t)HID * A2);
    net.o_fcb = add("0/2/b", HID);
  }
  if (arch == ARCH_FF) {
    net.o_piW = add("1/0/W", (int64_t)n_actions * HID);
    net.o_pib = add("1/0/b", n_actions);
    net.o_vW = add("2/0/W", HID);
    net.o_vb = add("2/0/b", 1);
  } else if (arch == ARCH_LSTM) {
    net.o_luW = add("1/upward/W", (int64_t)GATES * HID);
    net.o_lub = add("1/upward/b", GATES);
    net.o_llW = add("1/lateral/W", (int64_t)GATES * HID);
    net.o_piW = add("2/0/W", (int64_t)n_actions * HID);
    net.o_pib = add("2/0/b", n_actions);
    net.o_vW = add("3/0/W", HID);
    net.o_vb = add("3/0/b", 1);
  }
  net.param_floats = off;
  // ---- workspace
  const int64_t n = n_envs, T = t_max, T1 = T + 1, S = T * n, A = n_actions;
  net.norm_blocks = 256;
  int64_t slab = 0;
  slab = std::max(slab, (int64_t)FC_SPLIT * n * HID);
  slab = std::max(slab, conv_bwd_slab_floats((int)S));
  if (NAT) slab = nature_slab_floats(net);
  if (sts) slab = std::max(slab, states_slab_floats(net));
  net.slab_floats = slab;
  net.bufs.clear();
  int64_t wo = 0;
  auto buf = [&](const char* name, int64_t bytes) {
    Net::Buf b; b.name = name; b.off = wo; b.bytes = bytes;
    net.bufs.push_back(b);
    wo = align_up(wo + std::max<int64_t>(bytes, 1), 256);
    return b.off;
  };
  const bool L = arch == ARCH_LSTM;
  net.w_ctl = buf("ctl", CTL_SIZE * 8);
  net.w_frames = buf("frames", (int64_t)net.R * n * PLANE * (rgb ? 3 : stk ? 4 : sts ? 16 : 1));
  net.w_nvalid = buf("nvalid", (int64_t)net.R * n);
  net.w_reset = buf("reset", T1 * n);
  net.w_rewards = buf("rewards", S * 4);
  net.w_dones = buf("dones", S);
  const int64_t H = net.hid, nA1 = NAT ? NA1 : A1, nA2 = NAT ? NA2 : A2;
  net.w_a1 = buf("a1", T1 * n * nA1 * 4);
  net.w_a2 = buf("a2", T1 * n * nA2 * 4);
  // the FC backward's ReLU mask as bits, written by conv_fwd.hip (its f32-state / Nature paths write none)
  net.w_a2m = buf("a2_mask", (NAT || sts) ? 0 : T1 * n * A2W * 4);
  net.w_a3 = buf("a3", NAT ? T1 * n * NA3 * 4 : 0);
  net.w_hfc = buf("hfc", T1 * n * H * 4);
  net.w_gates = buf("gates", L ? T1 * n * GATES * 4 : 0);
  net.w_hbuf = buf("hbuf", L ? (T + 2) * n * HID * 4 : 0);
  net.w_cbuf = buf("cbuf", L ? (T + 2) * n * HID * 4 : 0);
  net.w_logits = buf("logits", T1 * n * A * 4);
  net.w_probs = buf("probs", T1 * n * A * 4);
  net.w_logp = buf("logp", T1 * n * A * 4);
  net.w_v = buf("v", T1 * n * 4);
  net.w_ent = buf("entropy", T1 * n * 4);
  net.w_logpa = buf("logp_a", T1 * n * 4);
  net.w_act = buf("actions", T1 * n * 4);
  net.w_dlogits = buf("dlogits", S * A * 4);
  net.w_dv = buf("dv", S * 4);
  net.w_dh = buf("dh", L ? S * HID * 4 : 0);
  net.w_dfc = buf("dfc", S * H * 4);
  net.w_dG = buf("dG", L ? S * GATES * 4 : 0);
  net.w_dhn = buf("dhn", L ? n * HID * 4 : 0);
  net.w_dcn = buf("dcn", L ? n * HID * 4 : 0);
  net.w_da2 = buf("da2", S * nA2 * 4);
  net.w_da1 = buf("da1", NAT ? S * NA1 * 4 : sts ? S * A1 * 4 : 0);
  net.w_da3 = buf("da3", NAT ? S * NA3 * 4 : 0);
  net.w_slab = buf("slab", slab * 4);
  net.w_norm = buf("norm_partials", (int64_t)NORM_SCRATCH * 8);   // partials, result, ticket (arl_internal.hpp)
  net.w_tick = buf("tickets", (int64_t)fc_fwd_tiles((int)n) * 4);
  net.w_fcb_part = buf("fc_bwd_partials", NAT ? 0 : fc_bwd_part_floats((int)S) * 4);
  net.w_fcb_tick = buf("fc_bwd_tickets", NAT ? 0 : (int64_t)fc_bwd_tickets() * 4);
  net.w_loss = buf("loss", n * 2 * 4);
  net.w_eval_h = buf("eval_h", L ? n * HID * 4 : 0);
  net.w_eval_c = buf("eval_c", L ? n * HID * 4 : 0);
  net.w_eval_hn = buf("eval_hn", L ? n * HID * 4 : 0);
  net.w_eval_cn = buf("eval_cn", L ? n * HID * 4 : 0);
  net.w_eval_reset = buf("eval_reset", L ? n : 0);
  net.w_zero = buf("zero_row", L ? ZERO_ROW_FLOATS * 4 : 0);
  net.w_fcplanes = buf("fc_planes", NAT ? 0 : FC_PLANES_BYTES);
  net.ws_bytes = wo;
  return true;
}

// ---------------------------------------------------------------- forward

// a2 > 0 bits of window slot t (conv_fwd.hip writes them, fc_bwd.hip's job B reads them as its ReLU
// mask); null for the nets whose conv forward is not conv_fwd.hip (Nature, f32 states)
static uint32_t* a2_mask(const Net& net, int t) {
  if (net.arch == ARCH_FF_NATURE || net.states) return nullptr;
  return net.at<uint32_t>(net.w_a2m) + (int64_t)t * net.N * A2W;
}

// the FC weight's split planes (fc.hip): rebuilt from the params when a writer bumped the parameter
// generation since they were built (bind, arl_net_params_changed); every update keeps them current
hipError_t ensure_fc_planes(Net& net, hipStream_t s) {
  if (net.planes_current() || net.arch == ARCH_FF_NATURE) return hipSuccess;
  ARL_TRY(launch_fc_planes(net.p + net.o_fcW, net.at<uint16_t>(net.w_fcplanes), s));
  net.planes_gen = net.param_gen;
  return hipSuccess;
}
static const uint16_t* fc_planes(const Net& net) { return net.at<uint16_t>(net.w_fcplanes); }

// head after conv1 (conv2 -> fc) for n rows, activations at a1/a2/hfc
static hipError_t fc_forward(const Net& net, int n, const float* a2, float* hfc, hipStream_t s) {
  return launch_fc_fwd(a2, n, fc_planes(net), net.p + net.o_fcb, net.at<float>(net.w_slab), net.at<int>(net.w_tick),
                       hfc, s);
}

// policy / value heads of window slot t (rows n of env 0..n-1) reading h
static PolicyArgs slot_policy_args(const Net& net, int t, int mode) {
  const float* P = net.p;
  const int A = net.A;
  const int64_t o = (int64_t)t * net.N;
  return make_policy_args(P + net.o_piW, P + net.o_pib, P + net.o_vW, P + net.o_vb, A, net.seed,
                          net.at<int64_t>(net.w_ctl), t, net.env_offset, mode, net.at<float>(net.w_logits) + o * A,
                          net.at<float>(net.w_probs) + o * A, net.at<float>(net.w_logp) + o * A,
                          net.at<float>(net.w_v) + o, net.at<float>(net.w_ent) + o, net.at<int32_t>(net.w_act) + o,
                          net.at<float>(net.w_logpa) + o);
}

// One lockstep step (conv -> fc [-> LSTM] -> policy) for envs [e0, e0 + ne)
// of window slot t.  Disjoint env ranges touch disjoint rows of every buffer
// (the FC split-K slab and tickets included: e0 is a multiple of the FC's
// 32-row tile), so ranges can run concurrently on separate streams.
hipError_t net_act(Net& net, int t, int mode, hipStream_t s, int e0, int ne) {
  if (ne < 0) {
    e0 = 0;
    ne = net.N;
  }
  if (net.arch == ARCH_FF_NATURE) {
    if (e0 != 0 || ne != net.N || mode > 2) return hipErrorInvalidValue;
    return nature_act(net, t, mode, s);
  }
  const int n = net.N, A = net.A;
  const int part = mode & (ACT_CONV_ONLY | ACT_AFTER_CONV);
  mode &= 3;
  // an env range forks from the caller's stream: stale planes rebuilt on one chain's stream would race
  // the other chains' FC reads (the ABI refuses that case first, arl_act_envs)
  if (ne != n && !net.planes_current()) return hipErrorNotReady;
  ARL_TRY(ensure_fc_planes(net, s));
  // a fused bootstrap launch whose learn never followed (a dropped window) must not make a later
  // window's learn skip its returns: any act of a window's step t < T starts a new window
  if (t < net.T) net.returns_done = false;
  // the bootstrap slot T feeds only the FC / heads forward: no backward reads its a1 or a2 mask
  // (the ring-frame conv kernels skip those stores: 25.6 KB an env)
  float* a1 = net.at<float>(net.w_a1) + (int64_t)t * n * A1;
  float* a1_bwd = t < net.T ? a1 : nullptr;
  uint32_t* mask_bwd = t < net.T ? a2_mask(net, t) : nullptr;
  float* a2 = net.at<float>(net.w_a2) + (int64_t)t * n * A2;
  float* hfc = net.at<float>(net.w_hfc) + ((int64_t)t * n + e0) * HID;
  const float* P = net.p;
  if (!(part & ACT_AFTER_CONV) && net.states) {
    if (e0 != 0 || ne != n) return hipErrorInvalidValue;   // one launch over all envs
    ARL_TRY(states_conv_fwd(net, t, a1, a2, s));
    ARL_TRY(stamp(net, STAGE_CONV_FWD, s));
  } else if (!(part & ACT_AFTER_CONV)) {
    ARL_TRY(launch_conv_fwd(net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid),
                            net.at<int64_t>(net.w_ctl), n, net.R, t, P + net.o_c1W, P + net.o_c1b, P + net.o_c2W,
                            P + net.o_c2b, a1_bwd, a2, s, net.layout, e0, ne, mask_bwd));
    ARL_TRY(stamp(net, STAGE_CONV_FWD, s));
  }
  if (part & ACT_CONV_ONLY) return hipSuccess;
  const int64_t o = (int64_t)t * n + e0;
  float* fc_slab = net.at<float>(net.w_slab) + (int64_t)FC_SPLIT * e0 * HID;
  const PolicyArgs pa = make_policy_args(P + net.o_piW, P + net.o_pib, P + net.o_vW, P + net.o_vb, A, net.seed,
                                         net.at<int64_t>(net.w_ctl), t, net.env_offset + e0, t < net.T ? mode : 0,
                                         net.at<float>(net.w_logits) + o * A, net.at<float>(net.w_probs) + o * A,
                                         net.at<float>(net.w_logp) + o * A, net.at<float>(net.w_v) + o,
                                         net.at<float>(net.w_ent) + o, net.at<int32_t>(net.w_act) + o,
                                         net.at<float>(net.w_logpa) + o);
  if (net.arch != ARCH_LSTM) {   // FF: split-K partials, reduce + relu + heads in one policy_fc launch
    ARL_TRY(launch_fc_fwd(a2 + (int64_t)e0 * A2, ne, fc_planes(net), P + net.o_fcb, fc_slab, nullptr, nullptr, s));
    ARL_TRY(stamp(net, STAGE_FC_FWD, s));
    if (t == net.T && net.fuse_returns && e0 == 0 && ne == n) {   // + the learner's returns (one env group)
      const Net::ReturnsCfg& r = net.ret;
      ARL_TRY(launch_policy_fc_returns(fc_slab, ne, P + net.o_fcb, hfc, pa, net.at<float>(net.w_rewards),
                                       net.at<uint8_t>(net.w_dones), net.at<float>(net.w_v),
                                       net.at<float>(net.w_probs), net.at<float>(net.w_logp),
                                       net.at<int32_t>(net.w_act), net.T, r.gamma, r.beta, r.vcoef, r.clip_reward,
                                       net.at<float>(net.w_dlogits), net.at<float>(net.w_dv),
                                       net.at<float>(net.w_loss), net.at<int64_t>(net.w_ctl), net.pi_coef,
                                       net.keep_scale, net.at<float>(net.w_hfc), net.at<float>(net.w_dfc), s));
      net.returns_done = true;
      net.norm_ready = false;   // a new gradient (as LEARN_RETURNS)
      return stamp(net, STAGE_POLICY, s);
    }
    ARL_TRY(launch_policy_fc(fc_slab, ne, P + net.o_fcb, hfc, pa, s));
    return stamp(net, STAGE_POLICY, s);
  }
  // LSTM: the FC's split-K partials, reduced + bias + relu either in the gate kernel's staging (XRED) or
  // by the FC's last-arriver ticket (lstm_xred); then the gates with the cell in their epilogue
  const bool xred = lstm_xred(ne);
  ARL_TRY(launch_fc_fwd(a2 + (int64_t)e0 * A2, ne, fc_planes(net), P + net.o_fcb, fc_slab,
                        xred ? nullptr : net.at<int>(net.w_tick) + fc_fwd_tiles(e0), xred ? nullptr : hfc, s));
  ARL_TRY(stamp(net, STAGE_FC_FWD, s));
  const int64_t r0 = (int64_t)t * n + e0;
  float* hout = net.at<float>(net.w_hbuf) + (r0 + n) * HID;
  ARL_TRY(launch_lstm_gates(xred ? nullptr : hfc, net.at<float>(net.w_hbuf) + r0 * HID,
                            net.at<uint8_t>(net.w_reset) + r0, P + net.o_luW, P + net.o_llW, P + net.o_lub,
                            net.at<float>(net.w_gates) + r0 * GATES, net.at<float>(net.w_cbuf) + r0 * HID,
                            net.at<float>(net.w_cbuf) + (r0 + n) * HID, hout, ne, true, s, xred ? fc_slab : nullptr,
                            xred ? P + net.o_fcb : nullptr, xred ? hfc : nullptr));
  ARL_TRY(stamp(net, STAGE_LSTM_GATES, s));
  ARL_TRY(launch_policy_args(hout, ne, pa, s, HID));
  return stamp(net, STAGE_POLICY, s);
}

// Policy arguments of a forward on explicit states (slot T): a sampled action
// draws from Philox stream 1 with a host counter, one per call, so repeated
// calls on the same state are independent draws and never collide with the
// window's draws (stream 0, counter = step + t).
PolicyArgs states_policy_args(Net& net, int mode) {
  PolicyArgs pa = slot_policy_args(net, net.T, mode);
  if (mode == 1) {
    pa.ctl = net.at<int64_t>(net.w_ctl) + CTL_ZERO;
    pa.step_off = net.eval_draws++;
    pa.stream = 1u;
  }
  return pa;
}

// Drop-in pi_and_v on explicit f32 states (dqn_phi output); results land in
// activation slot T (the bootstrap slot) of the workspace.  LSTM: the
// recurrent state is the pi_and_v state (eval_h / eval_c, reset flags
// eval_reset = "state is None"), separate from the lockstep window's; it
// advances unless keep (keep_same_state, a3c_ale.py:57-60).
hipError_t net_forward_f32(Net& net, const float* x, int n, int mode, hipStream_t s, bool keep) {
  if (net.arch == ARCH_FF_NATURE) return nature_forward_f32(net, x, n, mode, s);
  if (n > net.N) return hipErrorInvalidValue;
  const int T = net.T, N = net.N;
  float* a1 = net.at<float>(net.w_a1) + (int64_t)T * N * A1;
  float* a2 = net.at<float>(net.w_a2) + (int64_t)T * N * A2;
  float* hfc = net.at<float>(net.w_hfc) + (int64_t)T * N * HID;
  const float* P = net.p;
  ARL_TRY(ensure_fc_planes(net, s));
  const int K1 = (net.rgb ? 3 : 4) * 64;
  ARL_TRY((launch_gemm<64, 16, 32, 4, 1>(Conv1F32A{x, K1 / 64}, WeightT{P + net.o_c1W, K1},
                                                      EpiConv{a1, P + net.o_c1b, C1_OC, C1_P}, n * C1_P, C1_OC, K1,
                                                      1, s)));
  ARL_TRY((launch_gemm<32, 32, 32, 2, 2, GS, GK>(Conv2A{a1}, WeightT{P + net.o_c2W, 256},
                                                      EpiConv{a2, P + net.o_c2b, C2_OC, C2_P}, n * C2_P, C2_OC, 256,
                                                      1, s)));
  ARL_TRY(fc_forward(net, n, a2, hfc, s));
  const float* hpol = hfc;
  if (net.arch == ARCH_LSTM) {
    float* gates = net.at<float>(net.w_gates) + (int64_t)T * N * GATES;
    float* eh = net.at<float>(net.w_eval_h);
    float* ec = net.at<float>(net.w_eval_c);
    float* hn = net.at<float>(net.w_eval_hn);
    float* cn = net.at<float>(net.w_eval_cn);
    uint8_t* rs = net.at<uint8_t>(net.w_eval_reset);
    ARL_TRY(launch_lstm_gates(hfc, eh, rs, P + net.o_luW, P + net.o_llW, P + net.o_lub, gates, ec, cn, hn, n, true, s));
    const int64_t cnt = (int64_t)n * HID;
    if (!keep) {
      ARL_TRY(hipMemcpyAsync(eh, hn, cnt * 4, hipMemcpyDeviceToDevice, s));
      ARL_TRY(hipMemcpyAsync(ec, cn, cnt * 4, hipMemcpyDeviceToDevice, s));
      ARL_TRY(hipMemsetAsync(rs, 0, n, s));
    }
    hpol = hn;
  }
  const PolicyArgs pa = states_policy_args(net, mode);
  return launch_policy_args(hpol, n, pa, s, HID);
}

// A3CLSTM.reset_state (a3c_ale.py:65-66) for the pi_and_v state of rows [e0, e0 + n)
hipError_t net_reset_state(Net& net, int e0, int n, hipStream_t s) {
  if (net.arch != ARCH_LSTM) return hipSuccess;
  return hipMemsetAsync(net.at<uint8_t>(net.w_eval_reset) + e0, 1, n, s);
}

// ---------------------------------------------------------------- backward
// the folded clip norm's arguments (none unless arl_net_set_norm_fold): the
// conv tensors are [0, o_fcW) of the flat gradient, everything after is final
// before the conv slab reduce
static NormFold norm_fold_args(const Net& net) {
  if (!net.norm_fold) return NormFold{};
  return NormFold{net.at<double>(net.w_norm), net.g, net.o_fcW, net.param_floats, net.norm_rest_blocks};
}

// the fused conv backward (per-sample slabs) and its slab reduce (with the folded clip norm's
// partials when nf.parts is set): the learner's last part
static hipError_t conv_backward(Net& net, hipStream_t s, const NormFold& nf) {
  const int S = net.T * net.N;
  float* slab = net.at<float>(net.w_slab);
  ARL_TRY(launch_conv_bwd(net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid), net.at<int64_t>(net.w_ctl),
                          net.N, net.R, S, net.at<float>(net.w_a1), net.at<float>(net.w_da2), net.p + net.o_c2W, slab,
                          net.g + net.o_c2W, net.g + net.o_c2b, net.g + net.o_c1W, net.g + net.o_c1b, s,
                          /*reduce=*/false, net.layout));
  ARL_TRY(stamp(net, STAGE_CONV_BWD, s));
  ARL_TRY(launch_conv_reduce(slab, S, net.g + net.o_c2W, net.g + net.o_c2b, net.g + net.o_c1W, net.g + net.o_c1b, s,
                             net.layout, nf));
  return stamp(net, STAGE_CONV_REDUCE, s);
}

hipError_t net_learn(Net& net, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s) {
  if (net.arch == ARCH_FF_NATURE) return nature_learn(net, gamma, beta, vcoef, clip_reward, s);
  for (int part = 0; part < LEARN_CONV; ++part) ARL_TRY(net_learn_part(net, part, gamma, beta, vcoef, clip_reward, s));
  // the conv part last; with norm_fold its slab reduce also leaves the clip norm's partials
  // (every other gradient tensor is final by now: one stream)
  if (net.states) {   // the generic-GEMM conv backward has no folded norm: the update runs grad_sqnorm
    ARL_TRY(states_conv_bwd(net, s));
    net.norm_ready = false;
    return hipSuccess;
  }
  ARL_TRY(conv_backward(net, s, norm_fold_args(net)));
  net.norm_ready = net.norm_fold;
  return hipSuccess;
}

// LSTM gate weight gradients ([x | h_prev] operand, reset rows' h dropped) straight into the gradient
// and dfc = (dG Wu) * (hfc > 0), one launch (fc_bwd.hip's ShapeLSTM)
static hipError_t lstm_wgrad(Net& net, hipStream_t s) {
  const int S = net.T * net.N;
  return launch_lstm_wgrad(net.at<float>(net.w_dG), net.at<float>(net.w_hfc), net.at<float>(net.w_hbuf),
                           net.at<uint8_t>(net.w_reset), net.at<float>(net.w_zero), net.p + net.o_luW, S,
                           net.g + net.o_luW, net.g + net.o_llW, net.g + net.o_lub, net.at<float>(net.w_dfc),
                           net.at<float>(net.w_fcb_part), net.at<int>(net.w_fcb_tick), s);
}

// the heads' weight gradients ride on the FC backward launch (its job C)
static HeadsDW heads_dw(const Net& net) {
  const float* hh = net.arch == ARCH_LSTM ? net.at<float>(net.w_hbuf) + (int64_t)net.N * HID : net.at<float>(net.w_hfc);
  return HeadsDW{net.at<float>(net.w_dlogits), net.at<float>(net.w_dv), hh, net.A, net.g + net.o_piW,
                 net.g + net.o_pib, net.g + net.o_vW, net.g + net.o_vb};
}

static hipError_t fc_backward(Net& net, hipStream_t s) {
  const HeadsDW heads = heads_dw(net);
  return launch_fc_bwd(net.at<float>(net.w_dfc), net.at<float>(net.w_a2), net.p + net.o_fcW, net.T * net.N,
                       net.g + net.o_fcW, net.g + net.o_fcb, net.at<float>(net.w_da2), net.at<float>(net.w_fcb_part),
                       net.at<int>(net.w_fcb_tick), s, &heads, a2_mask(net, 0));
}

// One part of the NIPS learner (LEARN_* in arl_internal.hpp), in order on one stream
hipError_t net_learn_part(Net& net, int part, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s) {
  if (net.arch == ARCH_FF_NATURE) return hipErrorInvalidValue;
  const int n = net.N, T = net.T, A = net.A;
  const float* P = net.p;
  const bool L = net.arch == ARCH_LSTM;
  if (part == LEARN_RETURNS) {
    if (net.returns_done) {   // the bootstrap policy launch ran it (net_act, fuse_returns)
      net.returns_done = false;
      return hipSuccess;
    }
    // n-step returns + loss gradient wrt logits / v (a3c.py:82-126); also snapshots the step counter for
    // the optimizer's fused advance and, in the same launch, the heads' backward dh (FF: dfc = dh * (hfc > 0))
    net.norm_ready = false;   // a new gradient: no folded norm until net_learn's reduce
    ARL_TRY(launch_returns_heads(net.at<float>(net.w_rewards), net.at<uint8_t>(net.w_dones), net.at<float>(net.w_v),
                                 net.at<float>(net.w_probs), net.at<float>(net.w_logp), net.at<int32_t>(net.w_act), T,
                                 n, A, gamma, beta, vcoef, clip_reward, net.at<float>(net.w_dlogits),
                                 net.at<float>(net.w_dv), net.at<float>(net.w_loss), s, net.at<int64_t>(net.w_ctl),
                                 net.pi_coef, net.keep_scale, P + net.o_piW, P + net.o_vW,
                                 L ? nullptr : net.at<float>(net.w_hfc),
                                 L ? net.at<float>(net.w_dh) : net.at<float>(net.w_dfc)));
    return stamp(net, STAGE_RETURNS, s);
  }
  if (part == LEARN_CONV) {
    if (net.states) {
      ARL_TRY(states_conv_bwd(net, s));
      return stamp(net, STAGE_CONV_BWD, s);
    }
    // fused conv backward per sample (conv_bwd.hip): conv2 dW/db, da1 = conv_transpose(da2, W2) * (a1 > 0)
    // kept in LDS, conv1 dW/db straight from the frame ring; then its slab reduce
    return conv_backward(net, s, NormFold{});
  }
  if (part != LEARN_TRUNK) return hipErrorInvalidValue;
  // LSTM: truncated BPTT over the window (a3c.py:144), then the gate weight gradients and dfc
  if (L) {
    const float* gates = net.at<float>(net.w_gates);
    const float* cbuf = net.at<float>(net.w_cbuf);
    const uint8_t* rs = net.at<uint8_t>(net.w_reset);
    float* dG = net.at<float>(net.w_dG);
    float* dhn = net.at<float>(net.w_dhn);
    float* dcn = net.at<float>(net.w_dcn);
    const float* dH = net.at<float>(net.w_dh);
    const int64_t cnt = (int64_t)n * HID;
    // step T-1's cell, then per step t: dh_{t-1} = (dG_t Wl) * (no reset at t) and step t-1's cell in one
    // launch (lstm.hip)
    const int64_t oT = (int64_t)(T - 1) * n;
    hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, gates + oT * GATES,
                       cbuf + (oT + n) * HID, cbuf + oT * HID, rs + oT, dH + oT * HID, dhn, dcn, dG + oT * GATES, 1, cnt);
    ARL_TRY(hipGetLastError());
    ARL_TRY(stamp(net, STAGE_LSTM_CELL, s));
    for (int t = T - 1; t > 0; --t) {
      const int64_t o = (int64_t)t * n, op = o - n;
      ARL_TRY(launch_lstm_bptt(dG + o * GATES, P + net.o_llW, rs + o, gates + op * GATES, cbuf + (op + n) * HID,
                               cbuf + op * HID, rs + op, dH + op * HID, dcn, dG + op * GATES, dhn, n, true, s));
      ARL_TRY(stamp(net, STAGE_LSTM_BPTT, s));
    }
    ARL_TRY(lstm_wgrad(net, s));
    ARL_TRY(stamp(net, STAGE_LSTM_WGRAD, s));
  }
  // FC: dW + db straight into the gradient and da2 = (dfc W) * (a2 > 0), with the heads' weight
  // gradients, one launch (fc_bwd.hip)
  ARL_TRY(fc_backward(net, s));
  return stamp(net, STAGE_FC_BWD, s);
}

// One stage of a window on the current workspace contents (arl_run_stage):
// the same launches the window makes, isolated for timing.
hipError_t net_stage(Net& net, int stage, int t, hipStream_t s) {
  if (net.arch == ARCH_FF_NATURE) return nature_stage(net, stage, t, s);
  const int n = net.N, S = net.T * n;
  const float* P = net.p;
  float* G = net.g;
  float* slab = net.at<float>(net.w_slab);
  float* a2 = net.at<float>(net.w_a2);
  float* hfc = net.at<float>(net.w_hfc);
  if (net.states && (stage == STAGE_CONV_FWD || stage == STAGE_CONV_BWD || stage == STAGE_CONV_REDUCE)) {
    if (stage == STAGE_CONV_FWD)
      return states_conv_fwd(net, t, net.at<float>(net.w_a1) + (int64_t)t * n * A1, a2 + (int64_t)t * n * A2, s);
    return stage == STAGE_CONV_BWD ? states_conv_bwd(net, s) : hipSuccess;   // (no separate slab reduce)
  }
  switch (stage) {
    case STAGE_CONV_FWD:
      return launch_conv_fwd(net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid),
                             net.at<int64_t>(net.w_ctl), n, net.R, t, P + net.o_c1W, P + net.o_c1b, P + net.o_c2W,
                             P + net.o_c2b, net.at<float>(net.w_a1) + (int64_t)t * n * A1, a2 + (int64_t)t * n * A2,
                             s, net.layout, 0, -1, a2_mask(net, t));
    case STAGE_FC_FWD:   // as in net_act: FF (and the LSTM's XRED gate kernel) reduce the partials downstream
      ARL_TRY(ensure_fc_planes(net, s));
      if (net.arch != ARCH_LSTM || lstm_xred(n))
        return launch_fc_fwd(a2 + (int64_t)t * n * A2, n, fc_planes(net), P + net.o_fcb, slab, nullptr, nullptr, s);
      return fc_forward(net, n, a2 + (int64_t)t * n * A2, hfc + (int64_t)t * n * HID, s);
    case STAGE_POLICY: {
      const int64_t o = (int64_t)t * n;
      if (net.arch != ARCH_LSTM)
        return launch_policy_fc(slab, n, P + net.o_fcb, hfc + o * HID, slot_policy_args(net, t, 0), s);
      return launch_policy_args(net.at<float>(net.w_hbuf) + (o + n) * HID, n, slot_policy_args(net, t, 0), s, HID);
    }
    case STAGE_FC_BWD:   // with the heads' weight gradients (job C), as in LEARN_TRUNK
      return fc_backward(net, s);
    case STAGE_CONV_BWD:
      return launch_conv_bwd(net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid),
                             net.at<int64_t>(net.w_ctl), n, net.R, S, net.at<float>(net.w_a1),
                             net.at<float>(net.w_da2), P + net.o_c2W, slab, G + net.o_c2W, G + net.o_c2b,
                             G + net.o_c1W, G + net.o_c1b, s, /*reduce=*/false, net.layout);
    case STAGE_RETURNS:   // the LEARN_RETURNS launch (returns + loss gradient + heads dh), default coefficients
      return net_learn_part(net, LEARN_RETURNS, 0.99, 0.01f, 0.5f, 1, s);
    case STAGE_CONV_REDUCE:
      return launch_conv_reduce(slab, S, G + net.o_c2W, G + net.o_c2b, G + net.o_c1W, G + net.o_c1b, s, net.layout,
                                norm_fold_args(net));   // as arl_learn launches it
    case STAGE_GRAD_SQNORM:
      return launch_grad_sqnorm(net.g, net.param_floats, net.at<double>(net.w_norm), net.norm_blocks, s);
    case STAGE_LSTM_GATES: {   // as net_act's LSTM step over all envs
      if (net.arch != ARCH_LSTM) return hipErrorInvalidValue;
      const int64_t r0 = (int64_t)t * n;
      const bool xred = lstm_xred(n);
      return launch_lstm_gates(xred ? nullptr : hfc + r0 * HID, net.at<float>(net.w_hbuf) + r0 * HID,
                               net.at<uint8_t>(net.w_reset) + r0, P + net.o_luW, P + net.o_llW, P + net.o_lub,
                               net.at<float>(net.w_gates) + r0 * GATES, net.at<float>(net.w_cbuf) + r0 * HID,
                               net.at<float>(net.w_cbuf) + (r0 + n) * HID, net.at<float>(net.w_hbuf) + (r0 + n) * HID,
                               n, true, s, xred ? slab : nullptr, xred ? P + net.o_fcb : nullptr,
                               xred ? hfc + r0 * HID : nullptr);
    }
    case STAGE_LSTM_BPTT: {    // the BPTT step t -> t - 1 (t = T - 1 when t is 0)
      if (net.arch != ARCH_LSTM || net.T < 2) return hipErrorInvalidValue;
      const int tt = t > 0 && t < net.T ? t : net.T - 1;
      const int64_t o = (int64_t)tt * n, op = o - n;
      float* dG = net.at<float>(net.w_dG);
      const float* cbuf = net.at<float>(net.w_cbuf);
      const uint8_t* rs = net.at<uint8_t>(net.w_reset);
      return launch_lstm_bptt(dG + o * GATES, P + net.o_llW, rs + o, net.at<float>(net.w_gates) + op * GATES,
                              cbuf + (op + n) * HID, cbuf + op * HID, rs + op, net.at<float>(net.w_dh) + op * HID,
                              net.at<float>(net.w_dcn), dG + op * GATES, net.at<float>(net.w_dhn), n, true, s);
    }
    case STAGE_LSTM_WGRAD:
      if (net.arch != ARCH_LSTM) return hipErrorInvalidValue;
      return lstm_wgrad(net, s);
    case STAGE_RMSPROP:   // the update kernel as a window runs it (clip 40 from the last norm the window left), lr 0
      return launch_rmsprop(net.p, net.ms, net.g, net.param_floats, 0.0, 0.99, 0.1, net.at<double>(net.w_norm),
                            net.norm_ready ? conv_norm_parts(net.norm_rest_blocks) : net.norm_blocks, 40.f, nullptr, 0,
                            0, net.T, s);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t net_optimize(Net& net, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                        float clip, hipStream_t s, bool advance) {
  double* parts = net.at<double>(net.w_norm);
  const bool do_clip = clip > 0.f;
  // arl_learn left the step snapshot (returns kernel), so the update kernel
  // can also advance the window
  const bool fused = advance;
  const bool folded = do_clip && net.norm_ready;   // partials left by arl_learn's conv reduce
  net.norm_ready = false;
  if (do_clip && !folded) {
    ARL_TRY(launch_grad_sqnorm(net.g, net.param_floats, parts, net.norm_blocks, s));
    ARL_TRY(stamp(net, STAGE_GRAD_SQNORM, s));
  }
  const bool L = net.arch == ARCH_LSTM;
  // the update rewrites the FC weight's split planes with the new W (all of them, so they are current
  // afterwards even if they were not before)
  uint16_t* planes = net.arch == ARCH_FF_NATURE ? nullptr : net.at<uint16_t>(net.w_fcplanes);
  const AdvanceArgs adv{fused ? net.at<int64_t>(net.w_ctl) : nullptr, planes, net.o_fcW, net.at<uint8_t>(net.w_reset),
                        L ? net.at<float>(net.w_hbuf) : nullptr, L ? net.at<float>(net.w_cbuf) : nullptr, net.T,
                        net.N};
  if (planes != nullptr) net.planes_gen = net.param_gen;
  ARL_TRY(launch_rmsprop(net.p, net.ms, net.g, net.param_floats, lr0, alpha, eps, do_clip ? parts : nullptr,
                         folded ? conv_norm_parts(net.norm_rest_blocks) : net.norm_blocks, clip, total_steps > 0 ? net.at<int64_t>(net.w_ctl) : nullptr, total_steps,
                         n_total, net.T, s, &adv));
  ARL_TRY(stamp(net, STAGE_RMSPROP, s));
  return advance && !fused ? net_advance(net, s) : hipSuccess;
}

hipError_t net_advance(Net& net, hipStream_t s) {
  const bool L = net.arch == ARCH_LSTM;
  const int64_t cnt = L ? (int64_t)net.N * HID : net.N;
  hipLaunchKernelGGL(advance_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, net.at<int64_t>(net.w_ctl),
                     net.T, net.at<uint8_t>(net.w_reset), net.N, L ? net.at<float>(net.w_hbuf) : nullptr,
                     L ? net.at<float>(net.w_cbuf) : nullptr);
  return hipGetLastError();
}

}  // namespace arl
