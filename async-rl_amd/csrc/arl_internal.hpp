// Internal declarations shared by the HIP translation units of libasyncrl_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace arl {

// control block (device int64[16]), read by kernels so that a captured window
// replays with advancing step counters (no frozen kernel arguments)
// CTL_STEP_SNAP: the step counter as the learner saw it (written at learn start),
// read by the fused optimizer for the lr anneal so it can advance CTL_STEP itself
// CTL_ZERO: never written (0 after arl_net_reset); the step base of draws keyed by a host counter
enum { CTL_STEP = 0, CTL_WINDOW = 1, CTL_STEP_SNAP = 2, CTL_ZERO = 15, CTL_SIZE = 16 };

enum Arch { ARCH_FF = 0, ARCH_LSTM = 1, ARCH_FF_NATURE = 2 };
// arch flag: RGB (Doom) observations, train_a3c_doom.py:25-63 (NIPSDQNHead(n_input_channels=3)
// on one RGB screen); conv1 sees [0, R, G, B] so the fused kernels keep K = 256
constexpr int ARCH_RGB = 16;
// arch flag: observations are whole 4-screen stacks (ale.py:91-94 ALE.state), one per ring slot
// (frames (R, n, 4, 84, 84)) -- the layout of the reference-semantics A3C.act drop-in
constexpr int ARCH_STACK = 32;
// arch flag: observations are float32 (4, 84, 84) states -- whatever the A3C phi plugin returns
// (a3c.py:34,50,73; identity by default), one per ring slot (frames (R, n, 4, 84, 84) f32); the
// convs run on the generic implicit-GEMM template (states.hip)
constexpr int ARCH_STATES = 64;
// frame layout of the ring, as the conv kernels read it (conv input plane c of window step t):
//   FRAMES_RING  one screen per slot, plane c = slot (k - 3 + c) % R   (k = ctl[STEP] + t)
//   FRAMES_RGB   three planes per slot [0, R, G, B] of slot k % R
//   FRAMES_STACK four planes per slot, plane c of slot k % R
//   FRAMES_STATES four f32 planes per slot (ARCH_STATES), plane c of slot k % R
enum FrameLayout { FRAMES_RING = 0, FRAMES_RGB = 1, FRAMES_STACK = 2, FRAMES_STATES = 3 };

constexpr int PLANE = 84 * 84;         // 7056 B per screen
constexpr int PAIR = 2 * 210 * 160 * 3; // 201,600 B per frame pair
constexpr int C1_OC = 16, C1_P = 400;  // conv1: 16 x 20 x 20
constexpr int C2_OC = 32, C2_P = 81;   // conv2: 32 x 9 x 9
constexpr int A1 = C1_OC * C1_P;       // 6400
constexpr int A2 = C2_OC * C2_P;       // 2592
constexpr int A2W = A2 / 32;             // 81 u32 words of a2 > 0 bits per env-step (fc_bwd job B mask)
static_assert(A2 % 32 == 0, "mask words");
constexpr int HID = 256;
constexpr int GATES = 4 * HID;
constexpr int ZERO_ROW_FLOATS = 64;     // LSTM: the zero row a reset sample's h_prev is DMA'd from (fc_bwd.hip)
constexpr int MAXA = 32;               // max actions supported by the policy kernel
// NatureDQNHead (dqn_head.py:6-28): 4->32 k8 s4 (20x20), 32->64 k4 s2 (9x9),
// 64->64 k3 s1 (7x7), Linear 3136 -> 512
constexpr int NC1 = 32, NP1 = 400, NC2 = 64, NP2 = 81, NC3 = 64, NP3 = 49;
constexpr int NA1 = NC1 * NP1, NA2 = NC2 * NP2, NA3 = NC3 * NP3;   // 12800, 5184, 3136
constexpr int NHID = 512;

struct RingArgs {
  const uint8_t* pair_pool;   // (pool_len, n, 2, 210, 160, 3)
  const float* reward_pool;   // (pool_len, n) or null
  const uint8_t* done_pool;   // (pool_len, n) or null
  int64_t pool_len;
  uint8_t* frames;            // (R, n, 84, 84)
  uint8_t* nvalid;            // (R, n)
  uint8_t* reset_flags;       // (T+1, n)
  float* rewards;             // (T, n)
  uint8_t* dones;             // (T, n)
  const int64_t* ctl;
  int n, R, t, mode, force_reset;
  int H = 0, W = 0;           // RGB nets: pair_pool is an image pool (pool_len, n, H, W, 3)
  int e0 = 0, ne = -1;        // env range of this launch: e0 + blockIdx.y, ne envs (-1: all n)
  int esize = 1;              // stack_ring_kernel: bytes per stack element (1 uint8 screens, 4 f32 states)
};

// RGB (Doom) observations, train_a3c_doom.py:21-23 / doom_env.py:47
constexpr int RGB_MAX_W = 2048;   // staged source rows: 12 x W x 3 bytes of LDS
hipError_t launch_rgb_phi(const uint8_t* imgs, int64_t n, int H, int W, float* out, int mode, hipStream_t s);
hipError_t launch_rgb_ring(const RingArgs& a, hipStream_t s);
hipError_t launch_stack_ring(const RingArgs& a, hipStream_t s);   // ARCH_STACK / ARCH_STATES nets

hipError_t launch_current_screen(const uint8_t* cur, const uint8_t* prev, uint8_t* out, int64_t n,
                                 int mode, hipStream_t s);
hipError_t launch_phi_stack(const uint8_t* pairs, const uint8_t* prev_stack, const uint8_t* reset,
                            uint8_t* out_stack, int64_t n, int mode, hipStream_t s);
hipError_t launch_phi_ring(const RingArgs& a, hipStream_t s);
hipError_t launch_max_luminance(const uint8_t* cur, const uint8_t* prev, uint8_t* gray, int64_t npix,
                                hipStream_t s);
hipError_t launch_dqn_phi(const uint8_t* in, float* out, int64_t count, hipStream_t s);

// ---------------------------------------------------------------- network
struct ParamInfo {
  std::string name;   // Chainer namedparam / HDF5 path, e.g. "0/0/W"
  int64_t offset;     // floats into the flat buffer (64-float aligned)
  int64_t numel;
};

// window timeline (measurement, arl_stamps_*): while `on`, every stage launch of a window records a
// timing event on its stream right after the kernel(s) and remembers the stage (Stage) it closes, so
// the intervals between consecutive stamps split one eager window into its stages as it ran
struct Stamps {
  std::vector<hipEvent_t> ev;
  std::vector<int> stage;
  std::vector<int64_t> seq;   // the stamp call each recorded event answers
  int count = 0;
  bool on = false;
  int period = 0;             // > 0: sparse (arl_stamps_sparse): window w records only calls t - 1, t of its
  int64_t calls = 0;          //   period, t = w mod period
};

struct Net {
  int arch, A, N, T, R;
  Stamps* stamps = nullptr;   // null / off: stamp() is a no-op
  bool rgb = false;        // ARCH_RGB: 3 planes per obs step in the ring, conv1 W (16, 3, 8, 8)
  bool stack = false;      // ARCH_STACK: 4 planes (a whole stack) per obs step in the ring
  bool states = false;     // ARCH_STATES: 4 f32 planes (phi's output) per obs step in the ring
  int layout = FRAMES_RING;
  // loss options (a3c.py:110-121): pi_loss_coef, keep_loss_scale_same (arl_net_set_loss)
  float pi_coef = 1.f;
  int keep_scale = 0;
  int64_t eval_draws = 0;  // sampling forward_states calls so far (Philox stream 1 counter)
  // clip norm folded into the learner's conv reduce (arl_net_set_norm_fold; only valid when
  // nothing changes the gradient between arl_learn and the update, e.g. no all-reduce):
  // norm_ready = the last arl_learn left the partials, consumed by the next update
  bool norm_fold = false, norm_ready = false;
  // parameter generations: every writer of the params the library does not make itself bumps param_gen
  // (arl_net_bind, arl_net_params_changed); planes_gen = the generation the FC weight's split planes
  // (w_fcplanes) were built from.  A forward over all envs rebuilds stale planes on its own stream
  // (fc_planes_kernel); an env-range forward refuses them (arl_net_prepare first, before the streams
  // fork); every in-window update rewrites all planes from the new W (rmsprop_kernel).
  uint64_t param_gen = 1, planes_gen = 0;
  bool planes_current() const { return planes_gen == param_gen; }
  // the learner's returns folded into the bootstrap step's policy launch (FF, arl_run_window):
  // fuse_returns = on, with the learn arguments below, for the window's slot-T forward; returns_done = that
  // launch ran, so the window's LEARN_RETURNS part is a no-op
  struct ReturnsCfg { double gamma; float beta, vcoef; int clip_reward; };
  bool fuse_returns = false, returns_done = false;
  ReturnsCfg ret{};
  int norm_rest_blocks = 64;
  int hid;                 // width of the layer the heads read (256 NIPS / LSTM, 512 Nature)
  int env_offset;          // global id of env 0 on this rank (RNG stream)
  uint64_t seed;
  std::vector<ParamInfo> params;
  int64_t param_floats;    // padded flat length
  // parameter offsets (floats)
  int64_t o_c1W, o_c1b, o_c2W, o_c2b, o_fcW, o_fcb, o_luW, o_lub, o_llW, o_piW, o_pib, o_vW, o_vb;
  int64_t o_c3W = -1, o_c3b = -1;   // Nature head only
  // workspace layout (byte offsets)
  struct Buf { const char* name; int64_t off, bytes; };
  std::vector<Buf> bufs;
  int64_t ws_bytes;
  int64_t w_ctl, w_frames, w_nvalid, w_reset, w_rewards, w_dones, w_a1, w_a2, w_hfc, w_gates, w_hbuf,
      w_cbuf, w_logits, w_probs, w_logp, w_v, w_ent, w_logpa, w_act, w_dlogits, w_dv, w_dh, w_dfc,
      w_dG, w_dhn, w_dcn, w_da2, w_slab, w_norm, w_loss, w_tick, w_fcb_part = 0, w_fcb_tick = 0, w_zero = 0,
      w_a2m = 0,   // (T+1, N, 81) a2 > 0 bits (ring-frame NIPS nets; 0: none)
      w_fcplanes = 0;   // FC_PLANES_BYTES: the FC weight's bf16 split planes (NIPS nets)
  int64_t w_a3 = 0, w_da1 = 0, w_da3 = 0;   // Nature head only (w_da1 also ARCH_STATES)
  // LSTM recurrent state of pi_and_v on explicit states (A3CLSTM.pi_and_v, a3c_ale.py:55-63):
  // h, c (n, 256), the step's outputs hn, cn, and reset flags (1 = state is None)
  int64_t w_eval_h = 0, w_eval_c = 0, w_eval_hn = 0, w_eval_cn = 0, w_eval_reset = 0;
  int64_t slab_floats;
  int norm_blocks;
  // bound pointers
  float* p = nullptr;
  float* g = nullptr;
  float* ms = nullptr;
  char* ws = nullptr;
  template <class T> T* at(int64_t off) const { return reinterpret_cast<T*>(ws + off); }
};

bool net_init(Net& net, int arch, int n_actions, int n_envs, int t_max, int env_offset, uint64_t seed,
              std::string& err);
// mode: 0 none, 1 sample, 2 greedy, | ACT_CONV_ONLY / ACT_AFTER_CONV (env-group staggering:
// the step split after its conv launch); envs [e0, e0 + ne) (ne < 0: all)
constexpr int ACT_CONV_ONLY = 4, ACT_AFTER_CONV = 8;
hipError_t net_act(Net& net, int t, int mode, hipStream_t s, int e0 = 0, int ne = -1);
hipError_t ensure_fc_planes(Net& net, hipStream_t s);   // rebuild the FC weight planes if stale (net.hip)
// learner parts (net_learn_part), in this order on one stream
enum { LEARN_RETURNS = 0, LEARN_TRUNK, LEARN_CONV, LEARN_PARTS };
hipError_t net_learn_part(Net& net, int part, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s);
hipError_t net_learn(Net& net, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s);
// advance: also end the window, folded into the update kernel (arl_learn
// snapshots the step counter, so the update's lr anneal does not race it).
hipError_t net_optimize(Net& net, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                        float clip, hipStream_t s, bool advance = false);
hipError_t net_advance(Net& net, hipStream_t s);
enum Stage { STAGE_CONV_FWD = 1, STAGE_FC_FWD = 2, STAGE_POLICY = 3, STAGE_FC_BWD = 4, STAGE_CONV_BWD = 5,
             STAGE_RETURNS = 6, STAGE_CONV_REDUCE = 7, STAGE_GRAD_SQNORM = 8,
             STAGE_LSTM_GATES = 9, STAGE_LSTM_BPTT = 10, STAGE_LSTM_WGRAD = 11,
             // stamp-only stages (timeline, not arl_run_stage): the observation, the update kernel,
             // the separate LSTM cell launches, a caller's stamp (e.g. after a collective), others
             STAGE_PHI = 12, STAGE_RMSPROP = 13, STAGE_LSTM_CELL = 14, STAGE_HOST = 15, STAGE_OTHER = 16 };
// record the stamp closing `stage` on stream s (no-op unless the net's timeline is on)
inline hipError_t stamp(const Net& net, int stage, hipStream_t s) {
  Stamps* st = net.stamps;
  if (st == nullptr || !st->on || st->count >= (int)st->ev.size()) return hipSuccess;
  const int64_t q = st->calls++;
  if (st->period > 0) {
    const int64_t P = st->period, i = q % P, t = (q / P) % P;
    if (i != t && i != t - 1) return hipSuccess;
  }
  st->stage[st->count] = stage;
  st->seq[st->count] = q;
  return hipEventRecord(st->ev[st->count++], s);
}
hipError_t net_stage(Net& net, int stage, int t, hipStream_t s);
// keep: LSTM keep_same_state (the pi_and_v recurrent state is not advanced)
hipError_t net_forward_f32(Net& net, const float* x, int n, int mode, hipStream_t s, bool keep = false);
hipError_t net_reset_state(Net& net, int e0, int n, hipStream_t s);

// Nature head (nature.hip)
int64_t nature_slab_floats(const Net& net);
hipError_t nature_act(Net& net, int t, int mode, hipStream_t s);
hipError_t nature_forward_f32(Net& net, const float* x, int n, int mode, hipStream_t s);
hipError_t nature_learn(Net& net, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s);
hipError_t nature_stage(Net& net, int stage, int t, hipStream_t s);

// ARCH_STATES nets (states.hip): conv1 + conv2 forward of window slot t from the f32
// state ring (all envs), and the conv backward of the window (conv2 dW / db,
// da1, conv1 dW / db) on the generic GEMM, gradients straight into net.g
hipError_t states_conv_fwd(const Net& net, int t, float* a1, float* a2, hipStream_t s);
hipError_t states_conv_bwd(Net& net, hipStream_t s);
int64_t states_slab_floats(const Net& net);

// LSTM gate GEMM + bias (+ the F.lstm cell when cell) for rows [0, n) (lstm.hip)
hipError_t launch_lstm_bptt(const float* dG, const float* Wl, const uint8_t* rs_t, const float* gates, const float* c_t,
                            const float* c_prev, const uint8_t* rs, const float* dH, float* dcn, float* dG_out,
                            float* dhn, int n, bool cell, hipStream_t s);
hipError_t launch_lstm_gates(const float* x, const float* h, const uint8_t* reset, const float* Wu, const float* Wl,
                             const float* b, float* gates, const float* c_prev, float* c_out, float* h_out, int n,
                             bool cell, hipStream_t s, const float* fc_slab = nullptr, const float* fc_b = nullptr,
                             float* hfc = nullptr);

// shared pieces of the heads' backward (net.hip)
hipError_t launch_heads_bwd(const float* dl, const float* dv, const float* Wpi, const float* Wv, int A, int H,
                            const float* mask, float* out, int64_t S, hipStream_t s);

// layout: FrameLayout of the ring (FRAMES_RGB: conv1 W (16, 3, 8, 8) on input planes 1..3)
hipError_t launch_conv_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t,
                           const float* W1, const float* b1, const float* W2, const float* b2, float* a1, float* a2,
                           hipStream_t s, int layout = FRAMES_RING, int e0 = 0, int ne = -1, uint32_t* a2m = nullptr);
// the gradient's squared norm folded into the conv slab reduce (parts == null: not folded)
struct NormFold {
  double* parts;            // NORM_SCRATCH f64: conv_norm_parts(rest_blocks) partials
  const float* g;           // the flat gradient
  int64_t rest_begin, rest_end;   // floats of g outside the conv tensors (final before the reduce)
  int rest_blocks;
};
int conv_norm_parts(int rest_blocks);
hipError_t launch_conv_bwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int S,
                           const float* a1, const float* da2, const float* W2, float* slab, float* gW2, float* gb2,
                           float* gW1, float* gb1, hipStream_t s, bool reduce = true, int layout = FRAMES_RING,
                           const NormFold& nf = NormFold{});
int64_t conv_bwd_slab_floats(int S);
int conv_bwd_blocks(int S);       // workgroups (= slab slices) of launch_conv_bwd
// the slab reduce launch_conv_bwd(reduce = true) ends with, alone
hipError_t launch_conv_reduce(const float* slab, int S, float* gW2, float* gb2, float* gW1, float* gb1, hipStream_t s,
                              int layout, const NormFold& nf = NormFold{});

// arguments of the softmax policy / value heads (policy_rows.hpp)
struct PolicyArgs {
  const float *Wpi, *bpi, *Wv, *bv;
  int A;
  uint32_t seed_lo, seed_hi;
  const int64_t* ctl;       // step counter (Philox counter = ctl[STEP] + step_off)
  int64_t step_off;
  int env_offset, mode;     // mode: 0 none, 1 sample, 2 greedy
  uint32_t stream;          // Philox counter word 3: 0 = window draws, 1 = pi_and_v draws
  float *logits, *probs, *logp, *v, *ent;
  int32_t* act;
  float* logp_a;
};
inline PolicyArgs make_policy_args(const float* Wpi, const float* bpi, const float* Wv, const float* bv, int A,
                                   uint64_t seed, const int64_t* ctl, int64_t step_off, int env_offset, int mode,
                                   float* logits, float* probs, float* logp, float* v, float* ent, int32_t* act,
                                   float* logp_a) {
  return PolicyArgs{Wpi, bpi, Wv, bv, A, (uint32_t)seed, (uint32_t)(seed >> 32), ctl, step_off, env_offset, mode, 0u,
                    logits, probs, logp, v, ent, act, logp_a};
}

constexpr int FC_SPLIT = 8;   // fc forward split-K (one slice per XCD)
// The FC weight as three exact bf16 split planes (bf16split.hpp), the B operand of fc_fwd_kernel (fc.hip):
// [3][256][FC_PLANE_LD] bf16; split z's 324 columns at z * FC_PLANE_SLICE (16-byte aligned slices, 4 pad
// columns each), the first 320 of a slice permuted within each 32-block so that lane quarter g of a 16x16x32
// fragment reads its 8 k as one 16-byte run: stored 8 g + 4 h + r holds column k = 16 h + 4 g + r.
// Written by fc_planes_kernel (fc.hip) and, for every W the update changes, by rmsprop_kernel (optim.hip).
constexpr int FC_PLANE_SLICE = A2 / FC_SPLIT + 4, FC_PLANE_LD = FC_SPLIT * FC_PLANE_SLICE;   // 328, 2624
constexpr int64_t FC_PLANES_BYTES = (int64_t)3 * HID * FC_PLANE_LD * 2;
__host__ __device__ constexpr int fc_plane_pos(int local) {   // stored position of slice column `local`
  return local >= 320 ? local : (local & ~31) + 8 * ((local >> 2) & 3) + 4 * ((local >> 4) & 1) + (local & 3);
}
// 4 consecutive W elements (flat index e % 4 == 0 within the (256, 2592) tensor) -> 8 bytes per plane
__device__ inline void fc_planes_store(uint16_t* planes, int e, float4 w) {
  const int j = e / A2, k = e - j * A2, z = k / (A2 / FC_SPLIT), loc = k - z * (A2 / FC_SPLIT);
  const int64_t o = (int64_t)j * FC_PLANE_LD + z * FC_PLANE_SLICE + fc_plane_pos(loc);   // 4 consecutive stored
  const float v[4] = {w.x, w.y, w.z, w.w};
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t hb = __float_as_uint(v[i]) & 0xffff0000u;
    const float r1 = __fsub_rn(v[i], __uint_as_float(hb));
    const uint32_t mb = __float_as_uint(r1) & 0xffff0000u;
    const float r2 = __fsub_rn(r1, __uint_as_float(mb));
    h[i] = hb >> 16;
    m[i] = mb >> 16;
    l[i] = __float_as_uint(r2) >> 16;
  }
  constexpr int64_t P = (int64_t)HID * FC_PLANE_LD;
  *reinterpret_cast<uint2*>(planes + o) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  *reinterpret_cast<uint2*>(planes + P + o) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
  *reinterpret_cast<uint2*>(planes + 2 * P + o) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
}
hipError_t launch_fc_planes(const float* W, uint16_t* planes, hipStream_t s);
int fc_fwd_tiles(int n);      // tickets needed for n envs
bool fc_fwd_big(int n);       // launches over n envs run fc_fwd_big_kernel's 64-row tiles
// Wp: the FC weight's split planes (FC_PLANE_LD above); tickets == null: split-K partials only (the
// consumer reduces them); else the last-arriver reduce + bias + relu -> hfc in the same launch
hipError_t launch_fc_fwd(const float* a2, int n, const uint16_t* Wp, const float* b, float* slab, int* tickets,
                         float* hfc, hipStream_t s);
// FC backward (fc_bwd.hip): dW / db straight into the gradient, da2 = (dfc W) * (a2 > 0)
// weight gradients of the policy / value heads (a3c.py:126-130 through
// policy.py / v_function.py Linear layers): rows a < A from dlogits, row A
// from dv, over the S samples of h (fc_bwd's job C)
struct HeadsDW {
  const float* dl;   // (S, A)
  const float* dv;   // (S)
  const float* h;    // (S, HID) fed to the heads
  int A;
  float *gWpi, *gbpi, *gWv, *gbv;
};
hipError_t launch_fc_bwd(const float* dfc, const float* a2, const float* W, int S, float* gW, float* gb, float* da2,
                         float* part, int* tick, hipStream_t s, const HeadsDW* heads = nullptr,
                         const uint32_t* a2m = nullptr);
// LSTM gate weight gradients (upward W / b, lateral W) + dfc = (dG Wu) * (hfc > 0), the same kernel
hipError_t launch_lstm_wgrad(const float* dG, const float* hfc, const float* hprev, const uint8_t* reset,
                             const float* zero, const float* Wu, int S, float* gWu, float* gWl, float* gbu, float* dfc,
                             float* part, int* tick, hipStream_t s);
int64_t fc_bwd_part_floats(int S);   // workspace of its in-launch split reduction (both launches)
int fc_bwd_tickets();                 // int counters, zero before the first launch (re-armed by it)
hipError_t launch_policy_args(const float* h, int64_t n, const PolicyArgs& pa, hipStream_t s, int hid);
// policy arguments of a forward on explicit states (arl_forward_states): slot
// T, a sampled action from Philox stream 1 keyed by a per-call host counter
PolicyArgs states_policy_args(Net& net, int mode);
// FC split-K reduce (partials of launch_fc_fwd with tickets == nullptr) + bias
// + relu -> hfc, then the policy / value heads on the same 16 rows
hipError_t launch_policy_fc(const float* slab, int n, const float* fc_bias, float* hfc, const PolicyArgs& pa,
                            hipStream_t s);

// x / 255 correctly rounded, i.e. __fdiv_rn(x, 255.f), in three ops instead of the ~10 of the
// general division: q = x * RN(1/255), the exact residual r = x - 255 q (fma), q + r * RN(1/255)
// (fma).  scripts/div255_check.c compares it with IEEE division over every finite f32: equal
// except x = -0 (+0 instead of -0), which no caller passes (byte values; MFMA sums from +0
// accumulators).  Needs f32 denormals on (the kernels' default float_denorm_mode 3).
__device__ inline float div255(float x) {
  constexpr float inv = 1.f / 255.f;
  const float q = __fmul_rn(x, inv);
  return __fmaf_rn(__fmaf_rn(-q, 255.f, x), inv, q);
}

// end-of-window advance folded into the update (NIPS learner): the lr reads
// the learner's snapshot CTL_STEP_SNAP, so no workgroup reads CTL_STEP and one
// thread can move it without a ticket; reset flags (and the LSTM h / c carry)
// are copied grid-stride by all workgroups (optim.hip).
struct AdvanceArgs {
  int64_t* ctl;             // null: no advance
  uint16_t* fc_planes;      // non-null: also rewrite the FC weight's split planes ([fc_w0, fc_w0 + 256 x 2592))
  int64_t fc_w0;
  uint8_t* reset;           // (T+1, n): row T -> row 0
  float* hbuf;              // LSTM: (T+2, n, 256), row T -> row 0 (else null)
  float* cbuf;
  int T, n;
};
// GradientClipping's squared norm: f64 partials [0, nparts) (nparts <= NORM_MAX_PARTS) of the launch
// that sums them (grad_sqnorm_kernel, or reduce_conv_bwd_kernel with a NormFold), one per block;
// every block of the update kernel re-reduces them in block order
constexpr int NORM_MAX_PARTS = 1000, NORM_SCRATCH = 1024;
// norm_sq: the norm's partials [0, nparts), re-reduced by every block; null: no clip
hipError_t launch_rmsprop(float* p, float* ms, const float* g, int64_t n, double lr, double alpha, double eps,
                          const double* norm_sq, int nparts, float clip, const int64_t* ctl,
                          int64_t total_steps, int64_t n_total, int t_max, hipStream_t s,
                          const AdvanceArgs* adv = nullptr);
hipError_t launch_grad_sqnorm(const float* g, int64_t n, double* partials, int blocks, hipStream_t s);
hipError_t launch_stream_copy(const void* src, void* dst, int64_t bytes, int blocks, int mode, hipStream_t s);
hipError_t launch_policy(const float* h, int64_t n, const float* Wpi, const float* bpi, const float* Wv,
                         const float* bv, int A, uint64_t seed, const int64_t* ctl, int64_t step_off,
                         int env_offset, int mode, float* logits, float* probs, float* logp, float* v,
                         float* ent, int32_t* act, float* logp_a, hipStream_t s, int hid = HID);
// dones: bit 0 = the transition t -> t+1 ended the episode; bit 1 = step t lies
// past the end of this window (arl_truncate_window: no loss, no gradient).
// pcoef = pi_loss_coef; keep_scale: keep_loss_scale_same (a3c.py:110-121)
hipError_t launch_returns(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                          const float* logp, const int32_t* act, int T, int n, int A, double gamma, float beta,
                          float vcoef, int clip_reward, float* dlogits, float* dv, float* loss, hipStream_t s,
                          int64_t* ctl_snap = nullptr, float pcoef = 1.f, int keep_scale = 0);
// launch_returns + the heads' backward dh = dlogits Wpi + dv Wv (times
// mask > 0 when mask is given) for hidden width HID, one launch (T <= 64)
hipError_t launch_returns_heads(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                                const float* logp, const int32_t* act, int T, int n, int A, double gamma, float beta,
                                float vcoef, int clip_reward, float* dlogits, float* dv, float* loss, hipStream_t s,
                                int64_t* ctl_snap, float pcoef, int keep_scale, const float* Wpi, const float* Wv,
                                const float* mask, float* dh);
// launch_policy_fc of the bootstrap slot (no draw) + launch_returns_heads for the same n envs, one launch
// (policy.hip policy_fc_returns_kernel; v(s_T) handed over in LDS); bit-identical to the two launches
hipError_t launch_policy_fc_returns(const float* slab, int n, const float* fc_bias, float* hfc, const PolicyArgs& pa,
                                    const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                                    const float* logp, const int32_t* act, int T, double gamma, float beta,
                                    float vcoef, int clip_reward, float* dlogits, float* dv, float* loss,
                                    int64_t* ctl_snap, float pcoef, int keep_scale, const float* mask, float* dh,
                                    hipStream_t s);

}  // namespace arl
