/*
 * asyncrl_hip.h -- C ABI of libasyncrl_hip.so, the MI355X (gfx950) hot path of
 * batched A3C (phi + forward + sample + n-step update) for PeerM/async-rl.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * (passed as void*; NULL = the default stream).  Calls are asynchronous on
 * that stream, never allocate, never synchronise, and are graph-capturable.
 * Return value: 0 (ARL_OK) or an error code; arl_last_error() describes the
 * last failure of the calling thread.
 *
 * Each function names the reference interface it replaces (file:line in
 * PeerM/async-rl @ v0).  INTEGRATION.md shows the ctypes binding a maintainer
 * adds on the reference side.
 */
#ifndef ASYNCRL_HIP_H
#define ASYNCRL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARL_ABI_VERSION 4

#define ARL_OK 0
#define ARL_EINVAL 1   /* bad argument (shape, pointer, alignment) */
#define ARL_EHIP 2     /* HIP runtime error (launch failure) */
#define ARL_ESTATE 3   /* handle not bound / wrong arch for this call */

#define ARL_ARCH_FF 0     /* A3CFF   (a3c_ale.py:28-40) */
#define ARL_ARCH_LSTM 1   /* A3CLSTM (a3c_ale.py:43-70) */
#define ARL_ARCH_FF_NATURE 2  /* A3CFF with NatureDQNHead (dqn_head.py:6-28) instead of NIPSDQNHead */
#define ARL_ARCH_RGB 16   /* flag for FF / LSTM: the ViZDoom models of train_a3c_doom.py:25-63
                             (NIPSDQNHead(n_input_channels=3) on one RGB screen, no frame stack);
                             observations come through arl_observe_rgb */
#define ARL_ARCH_STACK 32 /* flag for FF / LSTM: observations are whole 4-screen stacks (ale.py:91-94
                             ALE.state, as A3C.act receives them, a3c.py:67,72-73), one per ring
                             slot; they come through arl_observe_stack */
#define ARL_ARCH_STATES 64 /* flag for FF / LSTM: observations are float32 (4, 84, 84) states -- the
                              output of A3C's phi plugin (a3c.py:34,50,73; identity by default) --
                              one per ring slot; they come through arl_observe_states */

#define ARL_RESIZE_SCALAR 0  /* OpenCV FixedPtCast vertical pass (canonical) */
#define ARL_RESIZE_SIMD 1    /* OpenCV VResizeLinearVec_32s8u (mulhi) pass */
#define ARL_RESIZE_CROP 2    /* flag: ale.py:73-82 crop_or_scale='crop' (84x110 resize, rows 18..101) */

int arl_abi_version(void);
const char* arl_last_error(void);

/* ------------------------------------------------------------------ phi */

/* ale.py:59-89 ALE.current_screen (crop_or_scale='scale'), batched.
 * rgb_cur, rgb_prev: (n, 210, 160, 3) uint8, 16-byte aligned.
 * out: (n, 84, 84) uint8.  max -> fp64 luminance -> uint8 -> 84x84 resize. */
int arl_current_screen(const uint8_t* rgb_cur, const uint8_t* rgb_prev, uint8_t* out, int64_t n,
                       int resize_mode, void* stream);

/* ale.py:62-69 alone: np.maximum of the two frames + float64 luminance +
 * astype(uint8), for npix pixels (rgb: (npix, 3) uint8) -> gray (npix,). */
int arl_max_luminance(const uint8_t* rgb_cur, const uint8_t* rgb_prev, uint8_t* gray, int64_t npix,
                      void* stream);

/* ale.py:135 + ale.py:155-158 (frame-stack deque), batched, materialised.
 * rgb_pairs: (n, 2, 210, 160, 3) uint8 (frame 4 and frame 3 of the skip);
 * prev_stack, out_stack: (n, 4, 84, 84) uint8, must not alias;
 * reset: (n,) uint8 or NULL -- 1 = episode start: [0, 0, 0, new]. */
int arl_phi_stack(const uint8_t* rgb_pairs, const uint8_t* prev_stack, const uint8_t* reset,
                  uint8_t* out_stack, int64_t n, int resize_mode, void* stream);

/* dqn_phi.py:4-17 dqn_phi, batched: (n, 4, 84, 84) uint8 -> float32 / 255. */
int arl_dqn_phi(const uint8_t* stack_u8, float* out, int64_t n, void* stream);

/* train_a3c_doom.py:21-23 phi, batched: cv2.resize(image_buffer, (84, 84))
 * per channel (INTER_LINEAR fixed point, resize_mode as above, no crop),
 * transpose(2, 0, 1), float32 / 255.  imgs: (n, H, W, 3) uint8 RGB24
 * (doom_env.py:47), 16-byte aligned, W % 16 == 0, W <= 2048; out: (n, 3,
 * 84, 84) f32. */
int arl_rgb_phi(const uint8_t* imgs, int64_t n, int H, int W, float* out, int resize_mode, void* stream);

/* ------------------------------------------------------------------ net */
typedef struct arl_net arl_net;

/* Describe an A3C model + lockstep actor-learner over n_envs envs and
 * t_max-step windows (a3c.py:33-61 A3C.__init__, a3c_ale.py:219-229).
 * env_offset: global id of this rank's env 0 (RNG stream); seed: Philox key. */
int arl_net_create(arl_net** out, int arch, int n_actions, int n_envs, int t_max, int env_offset,
                   uint64_t seed);
void arl_net_destroy(arl_net* net);

/* Flat parameter layout (Chainer namedparams order, each tensor 64-float
 * aligned).  The same layout is used for params, grads and RMSProp ms. */
int64_t arl_net_param_floats(const arl_net* net);
int arl_net_param_count(const arl_net* net);
int arl_net_param_info(const arl_net* net, int idx, int64_t* offset, int64_t* numel, char* name, int name_cap);

/* Caller-owned device workspace (activations, frame ring, rollout buffers). */
int64_t arl_net_workspace_bytes(const arl_net* net);
int arl_net_buffer(const arl_net* net, const char* name, int64_t* offset, int64_t* bytes);

/* Bind caller-owned device memory: params/grads/ms (param_floats f32 each,
 * 16-byte aligned; grads must be zeroed once by the caller) and workspace. */
int arl_net_bind(arl_net* net, float* params, float* grads, float* ms, void* workspace);

/* Parameter generations (ABI 4).  The FC forward reads the FC weight as bf16
 * split planes derived from the bound params; every arl_optimize* /
 * arl_run_window update keeps them current.  Any OTHER writer of the bound
 * params -- a checkpoint load, a copy from another model (copy_param.py,
 * serializers), arl_rmsprop on the params -- must bump the generation with
 * arl_net_params_changed; arl_net_bind bumps it too.  A forward over all envs
 * rebuilds stale planes on its own stream; arl_net_prepare rebuilds them on a
 * given stream (call it on the stream env-range chains fork from, and before
 * replaying a captured window after such a write: a replay has no rebuild);
 * arl_act_envs over a proper env range refuses stale planes with ARL_ESTATE.
 * arl_net_param_generation reads both generations (planes current iff equal).
 * No reference counterpart: the reference's forward reads the f32 params. */
int arl_net_params_changed(arl_net* net);
int arl_net_prepare(arl_net* net, void* stream);
int arl_net_param_generation(const arl_net* net, uint64_t* param_gen, uint64_t* planes_gen);

/* Reset the control block (step counters) and the frame ring; call once
 * before the first observation (async). */
int arl_net_reset(arl_net* net, void* stream);

/* Input pools (no reference counterpart: the reference's actors hand one frame
 * at a time to A3C.act).  The observation calls below read entry (control-block
 * step + t) % pool_len of caller-owned device pools, and a pointer carries no
 * extent, so the net keeps the extent of every pool it may read: register each
 * pool with its size in bytes before observing from it (kind ARL_POOL_FRAMES:
 * the frame-pair / image / stack / state pool; ARL_POOL_REWARDS; ARL_POOL_DONES;
 * up to 8 pools per kind, a later registration of the same base replaces the
 * earlier one, bytes == 0 removes it).  An observation whose non-NULL pool is
 * not inside a registered one, or whose pool_len entries of n_envs rows do not
 * fit before its end, fails with ARL_EINVAL before anything is launched. */
#define ARL_POOL_FRAMES 0
#define ARL_POOL_REWARDS 1
#define ARL_POOL_DONES 2
int arl_net_set_pool(arl_net* net, int kind, const void* pool, int64_t bytes);

/* Observation at window step t (0..t_max): phi of the env's frame pair into
 * the ring + stack bookkeeping + ingest of the reward/done that came with it
 * (a3c.py:69-75; ale.py:111-139).  Pools hold pool_len steps; the step used
 * is (control-block step + t) % pool_len.  pair_pool: (pool_len, n, 2, 210,
 * 160, 3) uint8; reward_pool: (pool_len, n) f32; done_pool: (pool_len, n)
 * uint8 (1 = the transition into this obs ended the episode, which also
 * resets the frame stack and LSTM state).  force_reset: treat every env as
 * starting an episode (first observation). */
int arl_observe(arl_net* net, int t, const uint8_t* pair_pool, const float* reward_pool,
                const uint8_t* done_pool, int64_t pool_len, int force_reset, int resize_mode, void* stream);

/* arl_observe for an ARL_ARCH_RGB net: the observation is the env's RGB
 * screen, img_pool (pool_len, n, H, W, 3) uint8 (W % 16 == 0, W <= 2048),
 * resized to 3 planes as arl_rgb_phi; same reward / done / reset handling
 * (the reset clears the LSTM state; there is no frame stack). */
int arl_observe_rgb(arl_net* net, int t, const uint8_t* img_pool, int H, int W, const float* reward_pool,
                    const uint8_t* done_pool, int64_t pool_len, int force_reset, int resize_mode, void* stream);

/* arl_observe for an ARL_ARCH_STACK net: stack_pool (pool_len, n, 4, 84, 84)
 * uint8 (ale.py:91-94 ALE.state: the 4 screens oldest first, zeros before
 * an episode's first screen), conv input = dqn_phi of it (dqn_phi.py:4-17).
 * stack_pool == NULL (t >= 1): ingest only the reward / done of the
 * transition into a terminal observation, whose state the reference never
 * feeds to the model (a3c.py:72-73, 165-167). */
int arl_observe_stack(arl_net* net, int t, const uint8_t* stack_pool, const float* reward_pool,
                      const uint8_t* done_pool, int64_t pool_len, int force_reset, void* stream);

/* arl_observe for an ARL_ARCH_STATES net: state_pool (pool_len, n, 4, 84, 84)
 * f32 (16-byte aligned), the conv input as phi returns it (a3c.py:73
 * np.expand_dims(self.phi(state), 0)); NULL (t >= 1): reward / done only, as
 * arl_observe_stack. */
int arl_observe_states(arl_net* net, int t, const float* state_pool, const float* reward_pool,
                       const uint8_t* done_pool, int64_t pool_len, int force_reset, void* stream);

/* The reference's early window end (a3c.py:77-78: an update at a terminal
 * after t_len < t_max steps): window steps [t_len, t_max) carry no loss and
 * no gradient in the next arl_learn (their done flags get bit 1, rewards 0).
 * Observations of the next window overwrite the flags again. */
int arl_truncate_window(arl_net* net, int t_len, void* stream);

/* Loss options of A3C.__init__ (a3c.py:33-36, 110-121): pi_loss_coef scales
 * the policy + entropy terms; keep_loss_scale_same scales both losses of a
 * segment that a terminal closed after len < t_max steps by t_max / len.
 * Host state of the handle, read when arl_learn launches (defaults 1, 0). */
int arl_net_set_loss(arl_net* net, double pi_loss_coef, int keep_loss_scale_same);

/* GradientClipping's squared norm (a3c_ale.py:226) folded into arl_learn:
 * with on != 0, arl_learn's conv slab reduce also leaves the f64 partial
 * sums of squares of the whole gradient (the conv tensors it writes, and the
 * rest, final by then), and the next arl_optimize / arl_optimize_advance
 * uses them instead of its own squared-norm launch.  Only valid when nothing
 * changes the gradient in between (turn it off when the gradient is
 * all-reduced across ranks); arl_learn_part never folds.  Default off. */
int arl_net_set_norm_fold(arl_net* net, int on);

/* The learner's returns + loss gradient + heads backward (arl_learn_part
 * ARL_LEARN_RETURNS, a3c.py:82-130) folded into the bootstrap step's policy
 * launch: with on != 0, the next arl_act / arl_act_mode at t == t_max over all
 * envs of an FF net with the NIPS head runs them in that launch with these
 * arguments, bit-identical, and the window's ARL_LEARN_RETURNS part (or
 * arl_learn's first launch) is then skipped.  arl_run_window does this
 * internally.  Host state of the handle; default off. */
int arl_net_set_returns_fusion(arl_net* net, int on, double gamma, double beta, double v_loss_coef, int clip_reward);

/* A3C.act forward + sample at window step t (a3c.py:154-164): pi_and_v of
 * the ring state, softmax policy output, Philox inverse-CDF action.  t ==
 * t_max is the bootstrap value of the window end (a3c.py:85, pre-update
 * params, LSTM state kept: a3c_ale.py:57-60); it samples nothing. */
int arl_act(arl_net* net, int t, void* stream);

/* arl_act with an explicit action mode: 0 = forward only (no action), 1 =
 * sample (as arl_act), 2 = greedy, the first argmax of the probabilities
 * (SoftmaxPolicyOutput.most_probable_actions, policy_output.py:37-39; the
 * evaluation policy of a3c_ale.py:73-89 / demo_a3c_ale.py:15-30). */
int arl_act_mode(arl_net* net, int t, int mode, void* stream);

/* Env groups: arl_observe / arl_observe_rgb and arl_act_mode restricted to
 * envs [e0, e0 + ne) of the net (no reference counterpart: the batched
 * form of running a3c.py:67-167 for a subset of the actors).  Disjoint
 * ranges touch disjoint workspace rows, so ranges issued on different
 * streams run concurrently (A3C.run_window(env_groups=G) forks one stream
 * per group for the T + 1 forward steps and joins before arl_learn).
 * e0 must be a multiple of ARL_ENV_GROUP_ALIGN; H, W are the screen size of
 * an ARL_ARCH_RGB net (ignored otherwise).  The Nature head accepts only
 * the full range. */
#define ARL_ENV_GROUP_ALIGN 32
int arl_observe_envs(arl_net* net, int t, int e0, int ne, const uint8_t* pool, int H, int W,
                     const float* reward_pool, const uint8_t* done_pool, int64_t pool_len, int force_reset,
                     int resize_mode, void* stream);
/* mode for arl_act_envs: 0 / 1 / 2 as arl_act_mode, optionally | one of
 * ARL_ACT_CONV_ONLY (launch only the step's conv layers) or
 * ARL_ACT_AFTER_CONV (the rest of the step): a stream can then record an
 * event between the two, which is how run_window staggers the groups. */
#define ARL_ACT_CONV_ONLY 4
#define ARL_ACT_AFTER_CONV 8
int arl_act_envs(arl_net* net, int t, int e0, int ne, int mode, void* stream);

/* Window update, gradient part (a3c.py:82-130): n-step returns with R = 0 at
 * terminals, advantage / entropy / value loss gradient, backward through
 * heads, [LSTM BPTT], FC, conv2, conv1 -> grads (overwritten). */
int arl_learn(arl_net* net, double gamma, double beta, double v_loss_coef, int clip_reward, void* stream);

/* arl_learn in parts (NIPS FF / LSTM heads; not the Nature head): parts 0..2
 * in order on one stream equal arl_learn (without its folded clip norm).
 * Part 0: returns + loss gradient + the heads' dh; part 1: LSTM BPTT and gate
 * weight gradients, the FC backward (dW, db, da2) and the heads' weight
 * gradients; part 2: the conv backward and its slab reduce, which write only
 * the conv tensors [0, offset of "0/2/W") of the gradient -- everything after
 * is final once part 1 is done (the N > 1 window all-reduces it meanwhile). */
#define ARL_LEARN_RETURNS 0
#define ARL_LEARN_TRUNK 1
#define ARL_LEARN_CONV 2
int arl_learn_part(arl_net* net, int part, double gamma, double beta, double v_loss_coef, int clip_reward,
                   void* stream);

/* GradientClipping(clip) + RMSpropAsync update (a3c_ale.py:224-226,
 * rmsprop_async.py:23-29) of the bound params / ms from the bound grads.
 * total_steps > 0 anneals lr on device (a3c_ale.py:111-112) with global_t =
 * (step + t_max) * n_total; otherwise lr = lr0.  clip <= 0 disables clipping. */
int arl_optimize(arl_net* net, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                 double clip, void* stream);

/* One stage of a window, run alone on the current workspace contents (the
 * same launches arl_act / arl_learn make), for per-kernel timing and
 * profiling.  t selects the window step for the forward stages.  Stages 1-11
 * and ARL_STAGE_RMSPROP. */
enum {
  ARL_STAGE_CONV_FWD = 1,   /* fused conv1 + conv2 forward from the frame ring */
  ARL_STAGE_FC_FWD = 2,     /* Linear(2592, 256): FF nets write the 8 split-K partials only; LSTM
                               nets reduce + bias + relu in the same launch */
  ARL_STAGE_POLICY = 3,     /* pi / v heads + softmax policy output (no action); FF nets first
                               reduce the FC partials + bias + relu into h (as in a window step) */
  ARL_STAGE_FC_BWD = 4,     /* FC dW / db and da2 GEMMs (+ the pi / v heads dW / db) */
  ARL_STAGE_CONV_BWD = 5,   /* fused conv backward (conv2 dW, convT, conv1 dW) into per-block slabs */
  ARL_STAGE_RETURNS = 6,    /* n-step returns + loss gradient + heads dh (gamma 0.99, beta 0.01, v coef 0.5,
                               clipped rewards): the learner's first launch */
  ARL_STAGE_CONV_REDUCE = 7,  /* the conv backward's slab reduce into the conv gradients */
  ARL_STAGE_GRAD_SQNORM = 8,  /* squared-norm partials of the whole gradient (GradientClipping) */
  ARL_STAGE_LSTM_GATES = 9,   /* LSTM: the gate kernel of slot t (cell in its epilogue) */
  ARL_STAGE_LSTM_BPTT = 10,   /* LSTM: one truncated-BPTT step (dh GEMM + the previous step's cell backward) */
  ARL_STAGE_LSTM_WGRAD = 11,  /* LSTM: the gate weight gradients + dfc (one launch) */
  /* timeline-only stages (arl_stamps_*, not arl_run_stage) */
  ARL_STAGE_PHI = 12,         /* the observation (phi into the frame ring) */
  ARL_STAGE_RMSPROP = 13,     /* clip + RMSProp (+ the window advance); arl_run_stage: the update
                                 kernel alone, lr 0, clip 40 at the norm the last window left */
  ARL_STAGE_LSTM_CELL = 14,   /* the LSTM cell backward of the window's last step */
  ARL_STAGE_HOST = 15,        /* a caller's stamp (arl_stamp), e.g. after a collective */
  ARL_STAGE_OTHER = 16
};
int arl_run_stage(arl_net* net, int stage, int t, void* stream);

/* Window timeline (measurement; no reference counterpart).  After
 * arl_stamps_begin(net, cap) every stage launch of the window (arl_observe*,
 * arl_act*, arl_learn*, arl_optimize*) records a timing event on its stream
 * right after its kernel(s), with the stage it closes (ARL_STAGE_*), up to cap
 * events; arl_stamp records one for the caller.  arl_stamps_end stops and
 * returns the count.  arl_stamps_read waits for stamp i0 + n - 1 and returns,
 * for i in [i0, i0 + n), ms[i - i0] = the time from stamp i - 1 to stamp i (0
 * for i = 0) and stage[i - i0]: consecutive intervals split an eager window
 * into its stages as it ran, launch boundaries included.
 * arl_stamps_sparse(net, P), right after arl_stamps_begin, for windows of P
 * stamp calls: window w records only its calls t - 1 and t, t = w mod P, so
 * each window carries at most two events and P windows time every stage once
 * nearly unperturbed; arl_stamps_read then returns ms = -1 for an interval
 * that is not between consecutive calls. */
int arl_stamps_begin(arl_net* net, int cap);
int arl_stamps_sparse(arl_net* net, int period);
int arl_stamp(arl_net* net, int stage, void* stream);
int arl_stamps_end(arl_net* net, int* count);
int arl_stamps_read(arl_net* net, int i0, int n, float* ms, int* stage);

/* One whole lockstep window in one call, for frame-pair nets with the NIPS
 * head (FF / LSTM): t = 0..t_max: arl_observe(t) (slot 0 only when first != 0,
 * with force_reset) + arl_act(t) (sampled; slot t_max the bootstrap forward,
 * a3c.py:85), then arl_learn and arl_optimize_advance (a3c.py:88-144) -- the
 * same launches in the same order as those calls one by one, issued without a
 * host round trip per step (A3C.run_window's single-chain window without
 * collectives). */
int arl_run_window(arl_net* net, const uint8_t* pair_pool, const float* reward_pool, const uint8_t* done_pool,
                   int64_t pool_len, int first, int resize_mode, double gamma, double beta, double v_loss_coef,
                   int clip_reward, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                   double clip, void* stream);

/* End of window: advance step counters, carry reset flags / LSTM state. */
int arl_advance(arl_net* net, void* stream);

/* arl_optimize followed by arl_advance (the end of a3c.py's update,
 * a3c.py:139-144) in one call; for the NIPS models the update kernel also
 * advances the window (one launch fewer). */
int arl_optimize_advance(arl_net* net, double lr0, int64_t total_steps, int64_t n_total, double alpha, double eps,
                         double clip, void* stream);

/* A3CFF / A3CLSTM.pi_and_v on explicit f32 states (a3c_ale.py:38-40,55-63;
 * input from dqn_phi), rows 0..n-1, n <= n_envs; outputs in the workspace's
 * bootstrap slot.  mode as arl_act_mode: 0 no action, 1 sampled
 * (action_indices from Philox stream 1, counter = number of sampling
 * forward_states calls so far on this handle: repeated calls draw afresh),
 * 2 greedy (most_probable_actions).  LSTM: the recurrent state is the
 * handle's pi_and_v state (not the lockstep window's); it advances unless
 * mode | ARL_FWD_KEEP_STATE (keep_same_state, a3c_ale.py:57-60). */
#define ARL_FWD_KEEP_STATE 16
int arl_forward_states(arl_net* net, const float* states, int64_t n, int mode, void* stream);

/* A3CLSTM.reset_state (a3c_ale.py:65-66) of the pi_and_v state, rows
 * [e0, e0 + n): the next forward starts from h = c = None.  No-op for FF. */
int arl_reset_state(arl_net* net, int64_t e0, int64_t n, void* stream);

/* ------------------------------------------------------------------ granular ops */

/* RMSpropAsync.update_one (rmsprop_async.py:23-38) on flat f32 arrays, with
 * optional Chainer GradientClipping (norm over g, scale if clip/norm < 1).
 * norm_partials: device f64[1024] scratch (needed when clip > 0): the norm
 * pass's per-block partials. */
int arl_rmsprop(float* param, float* ms, const float* grad, int64_t n, double lr, double alpha, double eps,
                double clip, double* norm_partials, void* stream);

/* SoftmaxPolicyOutput (policy_output.py:32-61) + FCSoftmaxPolicy / FCVFunction
 * heads (policy.py:53-58, v_function.py:29-34) for h: (n, 256) f32.  Samples
 * with Philox(seed; env_offset + row, step) when sample == 1 (step = *step_dev +
 * step_off); sample == 2 takes the first argmax (most_probable_actions);
 * sample == 0 writes no action. */
int arl_policy(const float* h, int64_t n, const float* W_pi, const float* b_pi, const float* W_v,
               const float* b_v, int n_actions, uint64_t seed, const int64_t* step_dev, int64_t step_off,
               int env_offset, int sample, float* logits, float* probs, float* log_probs, float* v,
               float* entropy, int32_t* actions, float* action_log_probs, void* stream);

/* a3c.py:82-126: returns + loss gradient over a (t_max, n) window. v, probs,
 * log_probs, actions are (t_max+1, n[, A]) with row t_max = bootstrap.
 * dones: bit 0 = the transition t -> t+1 ended the episode (R = 0), bit 1 =
 * step t is past the window's end (no loss).  loss: (n, 2) pi / v loss or
 * NULL. */
int arl_returns_lossgrad(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                         const float* log_probs, const int32_t* actions, int t_max, int64_t n, int n_actions,
                         double gamma, double beta, double pi_loss_coef, double v_loss_coef,
                         int keep_loss_scale_same, int clip_reward, float* dlogits, float* dv, float* loss,
                         void* stream);

/* ------------------------------------------------------------------ measurement */

/* Device-to-device copy of `bytes` (a multiple of 16, 16-byte aligned
 * buffers) by a grid of `blocks` 256-thread workgroups, 16-byte loads: the HBM
 * stream-copy peak the bench reports beside the 8 TB/s spec (SURVEY 8(d);
 * no reference counterpart).  mode 0: grid-stride, 4 loads in flight per lane;
 * mode 1: 64 KB blocks per workgroup, 16 non-temporal loads in flight per lane;
 * mode 2 / 3: a one-shot grid of bytes / 4 KB workgroups (`blocks` ignored), one
 * 16-byte load and store per lane (3: non-temporal). */
int arl_stream_copy(const void* src, void* dst, int64_t bytes, int blocks, int mode, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ASYNCRL_HIP_H */
