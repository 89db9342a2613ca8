// Policy / value heads, softmax policy output and action sampling; n-step
// returns and the loss gradient of the A3C objective.
//
// Reference: policy.py:28-29,53-58 (FCSoftmaxPolicy: logits = h W^T + b),
// v_function.py:29-34 (FCVFunction), policy_output.py:12-61
// (SoftmaxPolicyOutput: softmax, log_softmax, entropy, sampled actions and
// their log-probs), a3c.py:69-70 (reward clip), a3c.py:82-126 (n-step
// return, advantage, pi/v/entropy losses).
//
// policy_kernel: one 4-wave workgroup per 4 env rows (C3 window 1.0642-1.0678 -> 1.0582-1.0588 ms
// against 16 rows, 1.0635-1.0641 at 1 row, r5am).  The A logits and the
// value are one small GEMM on the matrix cores: [16 rows x 256] . [256 x
// (A + 1)] with v_mfma_f32_16x16x4_f32 (exact f32 products; each lane's h and
// W fragments are 16-byte loads covering 4 k-steps, k permuted identically on
// both sides); the 4 waves take one K quarter each and the partial tiles are
// summed in wave order.  The rows go through LDS to one lane
// per env, which accumulates the softmax, log-softmax and entropy serially
// (k = 0..A-1, the order NumPy uses for small rows) so the sampler's f32 CDF
// is reproducible by the CPU oracle.  The draw is inverse-CDF on a
// counter-based Philox4x32-10 uniform keyed by (seed; env id, step), so
// sampling needs no RNG state and a captured graph replays with fresh
// numbers; mode 2 takes the first argmax instead (most_probable_actions,
// policy_output.py:37-39).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "arl_internal.hpp"
#include "policy_rows.hpp"

namespace arl {

// HW = hidden width (256: NIPS head / LSTM; 512: Nature head)
constexpr int PK_ROWS = 4;   // env rows a workgroup (the MFMA tile's other rows repeat the last: bit-identical)
template <int HW>
__global__ void __launch_bounds__(256)
policy_kernel(const float* __restrict__ h, int64_t n, PolicyArgs pa) {
  __shared__ float part[4][16][MAXA + 2];
  __shared__ float zs[16][MAXA + 2];
  policy_rows16<HW, false, false, PK_ROWS>(h, (int64_t)blockIdx.x * PK_ROWS, n, pa, part, zs);
}

hipError_t launch_policy_args(const float* h, int64_t n, const PolicyArgs& pa, hipStream_t s, int hid) {
  if (n <= 0) return hipSuccess;
  if (hid == 512)
    hipLaunchKernelGGL(policy_kernel<512>, dim3((unsigned)((n + PK_ROWS - 1) / PK_ROWS)), dim3(256), 0, s, h, n, pa);
  else if (hid == HID)
    hipLaunchKernelGGL(policy_kernel<HID>, dim3((unsigned)((n + PK_ROWS - 1) / PK_ROWS)), dim3(256), 0, s, h, n, pa);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// FF act step: the FC forward's split-K reduce moved here from fc_fwd_kernel's
// last arriver (fc.hip).  The 8 partial slabs of this group's rows are
// summed in split order 0..7 from 0.f, then + bias, relu -- the same f32 op
// sequence as the ticket path, so hfc is bit-identical -- written to hfc (the
// backward reads it) and to LDS, where the heads read it.
// PF_ROWS env rows per workgroup (1: 256 workgroups at 256 envs, each reading
// 8 KB of partials; measured 4.33 us vs 4.57 at 2 rows, 4.62 at 4, 5.56 at 16,
// where the reduce ran on 16 CUs)
constexpr int PF_ROWS = 1;
__global__ void __launch_bounds__(256)
policy_fc_kernel(const float* __restrict__ slab, int n, const float* __restrict__ fc_bias, float* __restrict__ hfc,
                 PolicyArgs pa) {
  __shared__ float part[4][16][MAXA + 2];
  __shared__ float zs[16][MAXA + 2];
  __shared__ __attribute__((aligned(16))) float hl[PF_ROWS * HID];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * PF_ROWS;
  constexpr int NV = PF_ROWS * HID / 4;          // float4 per slab of this group
  constexpr int V4 = (NV + 255) / 256;           // per thread
  const HeadsPrefetch<HID> pf = heads_prefetch<HID>(pa);   // in flight with the slab loads
  f32x4v p[V4][FC_SPLIT];
#pragma unroll
  for (int z = 0; z < FC_SPLIT; ++z)
#pragma unroll
    for (int j = 0; j < V4; ++j) {
      const int idx = min(tid + 256 * j, NV - 1), r = idx / (HID / 4), c = 4 * (idx % (HID / 4));
      const int64_t m = min(row0 + r, (int64_t)n - 1);
      p[j][z] = *reinterpret_cast<const f32x4v*>(slab + ((int64_t)z * n + m) * HID + c);
    }
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int idx = tid + 256 * j, r = idx / (HID / 4), c = 4 * (idx % (HID / 4));
    if (idx >= NV) break;
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < FC_SPLIT; ++z)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], p[j][z][e]);
    const float4 b = *reinterpret_cast<const float4*>(fc_bias + c);
    float4 o;
    o.x = fmaxf(__fadd_rn(acc[0], b.x), 0.f); o.y = fmaxf(__fadd_rn(acc[1], b.y), 0.f);
    o.z = fmaxf(__fadd_rn(acc[2], b.z), 0.f); o.w = fmaxf(__fadd_rn(acc[3], b.w), 0.f);
    *reinterpret_cast<float4*>(hl + r * HID + c) = o;
    if (row0 + r < n) *reinterpret_cast<float4*>(hfc + (row0 + r) * HID + c) = o;
  }
  __syncthreads();
  policy_rows16<HID, false, true, PF_ROWS>(hl, row0, n, pa, part, zs, &pf);
}

hipError_t launch_policy_fc(const float* slab, int n, const float* fc_bias, float* hfc, const PolicyArgs& pa,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(policy_fc_kernel, dim3((unsigned)((n + PF_ROWS - 1) / PF_ROWS)), dim3(256), 0, s, slab, n, fc_bias, hfc, pa);
  return hipGetLastError();
}

hipError_t launch_policy(const float* h, int64_t n, const float* Wpi, const float* bpi, const float* Wv,
                         const float* bv, int A, uint64_t seed, const int64_t* ctl, int64_t step_off,
                         int env_offset, int mode, float* logits, float* probs, float* logp, float* v,
                         float* ent, int32_t* act, float* logp_a, hipStream_t s, int hid) {
  if (n <= 0) return hipSuccess;
  return launch_policy_args(h, n, make_policy_args(Wpi, bpi, Wv, bv, A, seed, ctl, step_off, env_offset, mode, logits,
                                                   probs, logp, v, ent, act, logp_a), s, hid);
}

// a3c.py:82-126 over a lockstep window, one thread per (step t, env).
// rewards/dones (T, n); v/probs/logp/act indexed (T+1, n[, A]) with row T =
// the bootstrap value v(s_T) computed with the pre-update parameters.
// R accumulates in float64 (Python float at a3c.py:83-92) and restarts at 0
// at every terminal (dones bit 0), so each episode segment in the window is
// one a3c update.  Thread (t, e) runs the reverse recurrence R = R*gamma + r
// from T-1 down to its own t -- the same operations in the same order as a
// sequential scan, so R_t is bit-identical -- with every reward / done of its
// env loaded up front (no dependent loads in the chain).  Steps flagged past
// the window's end (dones bit 1, arl_truncate_window: the reference's window
// closed early at a terminal, a3c.py:77-78) get no loss and a zero gradient.
// Loss scale (a3c.py:110-121): pi terms * pi_loss_coef, v terms * v_loss_coef,
// and with keep_loss_scale_same both * t_max / len for a segment that a
// terminal closed after len < t_max steps.  The per-env losses are then
// summed in the reference's order (t = T-1 .. 0) through LDS.  ctl != null:
// also snapshot the step counter (CTL_STEP_SNAP) for the optimizer's fused
// advance.  Block = EB envs x T steps (EB = 256 / T), env fastest.
struct ReturnsArgs {
  const float* rewards;
  const uint8_t* dones;
  const float* v;
  const float* probs;
  const float* logp;
  const int32_t* act;
  int T, n, A;
  double gamma;
  float beta, vcoef, pcoef;
  int clip_reward, keep_scale;
  float* dlogits;
  float* dv;
  float* loss;
  int64_t* ctl;
};

// dlogits / dv of (step t, env e); returns the two loss terms of the step
// (pi term without the sign, v term) through lpi / lv
// Every load of the thread is issued before the arithmetic that uses it
// (register arrays with static indices, clamped offsets): a load after a
// store the compiler cannot disambiguate, or under a per-lane branch, would
// wait for the one before it.  Windows up to RW steps keep their rewards /
// dones in registers; longer ones loop over memory.
constexpr int RW = 8;
// AM >= A: the action count the registers are sized for (4 / 8 / MAXA)
template <int AM>
struct RetIn {   // everything returns_one reads of step (t, e)
  float pr[AM], lp[AM], rw[RW];
  int dn[RW];
  float vboot, vi;
  int ac, di;
};
template <int AM>
__device__ inline void returns_load(const ReturnsArgs& a, int t, int e, RetIn<AM>& in) {
  const int T = a.T, n = a.n, A = a.A;
  const int64_t i = (int64_t)t * n + e;
#pragma unroll
  for (int k = 0; k < AM; ++k) {
    const int64_t o = i * A + min(k, A - 1);
    in.pr[k] = a.probs[o];
    in.lp[k] = a.logp[o];
  }
#pragma unroll
  for (int k = 0; k < RW; ++k) {
    const int64_t o = (int64_t)min(k, T - 1) * n + e;
    in.rw[k] = a.rewards[o];
    in.dn[k] = a.dones[o];
  }
  in.vboot = a.v[(int64_t)T * n + e];
  in.vi = a.v[i];
  in.ac = a.act[i];
  in.di = a.dones[i];
}
template <int AM>
__device__ inline void returns_compute(const ReturnsArgs& a, int t, int e, const RetIn<AM>& in, float& lpi, float& lv,
                                       float* sdl) {
  const int T = a.T, n = a.n, A = a.A;
  const int64_t i = (int64_t)t * n + e;
  const float* pr = in.pr;
  const float* lp = in.lp;
  const float* rw = in.rw;
  const int* dn = in.dn;
  const float vboot = in.vboot, vi = in.vi;
  const int ac = in.ac, di = in.di;
  float* dl = a.dlogits + i * A;
  if (di & 2) {   // past the end of this window
    for (int k = 0; k < A; ++k) dl[k] = 0.f;
    a.dv[i] = 0.f;
    if (sdl)
      for (int k = 0; k <= A; ++k) sdl[k] = 0.f;
    lpi = 0.f;
    lv = 0.f;
    return;
  }
  auto clip = [&](double r) { return a.clip_reward ? (r < -1.0 ? -1.0 : (r > 1.0 ? 1.0 : r)) : r; };
  double R = (double)vboot;
  int seg_end = -1;   // first terminal at or after t: closes t's segment
  int seg_start = 0;  // first step after the last terminal before t
  if (T <= RW) {
#pragma unroll
    for (int k = RW - 1; k >= 0; --k)
      if (k < T && k >= t) {
        if (dn[k] & 1) {
          R = 0.0;
          seg_end = k;
        }
        R = __dadd_rn(__dmul_rn(R, a.gamma), clip((double)rw[k]));
      }
#pragma unroll
    for (int k = 0; k < RW; ++k)
      if (k < t && (dn[k] & 1)) seg_start = k + 1;
  } else {
    for (int tt = T - 1; tt >= t; --tt) {
      const int64_t j = (int64_t)tt * n + e;
      if (a.dones[j] & 1) {
        R = 0.0;
        seg_end = tt;
      }
      R = __dadd_rn(__dmul_rn(R, a.gamma), clip((double)a.rewards[j]));
    }
    for (int tt = t - 1; tt >= 0; --tt)
      if (a.dones[(int64_t)tt * n + e] & 1) {
        seg_start = tt + 1;
        break;
      }
  }
  float pf = a.pcoef, vf = a.vcoef;
  if (a.keep_scale && seg_end >= 0) {
    const int len = seg_end - seg_start + 1;
    if (len < T) {
      const float factor = (float)((double)T / (double)len);
      pf = __fmul_rn(pf, factor);
      vf = __fmul_rn(vf, factor);
    }
  }
  const float Rf = (float)R;
  const float adv = __fsub_rn(Rf, vi);
  float H = 0.f, lpa = 0.f;
#pragma unroll
  for (int k = 0; k < AM; ++k)
    if (k < A) {
      H = __fadd_rn(H, __fmul_rn(pr[k], lp[k]));
      if (k == ac) lpa = lp[k];
    }
  H = -H;
#pragma unroll
  for (int k = 0; k < AM; ++k)
    if (k < A) {
      const float oh = (k == ac) ? 1.f : 0.f;
      const float t1 = __fmul_rn(-adv, __fsub_rn(oh, pr[k]));
      const float t2 = __fmul_rn(__fmul_rn(a.beta, pr[k]), __fadd_rn(lp[k], H));
      const float d = __fmul_rn(pf, __fadd_rn(t1, t2));
      dl[k] = d;
      if (sdl) sdl[k] = d;
    }
  const float dvv = __fsub_rn(vi, Rf);
  const float dvo = __fmul_rn(vf, dvv);
  a.dv[i] = dvo;
  if (sdl) sdl[A] = dvo;
  lpi = __fmul_rn(pf, __fadd_rn(__fmul_rn(lpa, adv), __fmul_rn(a.beta, H)));
  lv = __fmul_rn(vf, __fmul_rn(__fmul_rn(dvv, dvv), 0.5f));
}
__device__ inline void returns_one(const ReturnsArgs& a, int t, int e, float& lpi, float& lv) {
  RetIn<MAXA> in;
  returns_load(a, t, e, in);
  returns_compute(a, t, e, in, lpi, lv, nullptr);
}

// per-env losses summed in the reference's order (t = T-1 .. 0)
__device__ inline void env_loss(const ReturnsArgs& a, const float* lpi, const float* lv, int EB, int el, int e) {
  float pi_loss = 0.f, v_loss = 0.f;
  for (int tt = a.T - 1; tt >= 0; --tt) {
    pi_loss = __fsub_rn(pi_loss, lpi[tt * EB + el]);
    v_loss = __fadd_rn(v_loss, lv[tt * EB + el]);
  }
  a.loss[2 * e] = pi_loss;
  a.loss[2 * e + 1] = v_loss;
}

__global__ void __launch_bounds__(256)
returns_kernel(ReturnsArgs a) {
  __shared__ float lpi[256], lv[256];
  if (a.ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CTL_STEP_SNAP] = a.ctl[CTL_STEP];
  const int EB = 256 / a.T;
  const int tid = threadIdx.x, t = tid / EB, el = tid - t * EB;
  const int e = blockIdx.x * EB + el;
  const bool on = t < a.T && e < a.n;
  if (on) returns_one(a, t, e, lpi[tid], lv[tid]);
  if (a.loss == nullptr) return;
  __syncthreads();
  if (t == 0 && on) env_loss(a, lpi, lv, EB, el, e);
}

// returns_kernel + the heads' backward (a3c.py:129-130 through policy.py /
// v_function.py): dh[s][j] = sum_k dlogits[s][k] Wpi[k][j] + dv[s] Wv[j],
// times (mask[s][j] > 0) when mask is given, for the T steps of one env per
// block -- the rows the block's own threads just produced, handed over in
// LDS.  Thread j of the block owns column j (HID = 256 = blockDim): its Wpi /
// Wv column and its mask entries are loaded up front, beside the returns' own
// loads.  rh_load issues every load of a block, rh_finish does the rest, so
// the bootstrap step's policy launch can run both around its own work
// (policy_fc_returns_kernel).
// AM >= A actions, RB rows (steps) per pass: the register arrays (mask
// entries, head-weight column, loaded probs / log-probs) are sized for the
// window, e.g. 5 rows and 4 actions at C2 instead of 32 and 32
template <int AM, int RB>
struct RhState {
  float mv[RB];
  int64_t so[RB];
  float wc[AM + 1];
  RetIn<AM> in;
};

// mask entries of rows r0 .. r0 + RB - 1 (row r = step r of env e) for column j = threadIdx.x
// (unconditional loads at clamped offsets: a load under a per-lane branch would wait for each one in turn)
template <int AM, int RB>
__device__ inline void rh_rows(const ReturnsArgs& a, const float* __restrict__ mask, int e, int r0,
                               RhState<AM, RB>& st) {
  const int j = threadIdx.x;
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int r = r0 + u;
    st.so[u] = (r < a.T && e < a.n) ? ((int64_t)r * a.n + e) * HID + j : -1;
  }
#pragma unroll
  for (int u = 0; u < RB; ++u) st.mv[u] = mask != nullptr ? mask[st.so[u] < 0 ? j : st.so[u]] : 1.f;
}

template <int AM, int RB>
__device__ inline void rh_load(const ReturnsArgs& a, const float* __restrict__ Wpi, const float* __restrict__ Wv,
                               const float* __restrict__ mask, int e, RhState<AM, RB>& st) {
  const int T = a.T, A = a.A, j = threadIdx.x;
  rh_rows(a, mask, e, 0, st);
#pragma unroll
  for (int k = 0; k <= AM; ++k) st.wc[k] = k < A ? Wpi[min(k, A - 1) * HID + j] : Wv[j];
  returns_load(a, min((int)threadIdx.x, T - 1), min(e, a.n - 1), st.in);   // off threads: a valid step, discarded
}

// lpi / lv: 64 floats, sdl: 64 (AM + 1), w: (AM + 1) HID of LDS
template <int AM, int RB>
__device__ inline void rh_finish(const ReturnsArgs& a, const float* __restrict__ mask, float* __restrict__ dh, int e,
                                 RhState<AM, RB>& st, float* lpi, float* lv, float* sdl, float* w) {
  const int T = a.T, A = a.A;
  const int tid = threadIdx.x, t = tid, j = tid;
  const bool on = t < T && e < a.n;
#pragma unroll
  for (int k = 0; k <= AM; ++k)
    if (k <= A) w[k * HID + j] = k < A ? st.wc[k] : st.wc[AM];   // thread j's own column
  if (on) returns_compute(a, t, e, st.in, lpi[tid], lv[tid], sdl + tid * (A + 1));   // row tid = step t
  __syncthreads();
  if (a.loss != nullptr && t == 0 && on) env_loss(a, lpi, lv, 1, 0, e);
  for (int r0 = 0; r0 < T; r0 += RB) {
    if (r0 > 0) rh_rows(a, mask, e, r0, st);   // T > RB: the next RB rows
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      if (st.so[u] < 0) continue;
      const float* d = sdl + (r0 + u) * (A + 1);
      float acc = 0.f;
      for (int k = 0; k < A; ++k) acc = __fadd_rn(acc, __fmul_rn(d[k], w[k * HID + j]));
      acc = __fadd_rn(acc, __fmul_rn(d[A], w[A * HID + j]));
      dh[st.so[u]] = st.mv[u] > 0.f ? acc : 0.f;
    }
  }
}

template <int AM, int RB>
__global__ void __launch_bounds__(256)
returns_heads_kernel(ReturnsArgs a, const float* __restrict__ Wpi, const float* __restrict__ Wv,
                     const float* __restrict__ mask, float* __restrict__ dh) {
  __shared__ float lpi[64], lv[64];
  __shared__ float sdl[64 * (AM + 1)];
  __shared__ float w[(AM + 1) * HID];
  if (a.ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CTL_STEP_SNAP] = a.ctl[CTL_STEP];
  RhState<AM, RB> st;
  rh_load(a, Wpi, Wv, mask, blockIdx.x, st);
  rh_finish(a, mask, dh, blockIdx.x, st, lpi, lv, sdl, w);
}

// The FF window's bootstrap step (slot T, no draw) with the learner's first
// launch folded in: block e runs policy_fc_kernel's row e (the FC split-K
// reduce + relu + heads), then returns_heads_kernel's env e, whose bootstrap
// value v(s_T) is the row's own value head output, taken from LDS (the same
// f32 the policy stores to v).  Every load of the returns part is issued
// before the FC partials' loads.  Results are bit-identical to the two
// launches: the same per-element arithmetic in the same order.
template <int AM, int RB>
__global__ void __launch_bounds__(256)
policy_fc_returns_kernel(const float* __restrict__ slab, int n, const float* __restrict__ fc_bias,
                         float* __restrict__ hfc, PolicyArgs pa, ReturnsArgs ra, const float* __restrict__ mask,
                         float* __restrict__ dh) {
  __shared__ float part[4][16][MAXA + 2];
  __shared__ float zs[16][MAXA + 2];
  __shared__ __attribute__((aligned(16))) float hl[HID];
  __shared__ float lpi[64], lv[64];
  __shared__ float sdl[64 * (AM + 1)];
  __shared__ float w[(AM + 1) * HID];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int e = blockIdx.x;
  if (ra.ctl != nullptr && e == 0 && tid == 0) ra.ctl[CTL_STEP_SNAP] = ra.ctl[CTL_STEP];
  RhState<AM, RB> st;
  rh_load(ra, pa.Wpi, pa.Wv, mask, e, st);
  const HeadsPrefetch<HID> pf = heads_prefetch<HID>(pa);
  // policy_fc_kernel's row (PF_ROWS = 1): threads 0..63 hold one float4 column of the 8 partials
  const int c = 4 * (tid & 63);
  const int64_t m = min((int64_t)e, (int64_t)n - 1);
  f32x4v p[FC_SPLIT];
#pragma unroll
  for (int z = 0; z < FC_SPLIT; ++z) p[z] = *reinterpret_cast<const f32x4v*>(slab + ((int64_t)z * n + m) * HID + c);
  if (tid < HID / 4) {
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < FC_SPLIT; ++z)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = __fadd_rn(acc[k], p[z][k]);
    const float4 b = *reinterpret_cast<const float4*>(fc_bias + c);
    float4 o;
    o.x = fmaxf(__fadd_rn(acc[0], b.x), 0.f); o.y = fmaxf(__fadd_rn(acc[1], b.y), 0.f);
    o.z = fmaxf(__fadd_rn(acc[2], b.z), 0.f); o.w = fmaxf(__fadd_rn(acc[3], b.w), 0.f);
    *reinterpret_cast<float4*>(hl + c) = o;
    if (e < n) *reinterpret_cast<float4*>(hfc + (int64_t)e * HID + c) = o;
  }
  __syncthreads();
  policy_rows16<HID, false, true, 1>(hl, e, n, pa, part, zs, &pf);   // ends with a barrier
  st.in.vboot = zs[0][pa.A];   // v(s_T) of env e (heads_row_out stored zs[0][A] to v)
  rh_finish(ra, mask, dh, e, st, lpi, lv, sdl, w);
}

hipError_t launch_returns(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                          const float* logp, const int32_t* act, int T, int n, int A, double gamma, float beta,
                          float vcoef, int clip_reward, float* dlogits, float* dv, float* loss, hipStream_t s,
                          int64_t* ctl_snap, float pcoef, int keep_scale) {
  if (n <= 0) return hipSuccess;
  if (T < 1 || T > 256) return hipErrorInvalidValue;
  const int EB = 256 / T;
  const ReturnsArgs ra{rewards, dones, v, probs, logp, act, T, n, A, gamma, beta, vcoef, pcoef, clip_reward,
                       keep_scale, dlogits, dv, loss, ctl_snap};
  hipLaunchKernelGGL(returns_kernel, dim3((n + EB - 1) / EB), dim3(256), 0, s, ra);
  return hipGetLastError();
}

hipError_t launch_returns_heads(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                                const float* logp, const int32_t* act, int T, int n, int A, double gamma, float beta,
                                float vcoef, int clip_reward, float* dlogits, float* dv, float* loss, hipStream_t s,
                                int64_t* ctl_snap, float pcoef, int keep_scale, const float* Wpi, const float* Wv,
                                const float* mask, float* dh) {
  if (n <= 0) return hipSuccess;
  if (T < 1 || T > 64 || A < 1 || A > MAXA) return hipErrorInvalidValue;
  const ReturnsArgs ra{rewards, dones, v, probs, logp, act, T, n, A, gamma, beta, vcoef, pcoef, clip_reward,
                       keep_scale, dlogits, dv, loss, ctl_snap};
  const dim3 grid(n), blk(256);
  if (T <= 8) {
    if (A <= 4) hipLaunchKernelGGL((returns_heads_kernel<4, 8>), grid, blk, 0, s, ra, Wpi, Wv, mask, dh);
    else if (A <= 8) hipLaunchKernelGGL((returns_heads_kernel<8, 8>), grid, blk, 0, s, ra, Wpi, Wv, mask, dh);
    else hipLaunchKernelGGL((returns_heads_kernel<MAXA, 8>), grid, blk, 0, s, ra, Wpi, Wv, mask, dh);
  } else {
    hipLaunchKernelGGL((returns_heads_kernel<MAXA, 32>), grid, blk, 0, s, ra, Wpi, Wv, mask, dh);
  }
  return hipGetLastError();
}

hipError_t launch_policy_fc_returns(const float* slab, int n, const float* fc_bias, float* hfc, const PolicyArgs& pa,
                                    const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                                    const float* logp, const int32_t* act, int T, double gamma, float beta,
                                    float vcoef, int clip_reward, float* dlogits, float* dv, float* loss,
                                    int64_t* ctl_snap, float pcoef, int keep_scale, const float* mask, float* dh,
                                    hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int A = pa.A;
  if (T < 1 || T > 64 || A < 1 || A > MAXA) return hipErrorInvalidValue;
  const ReturnsArgs ra{rewards, dones, v, probs, logp, act, T, n, A, gamma, beta, vcoef, pcoef, clip_reward,
                       keep_scale, dlogits, dv, loss, ctl_snap};
  const dim3 grid(n), blk(256);
  if (T <= 8) {
    if (A <= 4)
      hipLaunchKernelGGL((policy_fc_returns_kernel<4, 8>), grid, blk, 0, s, slab, n, fc_bias, hfc, pa, ra, mask, dh);
    else if (A <= 8)
      hipLaunchKernelGGL((policy_fc_returns_kernel<8, 8>), grid, blk, 0, s, slab, n, fc_bias, hfc, pa, ra, mask, dh);
    else
      hipLaunchKernelGGL((policy_fc_returns_kernel<MAXA, 8>), grid, blk, 0, s, slab, n, fc_bias, hfc, pa, ra, mask,
                         dh);
  } else {
    hipLaunchKernelGGL((policy_fc_returns_kernel<MAXA, 32>), grid, blk, 0, s, slab, n, fc_bias, hfc, pa, ra, mask, dh);
  }
  return hipGetLastError();
}

}  // namespace arl
