// Policy / value heads, softmax policy output and action sampling; n-step
// returns and the loss gradient of the A3C objective.
//
// Reference: policy.py:28-29,53-58 (FCSoftmaxPolicy: logits = h W^T + b),
// v_function.py:29-34 (FCVFunction), policy_output.py:12-61
// (SoftmaxPolicyOutput: softmax, log_softmax, entropy, sampled actions and
// their log-probs), a3c.py:69-70 (reward clip), a3c.py:82-126 (n-step
// return, advantage, pi/v/entropy losses).
//
// policy_kernel: one 64-lane wave per env row.  Lane l holds h[4l..4l+3]
// (one 16-byte load); each of the A logits and the value is a 256-long dot
// product reduced across the wave with xor-shuffles; the softmax, the
// log-softmax and the entropy are then accumulated serially (k = 0..A-1, in
// the order NumPy uses for small rows) so the sampler's f32 CDF is
// reproducible by the CPU oracle.  The draw is inverse-CDF on a counter-based
// Philox4x32-10 uniform keyed by (seed; env id, step), so sampling needs no
// RNG state and a captured graph replays with fresh numbers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

__device__ inline uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ inline float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = __fadd_rn(x, __shfl_xor(x, o));
  return x;
}

__global__ void __launch_bounds__(256)
policy_kernel(const float* __restrict__ h, int64_t n, const float* __restrict__ Wpi, const float* __restrict__ bpi,
              const float* __restrict__ Wv, const float* __restrict__ bv, int A, uint32_t seed_lo,
              uint32_t seed_hi, const int64_t* __restrict__ ctl, int64_t step_off, int env_offset, int sample,
              float* __restrict__ logits, float* __restrict__ probs, float* __restrict__ logp,
              float* __restrict__ v, float* __restrict__ ent, int32_t* __restrict__ act,
              float* __restrict__ logp_a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float4 hv = reinterpret_cast<const float4*>(h + row * HID)[lane];
  auto dot = [&](const float* w) {
    const float4 wv = reinterpret_cast<const float4*>(w)[lane];
    float s = __fmul_rn(hv.x, wv.x);
    s = __fadd_rn(s, __fmul_rn(hv.y, wv.y));
    s = __fadd_rn(s, __fmul_rn(hv.z, wv.z));
    s = __fadd_rn(s, __fmul_rn(hv.w, wv.w));
    return wave_sum(s);
  };
  float z = 0.f;     // lane k < A holds logit k
  for (int k = 0; k < A; ++k) {
    const float d = __fadd_rn(dot(Wpi + (int64_t)k * HID), bpi[k]);
    if (lane == k) z = d;
  }
  const float vv = __fadd_rn(dot(Wv), bv[0]);
  // serial max / sum over k (policy_output.py:41-47; Chainer softmax, log_softmax)
  float m = __shfl(z, 0);
  for (int k = 1; k < A; ++k) m = fmaxf(m, __shfl(z, k));
  const float ez = expf(__fsub_rn(z, m));
  float se = 0.f;
  for (int k = 0; k < A; ++k) se = __fadd_rn(se, __shfl(ez, k));
  const float p = __fdiv_rn(ez, se);                 // softmax: exp(z-m) / sum
  const float lz = __fsub_rn(z, __fadd_rn(m, logf(se)));   // log_softmax: z - (m + log sum)
  float H = 0.f;                                     // entropy: -sum p log p
  for (int k = 0; k < A; ++k) H = __fadd_rn(H, __fmul_rn(__shfl(p, k), __shfl(lz, k)));
  H = -H;
  int a = A - 1;
  if (sample) {
    const int64_t step = ctl[CTL_STEP] + step_off;
    const uint4 r = philox4x32_10(make_uint4((uint32_t)(env_offset + row), (uint32_t)step,
                                             (uint32_t)((uint64_t)step >> 32), 0u), seed_lo, seed_hi);
    const float u = (float)(r.x >> 8) * 5.9604644775390625e-08f;
    float cdf = 0.f;
    bool found = false;
    for (int k = 0; k < A; ++k) {
      cdf = __fadd_rn(cdf, __shfl(p, k));
      if (!found && u < cdf) { a = k; found = true; }
    }
  }
  const float la = __shfl(lz, a);
  if (lane < A) {
    logits[row * A + lane] = z;
    probs[row * A + lane] = p;
    logp[row * A + lane] = lz;
  }
  if (lane == 0) {
    v[row] = vv;
    ent[row] = H;
    if (sample) {
      act[row] = a;
      logp_a[row] = la;
    }
  }
}

hipError_t launch_policy(const float* h, int64_t n, const float* Wpi, const float* bpi, const float* Wv,
                         const float* bv, int A, uint64_t seed, const int64_t* ctl, int64_t step_off,
                         int env_offset, int sample, float* logits, float* probs, float* logp, float* v,
                         float* ent, int32_t* act, float* logp_a, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(policy_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, h, n, Wpi, bpi, Wv, bv, A,
                     (uint32_t)seed, (uint32_t)(seed >> 32), ctl, step_off, env_offset, sample, logits, probs,
                     logp, v, ent, act, logp_a);
  return hipGetLastError();
}

// a3c.py:82-126 over a lockstep window, one thread per env.
// rewards/dones (T, n); v/probs/logp/act indexed (T+1, n[, A]) with row T =
// the bootstrap value v(s_T) computed with the pre-update parameters.
// R accumulates in float64 (Python float at a3c.py:83-92) and restarts at 0
// at every terminal, so each episode segment in the window is one a3c update.
__global__ void returns_kernel(const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
                               const float* __restrict__ v, const float* __restrict__ probs,
                               const float* __restrict__ logp, const int32_t* __restrict__ act, int T, int n,
                               int A, double gamma, float beta, float vcoef, int clip_reward,
                               float* __restrict__ dlogits, float* __restrict__ dv, float* __restrict__ loss) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double R = (double)v[(int64_t)T * n + e];
  float pi_loss = 0.f, v_loss = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const int64_t i = (int64_t)t * n + e;
    double r = (double)rewards[i];
    if (clip_reward) r = r < -1.0 ? -1.0 : (r > 1.0 ? 1.0 : r);
    if (dones[i]) R = 0.0;
    R = __dadd_rn(__dmul_rn(R, gamma), r);
    const float Rf = (float)R;
    const float vi = v[i];
    const float adv = __fsub_rn(Rf, vi);
    const float* pr = probs + i * A;
    const float* lp = logp + i * A;
    float H = 0.f;
    for (int k = 0; k < A; ++k) H = __fadd_rn(H, __fmul_rn(pr[k], lp[k]));
    H = -H;
    const int a = act[i];
    float* dl = dlogits + i * A;
    for (int k = 0; k < A; ++k) {
      const float oh = (k == a) ? 1.f : 0.f;
      const float t1 = __fmul_rn(-adv, __fsub_rn(oh, pr[k]));
      const float t2 = __fmul_rn(__fmul_rn(beta, pr[k]), __fadd_rn(lp[k], H));
      dl[k] = __fadd_rn(t1, t2);
    }
    const float dvv = __fsub_rn(vi, Rf);
    dv[i] = __fmul_rn(vcoef, dvv);
    pi_loss = __fsub_rn(pi_loss, __fadd_rn(__fmul_rn(lp[a], adv), __fmul_rn(beta, H)));
    v_loss = __fadd_rn(v_loss, __fmul_rn(vcoef, __fmul_rn(__fmul_rn(dvv, dvv), 0.5f)));
  }
  if (loss) {
    loss[2 * e] = pi_loss;
    loss[2 * e + 1] = v_loss;
  }
}

hipError_t launch_returns(const float* rewards, const uint8_t* dones, const float* v, const float* probs,
                          const float* logp, const int32_t* act, int T, int n, int A, double gamma, float beta,
                          float vcoef, int clip_reward, float* dlogits, float* dv, float* loss, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(returns_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rewards, dones, v, probs, logp, act, T,
                     n, A, gamma, beta, vcoef, clip_reward, dlogits, dv, loss);
  return hipGetLastError();
}

}  // namespace arl
