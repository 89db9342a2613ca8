// Policy / value heads, softmax policy output and action sampling; n-step
// returns and the loss gradient of the A3C objective.
//
// Reference: policy.py:28-29,53-58 (FCSoftmaxPolicy: logits = h W^T + b),
// v_function.py:29-34 (FCVFunction), policy_output.py:12-61
// (SoftmaxPolicyOutput: softmax, log_softmax, entropy, sampled actions and
// their log-probs), a3c.py:69-70 (reward clip), a3c.py:82-126 (n-step
// return, advantage, pi/v/entropy losses).
//
// policy_kernel: one 4-wave workgroup per 16 env rows.  The A logits and the
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

// HW = hidden width (256: NIPS head / LSTM; 512: Nature head)
template <int HW>
__global__ void __launch_bounds__(256)
policy_kernel(const float* __restrict__ h, int64_t n, const float* __restrict__ Wpi, const float* __restrict__ bpi,
              const float* __restrict__ Wv, const float* __restrict__ bv, int A, uint32_t seed_lo,
              uint32_t seed_hi, const int64_t* __restrict__ ctl, int64_t step_off, int env_offset, int mode,
              float* __restrict__ logits, float* __restrict__ probs, float* __restrict__ logp,
              float* __restrict__ v, float* __restrict__ ent, int32_t* __restrict__ act,
              float* __restrict__ logp_a) {
  // 4 waves split K = H into quarters; partial tiles summed in wave order
  constexpr int KW = HW / 4, NS = KW / 16;
  __shared__ float part[4][16][MAXA + 2];
  __shared__ float zs[16][MAXA + 2];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * 16;
  const int64_t rowc = min(row0 + col, n - 1);   // A row of this lane (rows past n: any valid row, not stored)
  f32x4 hv[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) hv[s] = *reinterpret_cast<const f32x4*>(h + rowc * HW + KW * w + 16 * s + 4 * g);
  for (int nt = 0; 16 * nt <= A; ++nt) {
    const int j = 16 * nt + col;   // head column: j < A -> pi logit j, j == A -> value
    const float* wrow = (j < A ? Wpi + (int64_t)j * HW : Wv) + KW * w;
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      f32x4 wv = {0.f, 0.f, 0.f, 0.f};
      if (j <= A) wv = *reinterpret_cast<const f32x4*>(wrow + 16 * s + 4 * g);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][0], wv[0], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][1], wv[1], c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][2], wv[2], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][3], wv[3], c1, 0, 0, 0);
    }
    if (j <= A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) part[w][4 * g + r][j] = __fadd_rn(c0[r], c1[r]);   // C row 4g + r = env
    }
  }
  __syncthreads();
  for (int i = tid; i < 16 * (A + 1); i += 256) {
    const int r = i / (A + 1), j = i - r * (A + 1);
    float z = __fadd_rn(__fadd_rn(part[0][r][j], part[1][r][j]), __fadd_rn(part[2][r][j], part[3][r][j]));
    zs[r][j] = __fadd_rn(z, j < A ? bpi[j] : bv[0]);
  }
  __syncthreads();
  const int64_t row = row0 + tid;
  if (tid >= 16 || row >= n) return;
  float* z = zs[tid];
  float* ez = part[0][tid];   // reused: exp(z - max) per action
  // serial max / sum over k (policy_output.py:41-47; Chainer softmax, log_softmax)
  float m = z[0];
  for (int k = 1; k < A; ++k) m = fmaxf(m, z[k]);
  float se = 0.f;
  for (int k = 0; k < A; ++k) {
    ez[k] = expf(__fsub_rn(z[k], m));
    se = __fadd_rn(se, ez[k]);
  }
  const float lse = __fadd_rn(m, logf(se));
  float u = 2.f;   // > any cdf: no draw
  if (mode == 1) {
    const int64_t step = ctl[CTL_STEP] + step_off;
    const uint4 r = philox4x32_10(make_uint4((uint32_t)(env_offset + row), (uint32_t)step,
                                             (uint32_t)((uint64_t)step >> 32), 0u), seed_lo, seed_hi);
    u = (float)(r.x >> 8) * 5.9604644775390625e-08f;
  }
  float H = 0.f, cdf = 0.f, best = -1.f, la = 0.f;
  int a = A - 1;
  bool found = false;
  for (int k = 0; k < A; ++k) {
    const float p = __fdiv_rn(ez[k], se);                       // softmax: exp(z-m) / sum
    const float lz = __fsub_rn(z[k], lse);                      // log_softmax: z - (m + log sum)
    H = __fadd_rn(H, __fmul_rn(p, lz));                         // entropy: -sum p log p
    logits[row * A + k] = z[k];
    probs[row * A + k] = p;
    logp[row * A + k] = lz;
    if (mode == 1) {
      cdf = __fadd_rn(cdf, p);
      if (!found && u < cdf) { a = k; la = lz; found = true; }
    } else if (mode == 2 && p > best) {
      best = p; a = k; la = lz;
    }
  }
  if (mode == 1 && !found) la = __fsub_rn(z[A - 1], lse);
  v[row] = z[A];
  ent[row] = -H;
  if (mode) {
    act[row] = a;
    logp_a[row] = la;
  }
}

hipError_t launch_policy(const float* h, int64_t n, const float* Wpi, const float* bpi, const float* Wv,
                         const float* bv, int A, uint64_t seed, const int64_t* ctl, int64_t step_off,
                         int env_offset, int mode, float* logits, float* probs, float* logp, float* v,
                         float* ent, int32_t* act, float* logp_a, hipStream_t s, int hid) {
  if (n <= 0) return hipSuccess;
  if (hid == 512)
    hipLaunchKernelGGL(policy_kernel<512>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, h, n, Wpi, bpi, Wv, bv,
                       A, (uint32_t)seed, (uint32_t)(seed >> 32), ctl, step_off, env_offset, mode, logits, probs,
                       logp, v, ent, act, logp_a);
  else if (hid == HID)
    hipLaunchKernelGGL(policy_kernel<HID>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, h, n, Wpi, bpi, Wv, bv,
                       A, (uint32_t)seed, (uint32_t)(seed >> 32), ctl, step_off, env_offset, mode, logits, probs,
                       logp, v, ent, act, logp_a);
  else
    return hipErrorInvalidValue;
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
