// Softmax policy / value heads for 16 env rows: the device body shared by
// policy_kernel (policy.hip) and the fused FC + policy tail of fc_fwd_kernel
// (fc.hip).  Reference: see policy.hip.
#pragma once
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

// One group of 16 env rows (row0 .. row0 + 15) of the softmax policy / value
// heads; part / zs are LDS scratch of the calling workgroup (all 256 threads
// call).  COH: h was written by other workgroups of the same launch (device
// scope, sc1) and is read with device-scope loads.  LOCAL: h holds only the
// group's 16 rows (row i at h + i * HW, e.g. LDS filled by the caller).
// ROWS < 16: only rows row0 .. row0 + ROWS - 1 are this group's (the other
// MFMA rows repeat the last one and are not stored).
template <int HW, bool COH, bool LOCAL = false, int ROWS = 16>
__device__ inline void policy_rows16(const float* __restrict__ h, int64_t row0, int64_t n, const PolicyArgs& pa,
                                     float (*part)[16][MAXA + 2], float (*zs)[MAXA + 2]) {
  // 4 waves split K = HW into quarters; partial tiles summed in wave order
  constexpr int KW = HW / 4, NS = KW / 16;
  const int A = pa.A;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int64_t rowc = min(row0 + (col < ROWS ? col : ROWS - 1), n - 1);   // A row of this lane (rows past n: any valid row, not stored)
  f32x4 hv[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const float* src = h + (LOCAL ? rowc - row0 : rowc) * HW + KW * w + 16 * s + 4 * g;
    if constexpr (COH) {
#pragma unroll
      for (int e = 0; e < 4; ++e) hv[s][e] = __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      hv[s] = *reinterpret_cast<const f32x4*>(src);
    }
  }
  for (int nt = 0; 16 * nt <= A; ++nt) {
    const int j = 16 * nt + col;   // head column: j < A -> pi logit j, j == A -> value
    const float* wrow = (j < A ? pa.Wpi + (int64_t)j * HW : pa.Wv) + KW * w;
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
    zs[r][j] = __fadd_rn(z, j < A ? pa.bpi[j] : pa.bv[0]);
  }
  __syncthreads();
  const int64_t row = row0 + tid;
  if (tid < ROWS && row < n) {
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
    const int mode = pa.mode;
    float u = 2.f;   // > any cdf: no draw
    if (mode == 1) {
      const int64_t step = pa.ctl[CTL_STEP] + pa.step_off;
      const uint4 r = philox4x32_10(make_uint4((uint32_t)(pa.env_offset + row), (uint32_t)step,
                                               (uint32_t)((uint64_t)step >> 32), pa.stream), pa.seed_lo, pa.seed_hi);
      u = (float)(r.x >> 8) * 5.9604644775390625e-08f;
    }
    float H = 0.f, cdf = 0.f, best = -1.f, la = 0.f;
    int a = A - 1;
    bool found = false;
    for (int k = 0; k < A; ++k) {
      const float p = __fdiv_rn(ez[k], se);                       // softmax: exp(z-m) / sum
      const float lz = __fsub_rn(z[k], lse);                      // log_softmax: z - (m + log sum)
      H = __fadd_rn(H, __fmul_rn(p, lz));                         // entropy: -sum p log p
      pa.logits[row * A + k] = z[k];
      pa.probs[row * A + k] = p;
      pa.logp[row * A + k] = lz;
      if (mode == 1) {
        cdf = __fadd_rn(cdf, p);
        if (!found && u < cdf) { a = k; la = lz; found = true; }
      } else if (mode == 2 && p > best) {
        best = p; a = k; la = lz;
      }
    }
    if (mode == 1 && !found) la = __fsub_rn(z[A - 1], lse);
    pa.v[row] = z[A];
    pa.ent[row] = -H;
    if (mode) {
      pa.act[row] = a;
      pa.logp_a[row] = la;
    }
  }
  __syncthreads();   // part / zs free for the caller's next group
}

}  // namespace arl
