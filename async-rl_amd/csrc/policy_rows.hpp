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
template <int HW> struct HeadsPrefetch;

// One group of 16 env rows (row0 .. row0 + 15) of the softmax policy / value
// heads; part / zs are LDS scratch of the calling workgroup (all 256 threads
// call).  COH: h was written by other workgroups of the same launch (device
// scope, sc1) and is read with device-scope loads.  LOCAL: h holds only the
// group's 16 rows (row i at h + i * HW, e.g. LDS filled by the caller).
// ROWS < 16: only rows row0 .. row0 + ROWS - 1 are this group's (the other
// MFMA rows repeat the last one and are not stored).
// Every global load of the heads, issued first (a caller can issue it before
// its own loads and pass it in): the B fragments of each 16-column head tile
// from clamped rows (a load under a per-lane branch is waited for at the
// branch's end; columns past A are zeroed at use), the bias of the zs entry
// the thread forms first, the step counter of the Philox draw.
template <int HW>
struct HeadsPrefetch {
  static constexpr int KW = HW / 4, NS = KW / 16, NTM = (MAXA + 1 + 15) / 16;
  f32x4 wv[NTM][NS];
  float bias;
  int64_t step;
};
// kq: the K quarter whose fragments this wave loads (-1: the wave's own, wave & 3 of a 4-wave group)
template <int HW>
__device__ inline HeadsPrefetch<HW> heads_prefetch(const PolicyArgs& pa, int kq = -1) {
  using P = HeadsPrefetch<HW>;
  const int A = pa.A;
  const int tid = threadIdx.x, w = kq >= 0 ? kq : tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  P pf;
#pragma unroll
  for (int nt = 0; nt < P::NTM; ++nt) {
    if (16 * nt > A) break;   // wave-uniform
    const int j = min(16 * nt + col, A);   // head column: j < A -> pi logit j, j == A -> value
    const float* wrow = (j < A ? pa.Wpi + (int64_t)j * HW : pa.Wv) + P::KW * w;
#pragma unroll
    for (int s = 0; s < P::NS; ++s) pf.wv[nt][s] = *reinterpret_cast<const f32x4*>(wrow + 16 * s + 4 * g);
  }
  const int bj = tid % (A + 1);
  pf.bias = bj < A ? pa.bpi[bj] : pa.bv[0];
  pf.step = pa.mode == 1 ? pa.ctl[CTL_STEP] + pa.step_off : 0;
  return pf;
}

// One wave's K-quarter partial of head tile nt (columns 16 nt .. 16 nt + 15) for 16 rows: lane (g, col)
// returns rows 4 g + r, column 16 nt + col.  hv / wv: the quarter's h and head-weight fragments (k
// permuted identically on both sides); valid == false: a column past A (zero weights).
template <int NS, int NTM>
__device__ inline f32x4 heads_quarter(const f32x4 (&hv)[NS], const f32x4 (&wv)[NTM][NS], int nt, bool valid) {
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const f32x4 wf = valid ? wv[nt][s] : f32x4{0.f, 0.f, 0.f, 0.f};
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][0], wf[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][1], wf[1], c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][2], wf[2], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][3], wf[3], c1, 0, 0, 0);
  }
  f32x4 c;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = __fadd_rn(c0[r], c1[r]);
  return c;
}

// One env row's softmax / log-softmax / entropy / draw from its A + 1 head
// outputs z (z[A] = value); ez: A floats of scratch (exp(z - max) per action).
__device__ inline void heads_row_out(const float* z, float* ez, int64_t row, const PolicyArgs& pa, int64_t step) {
  const int A = pa.A;
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

template <int HW, bool COH, bool LOCAL = false, int ROWS = 16>
__device__ inline void policy_rows16(const float* __restrict__ h, int64_t row0, int64_t n, const PolicyArgs& pa,
                                     float (*part)[16][MAXA + 2], float (*zs)[MAXA + 2],
                                     const HeadsPrefetch<HW>* pre = nullptr) {
  // 4 waves split K = HW into quarters; partial tiles summed in wave order
  constexpr int KW = HW / 4, NS = KW / 16;
  const int A = pa.A;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int64_t rowc = min(row0 + (col < ROWS ? col : ROWS - 1), n - 1);   // A row of this lane (rows past n: any valid row, not stored)
  const HeadsPrefetch<HW> pf = pre != nullptr ? *pre : heads_prefetch<HW>(pa);
  const f32x4 (&wv)[HeadsPrefetch<HW>::NTM][NS] = pf.wv;
  const float bias = pf.bias;
  const int64_t step = pf.step;
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
#pragma unroll
  for (int nt = 0; nt < HeadsPrefetch<HW>::NTM; ++nt) {
    if (16 * nt > A) break;   // wave-uniform
    const int j = 16 * nt + col;
    const f32x4 c = heads_quarter(hv, wv, nt, j <= A);
    if (j <= A) {
#pragma unroll
      for (int r = 0; r < 4; ++r) part[w][4 * g + r][j] = c[r];   // C row 4g + r = env
    }
  }
  __syncthreads();
  for (int i = tid; i < 16 * (A + 1); i += 256) {
    const int r = i / (A + 1), j = i - r * (A + 1);
    float z = __fadd_rn(__fadd_rn(part[0][r][j], part[1][r][j]), __fadd_rn(part[2][r][j], part[3][r][j]));
    zs[r][j] = __fadd_rn(z, i == tid ? bias : (j < A ? pa.bpi[j] : pa.bv[0]));   // (i != tid only for A >= 16)
  }
  __syncthreads();
  const int64_t row = row0 + tid;
  if (tid < ROWS && row < n) heads_row_out(zs[tid], part[0][tid], row, pa, step);
  __syncthreads();   // part / zs free for the caller's next group
}

}  // namespace arl
