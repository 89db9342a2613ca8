// Fused forward of the NIPS head's two conv layers (dqn_head.py:41-42,48-52)
// for one env per workgroup, straight from the uint8 frame ring:
//   a1 = relu(conv(x/255, W1, s4) + b1)   (16 x 20 x 20)  -> LDS + HBM (kept for backward)
//   a2 = relu(conv(a1, W2, s2) + b2)      (32 x 9 x 9)    -> HBM
// LDS: the 4 screens (28 KB, planes older than the env's last reset read as
// 0), W1 (16 KB), W2 (48 KB, k-major, padded) and a1 (25.6 KB) -- one
// 512-thread workgroup per CU, i.e. two waves per SIMD so one wave's LDS and
// dependency stalls hide behind the other's MFMAs (rocprof: one wave per SIMD
// left the MFMA pipe busy only ~26% of the time).
//
// conv1: C[p][oc], 25 position tiles x K 256, v_mfma_f32_16x16x4_f32 on the
// integer pixel values (1/255 applied to the sum in the epilogue; dqn_phi.py:16).
// The K order is permuted so one ds_read_b32 of 4 contiguous pixels feeds 4
// k-steps: k-step 4j + r, lane quarter q -> (ic, ky) = divmod(2j + (q >> 1), 8),
// kx = 4 (q & 1) + r; the weights follow the same permutation and live in 64
// VGPRs.  Two tiles in flight per wave.
// conv2: C[p][oc] with M = 81 (6 tiles), N = 32 (2 tiles), K = 256 = (ic, ky,
// kx) read from a1 in LDS: 12 tile jobs over 8 waves.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 1 conv1 MFMA, 2 conv2 MFMA, 4 staging loads)
#endif

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int NT = 512;      // threads per workgroup (8 waves)
constexpr int A1_LD = 401;   // a1 rows (per oc) in LDS, odd stride: lanes reading 16 oc hit 16 banks
constexpr int W1_LD = 257;   // W1 rows (per oc), odd stride for the same reason
constexpr int W2_LD = 48;    // W2 stored k-major: w2k[k * 48 + oc]; lanes (q, oc) -> banks 16q + oc
}  // namespace

struct ConvFwdArgs {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R, t;          // obs step = ctl[STEP] + t; env = blockIdx.x
  const float* W1;      // (16, 4, 8, 8)
  const float* b1;
  const float* W2;      // (32, 16, 4, 4)
  const float* b2;
  float* a1;            // (n, 16, 400)
  float* a2;            // (n, 32, 81)
};

__device__ inline float4 relu_scaled(f32x4 c, float bias) {
  float4 o;
  o.x = fmaxf(__fadd_rn(__fdiv_rn(c[0], 255.f), bias), 0.f);
  o.y = fmaxf(__fadd_rn(__fdiv_rn(c[1], 255.f), bias), 0.f);
  o.z = fmaxf(__fadd_rn(__fdiv_rn(c[2], 255.f), bias), 0.f);
  o.w = fmaxf(__fadd_rn(__fdiv_rn(c[3], 255.f), bias), 0.f);
  return o;
}

__global__ void __launch_bounds__(NT)
conv_fwd_kernel(ConvFwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[4 * PLANE];   // 28,224
  __shared__ float w1s[16 * W1_LD];                                 // 16,448
  __shared__ float w2k[256 * W2_LD];                                // 49,152
  __shared__ float a1s[C1_OC * A1_LD];                              // 25,664
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;
  const int e = blockIdx.x;
  // ---- stage screens + weights: every global load issued before the LDS
  // writes; the weight writes are laid out so 32 consecutive lanes hit 32 banks
  {
    const int64_t ks = a.ctl[CTL_STEP] + a.t;
    const int rs = (int)(ks % a.R);
    const int nv = a.nvalid[(int64_t)rs * a.n + e];
    int slot[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) slot[c] = (rs + a.R - 3 + c) % a.R;
    constexpr int V = PLANE / 16;            // 441 uint4 per screen
    constexpr int NX = (4 * V + NT - 1) / NT;  // 4
    uint4 xv[NX];
    float4 w1v[2], w2v[4];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      const int c = i / V, o = i - c * V;
      xv[j] = make_uint4(0, 0, 0, 0);
      if (!(ARL_ABLATE & 4) && i < 4 * V && c >= 4 - nv)
        xv[j] = reinterpret_cast<const uint4*>(a.frames + ((int64_t)slot[c] * a.n + e) * PLANE)[o];
    }
    // W1: thread -> (oc = i & 15, chunk = i >> 4); W2: (oc = i & 31, chunk = i >> 5)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + NT * j;
      w1v[j] = reinterpret_cast<const float4*>(a.W1)[(i & 15) * 64 + (i >> 4)];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + NT * j;
      w2v[j] = reinterpret_cast<const float4*>(a.W2)[(i & 31) * 64 + (i >> 5)];
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      if (i < 4 * V) reinterpret_cast<uint4*>(xs)[i] = xv[j];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + NT * j;
      float* d = w1s + (i & 15) * W1_LD + 4 * (i >> 4);
      d[0] = w1v[j].x; d[1] = w1v[j].y; d[2] = w1v[j].z; d[3] = w1v[j].w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + NT * j;
      const int oc = i & 31, k = 4 * (i >> 5);
      w2k[(k + 0) * W2_LD + oc] = w2v[j].x;
      w2k[(k + 1) * W2_LD + oc] = w2v[j].y;
      w2k[(k + 2) * W2_LD + oc] = w2v[j].z;
      w2k[(k + 3) * W2_LD + oc] = w2v[j].w;
    }
  }
  __syncthreads();
  // ---- conv1: permuted weights of this lane (B[k][n = oc = col])
  float wf[64];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int u = 2 * j + (q >> 1), ic = u >> 3, ky = u & 7;
#pragma unroll
    for (int r = 0; r < 4; ++r) wf[4 * j + r] = w1s[col * W1_LD + ic * 64 + ky * 8 + 4 * (q & 1) + r];
  }
  const float bias1 = a.b1[col];
  float* a1g = a.a1 + (int64_t)e * A1;
  // tile pairs (w, w+8), (w+16, w+24): 25 tiles over 8 waves
  for (int tA = wave; tA < 25; tA += 16) {
    const int tB = tA + 8;
    const bool hasB = tB < 25;
    const int pA = tA * 16 + col, pB = (hasB ? tB : tA) * 16 + col;
    const int oyA = pA / 20, oxA = pA - oyA * 20, oyB = pB / 20, oxB = pB - oyB * 20;
    const uint8_t* baseA = xs + (4 * oyA) * 84 + 4 * oxA + 4 * (q & 1);
    const uint8_t* baseB = xs + (4 * oyB) * 84 + 4 * oxB + 4 * (q & 1);
    f32x4 cA = {0.f, 0.f, 0.f, 0.f}, cB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < ((ARL_ABLATE & 1) ? 0 : 16); ++j) {
      const int u = 2 * j + (q >> 1), ic = u >> 3, ky = u & 7;
      const int off = ic * PLANE + ky * 84;
      const uint32_t wA = *reinterpret_cast<const uint32_t*>(baseA + off);
      const uint32_t wB = *reinterpret_cast<const uint32_t*>(baseB + off);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        cA = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((wA >> (8 * r)) & 0xff), wf[4 * j + r], cA, 0, 0, 0);
        cB = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((wB >> (8 * r)) & 0xff), wf[4 * j + r], cB, 0, 0, 0);
      }
    }
    // C rows q*4 + r -> positions tile*16 + q*4 + r, col = oc
    float4 o = relu_scaled(cA, bias1);
    int p0 = tA * 16 + q * 4;
    *reinterpret_cast<float4*>(a1g + col * C1_P + p0) = o;
    float* d = a1s + col * A1_LD + p0;
    d[0] = o.x; d[1] = o.y; d[2] = o.z; d[3] = o.w;
    if (hasB) {
      o = relu_scaled(cB, bias1);
      p0 = tB * 16 + q * 4;
      *reinterpret_cast<float4*>(a1g + col * C1_P + p0) = o;
      d = a1s + col * A1_LD + p0;
      d[0] = o.x; d[1] = o.y; d[2] = o.z; d[3] = o.w;
    }
  }
  __syncthreads();
  // ---- conv2: jobs j = wave, wave + 8 (< 12) -> (m-tile j >> 1, n-tile j & 1)
  {
    const int jA = wave, jB = wave + 8;
    const bool hasB = jB < 12;
    const int mtA = jA >> 1, ntA = jA & 1, mtB = hasB ? jB >> 1 : mtA, ntB = hasB ? jB & 1 : ntA;
    const int posA = 16 * mtA + col, posB = 16 * mtB + col;   // A row of this lane
    const bool okA = posA < C2_P, okB = posB < C2_P;
    const int pcA = okA ? posA : 0, pcB = okB ? posB : 0;
    const int rowA = (2 * (pcA / 9)) * 20 + 2 * (pcA % 9);
    const int rowB = (2 * (pcB / 9)) * 20 + 2 * (pcB % 9);
    const float* w2A = w2k + q * W2_LD + 16 * ntA + col;
    const float* w2B = w2k + q * W2_LD + 16 * ntB + col;
    f32x4 cA = {0.f, 0.f, 0.f, 0.f}, cB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < ((ARL_ABLATE & 2) ? 0 : 64); ++ks) {
      // k = 4 ks + q = (ic, ky, kx) = (ks >> 2, ks & 3, q)
      const int aoff = (ks >> 2) * A1_LD + (ks & 3) * 20 + q;
      const float afA = okA ? a1s[aoff + rowA] : 0.f;
      const float afB = okB ? a1s[aoff + rowB] : 0.f;
      cA = __builtin_amdgcn_mfma_f32_16x16x4f32(afA, w2A[4 * ks * W2_LD], cA, 0, 0, 0);
      cB = __builtin_amdgcn_mfma_f32_16x16x4f32(afB, w2B[4 * ks * W2_LD], cB, 0, 0, 0);
    }
    float* a2g = a.a2 + (int64_t)e * A2;
    {
      const int oc = 16 * ntA + col;
      const float b = a.b2[oc];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * mtA + q * 4 + r;
        if (p < C2_P) a2g[oc * C2_P + p] = fmaxf(__fadd_rn(cA[r], b), 0.f);
      }
    }
    if (hasB) {
      const int oc = 16 * ntB + col;
      const float b = a.b2[oc];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * mtB + q * 4 + r;
        if (p < C2_P) a2g[oc * C2_P + p] = fmaxf(__fadd_rn(cB[r], b), 0.f);
      }
    }
  }
}

hipError_t launch_conv_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t,
                           const float* W1, const float* b1, const float* W2, const float* b2, float* a1, float* a2,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  ConvFwdArgs a{frames, nvalid, ctl, n, R, t, W1, b1, W2, b2, a1, a2};
  hipLaunchKernelGGL(conv_fwd_kernel, dim3(n), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace arl
