// Fused forward of the NIPS head's two conv layers (dqn_head.py:41-42,48-52)
// for one env per workgroup, straight from the uint8 frame ring:
//   a1 = relu(conv(x/255, W1, s4) + b1)   (16 x 20 x 20)  -> LDS + HBM (kept for backward)
//   a2 = relu(conv(a1, W2, s2) + b2)      (32 x 9 x 9)    -> HBM
// Both contractions run on the bf16 matrix cores with exact bf16 splits of
// the f32 operands (bf16split.hpp): conv1 multiplies the integer pixel values
// (exact in bf16; 1/255 is applied to the sum) by W1 = h + m + l, 3 MFMAs per
// k-step; conv2 multiplies a1 = h + m + l by W2 = h + m + l, 6 MFMAs.
//
// LDS (145.5 KB, one 512-thread workgroup per CU = 2 waves per SIMD):
//   xb   4 screens as bf16 [ic][y][x]                         56,448 B
//   R1   W1 split planes [3][oc][k] (rows padded to 528 B),   25,344 B
//        then (after every wave holds its W1 fragments) the a1 split planes
//        [3][pixel][ic] with an XOR swizzle of the 16-byte slots  38,400 B
//   W2p  W2 split planes [3][oc][tap][ic] (rows 528 B)         50,688 B
//
// conv1: M = 400 positions (25 tiles), N = 16 oc, K = 256 ordered (ic, ky, kx):
//   k-step s, lane quarter g -> (ic, ky) = divmod(4 s + g, 8), kx = 0..7, i.e.
//   8 contiguous bf16 pixels per lane; W1 fragments live in 96 VGPRs.
// conv2: M = 81 positions (6 tiles), N = 32 oc (2 tiles), K = 256 ordered
//   (tap = ky*4 + kx, ic): k-step s, quarter g -> tap 2 s + (g >> 1), ic
//   8 (g & 1) + 0..7 = one 16-byte read of a channel-last a1 pixel.  Wave w
//   owns n-tile w & 1 (its W2 fragments in 96 VGPRs) and m-tiles w >> 1 and
//   (w >> 1) + 4: three jobs per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "bf16split.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 1 conv1 MFMA, 2 conv2 MFMA, 4 staging loads,
                       // 8 weight loads + splits, 16 epilogue /255 as a multiply)
#endif

namespace arl {

namespace {
constexpr int NT = 512;                  // threads per workgroup (8 waves)
constexpr int XB_ROW = 84 * 2;           // bytes per bf16 screen row
constexpr int XB_PLANE = PLANE * 2;      // 14,112 bytes per bf16 screen
constexpr int WROW = 528;                // bytes per oc row of a weight plane (512 + 16: conflict-free b128)
constexpr int W1P = 16 * WROW;           // 8,448 per W1 plane
constexpr int W2P = 32 * WROW;           // 16,896 per W2 plane
constexpr int A1P = C1_P * 32;           // 12,800 per a1 plane: 400 pixels x 16 ic bf16
constexpr int L_XB = 0;
constexpr int L_R1 = L_XB + 4 * XB_PLANE;   // 56,448
constexpr int L_W2 = L_R1 + 3 * A1P;        // 94,848
constexpr int L_END = L_W2 + 3 * W2P;       // 145,536
static_assert(3 * W1P <= 3 * A1P, "W1 planes fit the a1 region");
}  // namespace

// a1 plane byte offset of (pixel P, ic half h): 16-byte slot 2P + h with its
// low 4 bits XORed by P >> 3, so conv2's 16 lanes (positions 2 pixels apart)
// spread over the LDS banks
__device__ inline int a1_slot(int P, int h) { return (((2 * P + h) ^ ((P >> 3) & 15)) << 4); }

struct ConvFwdArgs {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R, t;          // obs step = ctl[STEP] + t; env = blockIdx.x
  const float* W1;      // (16, 4, 8, 8); RGB nets (16, 3, 8, 8) for input planes 1..3
  const float* b1;
  const float* W2;      // (32, 16, 4, 4)
  const float* b2;
  float* a1;            // (n, 16, 400)
  float* a2;            // (n, 32, 81)
  int layout;           // FrameLayout: FRAMES_RGB = (R, n, 3, 84, 84), planes [0, R, G, B] of slot ks % R;
                        // FRAMES_STACK = (R, n, 4, 84, 84), the 4 planes of slot ks % R
  int e0;               // first env of this launch (env = e0 + blockIdx.x)
};

__global__ void __launch_bounds__(NT)
conv_fwd_kernel(ConvFwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[L_END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const int e = a.e0 + blockIdx.x;
  // ---- stage: all global loads first, then bf16 conversion / splitting into LDS
  {
    const int64_t ks = a.ctl[CTL_STEP] + a.t;
    const int rs = (int)(ks % a.R);
    const int nv = a.nvalid[(int64_t)rs * a.n + e];
    int slot[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) slot[c] = (rs + a.R - 3 + c) % a.R;
    constexpr int V = PLANE / 16;              // 441 uint4 per screen
    constexpr int NX = (4 * V + NT - 1) / NT;  // 4
    uint4 xv[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      const int c = i / V, o = i - c * V;
      xv[j] = make_uint4(0, 0, 0, 0);
      if (!(ARL_ABLATE & 4) && i < 4 * V && c >= 4 - nv)   // planes older than the last reset read as 0
        xv[j] = reinterpret_cast<const uint4*>(
            a.frames + (a.layout == FRAMES_STACK ? ((int64_t)rs * a.n + e) * 4 + c
                        : a.layout == FRAMES_RGB ? ((int64_t)rs * a.n + e) * 3 + (c - 1)
                                                 : (int64_t)slot[c] * a.n + e) * PLANE)[o];
    }
    // W1: thread -> 8 consecutive k of one oc; W2: thread -> (oc, 4 ic, 4 taps)
    const int w1oc = tid >> 5, w1k = (8 * tid) & 255;
    const int w2oc = tid >> 4, ic4 = (tid >> 2) & 3, tg = tid & 3;
#if !(ARL_ABLATE & 8)
    float4 w1a = make_float4(0.f, 0.f, 0.f, 0.f), w1b = w1a;   // RGB: input plane 0 is the zero pad
    const bool rgb = a.layout == FRAMES_RGB;
    if (!rgb || w1k >= 64) {
      const float4* w1p = reinterpret_cast<const float4*>(rgb ? a.W1 + w1oc * 192 + w1k - 64 : a.W1 + 8 * tid);
      w1a = w1p[0];
      w1b = w1p[1];
    }
    float4 w2v[4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
      w2v[ii] = reinterpret_cast<const float4*>(a.W2)[(w2oc * 16 + 4 * ic4 + ii) * 4 + tg];
#endif
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      if (i < 4 * V) {
        const int c = i / V, o = i - c * V;
        uint4 lo, hi;
        lo.x = px_pair_bf16(xv[j].x, 0); lo.y = px_pair_bf16(xv[j].x, 1);
        lo.z = px_pair_bf16(xv[j].y, 0); lo.w = px_pair_bf16(xv[j].y, 1);
        hi.x = px_pair_bf16(xv[j].z, 0); hi.y = px_pair_bf16(xv[j].z, 1);
        hi.z = px_pair_bf16(xv[j].w, 0); hi.w = px_pair_bf16(xv[j].w, 1);
        uint4* d = reinterpret_cast<uint4*>(lds + L_XB + c * XB_PLANE + o * 32);
        d[0] = lo;
        d[1] = hi;
      }
    }
#if !(ARL_ABLATE & 8)
    {
      uint4 ph, pm, pl;
      split3_pack(w1a.x, w1a.y, ph.x, pm.x, pl.x);
      split3_pack(w1a.z, w1a.w, ph.y, pm.y, pl.y);
      split3_pack(w1b.x, w1b.y, ph.z, pm.z, pl.z);
      split3_pack(w1b.z, w1b.w, ph.w, pm.w, pl.w);
      uint8_t* d = lds + L_R1 + w1oc * WROW + w1k * 2;
      *reinterpret_cast<uint4*>(d) = ph;
      *reinterpret_cast<uint4*>(d + W1P) = pm;
      *reinterpret_cast<uint4*>(d + 2 * W1P) = pl;
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const float v0 = w2v[0][tt], v1 = w2v[1][tt], v2 = w2v[2][tt], v3 = w2v[3][tt];
      uint2 ph, pm, pl;
      split3_pack(v0, v1, ph.x, pm.x, pl.x);
      split3_pack(v2, v3, ph.y, pm.y, pl.y);
      uint8_t* d = lds + L_W2 + w2oc * WROW + ((4 * tg + tt) * 16 + 4 * ic4) * 2;
      *reinterpret_cast<uint2*>(d) = ph;
      *reinterpret_cast<uint2*>(d + W2P) = pm;
      *reinterpret_cast<uint2*>(d + 2 * W2P) = pl;
    }
#endif
  }
  __syncthreads();
  // ---- conv1 B fragments: lane (oc = col, g), k-step s -> k = 8 (4 s + g) + 0..7
  bf16x8 w1h[8], w1m[8], w1l[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int off = L_R1 + col * WROW + (4 * s + g) * 16;
    w1h[s] = lds_load<bf16x8>(lds, off);
    w1m[s] = lds_load<bf16x8>(lds, off + W1P);
    w1l[s] = lds_load<bf16x8>(lds, off + 2 * W1P);
  }
  __syncthreads();   // the W1 planes are overwritten by the a1 planes below
  const float bias1 = a.b1[col];
  float* a1g = a.a1 + (int64_t)e * A1;
  // tiles w, w + 8, w + 16 (and 24 on wave 0): 25 tiles over 8 waves in one pass,
  // 3-4 independent accumulator chains per wave (per-tile k order unchanged)
  {
    constexpr int TJ = 4;
    const bool has3 = wave + 24 < 25;   // wave-uniform
    int baseX[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int tl = (j < 3 || has3) ? wave + 8 * j : wave;
      const int p = tl * 16 + col, oy = p / 20, ox = p - oy * 20;
      baseX[j] = L_XB + (4 * oy) * XB_ROW + 8 * ox;
    }
    f32x4 big[TJ], sml[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) big[j] = sml[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < ((ARL_ABLATE & 1) ? 0 : 8); ++s) {
      const int u = 4 * s + g, off = (u >> 3) * XB_PLANE + (u & 7) * XB_ROW;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const bf16x8 xa = lds_load8_a8(lds, baseX[j] + off);
        mfma_x3(xa, w1h[s], w1m[s], w1l[s], big[j], sml[j]);
      }
      if (has3) {
        const bf16x8 xa = lds_load8_a8(lds, baseX[3] + off);
        mfma_x3(xa, w1h[s], w1m[s], w1l[s], big[3], sml[3]);
      }
    }
    // C rows g*4 + r -> positions tile*16 + g*4 + r, col = oc
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      if (j == 3 && !has3) break;
      const int p0 = (wave + 8 * j) * 16 + g * 4;
      float ov[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ov[r] = (ARL_ABLATE & 16) ? fmaxf(__fadd_rn(__fmul_rn(__fadd_rn(big[j][r], sml[j][r]), 1.f / 255.f), bias1), 0.f)
                                  : fmaxf(__fadd_rn(__fdiv_rn(__fadd_rn(big[j][r], sml[j][r]), 255.f), bias1), 0.f);
      *reinterpret_cast<float4*>(a1g + col * C1_P + p0) = make_float4(ov[0], ov[1], ov[2], ov[3]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        uint32_t h, m, l;
        split3(ov[r], h, m, l);
        const int off = L_R1 + a1_slot(p0 + r, col >> 3) + (col & 7) * 2;
        *reinterpret_cast<uint16_t*>(lds + off) = (uint16_t)h;
        *reinterpret_cast<uint16_t*>(lds + off + A1P) = (uint16_t)m;
        *reinterpret_cast<uint16_t*>(lds + off + 2 * A1P) = (uint16_t)l;
      }
    }
  }
  __syncthreads();
  // ---- conv2: wave -> n-tile nt = w & 1 (oc = 16 nt + col), m-tiles w >> 1, (w >> 1) + 4
  {
    const int nt = wave & 1, oc = 16 * nt + col;
    bf16x8 w2h[8], w2m[8], w2l[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int off = L_W2 + oc * WROW + (2 * s + (g >> 1)) * 32 + (g & 1) * 16;
      w2h[s] = lds_load<bf16x8>(lds, off);
      w2m[s] = lds_load<bf16x8>(lds, off + W2P);
      w2l[s] = lds_load<bf16x8>(lds, off + 2 * W2P);
    }
    const int mA = wave >> 1, mB = mA + 4;
    const bool hasB = mB < 6;
    const int posA = 16 * mA + col, posB = 16 * (hasB ? mB : mA) + col;   // A row of this lane
    const int pcA = posA < C2_P ? posA : 0, pcB = posB < C2_P ? posB : 0;
    const int oyA = pcA / 9, oxA = pcA - oyA * 9, oyB = pcB / 9, oxB = pcB - oyB * 9;
    const int PA0 = (2 * oyA) * 20 + 2 * oxA, PB0 = (2 * oyB) * 20 + 2 * oxB;
    f32x4 bigA = {0.f, 0.f, 0.f, 0.f}, smlA = bigA, bigB = bigA, smlB = bigA;
#pragma unroll
    for (int s = 0; s < ((ARL_ABLATE & 2) ? 0 : 8); ++s) {
      const int tap = 2 * s + (g >> 1), dP = (tap >> 2) * 20 + (tap & 3);
      const int offA = L_R1 + a1_slot(PA0 + dP, g & 1);
      const bf16x8 ahA = lds_load<bf16x8>(lds, offA), amA = lds_load<bf16x8>(lds, offA + A1P),
                   alA = lds_load<bf16x8>(lds, offA + 2 * A1P);
      mfma_x6(ahA, amA, alA, w2h[s], w2m[s], w2l[s], bigA, smlA);
      if (hasB) {
        const int offB = L_R1 + a1_slot(PB0 + dP, g & 1);
        const bf16x8 ahB = lds_load<bf16x8>(lds, offB), amB = lds_load<bf16x8>(lds, offB + A1P),
                     alB = lds_load<bf16x8>(lds, offB + 2 * A1P);
        mfma_x6(ahB, amB, alB, w2h[s], w2m[s], w2l[s], bigB, smlB);
      }
    }
    float* a2g = a.a2 + (int64_t)e * A2;
    const float b = a.b2[oc];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * mA + g * 4 + r;
      if (p < C2_P) a2g[oc * C2_P + p] = fmaxf(__fadd_rn(__fadd_rn(bigA[r], smlA[r]), b), 0.f);
    }
    if (hasB) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * mB + g * 4 + r;
        if (p < C2_P) a2g[oc * C2_P + p] = fmaxf(__fadd_rn(__fadd_rn(bigB[r], smlB[r]), b), 0.f);
      }
    }
  }
}

hipError_t launch_conv_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t,
                           const float* W1, const float* b1, const float* W2, const float* b2, float* a1, float* a2,
                           hipStream_t s, int layout, int e0, int ne) {
  if (n <= 0) return hipSuccess;
  if (ne < 0) ne = n;
  if (ne <= 0) return hipSuccess;
  ConvFwdArgs a{frames, nvalid, ctl, n, R, t, W1, b1, W2, b2, a1, a2, layout, e0};
  hipLaunchKernelGGL(conv_fwd_kernel, dim3(ne), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace arl
