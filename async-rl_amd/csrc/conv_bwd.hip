// Fused backward of the two conv layers of the NIPS head (dqn_head.py:41-42)
// for one lockstep window: per sample s
//   (1) dW2 += da2 (x) im2col(a1)           conv2 weight gradient, K = 81 positions
//   (2) da1  = conv_transpose(da2, W2) * (a1 > 0)        (stride-2 parity classes)
//   (3) dW1 += im2col(x)^T (x) da1           conv1 weight gradient, K = 400 positions
// with every operand of a sample resident in LDS (140 KB, one 512-thread
// workgroup per CU): da1 never touches HBM and a1 / da2 / x are read once.
// The next sample's a1 / da2 / screens are loaded into registers while the
// current one computes.
//
// Reference: a3c.py:129-130 (total_loss.backward through Chainer's
// Convolution2D backward: im2col + tensordot for gW, col2im for gx).
//
// (1) runs on v_mfma_f32_16x16x4_f32 (exact f32): M = 32 oc x N = 256 (ic,
//     ky, kx) x K = 81; wave w owns n-tiles 2w, 2w+1 of both m-tiles.
// (2) and (3) run on the bf16 matrix cores with exact bf16 splits of the f32
//     operands (bf16split.hpp; f32-accurate):
// (2) per parity class (py, px): M = 100 positions (7 tiles) x N = 16 ic x
//     K = 128 ordered (dy, dx, oc): A = da2 split planes stored channel-last
//     on an 11 x 11 grid with a zero border (so the shifted windows need no
//     bounds checks), B = W2 fragments of the wave's class held in 48 VGPRs;
//     6 MFMAs per k-step.  The masked result is written as da1 split planes.
// (3) the stride-4 im2col is made contiguous by splitting each screen row
//     into its 4 column phases b = x & 3 (X = x >> 2):
//       dW1[oc][ic][ky][4a + b] = sum_{oy, X} xph[ic][4 oy + ky][b][X + a] da1[oc][oy][X]
//     M = 256 (ic, ky, a, b) x N = 16 oc x K = 480 (oy, X padded 20 -> 24);
//     the A fragment is 8 contiguous pixels shifted by a bytes (v_alignbyte),
//     exact in bf16, so 3 MFMAs per k-step.  Wave w owns m-tiles 2w, 2w+1.
// Integer pixel values feed (3) and 1/255 is applied in the reduction.
// Each block sums a contiguous run of samples and writes one partial slab;
// reduce_conv_bwd_kernel sums the slabs in f64 in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "bf16split.hpp"
#include "conv_slab.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 8 step 1, 16 step 2, 32 step 3, 64 prefetch loads)
#endif

namespace arl {

namespace {
constexpr int NT = 512;                    // threads per workgroup (8 waves, 2 per SIMD)
constexpr int A1_LD = 401;                 // a1 f32 LDS row stride (odd: conflict-free oc spread)
constexpr int XQ = 4 * 84 * 6;             // screen items per sample: (plane, row, quad of 4 dwords)
constexpr int PX = (XQ + NT - 1) / NT;     // 4 per thread
constexpr int PA = (A1 / 4 + NT - 1) / NT; // 4 float4 of a1 per thread
constexpr int PD = (A2 / 4 + NT - 1) / NT; // 2 float4 of da2 per thread
// LDS map (bytes)
constexpr int XR = 24;                     // phase row: X = 0..20 (+ pad), uint8
constexpr int L_XPH = 0;                   // [ic][y][b][XR]                      32,256
constexpr int D1_ROW = 48;                 // da1 plane row (oy): 24 bf16, X 20..23 stay 0
constexpr int D1_OC = 20 * D1_ROW + 16;    // 976 = 61 16-byte slots (odd: oc rows spread over banks)
constexpr int D1P = 16 * D1_OC;            // 15,616 per plane
constexpr int L_D1 = L_XPH + 4 * 84 * 4 * XR;   // 32,256: 3 planes, 46,848
constexpr int D2P = 121 * 64;              // 11 x 11 cells x 32 oc bf16: 7,744 per plane
constexpr int L_D2 = L_D1 + 3 * D1P;       // 79,104: 3 planes, 23,232
constexpr int L_A1 = L_D2 + 3 * D2P;       // 102,336: a1 f32 [16][401]
constexpr int L_D2F = L_A1 + C1_OC * A1_LD * 4;   // 128,000: da2 f32 [32][81]
constexpr int L_RED = L_D2F + A2 * 4;      // 138,368: f32 [NT]
constexpr int L_END = L_RED + NT * 4;      // 140,416
static_assert(L_D1 % 16 == 0 && L_D2 % 16 == 0 && L_A1 % 16 == 0 && L_D2F % 16 == 0, "alignment");
}  // namespace

// da2 plane byte offset of (cell, oc group g = oc >> 3): slot 4 cell + g, low
// 2 bits XORed by cell >> 2 so runs of consecutive cells spread over banks
__device__ inline int d2_slot(int cell, int g) { return (((4 * cell + g) ^ ((cell >> 2) & 3)) << 4); }

struct ConvBwdArgs {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R;
  const float* a1;     // (S, 16, 400)
  const float* da2;    // (S, 32, 81), already masked by a2 > 0
  const float* W2;     // (32, 16, 4, 4)
  int S, spb;
  float* slab;         // (G, SLAB)
  int layout;          // FrameLayout (FRAMES_RGB: (R, n, 3, 84, 84), planes [0, R, G, B];
                       // FRAMES_STACK: (R, n, 4, 84, 84))
};

struct Prefetch {
  uint4 x[PX];
  float4 a[PA];
  float4 d[PD];
};

__device__ inline void prefetch_sample(const ConvBwdArgs& a, int s, Prefetch& r) {
  if (ARL_ABLATE & 64) return;
  const int tid = threadIdx.x;
  const int t = s / a.n, e = s - t * a.n;
  const int64_t ks = a.ctl[CTL_STEP] + t;
  const int rs = (int)(ks % a.R);
  const int nv = a.nvalid[(int64_t)rs * a.n + e];
  int slot[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) slot[c] = (rs + a.R - 3 + c) % a.R;
  // screens: item (plane c, row y, quad q) = dwords 4q..4q+3 of the row (q = 5: dword 20 only)
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int i = tid + NT * j;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < XQ) {
      const int c = i / 504, rem = i - c * 504, y = rem / 6, q = rem - y * 6;
      if (c >= 4 - nv) {
        const int64_t pl = a.layout == FRAMES_STACK ? ((int64_t)rs * a.n + e) * 4 + c
                           : a.layout == FRAMES_RGB ? ((int64_t)rs * a.n + e) * 3 + (c - 1)
                                                    : (int64_t)slot[c] * a.n + e;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.frames + pl * PLANE + y * 84) + 4 * q;
        if (q < 5) { v.x = src[0]; v.y = src[1]; v.z = src[2]; v.w = src[3]; }
        else v.x = src[0];
      }
    }
    r.x[j] = v;
  }
  const float4* g1 = reinterpret_cast<const float4*>(a.a1 + (int64_t)s * A1);
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int i = tid + NT * j;
    r.a[j] = i < A1 / 4 ? g1[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float4* g2 = reinterpret_cast<const float4*>(a.da2 + (int64_t)s * A2);
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int i = tid + NT * j;
    r.d[j] = i < A2 / 4 ? g2[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__device__ inline void commit_sample(const Prefetch& r, uint8_t* lds) {
  const int tid = threadIdx.x;
  // screens -> phase rows: the 4 dwords (X = 4q..4q+3, bytes b = 0..3) are
  // transposed so each phase b gets one dword of 4 consecutive X
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int i = tid + NT * j;
    if (i < XQ) {
      const int c = i / 504, rem = i - c * 504, y = rem / 6, q = rem - y * 6;
      const uint4 v = r.x[j];
      const uint32_t lo01 = __builtin_amdgcn_perm(v.y, v.x, 0x05010400u);
      const uint32_t hi01 = __builtin_amdgcn_perm(v.y, v.x, 0x07030602u);
      const uint32_t lo23 = __builtin_amdgcn_perm(v.w, v.z, 0x05010400u);
      const uint32_t hi23 = __builtin_amdgcn_perm(v.w, v.z, 0x07030602u);
      uint8_t* d = lds + L_XPH + (c * 84 + y) * 4 * XR + 4 * q;
      *reinterpret_cast<uint32_t*>(d) = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
      *reinterpret_cast<uint32_t*>(d + XR) = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
      *reinterpret_cast<uint32_t*>(d + 2 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
      *reinterpret_cast<uint32_t*>(d + 3 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
    }
  }
  float* a1s = reinterpret_cast<float*>(lds + L_A1);
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int i = tid + NT * j;
    if (i < A1 / 4) {
      const int oc = (4 * i) / C1_P, p = 4 * i - oc * C1_P;   // 400 % 4 == 0: one row per float4
      float* d = a1s + oc * A1_LD + p;
      d[0] = r.a[j].x; d[1] = r.a[j].y; d[2] = r.a[j].z; d[3] = r.a[j].w;
    }
  }
  float* d2s = reinterpret_cast<float*>(lds + L_D2F);
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int i = tid + NT * j;
    if (i < A2 / 4) {
      reinterpret_cast<float4*>(d2s)[i] = r.d[j];
      const float dv[4] = {r.d[j].x, r.d[j].y, r.d[j].z, r.d[j].w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int f = 4 * i + t, oc = f / C2_P, p = f - oc * C2_P, oy = p / 9, ox = p - oy * 9;
        uint32_t h, m, l;
        split3(dv[t], h, m, l);
        uint8_t* dd = lds + L_D2 + d2_slot((oy + 1) * 11 + ox + 1, oc >> 3) + (oc & 7) * 2;
        *reinterpret_cast<uint16_t*>(dd) = (uint16_t)h;
        *reinterpret_cast<uint16_t*>(dd + D2P) = (uint16_t)m;
        *reinterpret_cast<uint16_t*>(dd + 2 * D2P) = (uint16_t)l;
      }
    }
  }
}

__device__ inline bf16x8 frag_from_pairs(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3) {
  bf16x8 f;
  f[0] = (short)(p0 & 0xffff); f[1] = (short)(p0 >> 16);
  f[2] = (short)(p1 & 0xffff); f[3] = (short)(p1 >> 16);
  f[4] = (short)(p2 & 0xffff); f[5] = (short)(p2 >> 16);
  f[6] = (short)(p3 & 0xffff); f[7] = (short)(p3 >> 16);
  return f;
}

__global__ void __launch_bounds__(NT)
conv_bwd_kernel(ConvBwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[L_END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const float* a1s = reinterpret_cast<const float*>(lds + L_A1);
  const float* d2s = reinterpret_cast<const float*>(lds + L_D2F);
  float* red = reinterpret_cast<float*>(lds + L_RED);

  // zero the da1 / da2 split planes once: their padding (X 20..23, the grid
  // border) is never written and must read as 0
  for (int i = tid; i < (3 * D1P + 3 * D2P) / 16; i += NT)
    reinterpret_cast<uint4*>(lds + L_D1)[i] = make_uint4(0, 0, 0, 0);

  // (2) W2 fragments of this wave's parity class: lane (ic = col, g), k-step
  // ks = (dy, dx), k = oc = 8 g + j -> W2[oc][ic][py + 2 dy][px + 2 dx]
  const int cls = wave & 3, py = cls >> 1, px = cls & 1;
  bf16x8 w2h[4], w2m[4], w2l[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int tap = (py + 2 * (ks >> 1)) * 4 + px + 2 * (ks & 1);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = a.W2[((8 * g + j) * 16 + col) * 16 + tap];
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3_pack(v[2 * j], v[2 * j + 1], h[j], m[j], l[j]);
    w2h[ks] = frag_from_pairs(h[0], h[1], h[2], h[3]);
    w2m[ks] = frag_from_pairs(m[0], m[1], m[2], m[3]);
    w2l[ks] = frag_from_pairs(l[0], l[1], l[2], l[3]);
  }

  f32x4 acc2[2][2], big3[2], sml3[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc2[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    big3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    sml3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float b2sum = 0.f, b1sum = 0.f;

  // (3): m-tiles mt = 2 w + i -> ic = mt >> 2, ky = 2 (mt & 3) + (col >> 3),
  // a = (col >> 2) & 1, b = col & 3; A row base of lane (phase row of oy = 0)
  int xrow3[2];
  const int sh3 = (col >> 2) & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int mt = 2 * wave + i, ic = mt >> 2, ky = 2 * (mt & 3) + (col >> 3);
    xrow3[i] = L_XPH + ((ic * 84 + ky) * 4 + (col & 3)) * XR;
  }

  const int s0 = blockIdx.x * a.spb, s1 = min(a.S, s0 + a.spb);
  Prefetch pf;
  if (s0 < s1) prefetch_sample(a, s0, pf);
  for (int s = s0; s < s1; ++s) {
    __syncthreads();                 // previous sample fully consumed
    commit_sample(pf, lds);
    __syncthreads();
    if (s + 1 < s1) prefetch_sample(a, s + 1, pf);   // in flight during compute
    // ---- (1) conv2 weight gradient + bias; wave w: n-tiles (ic) 2w, 2w+1 x both m-tiles
    {
      const int oc = tid & 31, ch = tid >> 5;   // 16 chunks of <= 6 positions
      float t = 0.f;
      for (int p = ch * 6; p < min(C2_P, ch * 6 + 6); ++p) t = __fadd_rn(t, d2s[oc * C2_P + p]);
      b2sum = __fadd_rn(b2sum, t);
    }
    {
      const float* b0 = a1s + (2 * wave) * A1_LD + (col >> 2) * 20 + (col & 3);
      const float* b1 = b0 + A1_LD;
#pragma unroll 3
      for (int ps = 0; ps < ((ARL_ABLATE & 8) ? 0 : 21); ++ps) {
        const int p = 4 * ps + g;
        const bool pv = p < C2_P;
        const int pc = pv ? p : 0;
        const int oy = pc / 9, ox = pc - oy * 9;
        const float af0 = pv ? d2s[col * C2_P + pc] : 0.f;
        const float af1 = pv ? d2s[(16 + col) * C2_P + pc] : 0.f;
        const int boff = (2 * oy) * 20 + 2 * ox;
        const float bf0 = b0[boff], bf1 = b1[boff];
        acc2[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(af0, bf0, acc2[0][0], 0, 0, 0);
        acc2[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(af1, bf0, acc2[1][0], 0, 0, 0);
        acc2[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(af0, bf1, acc2[0][1], 0, 0, 0);
        acc2[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(af1, bf1, acc2[1][1], 0, 0, 0);
      }
    }
    // ---- (2) da1 = convT(da2, W2) * (a1 > 0) -> da1 split planes.
    // Wave: class cls, m-tiles (w >> 2) + 2 i, two in flight.
    for (int mA = wave >> 2; mA < 7; mA += 4) {
      const int mB = mA + 2;
      const bool hasB = mB < 7;
      const int rA = 16 * mA + col, rB = 16 * (hasB ? mB : mA) + col;
      const int cA = rA < 100 ? (rA / 10 + 1) * 11 + rA % 10 + 1 : 0;   // invalid rows read the zero border
      const int cB = rB < 100 ? (rB / 10 + 1) * 11 + rB % 10 + 1 : 0;
      f32x4 bigA = {0.f, 0.f, 0.f, 0.f}, smlA = bigA, bigB = bigA, smlB = bigA;
#pragma unroll
      for (int ks = 0; ks < ((ARL_ABLATE & 16) ? 0 : 4); ++ks) {
        const int dcell = (ks >> 1) * 11 + (ks & 1);
        const int oA = L_D2 + d2_slot(cA ? cA - dcell : 0, g);
        const int oB = L_D2 + d2_slot(cB ? cB - dcell : 0, g);
        const bf16x8 ahA = lds_load<bf16x8>(lds, oA), amA = lds_load<bf16x8>(lds, oA + D2P),
                     alA = lds_load<bf16x8>(lds, oA + 2 * D2P);
        const bf16x8 ahB = lds_load<bf16x8>(lds, oB), amB = lds_load<bf16x8>(lds, oB + D2P),
                     alB = lds_load<bf16x8>(lds, oB + 2 * D2P);
        mfma_x6(ahA, amA, alA, w2h[ks], w2m[ks], w2l[ks], bigA, smlA);
        mfma_x6(ahB, amB, alB, w2h[ks], w2m[ks], w2l[ks], bigB, smlB);
      }
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1 && !hasB) break;
        const f32x4 big = pass ? bigB : bigA, sml = pass ? smlB : smlA;
        const int mt = pass ? mB : mA;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = 16 * mt + 4 * g + rr;
          if (r < 100) {
            const int y2 = r / 10, x2 = r - y2 * 10;
            const int oy = 2 * y2 + py, ox = 2 * x2 + px;
            float v = __fadd_rn(big[rr], sml[rr]);
            if (!(a1s[col * A1_LD + oy * 20 + ox] > 0.f)) v = 0.f;
            b1sum = __fadd_rn(b1sum, v);
            uint32_t h, m, l;
            split3(v, h, m, l);
            uint8_t* d = lds + L_D1 + col * D1_OC + oy * D1_ROW + ox * 2;
            *reinterpret_cast<uint16_t*>(d) = (uint16_t)h;
            *reinterpret_cast<uint16_t*>(d + D1P) = (uint16_t)m;
            *reinterpret_cast<uint16_t*>(d + 2 * D1P) = (uint16_t)l;
          }
        }
      }
    }
    __syncthreads();
    // ---- (3) conv1 weight gradient: k-step ks, quarter g -> group G = 4 ks + g
    // = (oy, X0 = 8 c): 8 positions (oy, X0..X0+7)
#pragma unroll 3
    for (int ks = 0; ks < ((ARL_ABLATE & 32) ? 0 : 15); ++ks) {
      const int G = 4 * ks + g, oy = G / 3, c = G - 3 * oy;
      const int ob = L_D1 + col * D1_OC + oy * D1_ROW + 16 * c;
      const bf16x8 bh = lds_load<bf16x8>(lds, ob), bm = lds_load<bf16x8>(lds, ob + D1P),
                   bl = lds_load<bf16x8>(lds, ob + 2 * D1P);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int oa = xrow3[i] + oy * 16 * XR + 8 * c;
        const uint2 lo = lds_load<uint2>(lds, oa);
        const uint32_t nx = lds_load<uint32_t>(lds, oa + 8);
        const uint32_t w0 = __builtin_amdgcn_alignbyte(lo.y, lo.x, sh3);
        const uint32_t w1 = __builtin_amdgcn_alignbyte(nx, lo.y, sh3);
        const bf16x8 xa = frag_from_pairs(px_pair_bf16(w0, 0), px_pair_bf16(w0, 1), px_pair_bf16(w1, 0),
                                          px_pair_bf16(w1, 1));
        mfma_x3(xa, bh, bm, bl, big3[i], sml3[i]);
      }
    }
  }
  // ---- partial slab of this block
  float* out = a.slab + (int64_t)blockIdx.x * SLAB;
  // dW2: C map col = kk within n-tile 2w + jn, rows g*4+r -> oc = 16 mt + g*4 + r
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(16 * mt + g * 4 + r) * 256 + 16 * (2 * wave + jn) + col] = acc2[mt][jn][r];
  // dW1^T: m-tile 2w + i, C row g*4 + r -> (ky low bit, a, b) = (row >> 3, (row >> 2) & 1, row & 3)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int mt = 2 * wave + i, ic = mt >> 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = g * 4 + r;
      const int ky = 2 * (mt & 3) + (row >> 3), kx = 4 * ((row >> 2) & 1) + (row & 3);
      out[SLAB_W1 + (ic * 64 + ky * 8 + kx) * 16 + col] = __fadd_rn(big3[i][r], sml3[i][r]);
    }
  }
  red[tid] = b2sum;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int c = 0; c < NT / 32; ++c) t = __fadd_rn(t, red[c * 32 + tid]);
    out[SLAB_B2 + tid] = t;
  }
  __syncthreads();
  red[tid] = b1sum;   // lane's column = ic = tid & 15
  __syncthreads();
  if (tid < 16) {
    float t = 0.f;
    for (int c = 0; c < NT / 16; ++c) t = __fadd_rn(t, red[c * 16 + tid]);
    out[SLAB_B1 + tid] = t;
  }
}

__global__ void __launch_bounds__(256)
reduce_conv_bwd_kernel(const float* __restrict__ slab, int G, float* __restrict__ gW2, float* __restrict__ gb2,
                       float* __restrict__ gW1, float* __restrict__ gb1, int rgb) {
  __shared__ double part[16][16];
  const int o = blockIdx.x * 16 + (threadIdx.x & 15);
  const int zg = threadIdx.x >> 4;
  double t = 0.0;
  if (o < SLAB)
    for (int z = zg; z < G; z += 16) t += (double)slab[(int64_t)z * SLAB + o];
  part[zg][threadIdx.x & 15] = t;
  __syncthreads();
  if (zg == 0 && o < SLAB) {
    double v = 0.0;
    for (int g = 0; g < 16; ++g) v += part[g][threadIdx.x];
    conv_slab_put(o, v, gW2, gb2, gW1, gb1, rgb);
  }
}

int conv_bwd_blocks(int S) {   // slices actually launched: G0 <= 256 blocks of spb samples
  const int G0 = S < 256 ? S : 256;
  const int spb = (S + G0 - 1) / G0;
  return (S + spb - 1) / spb;
}
int64_t conv_bwd_slab_floats(int S) { return (int64_t)conv_bwd_blocks(S) * SLAB; }

hipError_t launch_conv_bwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int S,
                           const float* a1, const float* da2, const float* W2, float* slab, float* gW2, float* gb2,
                           float* gW1, float* gb1, hipStream_t s, bool reduce, int layout) {
  if (S <= 0) return hipSuccess;
  const int G0 = conv_bwd_blocks(S);
  const int spb = (S + G0 - 1) / G0;
  const int G = (S + spb - 1) / spb;
  ConvBwdArgs a{frames, nvalid, ctl, n, R, a1, da2, W2, S, spb, slab, layout};
  hipLaunchKernelGGL(conv_bwd_kernel, dim3(G), dim3(NT), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !reduce) return e;
  return launch_conv_reduce(slab, S, gW2, gb2, gW1, gb1, s, layout);
}

hipError_t launch_conv_reduce(const float* slab, int S, float* gW2, float* gb2, float* gW1, float* gb1, hipStream_t s,
                              int layout) {
  if (S <= 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_conv_bwd_kernel, dim3((SLAB + 15) / 16), dim3(256), 0, s, slab, conv_bwd_blocks(S), gW2,
                     gb2, gW1, gb1, layout == FRAMES_RGB ? 1 : 0);
  return hipGetLastError();
}

}  // namespace arl
