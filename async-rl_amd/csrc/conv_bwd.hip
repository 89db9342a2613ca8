// Fused backward of the two conv layers of the NIPS head (dqn_head.py:41-42)
// for one lockstep window: per sample s
//   (1) dW2 += da2 (x) im2col(a1)           conv2 weight gradient, K = 81 positions
//   (2) da1  = conv_transpose(da2, W2) * (a1 > 0)        (stride-2 parity classes)
//   (3) dW1 += im2col(x)^T (x) da1           conv1 weight gradient, K = 400 positions
// with a1 / da1, da2, the 4 uint8 screens and W2 resident in LDS (~97 KB,
// one workgroup per CU): da1 never touches HBM and a1 / da2 / x are read once.
// The next sample's a1 / da2 / screens are loaded into registers while the
// current one computes (one wave per SIMD leaves the VGPRs for it).
//
// Reference: a3c.py:129-130 (total_loss.backward through Chainer's
// Convolution2D backward: im2col + tensordot for gW, col2im for gx).
//
// All contractions are v_mfma_f32_16x16x4_f32 (exact f32 products):
//   (1) M = 32 oc (2 tiles) x N = 256 (ic,ky,kx) (16 tiles) x K = 81 (21 k-steps,
//       zero padded): each wave owns n-tiles 4w..4w+3 of both m-tiles (8
//       independent accumulators);
//   (2) per parity class (py,px): M = 100 positions (7 tiles) x N = 16 ic x
//       K = 128 (oc, dy, dx): 28 tile jobs, 7 per wave, two in flight; the
//       masked result overwrites a1 in place (each element has one producer);
//   (3) M = 256 k x N = 16 oc x K = 400: wave w owns input channel ic = w; its
//       4 accumulators are kx = 4 (row & 1) + i for i = 0..3, so one
//       ds_read_b32 of 4 contiguous pixels feeds all four MFMAs.
// Integer pixel values feed (3) and 1/255 is applied in the reduction.
// Each block sums a contiguous run of samples and writes one partial slab;
// reduce_conv_bwd_kernel sums the slabs in f64 in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 8 step 1, 16 step 2, 32 step 3, 64 prefetch loads)
#endif

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int NT = 512;                    // threads per workgroup (8 waves, 2 per SIMD)
constexpr int A1_LD = 401;                 // a1/da1 LDS row stride (odd: conflict-free oc spread)
constexpr int SLAB_W2 = C2_OC * 256;       // 8192
constexpr int SLAB_B2 = SLAB_W2;           // +32
constexpr int SLAB_W1 = SLAB_B2 + C2_OC;   // 8224: D1^T[k][oc], 4096
constexpr int SLAB_B1 = SLAB_W1 + 256 * 16;
constexpr int SLAB = SLAB_B1 + 16;         // 12336 floats per block
constexpr int XV = 4 * PLANE / 16;         // 1764 uint4 of screens per sample
constexpr int PX = (XV + NT - 1) / NT;     // 4 per thread
constexpr int PA = (A1 / 4 + NT - 1) / NT; // 4 float4 of a1 per thread
constexpr int PD = (A2 / 4 + NT - 1) / NT; // 2 float4 of da2 per thread
}  // namespace

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
  constexpr int V = PLANE / 16;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int i = tid + NT * j;
    uint4 v = make_uint4(0, 0, 0, 0);
    const int c = i / V, o = i - c * V;
    if (i < XV && c >= 4 - nv)
      v = reinterpret_cast<const uint4*>(a.frames + ((int64_t)slot[c] * a.n + e) * PLANE)[o];
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

__device__ inline void commit_sample(const Prefetch& r, uint8_t* xs, float* a1s, float* d2s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int i = tid + NT * j;
    if (i < XV) reinterpret_cast<uint4*>(xs)[i] = r.x[j];
  }
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int i = tid + NT * j;
    if (i < A1 / 4) {
      const int oc = (4 * i) / C1_P, p = 4 * i - oc * C1_P;   // 400 % 4 == 0: one row per float4
      float* d = a1s + oc * A1_LD + p;
      d[0] = r.a[j].x; d[1] = r.a[j].y; d[2] = r.a[j].z; d[3] = r.a[j].w;
    }
  }
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int i = tid + NT * j;
    if (i < A2 / 4) reinterpret_cast<float4*>(d2s)[i] = r.d[j];
  }
}

__global__ void __launch_bounds__(NT)
conv_bwd_kernel(ConvBwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[4 * PLANE];   // 28,224
  __shared__ float a1s[C1_OC * A1_LD];                              // 25,664
  __shared__ __attribute__((aligned(16))) float d2s[A2];            // 10,368
  __shared__ float w2t[C2_OC * 256];   // 32,768: W2 as [oc][tap = ky*4 + kx][ic]
  __shared__ float red[NT];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;

  {
    // thread -> (ic = i & 15, oc / tap chunk = i >> 4): reads W2[oc][ic][tap0..tap0+3]
    // (strided, L2), writes w2t[oc][tap][ic] with 16 consecutive ic per row
    float4 wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + NT * j;
      const int ic = i & 15, oc = (i >> 4) >> 2, tq = (i >> 4) & 3;
      wv[j] = reinterpret_cast<const float4*>(a.W2)[(oc * 16 + ic) * 4 + tq];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + NT * j;
      const int ic = i & 15, oc = (i >> 4) >> 2, tq = (i >> 4) & 3;
      float* d = w2t + (oc * 16 + 4 * tq) * 16 + ic;
      d[0] = wv[j].x; d[16] = wv[j].y; d[32] = wv[j].z; d[48] = wv[j].w;
    }
  }

  f32x4 acc2[2][2], acc1[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc2[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float b2sum = 0.f, b1sum = 0.f;

  // (3): wave w owns ic = w >> 1 and kx = 4 (row & 1) + 2 (w & 1) + i, i = 0, 1:
  // A row `col` reads the 2 contiguous pixels at this offset (+ position)
  const int ic3 = wave >> 1, h3 = wave & 1;
  const int xoff3 = ic3 * PLANE + (col >> 1) * 84 + 4 * (col & 1) + 2 * h3;

  const int s0 = blockIdx.x * a.spb, s1 = min(a.S, s0 + a.spb);
  Prefetch pf;
  if (s0 < s1) prefetch_sample(a, s0, pf);
  for (int s = s0; s < s1; ++s) {
    __syncthreads();                 // previous sample fully consumed
    commit_sample(pf, xs, a1s, d2s);
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
        const int p = 4 * ps + q;
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
    __syncthreads();   // a1s is overwritten by (2)
    // ---- (2) da1 = convT(da2, W2) * (a1 > 0), in place; job pairs (w, w+8), (w+16, w+24).
    // k-step ks, lane quarter q: k = 4 ks + q -> oc = ks, dy = q >> 1, dx = q & 1,
    // so a lane's operand addresses are affine in ks (stride 81 / 256 floats).
    {
      const int dy = q >> 1, dx = q & 1;
      for (int jobA = wave; jobA < 28; jobA += 16) {
        const int jobB = jobA + 8;
        const bool hasB = jobB < 28;
        const int clsA = jobA / 7, ttA = jobA - clsA * 7;
        const int clsB = hasB ? jobB / 7 : 0, ttB = hasB ? jobB - clsB * 7 : 0;
        const int pyA = clsA >> 1, pxA = clsA & 1, pyB = clsB >> 1, pxB = clsB & 1;
        const int rA = 16 * ttA + col, rB = 16 * ttB + col;
        const int oyA = rA / 10 - dy, oxA = rA % 10 - dx, oyB = rB / 10 - dy, oxB = rB % 10 - dx;
        const bool okA = rA < 100 && oyA >= 0 && oxA >= 0 && oyA < 9 && oxA < 9;
        const bool okB = hasB && rB < 100 && oyB >= 0 && oxB >= 0 && oyB < 9 && oxB < 9;
        const float* pa = d2s + (okA ? oyA * 9 + oxA : 0);
        const float* pb = d2s + (okB ? oyB * 9 + oxB : 0);
        const float* wa = w2t + ((pyA + 2 * dy) * 4 + pxA + 2 * dx) * 16 + col;
        const float* wb = w2t + ((pyB + 2 * dy) * 4 + pxB + 2 * dx) * 16 + col;
        f32x4 cA = {0.f, 0.f, 0.f, 0.f}, cB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int ks = 0; ks < ((ARL_ABLATE & 16) ? 0 : 32); ++ks) {
          const float afA = okA ? pa[ks * C2_P] : 0.f;
          const float afB = okB ? pb[ks * C2_P] : 0.f;
          cA = __builtin_amdgcn_mfma_f32_16x16x4f32(afA, wa[ks * 256], cA, 0, 0, 0);
          cB = __builtin_amdgcn_mfma_f32_16x16x4f32(afB, wb[ks * 256], cB, 0, 0, 0);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int posA = 16 * ttA + q * 4 + rr;
          if (posA < 100) {
            const int i2 = posA / 10, j2 = posA - i2 * 10;
            float* d = a1s + col * A1_LD + (2 * i2 + pyA) * 20 + 2 * j2 + pxA;
            *d = *d > 0.f ? cA[rr] : 0.f;
          }
          const int posB = 16 * ttB + q * 4 + rr;
          if (hasB && posB < 100) {
            const int i2 = posB / 10, j2 = posB - i2 * 10;
            float* d = a1s + col * A1_LD + (2 * i2 + pyB) * 20 + 2 * j2 + pxB;
            *d = *d > 0.f ? cB[rr] : 0.f;
          }
        }
      }
    }
    __syncthreads();
    // ---- (3) conv1 weight gradient + bias from da1 (in a1s)
    {
      const int oc = tid & 15, ch = tid >> 4;   // 32 chunks of <= 13 positions
      float t = 0.f;
      for (int p = ch * 13; p < min(C1_P, ch * 13 + 13); ++p) t = __fadd_rn(t, a1s[oc * A1_LD + p]);
      b1sum = __fadd_rn(b1sum, t);
    }
#pragma unroll 2
    for (int ps = 0; ps < ((ARL_ABLATE & 32) ? 0 : C1_P / 4); ++ps) {
      const int p = 4 * ps + q;
      const int oy = p / 20, ox = p - oy * 20;
      const uint32_t w2 = *reinterpret_cast<const uint16_t*>(xs + xoff3 + (4 * oy) * 84 + 4 * ox);
      const float bf = a1s[col * A1_LD + p];
      acc1[0] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(w2 & 0xff), bf, acc1[0], 0, 0, 0);
      acc1[1] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(w2 >> 8), bf, acc1[1], 0, 0, 0);
    }
  }
  // ---- partial slab of this block
  float* out = a.slab + (int64_t)blockIdx.x * SLAB;
  // dW2: C map col = kk within n-tile 2w + jn, rows q*4+r -> oc = 16 mt + q*4 + r
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(16 * mt + q * 4 + r) * 256 + 16 * (2 * wave + jn) + col] = acc2[mt][jn][r];
  // dW1^T: accumulator i, C row q*4 + r -> k = (ic3, ky = row >> 1, kx = 4 (row & 1) + 2 h3 + i)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = q * 4 + r;
      const int k = ic3 * 64 + (row >> 1) * 8 + 4 * (row & 1) + 2 * h3 + i;
      out[SLAB_W1 + k * 16 + col] = acc1[i][r];
    }
  red[tid] = b2sum;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int c = 0; c < NT / 32; ++c) t = __fadd_rn(t, red[c * 32 + tid]);
    out[SLAB_B2 + tid] = t;
  }
  __syncthreads();
  red[tid] = b1sum;
  __syncthreads();
  if (tid < 16) {
    float t = 0.f;
    for (int c = 0; c < NT / 16; ++c) t = __fadd_rn(t, red[c * 16 + tid]);
    out[SLAB_B1 + tid] = t;
  }
}

__global__ void __launch_bounds__(256)
reduce_conv_bwd_kernel(const float* __restrict__ slab, int G, float* __restrict__ gW2, float* __restrict__ gb2,
                       float* __restrict__ gW1, float* __restrict__ gb1) {
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
    if (o < SLAB_B2) gW2[o] = (float)v;                       // [oc][ic*16 + ky*4 + kx]
    else if (o < SLAB_W1) gb2[o - SLAB_B2] = (float)v;
    else if (o < SLAB_B1) {
      const int kk = o - SLAB_W1, k = kk >> 4, oc = kk & 15;
      gW1[oc * 256 + k] = (float)(v / 255.0);                 // integer pixels -> /255 here
    } else gb1[o - SLAB_B1] = (float)v;
  }
}

int conv_bwd_blocks(int S) { return S < 256 ? S : 256; }
int64_t conv_bwd_slab_floats(int S) { return (int64_t)conv_bwd_blocks(S) * SLAB; }

hipError_t launch_conv_bwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int S,
                           const float* a1, const float* da2, const float* W2, float* slab, float* gW2, float* gb2,
                           float* gW1, float* gb1, hipStream_t s) {
  if (S <= 0) return hipSuccess;
  const int G0 = conv_bwd_blocks(S);
  const int spb = (S + G0 - 1) / G0;
  const int G = (S + spb - 1) / spb;
  ConvBwdArgs a{frames, nvalid, ctl, n, R, a1, da2, W2, S, spb, slab};
  hipLaunchKernelGGL(conv_bwd_kernel, dim3(G), dim3(NT), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(reduce_conv_bwd_kernel, dim3((SLAB + 15) / 16), dim3(256), 0, s, slab, G, gW2, gb2, gW1, gb1);
  return hipGetLastError();
}

}  // namespace arl
