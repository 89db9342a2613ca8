// Fused backward of the two conv layers of the NIPS head (dqn_head.py:41-42)
// for one lockstep window: per sample s
//   (1) dW2 += da2 (x) im2col(a1)           conv2 weight gradient, K = 81 positions
//   (2) da1  = conv_transpose(da2, W2) * (a1 > 0)        (stride-2 parity classes)
//   (3) dW1 += im2col(x)^T (x) da1           conv1 weight gradient, K = 400 positions
// with a1 / da1, da2, the 4 uint8 screens and W2 resident in LDS (~97 KB,
// one workgroup per CU): da1 never touches HBM and a1 / da2 / x are read once.
//
// Reference: a3c.py:129-130 (total_loss.backward through Chainer's
// Convolution2D backward: im2col + tensordot for gW, col2im for gx).
//
// All contractions are v_mfma_f32_16x16x4_f32 (exact f32 products):
//   (1) M = 32 oc (2 tiles) x N = 256 (ic,ky,kx) (16 tiles) x K = 81 (21 k-steps,
//       zero padded): each wave owns n-tiles 4w..4w+3 of both m-tiles (32 acc regs);
//   (2) per parity class (py,px): M = 100 positions (7 tiles) x N = 16 ic x
//       K = 128 (oc, dy, dx): 28 tile jobs, 7 per wave; the masked result
//       overwrites a1 in place (each element has exactly one producer);
//   (3) M = 256 k (16 tiles, 4 per wave, 16 acc regs) x N = 16 oc x K = 400.
// Integer pixel values feed (3) and 1/255 is applied in the reduction.
// Each block sums a contiguous run of samples and writes one partial slab;
// reduce_conv_bwd_kernel sums the slabs in f64 in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int A1_LD = 401;                 // a1/da1 LDS row stride (odd: conflict-free oc spread)
constexpr int SLAB_W2 = C2_OC * 256;       // 8192
constexpr int SLAB_B2 = SLAB_W2;           // +32
constexpr int SLAB_W1 = SLAB_B2 + C2_OC;   // 8224: D1^T[k][oc], 4096
constexpr int SLAB_B1 = SLAB_W1 + 256 * 16;
constexpr int SLAB = SLAB_B1 + 16;         // 12336 floats per block
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

__global__ void __launch_bounds__(256)
conv_bwd_kernel(ConvBwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[4 * PLANE];   // 28,224
  __shared__ float a1s[C1_OC * A1_LD];                              // 25,664
  __shared__ __attribute__((aligned(16))) float d2s[A2];            // 10,368
  __shared__ __attribute__((aligned(16))) float w2s[C2_OC * 256];   // 32,768
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;

  for (int i = tid; i < C2_OC * 256 / 4; i += 256)
    reinterpret_cast<float4*>(w2s)[i] = reinterpret_cast<const float4*>(a.W2)[i];

  f32x4 acc2[2][4], acc1[4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) acc1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float b2sum = 0.f, b1sum = 0.f;

  // conv1 wgrad A rows of this lane: k = 16 (4 wave + i) + col
  int koff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 16 * (4 * wave + i) + col;
    koff[i] = (k >> 6) * PLANE + ((k >> 3) & 7) * 84 + (k & 7);
  }

  const int s0 = blockIdx.x * a.spb, s1 = min(a.S, s0 + a.spb);
  for (int s = s0; s < s1; ++s) {
    __syncthreads();
    // ---- stage x (ring), a1, da2
    {
      const int t = s / a.n, e = s - t * a.n;
      const int64_t ks = a.ctl[CTL_STEP] + t;
      const int nv = a.nvalid[(ks % a.R) * a.n + e];
      constexpr int V = PLANE / 16;
      for (int i = tid; i < 4 * V; i += 256) {
        const int c = i / V, o = i - c * V;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (c >= 4 - nv) {
          const int slot = (int)((ks + a.R - 3 + c) % a.R);
          v = reinterpret_cast<const uint4*>(a.frames + ((int64_t)slot * a.n + e) * PLANE)[o];
        }
        reinterpret_cast<uint4*>(xs + c * PLANE)[o] = v;
      }
      const float4* g1 = reinterpret_cast<const float4*>(a.a1 + (int64_t)s * A1);
      for (int i = tid; i < A1 / 4; i += 256) {
        const float4 v = g1[i];
        const int oc = (4 * i) / C1_P, p = 4 * i - oc * C1_P;   // 400 % 4 == 0: a float4 stays in one row
        float* d = a1s + oc * A1_LD + p;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
      const float4* g2 = reinterpret_cast<const float4*>(a.da2 + (int64_t)s * A2);
      for (int i = tid; i < A2 / 4; i += 256) reinterpret_cast<float4*>(d2s)[i] = g2[i];
    }
    __syncthreads();
    // ---- (1) conv2 weight gradient + bias
    {
      const int oc = tid & 31, ch = tid >> 5;   // 8 chunks of <= 11 positions
      float t = 0.f;
      for (int p = ch * 11; p < min(C2_P, ch * 11 + 11); ++p) t = __fadd_rn(t, d2s[oc * C2_P + p]);
      b2sum = __fadd_rn(b2sum, t);
    }
    for (int ps = 0; ps < 21; ++ps) {
      const int p = 4 * ps + q;
      const bool pv = p < C2_P;
      const int pc = pv ? p : 0;
      const int oy = pc / 9, ox = pc - oy * 9;
      const float af0 = pv ? d2s[col * C2_P + pc] : 0.f;
      const float af1 = pv ? d2s[(16 + col) * C2_P + pc] : 0.f;
      const int boff = (2 * oy + (col >> 2)) * 20 + 2 * ox + (col & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float bf = a1s[(4 * wave + j) * A1_LD + boff];   // ic = n-tile
        acc2[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af0, bf, acc2[0][j], 0, 0, 0);
        acc2[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af1, bf, acc2[1][j], 0, 0, 0);
      }
    }
    __syncthreads();   // a1s is overwritten by (2)
    // ---- (2) da1 = convT(da2, W2) * (a1 > 0), in place
    for (int job = wave; job < 28; job += 4) {
      const int cls = job / 7, tt = job - cls * 7;
      const int py = cls >> 1, px = cls & 1;
      const int r = 16 * tt + col;            // A row (position in class)
      const int ii = r / 10, jj = r - ii * 10;
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int ks = 0; ks < 32; ++ks) {
        const int k = 4 * ks + q;
        const int oc = k >> 2, dy = (k >> 1) & 1, dx = k & 1;
        const int oy = ii - dy, ox = jj - dx;
        const bool ok = r < 100 && oy >= 0 && ox >= 0 && oy < 9 && ox < 9;
        const float af = ok ? d2s[oc * C2_P + oy * 9 + ox] : 0.f;
        const float bf = w2s[(oc * 16 + col) * 16 + (py + 2 * dy) * 4 + px + 2 * dx];
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, c, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int pos = 16 * tt + q * 4 + rr;
        if (pos < 100) {
          const int i2 = pos / 10, j2 = pos - i2 * 10;
          float* d = a1s + col * A1_LD + (2 * i2 + py) * 20 + 2 * j2 + px;
          *d = *d > 0.f ? c[rr] : 0.f;
        }
      }
    }
    __syncthreads();
    // ---- (3) conv1 weight gradient + bias from da1 (in a1s)
    {
      const int oc = tid & 15, ch = tid >> 4;
      float t = 0.f;
      for (int p = ch * 25; p < ch * 25 + 25; ++p) t = __fadd_rn(t, a1s[oc * A1_LD + p]);
      b1sum = __fadd_rn(b1sum, t);
    }
    for (int ps = 0; ps < C1_P / 4; ++ps) {
      const int p = 4 * ps + q;
      const int oy = p / 20, ox = p - oy * 20;
      const int pbase = (4 * oy) * 84 + 4 * ox;
      const float bf = a1s[col * A1_LD + p];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float af = (float)xs[pbase + koff[i]];
        acc1[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, acc1[i], 0, 0, 0);
      }
    }
  }
  // ---- partial slab of this block
  float* out = a.slab + (int64_t)blockIdx.x * SLAB;
  // dW2: C map col = n (kk within tile), rows q*4+r -> oc = 16 mt + q*4 + r
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(16 * mt + q * 4 + r) * 256 + 16 * (4 * wave + j) + col] = acc2[mt][j][r];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[SLAB_W1 + (16 * (4 * wave + i) + q * 4 + r) * 16 + col] = acc1[i][r];
  red[tid] = b2sum;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int c = 0; c < 8; ++c) t = __fadd_rn(t, red[c * 32 + tid]);
    out[SLAB_B2 + tid] = t;
  }
  __syncthreads();
  red[tid] = b1sum;
  __syncthreads();
  if (tid < 16) {
    float t = 0.f;
    for (int c = 0; c < 16; ++c) t = __fadd_rn(t, red[c * 16 + tid]);
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
  hipLaunchKernelGGL(conv_bwd_kernel, dim3(G), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(reduce_conv_bwd_kernel, dim3((SLAB + 15) / 16), dim3(256), 0, s, slab, G, gW2, gb2, gW1, gb1);
  return hipGetLastError();
}

}  // namespace arl
