// conv1 of the NIPS head (dqn_head.py:41: Convolution2D(4, 16, 8, stride=4))
// straight from the uint8 frame ring: forward and weight gradient.
//
// Both kernels stage a sample's 4 screens (4 x 84 x 84 uint8 = 28 KB, planes
// older than the env's last reset zero-filled) into LDS with 16-byte loads
// and feed the fp32 MFMA (v_mfma_f32_16x16x4_f32) with the *integer* pixel
// values (exact in f32); the dqn_phi scale 1/255 (dqn_phi.py:16) is applied
// once to the accumulated sum in the epilogue / the reduction instead of to
// every operand -- the result differs from sum((x/255) * w) only by f32
// rounding (well inside the 1e-5 parity bound), and the gather loses its
// per-element division.
//
// Forward: C[p][oc] = sum_k X[p][k] W[oc][k], p = 400 positions, K = 256.
// The K order is permuted so that one ds_read_b32 fetches the operands of
// four consecutive MFMA k-steps: k-step 4j + r, lane quarter q reads
// (ic, ky) = divmod(2j + (q >> 1), 8), kx = 4 (q & 1) + r, i.e. the 4
// contiguous bytes at column 4 ox + 4 (q & 1).  The weights follow the same
// permutation and live in 64 VGPRs per lane for the whole block.
//
// Weight gradient: D[k][oc] = sum_{s,p} X_s[p][k] dY_s[oc][p] as a
// 256 x 16 MFMA product with the position axis as the reduction; each wave
// owns 4 k-tiles, each block a contiguous run of samples, and writes one
// partial slab (k x oc + the bias column) that reduce_conv1_grad sums in f64,
// in block order, into the flat gradient (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct RingView {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R, t0;
};

// stage sample s (= t*n + e relative to t0) into lds[4][7056]
__device__ inline void stage_state(const RingView& rv, int s, uint8_t* lds) {
  const int t = rv.t0 + s / rv.n, e = s % rv.n;
  const int64_t ks = rv.ctl[CTL_STEP] + t;
  const int nv = rv.nvalid[(ks % rv.R) * rv.n + e];
  constexpr int V = PLANE / 16;   // 441 uint4 per plane
  for (int i = threadIdx.x; i < 4 * V; i += blockDim.x) {
    const int c = i / V, o = i - c * V;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (c >= 4 - nv) {
      const int slot = (int)((ks + rv.R - 3 + c) % rv.R);
      v = reinterpret_cast<const uint4*>(rv.frames + ((int64_t)slot * rv.n + e) * PLANE)[o];
    }
    reinterpret_cast<uint4*>(lds + c * PLANE)[o] = v;
  }
}

// ------------------------------------------------------------------ forward
// grid: (n_samples, 2 halves of the 25 position tiles); block 256 (4 waves)
__global__ void __launch_bounds__(256)
conv1_fwd_kernel(RingView rv, const float* __restrict__ W, const float* __restrict__ b, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[4 * PLANE];
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, col = lane & 15;
  // weights in the permuted K order: wf[4j + r] = W[oc][ic*64 + ky*8 + kx]
  float wf[64];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int u = 2 * j + (q >> 1), ic = u >> 3, ky = u & 7;
#pragma unroll
    for (int r = 0; r < 4; ++r) wf[4 * j + r] = W[col * 256 + ic * 64 + ky * 8 + 4 * (q & 1) + r];
  }
  stage_state(rv, s, xs);
  __syncthreads();
  const float bias = b[col];
  const int tile0 = blockIdx.y * 13, tile1 = blockIdx.y ? 25 : 13;
  for (int tile = tile0 + wave; tile < tile1; tile += 4) {
    const int p = tile * 16 + col;          // A row (position) of this lane
    const int oy = p / 20, ox = p - oy * 20;
    const uint8_t* base = xs + (4 * oy) * 84 + 4 * ox + 4 * (q & 1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int u = 2 * j + (q >> 1), ic = u >> 3, ky = u & 7;
      const uint32_t w4 = *reinterpret_cast<const uint32_t*>(base + ic * PLANE + ky * 84);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(w4 & 0xff), wf[4 * j + 0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((w4 >> 8) & 0xff), wf[4 * j + 1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)((w4 >> 16) & 0xff), wf[4 * j + 2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(w4 >> 24), wf[4 * j + 3], acc, 0, 0, 0);
    }
    // C map: col = oc, rows (q*4 + r) -> positions tile*16 + q*4 + r
    float4 o;
    o.x = fmaxf(__fadd_rn(__fdiv_rn(acc[0], 255.f), bias), 0.f);
    o.y = fmaxf(__fadd_rn(__fdiv_rn(acc[1], 255.f), bias), 0.f);
    o.z = fmaxf(__fadd_rn(__fdiv_rn(acc[2], 255.f), bias), 0.f);
    o.w = fmaxf(__fadd_rn(__fdiv_rn(acc[3], 255.f), bias), 0.f);
    *reinterpret_cast<float4*>(out + (int64_t)s * A1 + col * C1_P + tile * 16 + q * 4) = o;
  }
}

// ------------------------------------------------------------------ weight gradient
constexpr int DY_LD = 401;   // LDS row stride of dY (oc-major), odd -> conflict-free oc spread
constexpr int C1G_SLAB = 256 * 16 + 16;   // D[k][oc] + bias[oc]

// grid: G blocks, block b handles samples [b*spb, min(S, (b+1)*spb))
__global__ void __launch_bounds__(256)
conv1_wgrad_kernel(RingView rv, const float* __restrict__ dY, int S, int spb, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[4 * PLANE];
  __shared__ float dys[C1_OC * DY_LD];
  __shared__ float bred[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, col = lane & 15;
  // this lane's 4 A rows: k = 16 * (4 wave + i) + col  ->  (ic, ky, kx)
  int koff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 16 * (4 * wave + i) + col;
    const int ic = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
    koff[i] = ic * PLANE + ky * 84 + kx;
  }
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const int s0 = blockIdx.x * spb;
  const int s1 = min(S, s0 + spb);
  for (int s = s0; s < s1; ++s) {
    __syncthreads();   // previous sample's LDS fully consumed
    stage_state(rv, s, xs);
    const float* dy = dY + (int64_t)s * A1;
    for (int i = threadIdx.x; i < A1; i += 256) {
      const int oc = i / C1_P, p = i - oc * C1_P;
      const float v = dy[i];
      dys[oc * DY_LD + p] = v;
    }
    __syncthreads();
    // bias: thread (oc = t & 15, chunk = t >> 4) sums 25 positions
    {
      const int oc = threadIdx.x & 15, ch = threadIdx.x >> 4;
      float t = 0.f;
      for (int p = ch * 25; p < ch * 25 + 25; ++p) t = __fadd_rn(t, dys[oc * DY_LD + p]);
      bsum = __fadd_rn(bsum, t);
    }
    for (int ps = 0; ps < C1_P / 4; ++ps) {
      const int p = 4 * ps + q;                // K index (position) of this lane
      const int oy = p / 20, ox = p - oy * 20;
      const int pbase = (4 * oy) * 84 + 4 * ox;
      const float bf = dys[col * DY_LD + p];   // B[k = p][n = oc]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float af = (float)xs[pbase + koff[i]];
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, acc[i], 0, 0, 0);
      }
    }
  }
  // D map: col = oc, rows q*4 + r -> k = 16 (4 wave + i) + q*4 + r
  float* out = slab + (int64_t)blockIdx.x * C1G_SLAB;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(16 * (4 * wave + i) + q * 4 + r) * 16 + col] = acc[i][r];
  bred[threadIdx.x] = bsum;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
    for (int c = 0; c < 16; ++c) t = __fadd_rn(t, bred[c * 16 + threadIdx.x]);
    out[256 * 16 + threadIdx.x] = t;
  }
}

// sum G slabs (f64, block order) -> grad W1[oc][k] (scaled by 1/255) and b1
__global__ void __launch_bounds__(256)
reduce_conv1_grad_kernel(const float* __restrict__ slab, int G, float* __restrict__ gW, float* __restrict__ gb) {
  // block: 64 outputs x 4 slab groups
  __shared__ double part[4][64];
  const int o = blockIdx.x * 64 + (threadIdx.x & 63);
  const int zg = threadIdx.x >> 6;
  double t = 0.0;
  if (o < C1G_SLAB)
    for (int z = zg; z < G; z += 4) t += (double)slab[(int64_t)z * C1G_SLAB + o];
  part[zg][threadIdx.x & 63] = t;
  __syncthreads();
  if (zg == 0 && o < C1G_SLAB) {
    const double v = ((part[0][threadIdx.x] + part[1][threadIdx.x]) + part[2][threadIdx.x]) + part[3][threadIdx.x];
    if (o < 256 * 16) {
      const int k = o >> 4, oc = o & 15;
      gW[oc * 256 + k] = (float)(v / 255.0);
    } else {
      gb[o - 256 * 16] = (float)v;
    }
  }
}

hipError_t launch_conv1_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t0,
                            int nsamples, const float* W, const float* b, float* out, hipStream_t s) {
  if (nsamples <= 0) return hipSuccess;
  RingView rv{frames, nvalid, ctl, n, R, t0};
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(nsamples, 2), dim3(256), 0, s, rv, W, b, out);
  return hipGetLastError();
}

int conv1_wgrad_blocks(int S) { return S < 640 ? S : 640; }
int64_t conv1_wgrad_slab_floats(int S) { return (int64_t)conv1_wgrad_blocks(S) * C1G_SLAB; }

hipError_t launch_conv1_wgrad(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R,
                              int S, const float* dY, float* slab, float* gW, float* gb, hipStream_t s) {
  if (S <= 0) return hipSuccess;
  const int G0 = conv1_wgrad_blocks(S);
  const int spb = (S + G0 - 1) / G0;
  const int G = (S + spb - 1) / spb;
  RingView rv{frames, nvalid, ctl, n, R, 0};
  hipLaunchKernelGGL(conv1_wgrad_kernel, dim3(G), dim3(256), 0, s, rv, dY, S, spb, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(reduce_conv1_grad_kernel, dim3((C1G_SLAB + 63) / 64), dim3(256), 0, s, slab, G, gW, gb);
  return hipGetLastError();
}

}  // namespace arl
