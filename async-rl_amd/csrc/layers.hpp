// Accessors, epilogues and the deterministic split-K slab reduction shared by
// the NIPS (net.hip) and Nature (nature.hip) heads on top of gemm.hpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "arl_internal.hpp"
#include "gemm.hpp"

namespace arl {

// ---------------------------------------------------------------- accessors
struct WeightT {        // B(k, n) = W[n][k]  (Chainer W is (out, in...))
  const float* __restrict__ w; int K;
  __device__ float load(int k, int n) const { return w[(int64_t)n * K + k]; }
  __device__ float4 load4(int k, int n) const {
    return *reinterpret_cast<const float4*>(w + (int64_t)n * K + k);
  }
};
struct HeadsGA {        // A(m, s) = m < A ? dlogits[s][m] : dv[s]
  const float* __restrict__ dl; const float* __restrict__ dv; int A;
  __device__ float load(int m, int s) const { return m < A ? dl[(int64_t)s * A + m] : dv[s]; }
};
struct OnesColB {       // B(s, j) = j < K ? X[s][j] : 1   (bias gradient column)
  const float* __restrict__ x; int K;
  __device__ float load(int s, int j) const { return j < K ? x[(int64_t)s * K + j] : 1.f; }
  __device__ float4 load4n(int s, int j) const {
    if (j + 3 < K) return *reinterpret_cast<const float4*>(x + (int64_t)s * K + j);
    return make_float4(load(s, j), load(s, j + 1), load(s, j + 2), load(s, j + 3));
  }
};

// im2col of an f32 activation tensor x[s][IC][IH][IH] for a KS x KS, stride ST
// convolution with OH x OH outputs: A(m, k), m = s*OH*OH + p, k = ic*KS*KS + ky*KS + kx
template <int IC, int IH, int KS, int ST, int OH>
struct Im2col {
  const float* __restrict__ x;
  __device__ float load(int m, int k) const {
    constexpr int OP = OH * OH, KK = KS * KS;
    const int s = m / OP, p = m - s * OP, oy = p / OH, ox = p - oy * OH;
    const int ic = k / KK, r = k - ic * KK, ky = r / KS, kx = r - ky * KS;
    return x[((int64_t)s * IC + ic) * (IH * IH) + (ST * oy + ky) * IH + ST * ox + kx];
  }
};

// B(m, j) = j < K ? X(m, j) : 1 -- weight-gradient operand with the bias column
template <class X>
struct OnesCol {
  X x; int K;
  __device__ float load(int m, int j) const { return j < K ? x.load(m, j) : 1.f; }
  __device__ float4 load4n(int m, int j) const {   // only instantiated for X with load4
    if (j + 3 < K) return x.load4(m, j);
    return make_float4(load(m, j), load(m, j + 1), load(m, j + 2), load(m, j + 3));
  }
};

// A(oc, m) = dy[s][oc][p], m = s*P + p (output gradient of a conv, transposed)
struct ConvDyT {
  const float* __restrict__ dy; int OC, P;
  __device__ float load(int oc, int m) const {
    const int s = m / P, p = m - s * P;
    return dy[((int64_t)s * OC + oc) * P + p];
  }
  __device__ float4 load4(int oc, int m) const {   // P % 4 == 0 only (conv1: 400)
    const int s = m / P, p = m - s * P;
    return *reinterpret_cast<const float4*>(dy + ((int64_t)s * OC + oc) * P + p);
  }
};

// stride-2, 4x4 transposed conv from OC channels of 9 x 9 back to IC channels of
// 20 x 20 (the second conv of both DQN heads, dqn_head.py:17,42) for one output
// parity class (py, px): y = 2 qy + py, x = 2 qx + px, qy, qx in [0, 10); k =
// oc*4 + jy*2 + jx covers exactly the taps ky = py + 2 jy, kx = px + 2 jx that
// reach (y, x) from oy = qy - jy, ox = qx - jx.
template <int OC, int IC>
struct ConvT2ClassA {
  const float* __restrict__ dy; int py, px;
  __device__ float load(int m, int k) const {
    const int s = m / 100, q = m - s * 100, qy = q / 10, qx = q - qy * 10;
    const int oc = k >> 2, jy = (k >> 1) & 1, jx = k & 1;
    const int oy = qy - jy, ox = qx - jx;
    if (oy < 0 || oy >= 9 || ox < 0 || ox >= 9) return 0.f;
    return dy[((int64_t)s * OC + oc) * 81 + oy * 9 + ox];
  }
};
template <int OC, int IC>
struct ConvT2ClassW {
  const float* __restrict__ w; int py, px;
  __device__ float load(int k, int ic) const {
    const int oc = k >> 2, ky = py + 2 * ((k >> 1) & 1), kx = px + 2 * (k & 1);
    return w[(((int64_t)oc * IC + ic) * 4 + ky) * 4 + kx];
  }
};

// ---------------------------------------------------------------- epilogues
template <int IC>
struct EpiT2Class {     // da1 of one parity class of ConvT2ClassA, times (a1 > 0)
  float* __restrict__ out; const float* __restrict__ mask; int py, px;
  __device__ void store(int m, int ic, float v, int) const {
    const int s = m / 100, q = m - s * 100, qy = q / 10, qx = q - qy * 10;
    const int64_t i = ((int64_t)s * IC + ic) * 400 + (2 * qy + py) * 20 + 2 * qx + px;
    out[i] = mask[i] > 0.f ? v : 0.f;
  }
};
struct EpiConv {        // out[s][n][p] = relu(v + b[n]); m = s*P + p
  float* __restrict__ out; const float* __restrict__ b; int OC, P;
  __device__ void store(int m, int n, float v, int) const {
    const int s = m / P, p = m - s * P;
    out[((int64_t)s * OC + n) * P + p] = fmaxf(__fadd_rn(v, b[n]), 0.f);
  }
};
struct EpiSlab {
  static constexpr bool kRow4 = false;
  float* __restrict__ slab; int M, N;
  __device__ void store(int m, int n, float v, int z) const {
    slab[((int64_t)z * M + m) * N + n] = v;
  }
};
struct EpiBias {        // out[m][n] = v + b[n]
  float* __restrict__ out; const float* __restrict__ b; int ld;
  __device__ void store(int m, int n, float v, int) const { out[(int64_t)m * ld + n] = __fadd_rn(v, b[n]); }
};
struct EpiMask {        // out[m][n] = mask[m][n] > 0 ? v : 0  (ReLU backward)
  static constexpr bool kRow4 = false;
  float* __restrict__ out; const float* __restrict__ mask; int ld;
  __device__ void store(int m, int n, float v, int) const {
    const int64_t i = (int64_t)m * ld + n;
    out[i] = mask[i] > 0.f ? v : 0.f;
  }
};

struct EpiMask4 {       // EpiMask with 16-byte row pieces (gemm_planes row epilogue; ld % 4 == 0)
  static constexpr bool kRow4 = true;
  float* __restrict__ out; const float* __restrict__ mask; int ld;
  __device__ void store4(int m, int n, float4 v, int) const {
    const int64_t i = (int64_t)m * ld + n;
    const float4 k = *reinterpret_cast<const float4*>(mask + i);
    *reinterpret_cast<float4*>(out + i) =
        make_float4(k.x > 0.f ? v.x : 0.f, k.y > 0.f ? v.y : 0.f, k.z > 0.f ? v.z : 0.f, k.w > 0.f ? v.w : 0.f);
  }
};
struct EpiSlab4 {       // EpiSlab with 16-byte row pieces (N % 4 == 0)
  static constexpr bool kRow4 = true;
  float* __restrict__ slab; int M, N;
  __device__ void store4(int m, int n, float4 v, int z) const {
    *reinterpret_cast<float4*>(slab + ((int64_t)z * M + m) * N + n) = v;
  }
};

// ---------------------------------------------------------------- reductions
// dense weight + bias: n < K -> g[oW + m*K + n]; n == K -> g[ob + m];
// (LSTM) n > K -> g[oL + m*K + n-K-1]
struct MapDense {
  float* g; int64_t oW, ob, oL; int K;
  __device__ void put(int m, int n, float v) const {
    if (n < K) g[oW + (int64_t)m * K + n] = v;
    else if (n == K) g[ob + m] = v;
    else g[oL + (int64_t)m * K + (n - K - 1)] = v;
  }
};
struct MapHeads {        // rows m < A: policy W / b; row A: value W / b (hidden width H)
  float* g; int64_t oPW, oPB, oVW, oVB; int A, H;
  __device__ void put(int m, int n, float v) const {
    if (m < A) { if (n < H) g[oPW + (int64_t)m * H + n] = v; else g[oPB + m] = v; }
    else { if (n < H) g[oVW + n] = v; else g[oVB] = v; }
  }
};
struct MapBiasRelu {     // split-K forward layer: out[m][n] = relu(v + b[n])
  float* out; const float* b; int ld;
  __device__ void put(int m, int n, float v) const { out[(int64_t)m * ld + n] = fmaxf(__fadd_rn(v, b[n]), 0.f); }
};

// block = 64 consecutive outputs x 4 slice groups; f64 sums combined in a
// fixed order (deterministic for any slice count)
template <class Map>
__global__ void __launch_bounds__(256)
reduce_grad_kernel(const float* __restrict__ slab, int splits, int M, int N, Map map) {
  __shared__ double part[4][64];
  const int64_t MN = (int64_t)M * N;
  const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int zg = threadIdx.x >> 6;
  double t = 0.0;
  if (i < MN)
    for (int z = zg; z < splits; z += 4) t += (double)slab[(int64_t)z * MN + i];
  part[zg][threadIdx.x & 63] = t;
  __syncthreads();
  if (zg == 0 && i < MN) {
    const int l = threadIdx.x;
    const double v = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
    map.put((int)(i / N), (int)(i % N), (float)v);
  }
}

template <class Map>
inline hipError_t launch_reduce_grad(const float* slab, int splits, int M, int N, const Map& map, hipStream_t s) {
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL((reduce_grad_kernel<Map>), dim3((unsigned)((MN + 63) / 64)), dim3(256), 0, s, slab, splits,
                     M, N, map);
  return hipGetLastError();
}

// ---------------------------------------------------------------- planning
inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// split-K factor: aim at ~1024 workgroups, each slice >= 4 K-chunks
inline int plan_splits(int tiles, int64_t K, int BK, int target = 1024) {
  int s = std::max(1, target / std::max(1, tiles));
  const int maxs = std::max(1, ceil_div(K, (int64_t)BK * 4));
  s = std::min(s, maxs);
  return s;
}

}  // namespace arl
