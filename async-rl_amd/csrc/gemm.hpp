// Generic fp32 implicit-GEMM on gfx950 MFMA (v_mfma_f32_16x16x4_f32).
//
//   C[m][n] = sum_k A(m,k) * B(k,n)        (exact f32 products, f32 accumulate)
//
// A and B are *accessors*: small structs whose load(m,k)/load(k,n) gather the
// operand on the fly (im2col for conv, ring-buffer planes for the frame stack,
// transposed weights, a "ones" column that yields bias gradients, ...).  The
// epilogue functor receives every output element with its split-K slice index
// z, so one template serves forward layers (bias+ReLU epilogue, z == 0) and the
// weight-gradient reductions (split K over workgroups, one partial slab per z,
// summed deterministically by reduce_slabs).
//
// Block = 256 threads = 4 waves of 64.  Output tile BM x BN is covered by 16x16
// MFMA tiles; wave w owns a (BM/WM) x (BN/WN) sub-block (WM*WN == 4).
// K is consumed in chunks of BK staged through LDS as f32 ([BK][BM+4] and
// [BK][BN+4]; the +4 pad breaks the 2-way ds_read_b32 conflict between the two
// k rows read by lanes 0-15 and 16-31).  The next chunk is gathered into
// registers while the current one feeds the MFMAs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// AKF / BKF: gather the A / B chunk with k fastest across threads (for
// operands that are contiguous along k, e.g. row-major activations, W[n][k]).
template <int BM, int BN, int BK, int WM, int WN, class AOp, class BOp, class EOp, bool AKF = false,
          bool BKF = false>
__global__ void __launch_bounds__(256)
gemm_kernel(AOp A, BOp B, EOp E, int M, int N, int K, int k_per_split) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / (16 * WM);   // MFMA tiles per wave along m
  constexpr int TN = BN / (16 * WN);   // along n
  static_assert(TM >= 1 && TN >= 1, "tile too small for wave layout");
  constexpr int LDA = AKF ? BM + 1 : BM + 4;
  constexpr int LDB = BKF ? BN + 1 : BN + 4;
  constexpr int A_PER = (BM * BK) / 256;   // A elements gathered per thread per chunk
  constexpr int B_PER = (BK * BN) / 256;
  static_assert(A_PER >= 1 && B_PER >= 1, "chunk too small");

  __shared__ float As[BK * LDA];
  __shared__ float Bs[BK * LDB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int z = blockIdx.z;
  const int kbeg = z * k_per_split;
  int kend = kbeg + k_per_split;
  if (kend > K) kend = K;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float ra[A_PER], rb[B_PER];

  // A chunk: element e = tid + 256*i -> (mm, kk), m fastest (or k fastest if AKF)
  // B chunk: element e -> (nn, kk), n fastest (or k fastest if BKF)
  auto a_mk = [](int e, int& mm, int& kk) {
    if (AKF) { kk = e % BK; mm = e / BK; } else { mm = e % BM; kk = e / BM; }
  };
  auto b_nk = [](int e, int& nn, int& kk) {
    if (BKF) { kk = e % BK; nn = e / BK; } else { nn = e % BN; kk = e / BN; }
  };
  auto gather = [&](int kc) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int mm, kk;
      a_mk(tid + 256 * i, mm, kk);
      const int m = m0 + mm, k = kc + kk;
      ra[i] = (m < M && k < kend) ? A.load(m, k) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      int nn, kk;
      b_nk(tid + 256 * i, nn, kk);
      const int n = n0 + nn, k = kc + kk;
      rb[i] = (n < N && k < kend) ? B.load(k, n) : 0.f;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int mm, kk;
      a_mk(tid + 256 * i, mm, kk);
      As[kk * LDA + mm] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      int nn, kk;
      b_nk(tid + 256 * i, nn, kk);
      Bs[kk * LDB + nn] = rb[i];
    }
  };

  if (kbeg < kend) {
    gather(kbeg);
    for (int kc = kbeg; kc < kend; kc += BK) {
      __syncthreads();           // previous chunk fully consumed
      commit();
      __syncthreads();
      if (kc + BK < kend) gather(kc + BK);   // overlap next gather with MFMAs
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        const int kr = ks * 4 + (lane >> 4);
        float af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = As[kr * LDA + wm * (BM / WM) + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = Bs[kr * LDB + wn * (BN / WN) + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // C/D map for 16x16x4 f32: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N) E.store(m, n, acc[i][j][r], z);
      }
    }
}

template <int BM, int BN, int BK, int WM, int WN, bool AKF = false, bool BKF = false, class AOp, class BOp,
          class EOp>
inline hipError_t launch_gemm(const AOp& A, const BOp& B, const EOp& E, int M, int N, int K,
                              int splits, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  splits = (K + kps - 1) / kps;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, AOp, BOp, EOp, AKF, BKF>), grid, dim3(256), 0, s,
                     A, B, E, M, N, K, kps);
  return hipGetLastError();
}

// Number of K slices actually launched by launch_gemm for a requested count.
template <int BK>
inline int effective_splits(int K, int splits) {
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  return (K + kps - 1) / kps;
}

// ---------------------------------------------------------------- accessors
struct RowMajor {            // X[m][k], leading dimension ld
  const float* p; int ld;
  __device__ float load(int m, int k) const { return p[(int64_t)m * ld + k]; }
};
struct ColMajor {            // element (r, c) = X[c][r]  (i.e. X transposed)
  const float* p; int ld;
  __device__ float load(int r, int c) const { return p[(int64_t)c * ld + r]; }
};

}  // namespace arl
