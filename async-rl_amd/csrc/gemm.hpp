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
// registers while the current one feeds the MFMAs.  gemm_tile<..., SP = true>
// (with BK a multiple of 32) runs each 32-deep piece of a chunk as one 16x16x32
// bf16 step per tile pair on exact bf16 splits of the f32 fragments
// (bf16split.hpp: 6 MFMAs, the 5 small terms in their own accumulator;
// f32-accurate) instead of 8 exact-f32 16x16x4 steps: 2.7x fewer matrix-pipe
// cycles for more VALU / LDS reads.  Off: these GEMMs wait on their register
// gathers and scalar LDS reads, not on the matrix pipe -- every GEMM on it took
// the LSTM C3 window 1.316 -> 1.377 ms (profiles/r02/gemm_split/).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bf16split.hpp"


namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Gather modes for the A / B chunk (template AV, BV):
//   GS (0): scalar, m (n) fastest across threads -- any accessor;
//   GK (1): 16-byte vectors of 4 consecutive k via load4(m, k) / load4(k, n)
//           (k-contiguous operands: row-major activations, W[n][k]);
//   GM (2): 16-byte vectors of 4 consecutive m (n) via load4m(m, k) /
//           load4n(k, n) (m / n-contiguous operands: W[k][n], X^T).
// Vector gathers need 16-byte aligned rows (leading dimension % 4 == 0);
// partial vectors at the K / M / N edges fall back to scalar loads.
enum { GS = 0, GK = 1, GM = 2 };

// Gather one BK-deep K chunk of the A (BM x BK) and B (BK x BN) tiles into
// registers (ra: A_PER, rb: B_PER values per thread); element order per mode
// is documented at the commit sites of the two kernels below.
template <int BM, int BN, int BK, int AV, int BV, int NTH, class AOp, class BOp>
__device__ inline void gemm_gather(const AOp& A, const BOp& B, int M, int N, int kend, int m0, int n0, int kc,
                                   int tid, float* ra, float* rb) {
  constexpr int A_PER = (BM * BK) / NTH;
  constexpr int B_PER = (BK * BN) / NTH;
  if constexpr (AV == GK) {
#pragma unroll
    for (int i = 0; i < A_PER / 4; ++i) {
      const int v = tid + NTH * i;
      const int kq = v % (BK / 4), mm = v / (BK / 4);
      const int m = m0 + mm, k = kc + 4 * kq;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M) {
        if (k + 3 < kend) x = A.load4(m, k);
        else {
          if (k < kend) x.x = A.load(m, k);
          if (k + 1 < kend) x.y = A.load(m, k + 1);
          if (k + 2 < kend) x.z = A.load(m, k + 2);
        }
      }
      ra[4 * i] = x.x; ra[4 * i + 1] = x.y; ra[4 * i + 2] = x.z; ra[4 * i + 3] = x.w;
    }
  } else if constexpr (AV == GM) {
#pragma unroll
    for (int i = 0; i < A_PER / 4; ++i) {
      const int v = tid + NTH * i;
      const int mq = v % (BM / 4), kk = v / (BM / 4);
      const int m = m0 + 4 * mq, k = kc + kk;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < kend) {
        if (m + 3 < M) x = A.load4m(m, k);
        else {
          if (m < M) x.x = A.load(m, k);
          if (m + 1 < M) x.y = A.load(m + 1, k);
          if (m + 2 < M) x.z = A.load(m + 2, k);
        }
      }
      ra[4 * i] = x.x; ra[4 * i + 1] = x.y; ra[4 * i + 2] = x.z; ra[4 * i + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int e = tid + NTH * i;
      const int mm = e % BM, kk = e / BM;
      const int m = m0 + mm, k = kc + kk;
      ra[i] = (m < M && k < kend) ? A.load(m, k) : 0.f;
    }
  }
  if constexpr (BV == GK) {
#pragma unroll
    for (int i = 0; i < B_PER / 4; ++i) {
      const int v = tid + NTH * i;
      const int kq = v % (BK / 4), nn = v / (BK / 4);
      const int n = n0 + nn, k = kc + 4 * kq;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < N) {
        if (k + 3 < kend) x = B.load4(k, n);
        else {
          if (k < kend) x.x = B.load(k, n);
          if (k + 1 < kend) x.y = B.load(k + 1, n);
          if (k + 2 < kend) x.z = B.load(k + 2, n);
        }
      }
      rb[4 * i] = x.x; rb[4 * i + 1] = x.y; rb[4 * i + 2] = x.z; rb[4 * i + 3] = x.w;
    }
  } else if constexpr (BV == GM) {
#pragma unroll
    for (int i = 0; i < B_PER / 4; ++i) {
      const int v = tid + NTH * i;
      const int nq = v % (BN / 4), kk = v / (BN / 4);
      const int n = n0 + 4 * nq, k = kc + kk;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < kend) {
        if (n + 3 < N) x = B.load4n(k, n);
        else {
          if (n < N) x.x = B.load(k, n);
          if (n + 1 < N) x.y = B.load(k, n + 1);
          if (n + 2 < N) x.z = B.load(k, n + 2);
        }
      }
      rb[4 * i] = x.x; rb[4 * i + 1] = x.y; rb[4 * i + 2] = x.z; rb[4 * i + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int e = tid + NTH * i;
      const int nn = e % BN, kk = e / BN;
      const int n = n0 + nn, k = kc + kk;
      rb[i] = (n < N && k < kend) ? B.load(k, n) : 0.f;
    }
  }
}

// an epilogue type with `static constexpr bool kTile = true` gets the whole
// output tile at once (E.tile) instead of per-element stores
template <class E, class = void>
struct epi_tile_flag { static constexpr bool value = false; };
template <class E>
struct epi_tile_flag<E, decltype((void)E::kTile)> { static constexpr bool value = E::kTile; };
template <class E>
constexpr bool epi_is_tile() { return epi_tile_flag<E>::value; }

// One BM x BN output tile (split-K slice z) of the implicit GEMM; the body of
// gemm_kernel and of gemm2_kernel (two independent GEMMs in one launch).
template <int BM, int BN, int BK, int WM, int WN, int AV, int BV, int NTH, class AOp, class BOp, class EOp,
          bool SP = false>
__device__ inline void gemm_tile(const AOp& A, const BOp& B, const EOp& E, int M, int N, int K, int k_per_split,
                                 int bx, int by, int z) {
  static_assert(WM * WN == NTH / 64, "one wave per WM x WN slot");
  constexpr int TM = BM / (16 * WM);   // MFMA tiles per wave along m
  constexpr int TN = BN / (16 * WN);   // along n
  static_assert(TM >= 1 && TN >= 1, "tile too small for wave layout");
  constexpr int LDA = AV == GK ? BM + 1 : BM + 4;
  constexpr int LDB = BV == GK ? BN + 1 : BN + 4;
  constexpr int A_PER = (BM * BK) / NTH;   // A elements gathered per thread per chunk
  constexpr int B_PER = (BK * BN) / NTH;
  static_assert(A_PER >= 1 && B_PER >= 1, "chunk too small");
  static_assert(AV == GS || A_PER % 4 == 0, "vector A gather needs whole 4-vectors per thread");
  static_assert(BV == GS || B_PER % 4 == 0, "vector B gather needs whole 4-vectors per thread");

  __shared__ __attribute__((aligned(16))) float As[BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int m0 = bx * BM;
  const int n0 = by * BN;
  const int kbeg = z * k_per_split;
  int kend = kbeg + k_per_split;
  if (kend > K) kend = K;

  // bf16-split steps (bf16split.hpp) when the chunk is whole 32-deep steps
  constexpr bool SPLIT = SP && BK % 32 == 0;
  f32x4 acc[TM][TN], sml[SPLIT ? TM : 1][SPLIT ? TN : 1];   // sml: the split's 5 small terms
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < (SPLIT ? TM : 1); ++i)
#pragma unroll
    for (int j = 0; j < (SPLIT ? TN : 1); ++j) sml[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float ra[A_PER], rb[B_PER];

  auto gather = [&](int kc) { gemm_gather<BM, BN, BK, AV, BV, NTH>(A, B, M, N, kend, m0, n0, kc, tid, ra, rb); };
  auto commit = [&]() {
    if constexpr (AV == GK) {
#pragma unroll
      for (int i = 0; i < A_PER / 4; ++i) {
        const int v = tid + NTH * i;
        const int kq = v % (BK / 4), mm = v / (BK / 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) As[(4 * kq + r) * LDA + mm] = ra[4 * i + r];
      }
    } else if constexpr (AV == GM) {
#pragma unroll
      for (int i = 0; i < A_PER / 4; ++i) {
        const int v = tid + NTH * i;
        const int mq = v % (BM / 4), kk = v / (BM / 4);
        *reinterpret_cast<float4*>(&As[kk * LDA + 4 * mq]) =
            make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const int e = tid + NTH * i;
        As[(e / BM) * LDA + (e % BM)] = ra[i];
      }
    }
    if constexpr (BV == GK) {
#pragma unroll
      for (int i = 0; i < B_PER / 4; ++i) {
        const int v = tid + NTH * i;
        const int kq = v % (BK / 4), nn = v / (BK / 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) Bs[(4 * kq + r) * LDB + nn] = rb[4 * i + r];
      }
    } else if constexpr (BV == GM) {
#pragma unroll
      for (int i = 0; i < B_PER / 4; ++i) {
        const int v = tid + NTH * i;
        const int nq = v % (BN / 4), kk = v / (BN / 4);
        *reinterpret_cast<float4*>(&Bs[kk * LDB + 4 * nq]) =
            make_float4(rb[4 * i], rb[4 * i + 1], rb[4 * i + 2], rb[4 * i + 3]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        const int e = tid + NTH * i;
        Bs[(e / BN) * LDB + (e % BN)] = rb[i];
      }
    }
  };

  if (kbeg < kend) {
    gather(kbeg);
    for (int kc = kbeg; kc < kend; kc += BK) {
      __syncthreads();           // previous chunk fully consumed
      commit();
      __syncthreads();
      if (kc + BK < kend) gather(kc + BK);   // overlap next gather with MFMAs
      if constexpr (SPLIT) {
        // 32-deep steps on bf16 splits: element e of lane (col, q) is k = 4 e + q,
        // the rows the f32 steps below read
#pragma unroll
        for (int kb = 0; kb < BK; kb += 32) {
          bf16x8 bh[TN], bm[TN], bl[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = Bs[(kb + 4 * e + (lane >> 4)) * LDB + wn * (BN / WN) + j * 16 + (lane & 15)];
            split3_x8(x, bh[j], bm[j], bl[j]);
          }
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            float x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = As[(kb + 4 * e + (lane >> 4)) * LDA + wm * (BM / WM) + i * 16 + (lane & 15)];
            bf16x8 ah, am, al;
            split3_x8(x, ah, am, al);
#pragma unroll
            for (int j = 0; j < TN; ++j) mfma_x6(ah, am, al, bh[j], bm[j], bl[j], acc[i][j], sml[i][j]);
          }
        }
      } else {
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
  }
  if constexpr (SPLIT) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += sml[i][j];
  }

  // C/D map for 16x16x4 f32: col = lane & 15, row = (lane >> 4) * 4 + r
  if constexpr (epi_is_tile<EOp>()) {
    // whole-tile epilogue (e.g. the LSTM cell on a gate tile): the raw tile in
    // LDS (the B staging area, row stride BN), then E.tile on all threads
    static_assert(BK * LDB >= BM * BN, "tile fits the B staging area");
    __syncthreads();   // the last chunk is consumed
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Bs[(wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r) * BN + wn * (BN / WN) + j * 16 + (lane & 15)] =
              acc[i][j][r];
    __syncthreads();
    E.template tile<BM, BN, NTH>(Bs, m0, n0, M, N);
  } else {
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
}

template <int BM, int BN, int BK, int WM, int WN, class AOp, class BOp, class EOp, int AV = GS, int BV = GS>
__global__ void __launch_bounds__(256)
gemm_kernel(AOp A, BOp B, EOp E, int M, int N, int K, int k_per_split) {
  gemm_tile<BM, BN, BK, WM, WN, AV, BV, 256>(A, B, E, M, N, K, k_per_split, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Two independent GEMMs of the same tile shape in one launch: workgroups
// [0, g1) run the first (tile-major: x fastest, then y, then split z), the rest
// the second.  Latency-bound GEMMs that would run back to back share the chip.
template <class AOp, class BOp, class EOp>
struct GemmJob {
  AOp A; BOp B; EOp E;
  int M, N, K, kps, gx, gy, gz;
};

template <int BM, int BN, int BK, int WM, int WN, int NTH, int AV1, int BV1, int AV2, int BV2, class J1, class J2>
__global__ void __launch_bounds__(NTH)
gemm2_kernel(J1 j1, J2 j2) {
  int b = blockIdx.x;
  const int g1 = j1.gx * j1.gy * j1.gz;
  if (b < g1) {
    const int x = b % j1.gx, y = (b / j1.gx) % j1.gy, z = b / (j1.gx * j1.gy);
    gemm_tile<BM, BN, BK, WM, WN, AV1, BV1, NTH, decltype(j1.A), decltype(j1.B), decltype(j1.E), false>(j1.A, j1.B, j1.E, j1.M, j1.N, j1.K, j1.kps, x, y, z);
  } else {
    b -= g1;
    const int x = b % j2.gx, y = (b / j2.gx) % j2.gy, z = b / (j2.gx * j2.gy);
    gemm_tile<BM, BN, BK, WM, WN, AV2, BV2, NTH, decltype(j2.A), decltype(j2.B), decltype(j2.E), false>(j2.A, j2.B, j2.E, j2.M, j2.N, j2.K, j2.kps, x, y, z);
  }
}

template <int BM, int BK, class AOp, class BOp, class EOp>
inline GemmJob<AOp, BOp, EOp> gemm_job(const AOp& A, const BOp& B, const EOp& E, int M, int N, int K, int splits,
                                       int BN) {
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  splits = (K + kps - 1) / kps;
  return GemmJob<AOp, BOp, EOp>{A, B, E, M, N, K, kps, (M + BM - 1) / BM, (N + BN - 1) / BN, splits};
}

// NTH threads per workgroup (WM x WN = NTH / 64 waves)
template <int BM, int BN, int BK, int WM, int WN, int NTH, int AV1, int BV1, int AV2, int BV2, class J1, class J2>
inline hipError_t launch_gemm2_nt(const J1& j1, const J2& j2, hipStream_t s) {
  const int g = j1.gx * j1.gy * j1.gz + j2.gx * j2.gy * j2.gz;
  if (g <= 0) return hipSuccess;
  hipLaunchKernelGGL((gemm2_kernel<BM, BN, BK, WM, WN, NTH, AV1, BV1, AV2, BV2, J1, J2>), dim3(g), dim3(NTH), 0, s,
                     j1, j2);
  return hipGetLastError();
}

template <int BM, int BN, int BK, int WM, int WN, int AV1, int BV1, int AV2, int BV2, class J1, class J2>
inline hipError_t launch_gemm2(const J1& j1, const J2& j2, hipStream_t s) {
  return launch_gemm2_nt<BM, BN, BK, WM, WN, 256, AV1, BV1, AV2, BV2>(j1, j2, s);
}

template <int BM, int BN, int BK, int WM, int WN, int AV = GS, int BV = GS, class AOp, class BOp, class EOp>
inline hipError_t launch_gemm(const AOp& A, const BOp& B, const EOp& E, int M, int N, int K,
                              int splits, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  splits = (K + kps - 1) / kps;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, AOp, BOp, EOp, AV, BV>), grid, dim3(256), 0, s,
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
  __device__ float4 load4(int m, int k) const {   // k % 4 == 0, ld % 4 == 0
    return *reinterpret_cast<const float4*>(p + (int64_t)m * ld + k);
  }
  __device__ float4 load4n(int k, int n) const {  // as a B operand: 4 consecutive n
    return *reinterpret_cast<const float4*>(p + (int64_t)k * ld + n);
  }
};
struct ColMajor {            // element (r, c) = X[c][r]  (i.e. X transposed)
  const float* p; int ld;
  __device__ float load(int r, int c) const { return p[(int64_t)c * ld + r]; }
  __device__ float4 load4m(int r, int c) const {   // 4 consecutive r (A operand)
    return *reinterpret_cast<const float4*>(p + (int64_t)c * ld + r);
  }
};

}  // namespace arl
