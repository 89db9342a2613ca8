// f32-accurate GEMM on the bf16 matrix cores from PRE-SPLIT operands.
//
//   C[m][n] = sum_k A(m,k) * B(k,n),   A = Ah + Am + Al,  B = Bh + Bm + Bl
//
// Every f32 operand is stored as three bf16 planes (bf16split.hpp: exact
// 3-way split by truncation), written once by the kernel that produces the
// value (the optimizer for weights, the layer for activations / gradients),
// so the GEMM itself does no conversion work: it stages bf16 bytes and runs
// the 6 significant cross terms per k-step on v_mfma_f32_16x16x32_bf16 into a
// big (hh) and a small (the 5 others) accumulator -- the same arithmetic and
// error bound as gemm_x6_kernel / the fused conv kernels.
//
// Operand storage, per plane (ld = row pitch in elements, multiple of 8):
//   A_TR = false: A(m, k) at a[m * lda + k]   (k contiguous)
//   A_TR = true:  A(m, k) at a[k * lda + m]   (m contiguous)
//   B_TR = false: B(k, n) at b[n * ldb + k]   (k contiguous)
//   B_TR = true:  B(k, n) at b[k * ldb + n]   (n contiguous)
// k-contiguous tiles land in LDS as [row][BK] and feed the MFMA through
// ds_read_b128; m / n-contiguous tiles land as [BK][row] and are read
// transposed by ds_read_b64_tr_b16 (gfx950), so no operand is ever
// re-laid-out in memory.  Requirements (checked by the launcher): K % 8 == 0,
// and M (N) % 8 == 0 for a transposed A (B); rows / k past the edges are
// zero-filled per 16-byte vector.
//
// Block = 256 threads = 4 waves (WM x WN), tile BM x BN, K chunk BK staged in
// registers one chunk ahead (global -> VGPR -> ds_write_b128).  Epilogue:
// EOp::store(m, n, v, z) per element from the MFMA layout, or, when
// EOp::kRow4, the tile goes through LDS and EOp::store4(m, n, float4, z) gets
// whole 16-byte row pieces (n % 4 == 0, N % 4 == 0 required by the functor).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bf16split.hpp"

namespace arl {

struct Planes {            // three bf16 planes of one f32 operand
  const uint16_t* p;       // plane h; m = p + stride, l = p + 2 * stride
  int64_t stride;          // elements between planes
  int ld;                  // row pitch (elements)
};

typedef short bf16x4_t __attribute__((ext_vector_type(4)));

__device__ inline bf16x8 tr_pair(const uint16_t* lo, const uint16_t* hi) {
  const bf16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4_t*)(lo));
  const bf16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4_t*)(hi));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int BM, int BN, int BK, int WM, int WN, bool A_TR, bool B_TR, class EOp>
__global__ void __launch_bounds__(256)
gemm_planes_kernel(Planes A, Planes B, EOp E, int M, int N, int K, int k_per_split) {
  static_assert(WM * WN == 4, "4 waves");
  static_assert(BK % 32 == 0, "32-deep k-steps");
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  // LDS images (bf16 elements); +8 pad per row spreads rows over banks
  constexpr int A_ROWS = A_TR ? BK : BM, A_COLS = A_TR ? BM : BK;
  constexpr int B_ROWS = B_TR ? BK : BN, B_COLS = B_TR ? BN : BK;
  constexpr int LA = A_COLS + 8, LB = B_COLS + 8;
  constexpr int PA = A_ROWS * LA, PB = B_ROWS * LB;     // per plane
  // staging: 16-byte vectors (8 bf16) per plane
  constexpr int AV = A_ROWS * (A_COLS / 8), BV = B_ROWS * (B_COLS / 8);
  constexpr int AVT = (AV + 255) / 256, BVT = (BV + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint16_t lds[3 * (PA + PB)];
  uint16_t* const la = lds;
  uint16_t* const lb = lds + 3 * PA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, z = blockIdx.z;
  const int kbeg = z * k_per_split;
  const int kend = min(kbeg + k_per_split, K);

  uint4 ra[3][AVT], rb[3][BVT];
  auto gather = [&](int kc) {
#pragma unroll
    for (int i = 0; i < AVT; ++i) {
      const int v = tid + 256 * i;
      const int r = v / (A_COLS / 8), c = 8 * (v % (A_COLS / 8));
      // (row of the image, first element) -> (m, k)
      const int m = A_TR ? m0 + c : m0 + r, k = A_TR ? kc + r : kc + c;
      const bool ok = v < AV && m < M && k < kend;
      const int64_t off = A_TR ? (int64_t)k * A.ld + m : (int64_t)m * A.ld + k;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        ra[p][i] = ok ? *reinterpret_cast<const uint4*>(A.p + p * A.stride + off) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BVT; ++i) {
      const int v = tid + 256 * i;
      const int r = v / (B_COLS / 8), c = 8 * (v % (B_COLS / 8));
      const int n = B_TR ? n0 + c : n0 + r, k = B_TR ? kc + r : kc + c;
      const bool ok = v < BV && n < N && k < kend;
      const int64_t off = B_TR ? (int64_t)k * B.ld + n : (int64_t)n * B.ld + k;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        rb[p][i] = ok ? *reinterpret_cast<const uint4*>(B.p + p * B.stride + off) : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < AVT; ++i) {
      const int v = tid + 256 * i;
      if (v < AV) {
        const int r = v / (A_COLS / 8), c = 8 * (v % (A_COLS / 8));
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4*>(la + p * PA + r * LA + c) = ra[p][i];
      }
    }
#pragma unroll
    for (int i = 0; i < BVT; ++i) {
      const int v = tid + 256 * i;
      if (v < BV) {
        const int r = v / (B_COLS / 8), c = 8 * (v % (B_COLS / 8));
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4*>(lb + p * PB + r * LB + c) = rb[p][i];
      }
    }
  };

  f32x4 big[TM][TN], sml[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) big[i][j] = sml[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, pp = l16 & 3;
  if (kbeg < kend) {
    gather(kbeg);
    for (int kc = kbeg; kc < kend; kc += BK) {
      __syncthreads();
      commit();
      __syncthreads();
      if (kc + BK < kend) gather(kc + BK);
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[3][TM], bf[3][TN];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int mr = wm * (BM / WM) + 16 * i;   // first row of the 16-row tile
            if constexpr (A_TR) {
              // group g: rows k = 32 ks + 8 g + {0..3} / {4..7}, columns mr + 4 pp .. of row q
              const uint16_t* base = la + p * PA + (32 * ks + 8 * g + q) * LA + mr + 4 * pp;
              af[p][i] = tr_pair(base, base + 4 * LA);
            } else {
              af[p][i] = *reinterpret_cast<const bf16x8*>(la + p * PA + (mr + l16) * LA + 32 * ks + 8 * g);
            }
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int nr = wn * (BN / WN) + 16 * j;
            if constexpr (B_TR) {
              const uint16_t* base = lb + p * PB + (32 * ks + 8 * g + q) * LB + nr + 4 * pp;
              bf[p][j] = tr_pair(base, base + 4 * LB);
            } else {
              bf[p][j] = *reinterpret_cast<const bf16x8*>(lb + p * PB + (nr + l16) * LB + 32 * ks + 8 * g);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            mfma_x6(af[0][i], af[1][i], af[2][i], bf[0][j], bf[1][j], bf[2][j], big[i][j], sml[i][j]);
      }
    }
  }
  if constexpr (EOp::kRow4) {
    // epilogue through LDS: whole 16-byte row segments per thread (coalesced
    // stores and mask loads) instead of the MFMA layout's 64-byte pieces
    static_assert(BM * (BN + 4) * 4 <= 3 * (PA + PB) * 2, "C tile fits the staging LDS");
    constexpr int LC = BN + 4;
    float* ct = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(wm * (BM / WM) + i * 16 + g * 4 + r) * LC + wn * (BN / WN) + j * 16 + l16] =
              __fadd_rn(big[i][j][r], sml[i][j][r]);
    __syncthreads();
    for (int v = tid; v < BM * (BN / 4); v += 256) {
      const int r = v / (BN / 4), c = 4 * (v % (BN / 4));
      const int m = m0 + r, n = n0 + c;
      if (m < M && n < N) E.store4(m, n, *reinterpret_cast<const float4*>(ct + r * LC + c), z);
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / WN) + j * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * (BM / WM) + i * 16 + g * 4 + r;
          if (m < M && n < N) E.store(m, n, __fadd_rn(big[i][j][r], sml[i][j][r]), z);
        }
      }
  }
}

template <int BM, int BN, int BK, int WM, int WN, bool A_TR, bool B_TR, class EOp>
inline hipError_t launch_gemm_planes(const Planes& A, const Planes& B, const EOp& E, int M, int N, int K, int splits,
                                     hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  // 16-byte vectors: K % 8 == 0 and 8-element row pitches; a transposed operand's
  // rows must be padded to a multiple of 8 columns (the caller's ld >= M / N
  // rounded up, padding finite) -- vectors starting below M / N are read whole
  if (K % 8 || A.ld % 8 || B.ld % 8 || (A_TR && A.ld < (M + 7) / 8 * 8) || (B_TR && B.ld < (N + 7) / 8 * 8))
    return hipErrorInvalidValue;
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  splits = (K + kps - 1) / kps;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  hipLaunchKernelGGL((gemm_planes_kernel<BM, BN, BK, WM, WN, A_TR, B_TR, EOp>), grid, dim3(256), 0, s, A, B, E, M, N,
                     K, kps);
  return hipGetLastError();
}

// exact 3-way split of rows of f32 values into planes h / m / l (stride elements
// apart): x[r][c] (pitch ldx) -> out[r][c] (pitch ldo), r < rows, c < cols
template <int UNUSED = 0>
__global__ void __launch_bounds__(256)
split_planes_kernel(const float* __restrict__ x, int rows, int cols, int ldx, uint16_t* __restrict__ out, int ldo,
                    int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
  uint32_t h, m, l;
  split3(x[(int64_t)r * ldx + c], h, m, l);
  uint16_t* o = out + (int64_t)r * ldo + c;
  o[0] = (uint16_t)h;
  o[stride] = (uint16_t)m;
  o[2 * stride] = (uint16_t)l;
}

inline hipError_t launch_split_planes(const float* x, int rows, int cols, int ldx, uint16_t* out, int ldo,
                                      int64_t stride, hipStream_t s) {
  const int64_t n = (int64_t)rows * cols;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(split_planes_kernel<0>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, rows, cols, ldx,
                     out, ldo, stride);
  return hipGetLastError();
}

}  // namespace arl
