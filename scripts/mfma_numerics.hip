// Dev check: accuracy of f32 GEMM emulated with bf16 MFMA operand splits
// (x = hi + mid + lo, each bf16) against f64, next to the exact-f32 MFMA.
//   case 0: A = integers 0..255 (exact in bf16, like uint8 pixels), B = f32
//           -> 3 MFMAs per k-step (A * B_hi, A * B_mid, A * B_lo)
//   case 1: A, B = f32 -> 6 MFMAs (hh, hm, mh, hl, mm, lh)
// Prints max |err| / sum|a*b| per case and per method.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_numerics scripts/mfma_numerics.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ inline unsigned short bf16_rn(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
__device__ inline float bf16_f(unsigned short h) { return __uint_as_float((uint32_t)h << 16); }
__device__ inline void split3(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf16_rn(x);
  const float r1 = x - bf16_f(h);
  m = bf16_rn(r1);
  const float r2 = r1 - bf16_f(m);
  l = bf16_rn(r2);
}

constexpr int K = 256;

// one 16x16 tile: A (16 x K) row-major, B (K x 16) row-major
__global__ void gemm_bf16split(const float* A, const float* B, float* C, int terms) {
  const int lane = threadIdx.x, row = lane & 15, g = lane >> 4;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < K / 32; ++s) {
    bf16x8 ah, am, al, bh, bm, bl;
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * g + j;
      unsigned short h, m, l;
      split3(A[row * K + k], h, m, l);
      ah[j] = h; am[j] = m; al[j] = l;
      split3(B[k * 16 + row], h, m, l);
      bh[j] = h; bm[j] = m; bl[j] = l;
    }
    if (terms == 3) {   // A exact in bf16
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
    } else {
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
    }
  }
  for (int r = 0; r < 4; ++r) C[(g * 4 + r) * 16 + row] = c[r];
}

// same tile with separate accumulators per term, summed small-first at the end
__global__ void gemm_bf16split_sep(const float* A, const float* B, float* C, int terms) {
  const int lane = threadIdx.x, row = lane & 15, g = lane >> 4;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  for (int s = 0; s < K / 32; ++s) {
    bf16x8 ah, am, al, bh, bm, bl;
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * g + j;
      unsigned short h, m, l;
      split3(A[row * K + k], h, m, l);
      ah[j] = h; am[j] = m; al[j] = l;
      split3(B[k * 16 + row], h, m, l);
      bh[j] = h; bm[j] = m; bl[j] = l;
    }
    if (terms == 3) {
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c0, 0, 0, 0);
    } else {
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c0, 0, 0, 0);
    }
  }
  for (int r = 0; r < 4; ++r) C[(g * 4 + r) * 16 + row] = c0[r] + c1[r];
}

__global__ void gemm_f32(const float* A, const float* B, float* C) {
  const int lane = threadIdx.x, row = lane & 15, g = lane >> 4;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < K / 4; ++s)
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A[row * K + 4 * s + g], B[(4 * s + g) * 16 + row], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(g * 4 + r) * 16 + row] = c[r];
}

static double frand() { return rand() / (RAND_MAX + 1.0); }

int main() {
  float *A, *B, *C;
  hipMallocManaged(&A, 16 * K * 4);
  hipMallocManaged(&B, K * 16 * 4);
  hipMallocManaged(&C, 256 * 4);
  for (int cs = 0; cs < 2; ++cs) {
    double worst[3] = {0, 0, 0};
    for (int trial = 0; trial < 50; ++trial) {
      for (int i = 0; i < 16 * K; ++i) {
        if (cs == 0) A[i] = (float)(rand() % 256);
        else A[i] = (float)(frand() < 0.5 ? 0.0 : frand() * 3.0);   // relu-like activations
      }
      for (int i = 0; i < K * 16; ++i) B[i] = (float)((frand() - 0.5) * 0.1);
      for (int method = 0; method < 3; ++method) {
        if (method == 0) hipLaunchKernelGGL(gemm_f32, dim3(1), dim3(64), 0, 0, A, B, C);
        else if (method == 1) hipLaunchKernelGGL(gemm_bf16split, dim3(1), dim3(64), 0, 0, A, B, C, cs == 0 ? 3 : 6);
        else hipLaunchKernelGGL(gemm_bf16split_sep, dim3(1), dim3(64), 0, 0, A, B, C, cs == 0 ? 3 : 6);
        hipDeviceSynchronize();
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            double ref = 0, mag = 0;
            for (int k = 0; k < K; ++k) {
              ref += (double)A[i * K + k] * B[k * 16 + j];
              mag += fabs((double)A[i * K + k] * B[k * 16 + j]);
            }
            const double e = fabs(C[i * 16 + j] - ref) / mag;
            if (e > worst[method]) worst[method] = e;
          }
      }
    }
    printf("case %d (%s): max|err|/sum|ab|  f32-mfma %.3e   bf16x%d %.3e   bf16x%d-sep %.3e\n", cs,
           cs == 0 ? "int8 x f32" : "f32 x f32", worst[0], cs == 0 ? 3 : 6, worst[1], cs == 0 ? 3 : 6, worst[2]);
  }
  return 0;
}
