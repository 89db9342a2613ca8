// Fully connected layer of the NIPS head (dqn_head.py:43, Linear(2592, 256)
// followed by relu at dqn_head.py:52):  hfc = relu(a2 . W^T + b)  for the n
// envs of one lockstep step.
//
// M = n (envs), N = 256, K = 2592: latency-bound at these sizes, so the shape
// is chosen for one short dependency chain per workgroup:
//   * split-K 8 ways, one K slice (324) per XCD (blockIdx % 8 = split): each
//     XCD's L2 holds just its 324-column slice of a2 and W;
//   * 32 x 64 output tile per workgroup; the whole 96 x 324 operand block
//     (124 KB) is staged by LDS-DMA (global_load_lds_dwordx4) in one burst --
//     every load in flight at once, one wait, one barrier;
//   * v_mfma_f32_16x16x4_f32, 8 waves with one 16 x 16 sub-tile each, operands read as
//     ds_read_b128 feeding 4 k-steps each (k permuted identically for A/B);
//   * partial tiles go to a slab; the last workgroup of each tile (device
//     ticket) sums the 8 partials in split order 0..7 -- deterministic and
//     independent of arrival order -- adds the bias, applies relu and writes
//     hfc, then re-arms the ticket.  No second launch.
//   * tickets == nullptr (FF act steps): partials only; policy_fc_kernel
//     (policy.hip) sums them in the same order and runs the heads, so the
//     ticket round trip and the last-arriver tail leave the step's chain.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 128 staging, 256 ticket/reduce, 512 MFMA)
#endif

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int FBM = 32, FBN = 64, FSPLIT = FC_SPLIT;
constexpr int FKS = A2 / FSPLIT;          // 324 columns per split
constexpr int FROWS = FBM + FBN;          // 96 staged rows (32 of a2, 64 of W)
constexpr int FV = FKS / 4;               // 81 float4 per row
constexpr int FVEC = FROWS * FV;          // 7776 float4 per workgroup
constexpr int FINSTR = (FVEC + 63) / 64;  // 122 wave-instructions of LDS-DMA
constexpr int FT = 512;                   // threads: 8 waves, one 16 x 16 output sub-tile each
constexpr int FW = FT / 64;
static_assert(A2 % (4 * FSPLIT) == 0, "K slice must be whole float4s");
static_assert(HID % FBN == 0, "N tiles");
}  // namespace

__global__ void __launch_bounds__(FT)
fc_fwd_kernel(const float* __restrict__ a2, int n, const float* __restrict__ W, const float* __restrict__ bias,
              float* __restrict__ slab, int* __restrict__ tickets, float* __restrict__ hfc) {
  __shared__ __attribute__((aligned(16))) float S[FROWS * FKS];   // 124,416 B
  __shared__ int is_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x % FSPLIT, tile = blockIdx.x / FSPLIT;
  constexpr int NTN = HID / FBN;
  const int m0 = (tile / NTN) * FBM, n0 = (tile % NTN) * FBN, k0 = split * FKS;

  // ---- stage: float4 i -> row i / 81, column 4 (i % 81); LDS image is the
  // unpadded [96][324] block, lane-linear per wave-instruction
  for (int it = wave; it < ((ARL_ABLATE & 128) ? 0 : FINSTR); it += FW) {
    const int i = it * 64 + lane;
    if (i < FVEC) {
      const int r = i / FV, c = i - r * FV;
      const float* src;
      if (r < FBM) src = a2 + (int64_t)min(m0 + r, n - 1) * A2;   // rows past n: any valid row, never stored
      else src = W + (int64_t)(n0 + r - FBM) * A2;
      __builtin_amdgcn_global_load_lds(src + k0 + 4 * c, (__attribute__((address_space(3))) void*)(S + it * 256),
                                       16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- MFMA: wave -> m sub-tile (wave & 1), n sub-tile (wave >> 1)
  const int q = lane >> 4, col = lane & 15;
  const int ms = wave & 1, ns = wave >> 1;
  const float* Ar = S + (ms * 16 + col) * FKS + 4 * q;
  const float* B0 = S + (FBM + ns * 16 + col) * FKS + 4 * q;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
  for (int s = 0; s < ((ARL_ABLATE & 512) ? 0 : FKS / 16); ++s) {   // 20 groups of 16 k: lane quarter q holds k = 16 s + 4 q + r
    const f32x4 av = *reinterpret_cast<const f32x4*>(Ar + 16 * s);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(B0 + 16 * s);
#pragma unroll
    for (int r = 0; r < 4; ++r) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r], b0[r], c0, 0, 0, 0);
  }
  {  // tail k = 320 + q
    constexpr int KT = (FKS / 16) * 16;
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ar[KT - 3 * q], B0[KT - 3 * q], c0, 0, 0, 0);
  }
  static_assert(FKS - (FKS / 16) * 16 == 4, "one tail k-step");

  // ---- partials: C row q*4 + r -> env m, col -> hidden unit.  Partials and
  // ticket use device-scope (sc1) accesses, which bypass the per-XCD L2s'
  // non-coherent state; no device-scope fence (an L2 writeback per workgroup
  // cost ~30 us here).  vmcnt(0) + barrier: every store of this workgroup has
  // been acknowledged at device scope before the ticket is taken.
  float* part = slab + (int64_t)split * n * HID;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + ms * 16 + q * 4 + r;
    if (m < n)
      __hip_atomic_store(part + (int64_t)m * HID + n0 + ns * 16 + col, c0[r], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if ((ARL_ABLATE & 256) || tickets == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    is_last = __hip_atomic_fetch_add(&tickets[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == FSPLIT - 1;
  __syncthreads();
  if (!is_last) return;
  // ---- last arrival: sum splits 0..7 in order, bias, relu (RJ float4 per thread,
  // all device-scope loads in flight before one wait)
  constexpr int RJ = FBM * FBN / 4 / FT;
  f32x4 p[RJ][FSPLIT];
  int mrow[RJ], ccol[RJ];
#pragma unroll
  for (int j = 0; j < RJ; ++j) {
    const int idx = tid + FT * j;           // 32 rows x 16 float4
    mrow[j] = m0 + (idx >> 4);
    ccol[j] = n0 + 4 * (idx & 15);
  }
#pragma unroll
  for (int z = 0; z < FSPLIT; ++z) {
    // one descriptor per split slab (wave-uniform base), aux 16 = sc1
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(slab + (int64_t)z * n * HID, 0, n * HID * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < RJ; ++j)
      p[j][z] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (min(mrow[j], n - 1) * HID + ccol[j]) * 4, 0, 16));
  }
#pragma unroll
  for (int j = 0; j < RJ; ++j) {
    if (mrow[j] < n) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int z = 0; z < FSPLIT; ++z)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], p[j][z][e]);
      const float4 b = *reinterpret_cast<const float4*>(bias + ccol[j]);
      float4 o;
      o.x = fmaxf(__fadd_rn(acc[0], b.x), 0.f); o.y = fmaxf(__fadd_rn(acc[1], b.y), 0.f);
      o.z = fmaxf(__fadd_rn(acc[2], b.z), 0.f); o.w = fmaxf(__fadd_rn(acc[3], b.w), 0.f);
      *reinterpret_cast<float4*>(hfc + (int64_t)mrow[j] * HID + ccol[j]) = o;
    }
  }
  if (tid == 0) __hip_atomic_store(&tickets[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int fc_fwd_tiles(int n) { return ((n + FBM - 1) / FBM) * (HID / FBN); }

hipError_t launch_fc_fwd(const float* a2, int n, const float* W, const float* b, float* slab, int* tickets,
                         float* hfc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fc_fwd_kernel, dim3((unsigned)(fc_fwd_tiles(n) * FSPLIT)), dim3(FT), 0, s, a2, n, W, b, slab,
                     tickets, hfc);
  return hipGetLastError();
}

}  // namespace arl
