// Fully connected layer of the NIPS head (dqn_head.py:43, Linear(2592, 256)
// followed by relu at dqn_head.py:52):  hfc = relu(a2 . W^T + b)  for the n
// envs of one lockstep step.
//
// M = n (envs), N = 256, K = 2592: latency-bound at these sizes, so the shape
// is chosen for one short dependency chain per workgroup:
//   * split-K 8 ways, one K slice (324) per XCD (blockIdx % 8 = split): each
//     XCD's L2 holds just its 324-column slice of a2 and W;
//   * 32 x 64 output tile per workgroup; the whole 96 x 324 operand block
//     (124 KB) is staged by LDS-DMA (global_load_lds_dwordx4) in one burst of
//     three K chunks -- every load in flight at once; the MFMAs of a chunk
//     start when it has landed (one wait + barrier per chunk);
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

#include <cstdlib>

#include "arl_internal.hpp"


namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int FBM = 32, FBN = 64, FSPLIT = FC_SPLIT;
constexpr int FKS = A2 / FSPLIT;          // 324 columns per split
constexpr int FROWS = FBM + FBN;          // 96 staged rows (32 of a2, 64 of W)
constexpr int FT = 512;                   // threads: 8 waves, one 16 x 16 output sub-tile each
constexpr int FW = FT / 64;
static_assert(A2 % (4 * FSPLIT) == 0, "K slice must be whole float4s");
static_assert(HID % FBN == 0, "N tiles");
// The K slice is staged in three chunks (112 + 112 + 100 columns), each a
// [96][stride] block of LDS (row strides 29 / 29 / 26 float4: 116 / 116 / 104
// floats put the 16 rows a b128 read touches on distinct bank quads); the
// chunks are issued back to back, and the MFMAs of chunk c run while chunks
// c+1.. are still landing.  A pad slot of a row (the 29th float4 of a 28-wide
// chunk, 26th of the 25-wide one) re-loads the row's last float4.
constexpr int FCH = 3;
__host__ __device__ constexpr int ch_k0(int c) { return c == 0 ? 0 : c == 1 ? 112 : 224; }
__host__ __device__ constexpr int ch_w(int c) { return c < 2 ? 28 : 25; }          // float4 used per row
__host__ __device__ constexpr int ch_ld(int c) { return c < 2 ? 29 : 26; }         // float4 per row (padded)
__host__ __device__ constexpr int ch_pieces(int c) { return (FROWS * ch_ld(c) + 63) / 64; }   // 44, 44, 39
// float4 offset of chunk c: whole pieces, so a chunk's last (partly past-the-end) piece lands in
// its own region, never in the next chunk's
__host__ __device__ constexpr int ch_base(int c) { return c == 0 ? 0 : c == 1 ? 44 * 64 : 88 * 64; }
static_assert(ch_pieces(0) == 44 && ch_pieces(1) == 44, "chunk bases");
constexpr int FLDS4 = ch_base(2) + ch_pieces(2) * 64;   // float4 of LDS incl. the last piece's overhang
static_assert(ch_k0(2) + 100 == FKS && ch_w(0) * 4 == 112 && ch_w(2) * 4 == 100, "chunks cover the slice");
// pieces of wave w in chunk c (piece it -> wave it % 8)
__host__ __device__ constexpr int ch_wave_pieces(int c, int w) { return (ch_pieces(c) - w + FW - 1) / FW; }
}  // namespace

__device__ inline void fc_wait_vm(int n) {   // s_waitcnt vmcnt(n), n wave-uniform, 0..16
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// The MFMAs of one staged chunk: fragments read per 16-k group, each group's reads waited for right
// before its four MFMAs (reading every fragment first measured slower: 9.7 -> 10.5 us at 512 envs, r3s)
template <int G>
__device__ inline f32x4 fc_chunk_mfma(const float* Ar, const float* B0, f32x4 c0) {
  f32x4 av[G], bv[G];
#pragma unroll
  for (int s = 0; s < G; ++s) {
    av[s] = *reinterpret_cast<const f32x4*>(Ar + 16 * s);
    bv[s] = *reinterpret_cast<const f32x4*>(B0 + 16 * s);
#pragma unroll
      for (int r = 0; r < 4; ++r) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s][r], bv[s][r], c0, 0, 0, 0);
  }
  return c0;
}

__global__ void __launch_bounds__(FT)
fc_fwd_kernel(const float* __restrict__ a2, int n, const float* __restrict__ W, const float* __restrict__ bias,
              float* __restrict__ slab, int* __restrict__ tickets, float* __restrict__ hfc) {
  __shared__ __attribute__((aligned(16))) float S[FLDS4 * 4];   // 130,048 B
  __shared__ int is_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x % FSPLIT, tile = blockIdx.x / FSPLIT;
  constexpr int NTN = HID / FBN;
  const int m0 = (tile / NTN) * FBM, n0 = (tile % NTN) * FBN, k0 = split * FKS;

  // ---- stage: every chunk's LDS-DMA pieces issued back to back; slot i of
  // chunk c -> row i / ld, float4 column min(i % ld, w - 1) of the chunk
#pragma unroll
  for (int c = 0; c < FCH; ++c) {
    for (int it = wave; it < ch_pieces(c); it += FW) {
      const int i = min(it * 64 + lane, FROWS * ch_ld(c) - 1);
      const int r = i / ch_ld(c), cc = min(i - r * ch_ld(c), ch_w(c) - 1);
      const float* src = r < FBM ? a2 + (int64_t)min(m0 + r, n - 1) * A2   // rows past n: any valid row, never stored
                                 : W + (int64_t)(n0 + r - FBM) * A2;
      __builtin_amdgcn_global_load_lds(src + k0 + ch_k0(c) + 4 * cc,
                                       (__attribute__((address_space(3))) void*)(S + 4 * (ch_base(c) + it * 64)), 16,
                                       0, 0);
    }
  }

  // ---- MFMA: wave -> m sub-tile (wave & 1), n sub-tile (wave >> 1); chunk c
  // after this wave's pieces of it have landed and a barrier (everyone's)
  const int q = lane >> 4, col = lane & 15;
  const int ms = wave & 1, ns = wave >> 1;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < FCH; ++c) {
    int later = 0;
#pragma unroll
    for (int c2 = c + 1; c2 < FCH; ++c2) later += ch_wave_pieces(c2, wave);
    fc_wait_vm(later);
    // LDS-only barrier: __syncthreads()'s fence would drain vmcnt, i.e. wait for the later chunks too
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const float* Ar = S + 4 * ch_base(c) + (ms * 16 + col) * 4 * ch_ld(c) + 4 * q;
    const float* B0 = S + 4 * ch_base(c) + (FBM + ns * 16 + col) * 4 * ch_ld(c) + 4 * q;
    constexpr int G16[FCH] = {7, 7, 6};   // whole 16-k groups per chunk
    // lane quarter q holds k = 16 s + 4 q + r
    c0 = G16[c] == 7 ? fc_chunk_mfma<7>(Ar, B0, c0) : fc_chunk_mfma<6>(Ar, B0, c0);
    if (c == FCH - 1) {   // tail k = 320 + q (chunk column 96 + q)
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ar[96 - 3 * q], B0[96 - 3 * q], c0, 0, 0, 0);
    }
  }

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
  if (tickets == nullptr) return;
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

// ---- partials-only launches over >= 512 envs: 64 x 64 output tiles on 16
// waves (one 16 x 16 sub-tile each), so 512 envs are one workgroup per CU (256
// workgroups) instead of two rounds of the 32 x 64 form, and each staged byte
// feeds twice the MFMAs.  The same three K chunks in the same k order
// (bit-identical partials), staged through two LDS buffers: chunks 0 and 1 are
// issued together, chunk 2 into chunk 0's buffer once its MFMAs are done.
namespace {
constexpr int GBM = 64, GT = 1024, GW = GT / 64;
constexpr int GROWS = GBM + FBN;                  // 128 staged rows (64 of a2, 64 of W)
__host__ __device__ constexpr int g_pieces(int c) { return (GROWS * ch_ld(c) + 63) / 64; }   // 58, 58, 52
constexpr int GBUF4 = g_pieces(0) * 64;           // float4 per buffer
static_assert(g_pieces(1) == g_pieces(0) && g_pieces(2) <= g_pieces(0), "chunk buffers");
__host__ __device__ constexpr int g_wave_pieces(int c, int w) { return (g_pieces(c) - w + GW - 1) / GW; }
}  // namespace

__global__ void __launch_bounds__(GT)
fc_fwd_big_kernel(const float* __restrict__ a2, int n, const float* __restrict__ W, float* __restrict__ slab,
                  int* __restrict__ tickets, const float* __restrict__ bias, float* __restrict__ hfc) {
  __shared__ __attribute__((aligned(16))) float S[2 * GBUF4 * 4];   // 118,784 B
  __shared__ int is_last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int split = blockIdx.x % FSPLIT, tile = blockIdx.x / FSPLIT;
  constexpr int NTN = HID / FBN;
  const int m0 = (tile / NTN) * GBM, n0 = (tile % NTN) * FBN, k0 = split * FKS;
  auto issue = [&](int c) {   // slot i of chunk c -> row i / ld, float4 column min(i % ld, w - 1)
    float* buf = S + 4 * (c & 1) * GBUF4;
    for (int it = wave; it < g_pieces(c); it += GW) {
      const int i = min(it * 64 + lane, GROWS * ch_ld(c) - 1);
      const int r = i / ch_ld(c), cc = min(i - r * ch_ld(c), ch_w(c) - 1);
      const float* src = r < GBM ? a2 + (int64_t)min(m0 + r, n - 1) * A2   // rows past n: never stored
                                 : W + (int64_t)(n0 + r - GBM) * A2;
      __builtin_amdgcn_global_load_lds(src + k0 + ch_k0(c) + 4 * cc,
                                       (__attribute__((address_space(3))) void*)(buf + 4 * it * 64), 16, 0, 0);
    }
  };
  issue(0);
  issue(1);
  const int q = lane >> 4, col = lane & 15;
  const int ms = wave & 3, ns = wave >> 2;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < FCH; ++c) {
    // this wave's pieces of chunk c have landed (chunk c + 1's may still fly), then everyone's
    fc_wait_vm(c + 1 < FCH ? g_wave_pieces(c + 1, wave) : 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const float* buf = S + 4 * (c & 1) * GBUF4;
    const float* Ar = buf + (ms * 16 + col) * 4 * ch_ld(c) + 4 * q;
    const float* B0 = buf + (GBM + ns * 16 + col) * 4 * ch_ld(c) + 4 * q;
    constexpr int G16[FCH] = {7, 7, 6};
    c0 = G16[c] == 7 ? fc_chunk_mfma<7>(Ar, B0, c0) : fc_chunk_mfma<6>(Ar, B0, c0);
    if (c == FCH - 1) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Ar[96 - 3 * q], B0[96 - 3 * q], c0, 0, 0, 0);
    if (c == 0) {   // every wave is done reading buffer 0: chunk 2 goes there
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(2);
    }
  }
  float* part = slab + (int64_t)split * n * HID;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + ms * 16 + q * 4 + r;
    if (m < n)
      __hip_atomic_store(part + (int64_t)m * HID + n0 + ns * 16 + col, c0[r], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tickets == nullptr) return;
  // the last of the tile's FSPLIT workgroups sums the partials in split order, adds the bias, applies
  // relu and writes hfc (as fc_fwd_kernel's tail: sc1 stores drained before the relaxed agent-scope
  // ticket, sc1 loads after it); one float4 of the 64 x 64 tile per thread
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid == 0) is_last = __hip_atomic_fetch_add(&tickets[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == FSPLIT - 1;
  __syncthreads();
  if (!is_last) return;
  const int mrow = m0 + (tid >> 4), ccol = n0 + 4 * (tid & 15);
  f32x4 p[FSPLIT];
#pragma unroll
  for (int z = 0; z < FSPLIT; ++z) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(slab + (int64_t)z * n * HID, 0, n * HID * 4, 0x00020000);
    p[z] = __builtin_bit_cast(f32x4,
                              __builtin_amdgcn_raw_buffer_load_b128(rsrc, (min(mrow, n - 1) * HID + ccol) * 4, 0, 16));
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int z = 0; z < FSPLIT; ++z)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], p[z][e]);
  const float4 b = *reinterpret_cast<const float4*>(bias + ccol);
  f32x4 o;
  o[0] = fmaxf(__fadd_rn(acc[0], b.x), 0.f); o[1] = fmaxf(__fadd_rn(acc[1], b.y), 0.f);
  o[2] = fmaxf(__fadd_rn(acc[2], b.z), 0.f); o[3] = fmaxf(__fadd_rn(acc[3], b.w), 0.f);
  if (mrow < n) *reinterpret_cast<f32x4*>(hfc + (int64_t)mrow * HID + ccol) = o;
  if (tid == 0) __hip_atomic_store(&tickets[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int fc_fwd_tiles(int n) { return ((n + FBM - 1) / FBM) * (HID / FBN); }

bool fc_fwd_big(int n) {
  // partials-only launches over >= 512 envs on the 64-row tiles (C4 0.503 -> 0.497 ms at one env group,
  // C3 1.215 -> 1.162 ms; at 256-env launches, 128 workgroups of them lose: profiles/r03/r3l);
  // ARL_FC_BIG=0 / 1 forces one form (A/B timing)
  static const char* big = getenv("ARL_FC_BIG");
  return (big && (big[0] == '0' || big[0] == '1')) ? big[0] == '1' : n >= 512;
}

hipError_t launch_fc_fwd(const float* a2, int n, const float* W, const float* b, float* slab, int* tickets,
                         float* hfc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (fc_fwd_big(n)) {
    // its 64-row tiles use the first half of the 32-row tiles' tickets
    const int tiles = ((n + GBM - 1) / GBM) * (HID / FBN);
    hipLaunchKernelGGL(fc_fwd_big_kernel, dim3((unsigned)(tiles * FSPLIT)), dim3(GT), 0, s, a2, n, W, slab, tickets, b,
                       hfc);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(fc_fwd_kernel, dim3((unsigned)(fc_fwd_tiles(n) * FSPLIT)), dim3(FT), 0, s, a2, n, W, b, slab,
                     tickets, hfc);
  return hipGetLastError();
}

}  // namespace arl
