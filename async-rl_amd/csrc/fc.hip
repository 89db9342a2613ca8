// Fully connected layer of the NIPS head (dqn_head.py:43, Linear(2592, 256)
// followed by relu at dqn_head.py:52):  hfc = relu(a2 . W^T + b)  for the n
// envs of one lockstep step.
//
// M = n (envs), N = 256, K = 2592: latency-bound at these sizes, so the shape
// is chosen for one short dependency chain per workgroup:
//   * split-K 8 ways, one K slice (324) per XCD (blockIdx % 8 = split): each
//     XCD's L2 holds just its 324-column slice of a2 and W;
//   * BM x 64 output tile per workgroup (BM = 32: 4 waves; BM = 64 for
//     launches over >= 512 envs: 8 waves, so 512 envs are one workgroup per
//     CU), two 16 x 16 output sub-tiles per wave along N, so one exact split
//     of the wave's a2 fragment feeds both (fc_fwd 10.7 -> 9.9 us at C4
//     against one sub-tile a wave, r5p);
//   * the f32 products on the bf16 matrix cores: a2 (f32) is split exactly
//     into three bf16 parts in registers, W comes pre-split as three bf16
//     planes (fc_planes_kernel / the RMSProp kernel write them whenever W
//     changes), 6 v_mfma_f32_16x16x32_bf16 per 32-deep k-step (bf16split.hpp:
//     f32-accurate, 2.7x fewer matrix cycles than the exact-f32 16x16x4 form);
//     the last 4 k of a slice on one exact-f32 v_mfma_f32_16x16x4_f32;
//   * operands staged by LDS-DMA (global_load_lds_dwordx4) in four K chunks
//     (96, 96, 96, 36 columns) through two LDS buffers; a chunk's MFMAs start
//     when it has landed (one counted wait + LDS-only barrier per chunk);
//   * partial tiles go to a slab; with tickets, the last workgroup of each tile
//     (device ticket) sums the 8 partials in split order 0..7 -- deterministic
//     and independent of arrival order -- adds the bias, applies relu and
//     writes hfc, then re-arms the ticket;
//   * tickets == nullptr (FF act steps, the LSTM's XRED steps): partials only;
//     policy_fc_kernel (policy.hip) or the LSTM gate kernel sums them in the
//     same order.
// Both tile heights run the same per-sub-tile MFMA sequence: bit-identical.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "arl_internal.hpp"
#include "bf16split.hpp"

namespace arl {

namespace {
constexpr int FBN = 64, FSPLIT = FC_SPLIT;
constexpr int FKS = A2 / FSPLIT;          // 324 columns per split
static_assert(A2 % (4 * FSPLIT) == 0 && FKS == 10 * 32 + 4, "K slice: ten 32-deep k-steps + a 4-deep tail");
static_assert(HID % FBN == 0, "N tiles");
constexpr int PSLICE = FC_PLANE_SLICE;    // 328 stored columns per split (arl_internal.hpp fc_plane_pos)
constexpr int64_t PLANE_ELEMS = (int64_t)HID * FC_PLANE_LD;
// chunk c: slice columns [96 c, 96 c + 96) (c < 3), [288, 324) (c = 3); A rows of 26 slots (416 B), B plane
// rows of 14 slots (224 B): conflict-free ds_read_b128 lane groups for both (scripts/lds_banks.py model)
constexpr int FCH = 4;
__host__ __device__ constexpr int ck_a(int c) { return c < 3 ? 24 : 9; }    // A float4 per row
__host__ __device__ constexpr int ck_b(int c) { return c < 3 ? 12 : 5; }    // B 16-byte slots per plane row
constexpr int A_LD = 26, B_LD = 14;                                            // 16-byte slots per row
template <int BM>
struct FcLay {
  static constexpr int NT = BM * 8;                      // threads: two 16 x 16 sub-tiles per wave (along N)
  static constexpr int NW = NT / 64;
  static constexpr int A_SLOTS = BM * A_LD;
  static constexpr int B_PLANE = FBN * B_LD;             // slots per B plane
  static constexpr int SLOTS = A_SLOTS + 3 * B_PLANE;
  static constexpr int PIECES = (SLOTS + 63) / 64;        // 1 KB LDS-DMA pieces per chunk
  static constexpr int BUF = PIECES * 64;                 // slots per buffer (incl. the last piece's overhang)
  static constexpr int PW_MAX = (PIECES + NW - 1) / NW;
};
static_assert(2 * FcLay<64>::BUF * 16 <= 160 * 1024 && 2 * FcLay<32>::BUF * 16 <= 160 * 1024, "LDS");
static_assert(FcLay<64>::PW_MAX <= 16 && FcLay<32>::PW_MAX <= 16, "fc_wait_vm range");
}  // namespace

__device__ inline void fc_wait_vm(int n) {   // s_waitcnt vmcnt(n), n wave-uniform, 0..12
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
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int BM>
__global__ void __launch_bounds__(FcLay<BM>::NT)
fc_fwd_kernel(const float* __restrict__ a2, int n, const uint16_t* __restrict__ Wp, const float* __restrict__ bias,
              float* __restrict__ slab, int* __restrict__ tickets, float* __restrict__ hfc) {
  using LY = FcLay<BM>;
  constexpr int NT = LY::NT, NW = LY::NW;
  __shared__ __attribute__((aligned(16))) uint8_t S[2 * LY::BUF * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x % FSPLIT, tile = blockIdx.x / FSPLIT;
  constexpr int NTN = HID / FBN;
  const int m0 = (tile / NTN) * BM, n0 = (tile % NTN) * FBN, k0 = split * FKS;
  // slot i of a buffer -> A row i / A_LD (f32 float4 column min(i % A_LD, ck_a - 1)) or B plane p row j
  // (16-byte column min(.., ck_b - 1)); pad slots re-load a valid 16 bytes
  auto issue = [&](int c) {
    uint8_t* buf = S + 16 * (c & 1) * LY::BUF;
#pragma unroll
    for (int ii = 0; ii < LY::PW_MAX; ++ii) {
      const int it = min(wave + NW * ii, LY::PIECES - 1);   // (every wave issues PW_MAX pieces: exact waits)
      const int i = min(it * 64 + lane, LY::SLOTS - 1);
      const void* src;
      if (i < LY::A_SLOTS) {
        const int r = i / A_LD, cc = min(i - r * A_LD, ck_a(c) - 1);
        src = a2 + (int64_t)min(m0 + r, n - 1) * A2 + k0 + 96 * c + 4 * cc;   // rows past n: never stored
      } else {
        const int ib = i - LY::A_SLOTS, p = ib / LY::B_PLANE, rem = ib - p * LY::B_PLANE;
        const int j = rem / B_LD, cc = min(rem - j * B_LD, ck_b(c) - 1);
        src = Wp + p * PLANE_ELEMS + (int64_t)(n0 + j) * FC_PLANE_LD + split * PSLICE + 96 * c + 8 * cc;
      }
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(buf + 16 * it * 64), 16, 0, 0);
    }
  };
  issue(0);
  issue(1);
  const int g = lane >> 4, col = lane & 15;
  // wave: m sub-tile ms, n sub-tiles 2 np and 2 np + 1 (one A split feeds both)
  const int ms = wave % (BM / 16), np = wave / (BM / 16);
  f32x4 big[2], sml[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) big[u] = sml[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < FCH; ++c) {
    // this wave's pieces of chunk c have landed (chunk c + 1's may still fly), then everyone's
    fc_wait_vm(c + 1 < FCH ? LY::PW_MAX : 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const uint8_t* buf = S + 16 * (c & 1) * LY::BUF;
    const float* Ar = reinterpret_cast<const float*>(buf) + (ms * 16 + col) * (4 * A_LD);
    const uint8_t* Br0 = buf + 16 * (LY::A_SLOTS + (2 * np * 16 + col) * B_LD);
#pragma unroll
    for (int s = 0; s < (c < 3 ? 3 : 1); ++s) {
      // lane quarter g: k = 32 s + 16 h + 4 g + r (element 4 h + r) on both sides
      float x[8];
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(Ar + 32 * s + 4 * g);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(Ar + 32 * s + 16 + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = a0[r];
        x[4 + r] = a1[r];
      }
      bf16x8 ah, am, al;
      split3_x8(x, ah, am, al);
      const int bo = 64 * s + 16 * g;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint8_t* Br = Br0 + 16 * 16 * B_LD * u;
        const bf16x8 bh = lds_load<bf16x8>(Br, bo), bm = lds_load<bf16x8>(Br, bo + 16 * LY::B_PLANE),
                     bl = lds_load<bf16x8>(Br, bo + 32 * LY::B_PLANE);
        mfma_x6(ah, am, al, bh, bm, bl, big[u], sml[u]);
      }
    }
    if (c == FCH - 1) {   // the slice's last 4 k (chunk columns 32 + g): exact f32, W rebuilt from its planes
      const float at = Ar[32 + g];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint16_t* bt = reinterpret_cast<const uint16_t*>(Br0 + 16 * 16 * B_LD * u) + 32 + g;
        const float wt = __fadd_rn(__fadd_rn(__uint_as_float((uint32_t)bt[0] << 16),
                                             __uint_as_float((uint32_t)bt[8 * LY::B_PLANE] << 16)),
                                   __uint_as_float((uint32_t)bt[16 * LY::B_PLANE] << 16));
        sml[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(at, wt, sml[u], 0, 0, 0);
      }
    }
    if (c + 2 < FCH) {   // every wave is done reading buffer c & 1: chunk c + 2 goes there
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(c + 2);
    }
  }

  // ---- partials: C row 4 g + r -> env m, col -> hidden unit.  Partials and
  // ticket use device-scope (sc1) accesses, which bypass the per-XCD L2s'
  // non-coherent state; no device-scope fence (an L2 writeback per workgroup
  // cost ~30 us here).  vmcnt(0) + barrier: every store of this workgroup has
  // been acknowledged at device scope before the ticket is taken.
  float* part = slab + (int64_t)split * n * HID;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + ms * 16 + g * 4 + r;
      if (m < n)
        __hip_atomic_store(part + (int64_t)m * HID + n0 + (2 * np + u) * 16 + col, __fadd_rn(big[u][r], sml[u][r]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (tickets == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int& is_last = *reinterpret_cast<int*>(S);   // the staging array (every read of it is done): no second
  if (tid == 0)                                // __shared__ object, which would make the compiler drain the DMA
    is_last = __hip_atomic_fetch_add(&tickets[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == FSPLIT - 1;
  __syncthreads();
  if (!is_last) return;
  // ---- last arrival: sum splits 0..7 in order, bias, relu; RJ float4 of the BM x 64 tile per thread,
  // all device-scope loads in flight before one wait
  constexpr int RJ = BM * FBN / 4 / NT;
  f32x4 p[RJ][FSPLIT];
  int mrow[RJ], ccol[RJ];
#pragma unroll
  for (int j = 0; j < RJ; ++j) {
    const int idx = tid + NT * j;           // BM rows x 16 float4
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

// FC W (256, 2592) f32 -> the three bf16 split planes in fc_fwd_kernel's stored order (4 columns a thread:
// one float4 read, one 8-byte store per plane; the 4 pad columns of each slice are never read as data)
__global__ void __launch_bounds__(256) fc_planes_kernel(const float* __restrict__ W, uint16_t* __restrict__ planes) {
  const int q = blockIdx.x * 256 + threadIdx.x;   // float4 of W
  if (q >= HID * A2 / 4) return;
  fc_planes_store(planes, 4 * q, reinterpret_cast<const float4*>(W)[q]);
}

int fc_fwd_tiles(int n) { return ((n + 31) / 32) * (HID / FBN); }

bool fc_fwd_big(int n) {
  // launches over >= 512 envs on the 64-row tiles (C4 0.503 -> 0.497 ms at one env group, C3 1.215 -> 1.162
  // ms; at 256-env launches, 128 workgroups of them lose: profiles/r03/r3l); ARL_FC_BIG=0 / 1 forces one
  // form (the bitwise arm of test_conv_fwd_two_envs_identical)
  static const char* big = getenv("ARL_FC_BIG");
  return (big && (big[0] == '0' || big[0] == '1')) ? big[0] == '1' : n >= 512;
}

hipError_t launch_fc_planes(const float* W, uint16_t* planes, hipStream_t s) {
  hipLaunchKernelGGL(fc_planes_kernel, dim3((HID * A2 / 4 + 255) / 256), dim3(256), 0, s, W, planes);
  return hipGetLastError();
}

hipError_t launch_fc_fwd(const float* a2, int n, const uint16_t* Wp, const float* b, float* slab, int* tickets,
                         float* hfc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (fc_fwd_big(n)) {   // its 64-row tiles use the first half of the 32-row tiles' tickets
    const int tiles = ((n + 63) / 64) * (HID / FBN);
    hipLaunchKernelGGL(fc_fwd_kernel<64>, dim3((unsigned)(tiles * FSPLIT)), dim3(FcLay<64>::NT), 0, s, a2, n, Wp, b,
                       slab, tickets, hfc);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(fc_fwd_kernel<32>, dim3((unsigned)(fc_fwd_tiles(n) * FSPLIT)), dim3(FcLay<32>::NT), 0, s, a2, n,
                     Wp, b, slab, tickets, hfc);
  return hipGetLastError();
}

}  // namespace arl
