// Backward of the NIPS head's fully connected layer (dqn_head.py:43,52,
// Linear(2592, 256) + relu) over the S = t_max * n samples of a window
// (a3c.py:129-130):
//   dW[j][k] = sum_s dfc[s][j] a2[s][k],  db[j] = sum_s dfc[s][j]
//   da2[s][k] = (sum_j dfc[s][j] W[j][k]) * (a2[s][k] > 0)
// (dfc is already masked by hfc > 0).  One launch, two independent jobs:
//   job A (dW, db): 256 (all j) x 32 (k) tiles -- every dfc row staged once
//     per tile feeds 256 x 32 outputs, so the LDS-DMA bytes per FLOP stay
//     under what a CU can stream -- over one of Z contiguous sample ranges.
//     The Z range partials of a tile meet in the same launch: each workgroup
//     takes a ticket when its range is done; the first Z - 1 publish their
//     partial (write-through stores, then a per-tile "published" count), the
//     last waits for that count, sums the Z partials in range order
//     (deterministic whatever the arrival order) and writes dW / db straight
//     into the flat gradient.  The last arriver's own partial never leaves
//     its registers.  MFMA accumulators restart every 32-sample chunk; chunk
//     sums are added in f64.  db: the k-tile 0 workgroups add the A fragments
//     they already hold.
//   job B (da2): 128 (s) x 128 (k) tiles over K = 256, ReLU mask in the
//     epilogue.
// Operands stream HBM/L2 -> LDS by LDS-DMA (global_load_lds dwordx4) into two
// 36 KB stages (K chunks of 32; the next chunk in flight while the current one
// feeds the MFMAs); exact f32 MFMA (v_mfma_f32_16x16x4_f32); 512 threads.
// The DMA writes lane-linear, so the LDS images are XOR-swizzled through the
// global source address (physical 16-byte chunk = logical chunk ^ key):
//   job A  A: dfc rows s, 256 floats of j, key 4*(row & 3)         b32 reads, rows kb + q
//          B: a2 rows s, 32 floats of k,   key 4*((row >> 1) & 1)  b32 reads, rows kb + q
//   job B  A: dfc rows s, 32 floats of j,  key (row >> 1) & 7      b128 reads (k-permuted)
//          B: W rows j, 128 floats of k,   key 4*((row >> 2) & 3)  b32 reads, rows 16g + 4q + r
// so every fragment read is free of bank conflicts.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "arl_internal.hpp"

namespace arl {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NT = 512;                 // 8 waves
constexpr int NW = NT / 64;
constexpr int BK = 32;                  // K chunk (rows of a stage)
constexpr int STAGE = 9216;             // floats per LDS stage (job A: 32 x 256 + 32 x 32)
constexpr int AK = 32;                  // job A: k columns per tile
constexpr int NKA = A2 / AK;            // 81 job A tiles per range
constexpr int BM = 128, BN = 128;       // job B tile
constexpr int NKB = (A2 + BN - 1) / BN; // 21 (the last one a quarter full)
constexpr int PART = HID * AK + HID;    // floats per published partial (dW tile + db)
static_assert(A2 % AK == 0 && HID == 256, "tiles");

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ inline void barrier_lds() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Stage R rows x WC floats of a row-major matrix into LDS at dst by LDS-DMA:
// tile row r = global row min(row0 + r, rmax); logical 16-byte chunk c of
// row r lands at physical chunk c ^ key(r).  Wave w issues the 1 KB pieces
// w, w + NW, ...
template <int R, int WC, int KEY>
__device__ inline void stage_tile(float* dst, const float* __restrict__ g, int64_t ld, int row0, int rmax, int col0) {
  constexpr int CPR = WC / 4;                 // chunks per row
  constexpr int NI = R * WC * 4 / 1024;       // 1 KB pieces
  static_assert(NI % NW == 0 || NI < NW, "pieces per wave");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int it = wave; it < NI; it += NW) {
    const int i = it * 64 + lane;             // chunk index in the tile image
    const int r = i / CPR, pc = i - r * CPR;
    int key;
    if constexpr (KEY == 0) key = 4 * (r & 3);
    else if constexpr (KEY == 1) key = 4 * ((r >> 1) & 1);
    else if constexpr (KEY == 2) key = (r >> 1) & 7;
    else key = 4 * ((r >> 2) & 3);
    const int row = min(row0 + r, rmax);
    const float* src = g + (int64_t)row * ld + col0 + 4 * (pc ^ key);
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(dst + it * 256), 16, 0, 0);
  }
}

struct FcBwdArgs {
  const float* dfc;   // (S, 256)
  const float* a2;    // (S, 2592)
  const float* W;     // (256, 2592)
  int S, Z, kpz;      // job A: Z sample ranges of kpz samples (multiple of BK)
  float* gW;          // (256, 2592)
  float* gb;          // (256)
  float* da2;         // (S, 2592)
  float* part;        // (NKA, Z, PART) published job A partials (slot z = range z)
  int* tick;          // (2 * NKA): arrival ticket, published count per k tile
  int b0;             // first job index of this launch (timing experiments)
  int abl;            // ARL_FC_BWD_ABL bits (timing experiments only): 1 no MFMA, 2 no staging
};

// ---------------------------------------------------------------- job A: dW, db
__device__ void job_dw(const FcBwdArgs& a, int tile, float* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;
  const int kt = tile % NKA, z = tile / NKA;
  const int k0 = kt * AK;
  const int r0 = z * a.kpz, r1 = min(a.S, r0 + a.kpz);
  const bool bias = kt == 0;
  const int nchunks = (r1 - r0 + BK - 1) / BK;
  double tot[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) tot[i][jj][e] = 0.0;
  float bsum[2] = {0.f, 0.f};
  auto issue = [&](int c) {
    if (a.abl & 2) return;
    float* st = lds + (c & 1) * STAGE;
    stage_tile<BK, HID, 0>(st, a.dfc, HID, r0 + c * BK, r1 - 1, 0);          // dfc[s][0..255]
    stage_tile<BK, AK, 1>(st + BK * HID, a.a2, A2, r0 + c * BK, r1 - 1, k0);  // a2[s][k0..k0+31]
  };
  if (nchunks > 0) issue(0);
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) {
      issue(c + 1);
      // DMA pieces per wave per chunk: 4 of dfc, + 1 of a2 on waves 0..3
      if (wave < 4) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_lds();
    const float* As = lds + (c & 1) * STAGE;
    const float* Bs = As + BK * HID;
    const int kvalid = r1 - (r0 + c * BK);   // rows >= kvalid: clamped copies, masked to 0
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int ks = 0; ks < ((a.abl & 1) ? 0 : BK / 4); ++ks) {
      const int r = 4 * ks + q;
      const bool ok = r < kvalid;
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = wave * 32 + i * 16 + col;
        const float v = As[r * HID + (((m >> 2) ^ (4 * q)) << 2) + (m & 3)];
        av[i] = ok ? v : 0.f;
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int n = jj * 16 + col;
        bv[jj] = Bs[r * AK + (((n >> 2) ^ (4 * ((r >> 1) & 1))) << 2) + (n & 3)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[jj], acc[i][jj], 0, 0, 0);
      if (bias) {
        bsum[0] = __fadd_rn(bsum[0], av[0]);
        bsum[1] = __fadd_rn(bsum[1], av[1]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) tot[i][jj][e] += (double)acc[i][jj][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_lds();   // this stage is restaged two chunks on
  }
  // this range's partial, rounded to f32 (every range's partial is, whoever arrives last)
  float p[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) p[i][jj][e] = (float)tot[i][jj][e];
  float pb[2] = {0.f, 0.f};
  if (bias) {   // lanes (col, q) hold sums over rows = q (mod 4): fixed-order quarter reduction
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v = bsum[i];
      v = __fadd_rn(v, __shfl_xor(v, 16));
      pb[i] = __fadd_rn(v, __shfl_xor(v, 32));
    }
  }
  // C layout (16x16x4): lane (col, q) holds rows 4q + e of column col
  auto out_index = [&](int i, int jj, int e) { return (wave * 32 + i * 16 + 4 * q + e) * AK + jj * 16 + col; };
  if (a.Z > 1) {
    int* flag = reinterpret_cast<int*>(lds);   // the stages are free after the k loop's last barrier
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(&a.tick[kt], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = t == a.Z - 1;
    }
    __syncthreads();   // (no DMA in flight here: its vmcnt(0) is free)
    const int last = *flag;
    if (!last) {   // publish into slot z: write-through (sc1) stores, drained, then the count
      float* dst = a.part + ((int64_t)kt * a.Z + z) * PART;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __hip_atomic_store(dst + out_index(i, jj, e), p[i][jj][e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (bias && q == 0)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __hip_atomic_store(dst + HID * AK + wave * 32 + i * 16 + col, pb[i], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&a.tick[NKA + kt], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    // last arriver: wait until the other Z - 1 partials are published (their
    // workgroups already hold a ticket, so they are resident); bounded spin
    if (tid == 0) {
      for (int spin = 0; spin < (1 << 24); ++spin) {
        if (__hip_atomic_load(&a.tick[NKA + kt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.Z - 1) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every partial load below is sc1
  }
  // sum the Z partials in range order (own range from registers), f64
  double s[2][2][4];
  double sb[2] = {0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[i][jj][e] = 0.0;
  for (int zz = 0; zz < a.Z; ++zz) {
    // a whole slot's values into registers first (one branch per slot, all
    // loads in flight together), then the ordered f64 adds
    float v[2][2][4], vb[2];
    if (zz == z) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        vb[i] = pb[i];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[i][jj][e] = p[i][jj][e];
      }
    } else {
      const float* src = a.part + ((int64_t)kt * a.Z + zz) * PART;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        vb[i] = __hip_atomic_load(src + HID * AK + wave * 32 + i * 16 + col, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[i][jj][e] = __hip_atomic_load(src + out_index(i, jj, e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sb[i] += (double)vb[i];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[i][jj][e] += (double)v[i][jj][e];
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = wave * 32 + i * 16 + 4 * q + e;
        a.gW[(int64_t)j * A2 + k0 + jj * 16 + col] = (float)s[i][jj][e];
      }
  if (bias && q == 0)
#pragma unroll
    for (int i = 0; i < 2; ++i) a.gb[wave * 32 + i * 16 + col] = (float)sb[i];
  if (a.Z > 1 && tid == 0) {   // re-arm for the next launch (a captured graph replays this one)
    __hip_atomic_store(&a.tick[kt], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.tick[NKA + kt], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- job B: da2
__device__ void job_da2(const FcBwdArgs& a, int tile, float* lds) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;   // wave: 32 s x 64 k
  const int kt = tile % NKB, st = tile / NKB;
  const int s0 = st * BM, k0 = kt * BN;
  constexpr int NCH = HID / BK;              // 8 chunks of 32 j
  auto issue = [&](int c) {
    if (a.abl & 2) return;
    float* sg = lds + (c & 1) * STAGE;
    stage_tile<BM, BK, 2>(sg, a.dfc + c * BK, HID, s0, a.S - 1, 0);                    // dfc[s][j]
    stage_tile<BK, BN, 3>(sg + BM * BK, a.W + (int64_t)c * BK * A2, A2, 0, BK - 1, k0);  // W[j][k0..k0+127]
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  issue(0);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) {
      issue(c + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // 2 + 2 DMA pieces per wave per chunk
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_lds();
    const float* As = lds + (c & 1) * STAGE;
    const float* Bs = As + BM * BK;
#pragma unroll
    for (int g = 0; g < ((a.abl & 1) ? 0 : BK / 16); ++g) {
      f32x4 av[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = wm * 32 + i * 16 + col;
        av[i] = *reinterpret_cast<const f32x4*>(As + m * BK + (((4 * g + q) ^ ((m >> 1) & 7)) << 2));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * g + 4 * q + r;
        float bv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int n = wn * 64 + jj * 16 + col;
          bv[jj] = Bs[row * BN + (((n >> 2) ^ (4 * q)) << 2) + (n & 3)];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][r], bv[jj], acc[i][jj], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_lds();
  }
  // ReLU mask: every a2 value loaded first (clamped rows / columns, all in
  // flight at once), then the guarded stores
  float mk[2][4][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int k = min(k0 + wn * 64 + jj * 16 + col, A2 - 1);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = min(s0 + wm * 32 + i * 16 + 4 * q + e, a.S - 1);
        mk[i][jj][e] = a.a2[(int64_t)s * A2 + k];
      }
    }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int k = k0 + wn * 64 + jj * 16 + col;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = s0 + wm * 32 + i * 16 + 4 * q + e;
        if (s < a.S && k < A2) a.da2[(int64_t)s * A2 + k] = mk[i][jj][e] > 0.f ? acc[i][jj][e] : 0.f;
      }
    }
}

__global__ void __launch_bounds__(NT)
fc_bwd_kernel(FcBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];   // 72 KB, the only LDS object
  const int b = a.b0 + blockIdx.x;
  const int na = NKA * a.Z;
  if (b < na) job_dw(a, b, lds);
  else job_da2(a, b - na, lds);
}

int fc_bwd_ranges(int S) { return std::max(1, std::min(3, (S + 4 * BK - 1) / (4 * BK))); }
}  // namespace

int64_t fc_bwd_part_floats(int S) { return (int64_t)NKA * fc_bwd_ranges(S) * PART; }
int fc_bwd_tickets() { return 2 * NKA; }

// Job B's last k tile stages W columns 2560..2687: the floats past the end of
// W belong to the next parameters of the flat buffer (never stored).
hipError_t launch_fc_bwd(const float* dfc, const float* a2, const float* W, int S, float* gW, float* gb, float* da2,
                         float* part, int* tick, hipStream_t s) {
  if (S <= 0) return hipSuccess;
  const int Z = fc_bwd_ranges(S);
  int kpz = (S + Z - 1) / Z;
  kpz = (kpz + BK - 1) / BK * BK;
  const int na = NKA * Z, nb = ((S + BM - 1) / BM) * NKB;
  // ARL_FC_BWD_JOBS=a / b: launch one job alone (timing experiments only)
  static const char* only = getenv("ARL_FC_BWD_JOBS");
  const int b0 = (only && only[0] == 'b') ? na : 0;
  const int grid = (only && only[0] == 'a') ? na : (only && only[0] == 'b') ? nb : na + nb;
  static const char* abl = getenv("ARL_FC_BWD_ABL");
  FcBwdArgs args{dfc, a2, W, S, Z, kpz, gW, gb, da2, part, tick, b0, abl ? atoi(abl) : 0};
  hipLaunchKernelGGL(fc_bwd_kernel, dim3(grid), dim3(NT), 0, s, args);
  return hipGetLastError();
}

}  // namespace arl
