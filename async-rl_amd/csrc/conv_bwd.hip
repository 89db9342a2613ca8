// Fused backward of the two conv layers of the NIPS head (dqn_head.py:41-42)
// for one lockstep window: per sample s
//   (1) dW2 += da2 (x) im2col(a1)           conv2 weight gradient, K = 81 positions
//   (2) da1  = conv_transpose(da2, W2) * (a1 > 0)        (stride-2 parity classes)
//   (3) dW1 += im2col(x)^T (x) da1           conv1 weight gradient, K = 400 positions
// with every operand of a sample resident in LDS: da1 never touches HBM and
// a1 / da2 / x are read once.
//
// Reference: a3c.py:129-130 (total_loss.backward through Chainer's
// Convolution2D backward: im2col + tensordot for gW, col2im for gx).
//
// One workgroup per CU; every operand of a sample has its own LDS region
// (152 KB).  Workgroup b handles samples b, b + G, ...  Two forms, bit-identical:
// * conv_bwd_ws_kernel (the default, below): 1,024 threads; waves 0-7 run (2)
//   and (3), waves 8-15 run (1) and the commits, two barriers a sample;
// * conv_bwd_kernel (ARL_CB_WS=0, the test arm): 512 threads (8 waves, 2 per
//   SIMD), a sample in four barrier-separated phases: commit, (1) + mask, (2),
//   (3); the next sample's a1 / da2 / screens are loaded into registers
//   (unconditional loads from clamped addresses: no load waits for another)
//   while the current one computes.
//
// All three run on the bf16 matrix cores with exact bf16 splits of the f32
// operands (bf16split.hpp; f32-accurate):
// (1) M = 32 oc x N = 256 (ic, ky, kx) x K = 81 positions p = 9 oy + ox (3
//     k-steps of 32, positions past 80 zero on the A side); wave w owns n-tiles
//     2w, 2w+1 of both m-tiles.  A = da2 split planes [oc][p], written at commit
//     time; B = 8 consecutive positions of one (ic, ky, kx) column gathered from
//     the f32 a1 rows and split in registers -- no convert pass, 6 MFMAs per
//     tile pair and k-step (72 issues of 16 cycles a wave, was 84 exact-f32
//     16x16x4 of 32).
// (2) per parity class (py, px) = wave & 3: C^T = W2 (16 ic rows) x the da2
//     split planes stored channel-last on an 11 x 11 grid with a zero border
//     (16 consecutive grid cells per tile, 7 tiles; the shifted windows need
//     no bounds checks), K = 128 ordered (dy, dx, oc); 6 MFMAs per k-step.
//     Waves w and w + 4 share a class (tiles 0-3 / 4-6).  The masked result
//     is written as da1 split planes.
// (3) the stride-4 im2col is made contiguous by splitting each screen row
//     into its 4 column phases b = x & 3 (X = x >> 2):
//       dW1[oc][ic][ky][4a + b] = sum_{oy, X} xph[ic][4 oy + ky][b][X + a] da1[oc][oy][X]
//     M = 256 (ic, ky, a, b) x N = 16 oc x K = 480 (oy, X padded 20 -> 24);
//     the A fragment is 8 contiguous pixels shifted by a bytes (v_alignbyte),
//     exact in bf16, so 3 MFMAs per k-step.  Wave w owns screen ic = w >> 1,
//     ky = 4 (w & 1) + 0..3, both a (2 tiles sharing one pixel conversion).
// Integer pixel values feed (3) and 1/255 is applied in the reduction.
// Each workgroup writes one partial slab; reduce_conv_bwd_kernel sums the
// slabs in f64 in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "bf16split.hpp"
#include "conv_slab.hpp"

namespace arl {

namespace {
constexpr int NT = 512;                    // threads per workgroup (8 waves; one workgroup per CU)
constexpr int PX = 4;                      // screens per sample (one load of 4 dwords per thread each)
constexpr int GI = 121 * 4;                // da2 grid items: (oc group, cell)
constexpr int PG = (GI + NT - 1) / NT;     // 1 per thread
// LDS map (bytes).  Strides are chosen for conflict-free banking of the hot
// reads (scripts/lds_banks.py models every site): a1 rows of 24 floats, da2
// [p][oc] rows of 48 floats, grid slot = g * 128 + cell, da1 oc rows of 62
// 16-byte slots.
constexpr int A1R = 24;                    // a1 f32 row stride (20 used)
constexpr int A1C = 20 * A1R;              // a1 f32 channel stride
constexpr int XR = 24;                     // phase row: X = 0..20 (+ pad), uint8
constexpr int D1_ROW = 48;                 // da1 plane row (oy): 24 bf16, X 20..23 zero
constexpr int D1_OC = 992;                 // da1 plane oc row: 62 16-byte slots
constexpr int D1P = 16 * D1_OC;            // 15,872 per plane
constexpr int GRID_G = 128;                // grid slots per oc group (121 cells used)
constexpr int D2P = 4 * GRID_G * 16;       // 8,192 per plane
constexpr int L_D1 = 0;                    // da1 split planes, 3 x D1P            47,616
constexpr int L_XPH = L_D1 + 3 * D1P;      // [ic][y][b][XR]                        32,256
constexpr int L_D2 = L_XPH + 4 * 84 * 4 * XR;   // da2 split grid, 3 x D2P          24,576
constexpr int L_MASK = L_D2 + 3 * D2P;     // a1 > 0, u16 of 16 channel bits per pixel 800
constexpr int L_A1 = L_MASK + 800;         // a1 f32 [16][20][A1R]                  30,720
// (1)'s A operand: da2 split planes [3][oc][p] (row 208 B = 13 16-byte slots, an odd count, so the 16
// rows a ds_read_b128 lane group reads land on distinct bank quads); positions 81..103 stay 0
constexpr int DA_ROW = 208;
constexpr int DAP = 32 * DA_ROW;           // 6,656 per plane
constexpr int L_DA = L_A1 + C1_OC * A1C * 4;    // 3 x DAP                             19,968
constexpr int L_END = L_DA + 3 * DAP;      // 155,936
static_assert(L_DA % 16 == 0, "alignment");
constexpr int L_RED = 0;                   // end: f32 [16][128] (after the last sample)
static_assert(L_END <= 160 * 1024, "LDS");
static_assert(L_XPH % 16 == 0 && L_D2 % 16 == 0 && L_A1 % 16 == 0 && L_MASK % 8 == 0, "alignment");
}  // namespace

// da2 plane byte offset of (cell, oc group g = oc >> 3): the 16 cells a
// b128 lane group reads are consecutive, so slot g * 128 + cell spreads them
// over all 64 banks
__device__ inline int d2_slot(int cell, int g) { return (g * GRID_G + cell) << 4; }

struct ConvBwdArgs {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R;
  const float* a1;     // (S, 16, 400)
  const float* da2;    // (S, 32, 81), already masked by a2 > 0
  const float* W2;     // (32, 16, 4, 4)
  int S, G;            // samples; workgroups (workgroup b: samples b, b + G, ...)
  float* slab;         // (G, SLAB)
  int layout;          // FrameLayout (FRAMES_RGB: (R, n, 3, 84, 84), planes [0, R, G, B];
                       // FRAMES_STACK: (R, n, 4, 84, 84))
};

// a1 / da2 of a sample: a1 as float4 runs, da2 as (oc group, grid cell) items
// of 8 channels.  The prefetches are pure loads from clamped, always-valid
// addresses (no branch, no zero-fill of a load's destination register, so no
// load waits for another); validity is applied at commit time.
struct PrefetchA {
  float d[PG][8];
};
struct PrefetchX {
  uint4 x[PX];
  int nv;   // lane 0: nvalid of the sample's (slot, env); other lanes: other envs (read at commit)
};

__device__ inline void grid_item(int i, int& grp, int& cell, bool& v, int& p) {
  grp = i / 121;
  cell = i - grp * 121;
  const int cy = cell / 11, cx = cell - cy * 11;
  v = i < GI && cy >= 1 && cy <= 9 && cx >= 1 && cx <= 9;
  p = v ? (cy - 1) * 9 + cx - 1 : 0;
}

__device__ inline void prefetch_a(const ConvBwdArgs& a, int s, PrefetchA& r) {
  const int tid = threadIdx.x;
  const float* g2 = a.da2 + (int64_t)s * A2;
#pragma unroll
  for (int j = 0; j < PG; ++j) {
    int grp, cell, p;
    bool v;
    grid_item(tid + NT * j, grp, cell, v, p);
    const float* src = g2 + (v ? 8 * grp * C2_P + p : 0);   // k-th load at a constant offset
#pragma unroll
    for (int k = 0; k < 8; ++k) r.d[j][k] = src[k * C2_P];
  }
}

// screens: load j = plane c covers the plane's 504 items (row y, quad q) =
// dwords 4q..4q+3 of the row on threads 0..503; q = 5 holds the row's last
// dword (20), loaded as dwords 17..20 so no read passes the row.  The plane
// base is uniform (scalar address + one offset VGPR per item).
__device__ inline void prefetch_x(const ConvBwdArgs& a, int64_t step0, int s, PrefetchX& r) {
  const int tid = threadIdx.x;
  const int t = s / a.n, e = s - t * a.n;
  const int64_t ks = step0 + t;
  const int rs = (int)(ks % a.R);
  // a lane-varying address keeps the load a vector load that nothing waits
  // for until commit_x broadcasts lane 0 (a uniform one would be moved to an
  // SGPR right after the load, i.e. waited for at once)
  r.nv = a.nvalid[(int64_t)rs * a.n + min(e + (tid & 63), a.n - 1)];
  const int it = tid < 504 ? tid : 0;
  const int y = it / 6, q = it - 6 * (it / 6);
  const int off = y * 84 + (q < 5 ? 16 * q : 68);
#pragma unroll
  for (int c = 0; c < PX; ++c) {
    const int64_t pl = a.layout == FRAMES_STACK ? ((int64_t)rs * a.n + e) * 4 + c
                       : a.layout == FRAMES_RGB ? ((int64_t)rs * a.n + e) * 3 + (c > 0 ? c - 1 : 0)
                                                : (int64_t)((rs + a.R - 3 + c) % a.R) * a.n + e;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.frames + pl * PLANE + off);
    r.x[c] = make_uint4(src[0], src[1], src[2], src[3]);
  }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// a1 of sample s straight into its padded LDS rows by LDS-DMA (no registers):
// image chunk i = (ic, y, 16-byte column xq of 6; xq = 5 is row padding and
// re-reads column 4)
constexpr int A1_PIECES = C1_OC * 20 * (A1R / 4) / 64;   // 30 pieces of 1 KB
__device__ inline void dma_a1(const ConvBwdArgs& a, int s, uint8_t* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* g1 = a.a1 + (int64_t)s * A1;
#pragma unroll
  for (int ii = 0; ii < (A1_PIECES + NT / 64 - 1) / (NT / 64); ++ii) {
    const int it = ii * (NT / 64) + wave;
    if (it < A1_PIECES) {   // wave-uniform
      const int i = it * 64 + lane;
      const int ic = i / 120, rem = i - ic * 120, y = rem / 6, xq = rem - y * 6;
      __builtin_amdgcn_global_load_lds(g1 + ic * C1_P + y * 20 + 4 * min(xq, 4),
                                       (lds_ptr_t)(lds + L_A1 + it * 1024), 16, 0, 0);
    }
  }
}

// da2 of a sample: the split grid of (2) (border cells written as 0), the [oc][p] split planes of (1),
// and the thread's running conv2 bias sums b2a (its item's 8 channels)
__device__ inline void commit_a(const PrefetchA& r, uint8_t* lds, float (&b2a)[8]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < PG; ++j) {
    const int i = tid + NT * j;
    if (i < GI) {
      int grp, cell, p;
      bool v;
      grid_item(i, grp, cell, v, p);
      float d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = v ? r.d[j][k] : 0.f;
      uint32_t h[4], m[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) split3_pack(d[2 * k], d[2 * k + 1], h[k], m[k], l[k]);
      uint8_t* dd = lds + L_D2 + d2_slot(cell, grp);
      *reinterpret_cast<uint4*>(dd) = make_uint4(h[0], h[1], h[2], h[3]);
      *reinterpret_cast<uint4*>(dd + D2P) = make_uint4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<uint4*>(dd + 2 * D2P) = make_uint4(l[0], l[1], l[2], l[3]);
      if (v) {
        uint8_t* da = lds + L_DA + (8 * grp) * DA_ROW + 2 * p;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int sh = 16 * (k & 1);
          *reinterpret_cast<uint16_t*>(da + k * DA_ROW) = (uint16_t)(h[k >> 1] >> sh);
          *reinterpret_cast<uint16_t*>(da + k * DA_ROW + DAP) = (uint16_t)(m[k >> 1] >> sh);
          *reinterpret_cast<uint16_t*>(da + k * DA_ROW + 2 * DAP) = (uint16_t)(l[k >> 1] >> sh);
          b2a[k] = __fadd_rn(b2a[k], d[k]);
        }
      }
    }
  }
}

// screens -> phase rows: the 4 dwords (X = 4q..4q+3, bytes b = 0..3) are
// transposed so each phase b gets one dword of 4 consecutive X; planes older
// than the last reset (c < 4 - nvalid) read as 0
__device__ inline void commit_x(const PrefetchX& r, uint8_t* lds) {
  const int tid = threadIdx.x;
  const int nv = __shfl(r.nv, 0);
  if (tid >= 504) return;
  const int y = tid / 6, q = tid - 6 * (tid / 6);
#pragma unroll
  for (int c = 0; c < PX; ++c) {
    uint4 v = r.x[c];
    if (q == 5) v = make_uint4(v.w, 0, 0, 0);
    if (c < 4 - nv) v = make_uint4(0, 0, 0, 0);
    const uint32_t lo01 = __builtin_amdgcn_perm(v.y, v.x, 0x05010400u);
    const uint32_t hi01 = __builtin_amdgcn_perm(v.y, v.x, 0x07030602u);
    const uint32_t lo23 = __builtin_amdgcn_perm(v.w, v.z, 0x05010400u);
    const uint32_t hi23 = __builtin_amdgcn_perm(v.w, v.z, 0x07030602u);
    uint8_t* d = lds + L_XPH + (c * 84 + y) * 4 * XR + 4 * q;
    *reinterpret_cast<uint32_t*>(d) = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    *reinterpret_cast<uint32_t*>(d + XR) = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    *reinterpret_cast<uint32_t*>(d + 2 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    *reinterpret_cast<uint32_t*>(d + 3 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
  }
}

// Workgroup barrier for LDS traffic only: this wave's LDS operations are
// complete, then s_barrier.  Unlike __syncthreads() it does not wait for the
// wave's outstanding global loads / LDS-DMA (the fence before s_barrier would
// drain vmcnt), so the prefetches stay in flight across phases; a phase that
// reads DMA'd LDS waits for it explicitly (s_waitcnt vmcnt).
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ inline bf16x8 frag_from_pairs(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(bf16x8, (u32x4{p0, p1, p2, p3}));
}

__device__ inline void slab_store(float* p, float v) { *p = v; }

__global__ void __launch_bounds__(NT)
conv_bwd_kernel(ConvBwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[L_END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  const float* a1s = reinterpret_cast<const float*>(lds + L_A1);
  // zero once: the da1 pad columns X 20..23 ((2) writes only X < 20) and the da2 [oc][p] planes (commit_a
  // writes only p < 81; (1) reads positions up to 95 as zeros)
  for (int i = tid; i < 3 * 16 * 20; i += NT) {
    const int pl = i / 320, r = i - pl * 320;
    *reinterpret_cast<uint2*>(lds + L_D1 + pl * D1P + (r / 20) * D1_OC + (r % 20) * D1_ROW + 40) = make_uint2(0, 0);
  }
  for (int i = tid; i < 3 * DAP / 16; i += NT) reinterpret_cast<uint4*>(lds + L_DA)[i] = make_uint4(0, 0, 0, 0);

  // (2) W2 fragments of this wave's parity class: lane (ic = col, g), k-step
  // ks = (dy, dx), k = oc = 8 g + j -> W2[oc][ic][py + 2 dy][px + 2 dx]
  const int cls = wave & 3, py = cls >> 1, px = cls & 1;
  bf16x8 w2h[4], w2m[4], w2l[4];
  {
    const float* w2src = a.W2 + (8 * g * 16 + col) * 16 + py * 4 + px;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = w2src[j * 256 + (ks >> 1) * 8 + 2 * (ks & 1)];
      uint32_t h[4], m[4], l[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) split3_pack(v[2 * j], v[2 * j + 1], h[j], m[j], l[j]);
      w2h[ks] = frag_from_pairs(h[0], h[1], h[2], h[3]);
      w2m[ks] = frag_from_pairs(m[0], m[1], m[2], m[3]);
      w2l[ks] = frag_from_pairs(l[0], l[1], l[2], l[3]);
    }
  }

  f32x4 acc1[2][2], big3[2], sml3[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc1[0][i] = acc1[1][i] = big3[i] = sml3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float b1s[4] = {0.f, 0.f, 0.f, 0.f};   // b1s[rr]: channel 4 g + rr
  float b2a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // conv2 bias sums of this thread's da2 item

  // (3): wave w -> screen ic = w >> 1, ky = 4 kyq + (col >> 2) with kyq = w & 1,
  // kx = 4 a + (col & 3) (tile a = 0, 1); A row base of lane (phase row b = col & 3)
  const int xrow3 = L_XPH + (((wave >> 1) * 84 + 4 * (wave & 1) + (col >> 2)) * 4 + (col & 3)) * XR;

  const int G = a.G;
  PrefetchA pa;
  PrefetchX px_;
  const int64_t step0 = a.ctl[CTL_STEP];
  prefetch_a(a, blockIdx.x, pa);
  prefetch_x(a, step0, blockIdx.x, px_);
  dma_a1(a, blockIdx.x, lds);
  for (int s = blockIdx.x; s < a.S; s += G) {
    lds_barrier();                 // B0: the previous sample is done with every region
    commit_a(pa, lds, b2a);
    commit_x(px_, lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this sample's a1 DMA has landed
    lds_barrier();                 // B1
    {
      const int sn = min(s + G, a.S - 1);   // unconditional: the registers are redefined here
      prefetch_a(a, sn, pa);                // in flight during (1)-(3)
      prefetch_x(a, step0, sn, px_);
    }
    // ---- (1) conv2 weight gradient; wave w: n-tiles (ic) 2w, 2w+1 x both m-tiles.  k-step ks, lane
    // (col, g): positions p = 32 ks + 8 g + j, j = 0..7.  A: da2 planes row oc = 16 mt + col, one b128 a
    // plane; B: a1[ic][2 oy + ky][2 ox + kx] of the lane's column (ky, kx) = divmod(col, 4) at those
    // positions, 8 f32 LDS reads (offset 48 oy + 2 ox: the 8 positions wrap a row at most once; past
    // position 80 they read finite bytes beyond the row block, times A's zeros), split in registers.
    {
      const float* b0 = a1s + (2 * wave) * A1C + (col >> 2) * A1R + (col & 3);
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int p0 = 32 * ks + 8 * g, oy0 = p0 / 9, ox0 = p0 - 9 * oy0;
        const int off0 = 48 * oy0 + 2 * ox0, wrap = 9 - ox0;   // j >= wrap: the next output row
        bf16x8 av[2][3];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int h = 0; h < 3; ++h)
            av[mt][h] = lds_load<bf16x8>(lds, L_DA + (16 * mt + col) * DA_ROW + h * DAP + 2 * p0);
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) {
          float x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = b0[jn * A1C + off0 + 2 * j + (j >= wrap ? 30 : 0)];
          bf16x8 bh, bm, bl;
          split3_x8(x, bh, bm, bl);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            acc1[mt][jn] = mfma_x6_acc(av[mt][0], av[mt][1], av[mt][2], bh, bm, bl, acc1[mt][jn]);
        }
      }
    }
    // a1 > 0 per pixel as 16 channel bits
    if (tid < C1_P) {
      const float* ap = a1s + (tid / 20) * A1R + tid % 20;
      uint32_t m = 0;
#pragma unroll
      for (int ic = 0; ic < C1_OC; ++ic) m |= (ap[ic * A1C] > 0.f ? 1u : 0u) << ic;
      reinterpret_cast<uint16_t*>(lds + L_MASK)[tid] = (uint16_t)m;
    }
    lds_barrier();                 // B2: a1 and the mask are consumed
    dma_a1(a, min(s + G, a.S - 1), lds);   // next sample's a1, in flight during (2)-(3)
    // ---- (2) da1 = convT(da2, W2) * (a1 > 0) -> da1 split planes.
    {
      // C^T form: rows = ic (A = the W2 fragments), columns = 16 grid cells
      // 12 + 16 mt + col (B = the da2 split grid); cells in the border column or
      // past the grid are computed and dropped.  Lane (col, g) ends up with
      // channels ic = 4 g + rr of one position.  Waves w < 4: tiles 0-3, w >= 4: 4-6.
      const int mt0 = wave < 4 ? 0 : 4, mt1 = wave < 4 ? 4 : 7;
#pragma unroll 1
      for (int mt = mt0; mt < mt1; ++mt) {
        const int cell = 12 + 16 * mt + col;
        // the position, its a1 > 0 mask and the da1 address first (clamped for dropped
        // cells): the mask read is in flight with the B operand reads
        const int cy = cell / 11, cx = cell - cy * 11;
        const bool keep = cell < 121 && cx != 0;
        const int oy = keep ? 2 * (cy - 1) + py : 0, ox = keep ? 2 * (cx - 1) + px : 0;
        const uint32_t m = reinterpret_cast<const uint16_t*>(lds + L_MASK)[oy * 20 + ox];
        f32x4 big = {0.f, 0.f, 0.f, 0.f}, sml = big;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int dcell = (ks >> 1) * 11 + (ks & 1);
          const int o = L_D2 + d2_slot(cell < 121 ? cell - dcell : 0, g);
          const bf16x8 bh = lds_load<bf16x8>(lds, o), bm = lds_load<bf16x8>(lds, o + D2P),
                       bl = lds_load<bf16x8>(lds, o + 2 * D2P);
          mfma_x6(w2h[ks], w2m[ks], w2l[ks], bh, bm, bl, big, sml);
        }
        if (keep) {
          uint8_t* d = lds + L_D1 + (4 * g) * D1_OC + oy * D1_ROW + ox * 2;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float v = __fadd_rn(big[rr], sml[rr]);
            if (!((m >> (4 * g + rr)) & 1)) v = 0.f;
            b1s[rr] = __fadd_rn(b1s[rr], v);
            uint32_t h, mm, l;
            split3(v, h, mm, l);
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC) = (uint16_t)h;
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC + D1P) = (uint16_t)mm;
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC + 2 * D1P) = (uint16_t)l;
          }
        }
      }
    }
    lds_barrier();                 // B3
    // ---- (3) conv1 weight gradient: k-step ks, quarter g -> group Gk = 4 ks + g
    // = (oy, X0 = 8 c): 8 positions (oy, X0..X0+7).  Tile a = rows (ky, kx =
    // 4 a + (col & 3)): the a = 0 and a = 1 fragments of a lane are pixels
    // X0..X0+7 and X0+1..X0+8 of one phase row, converted once and packed twice.
#pragma unroll 3
    for (int ks = 0; ks < 15; ++ks) {
      const int Gk = 4 * ks + g, oy = Gk / 3, c = Gk - 3 * oy;
      const int ob = L_D1 + col * D1_OC + oy * D1_ROW + 16 * c;
      const bf16x8 bh = lds_load<bf16x8>(lds, ob), bm = lds_load<bf16x8>(lds, ob + D1P),
                   bl = lds_load<bf16x8>(lds, ob + 2 * D1P);
      const int oa = xrow3 + oy * 16 * XR + 8 * c;
      const uint2 lo = lds_load<uint2>(lds, oa);
      const uint32_t nx = lds_load<uint32_t>(lds, oa + 8);
      uint32_t f[9];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f[k] = __float_as_uint((float)((lo.x >> (8 * k)) & 0xffu));
        f[4 + k] = __float_as_uint((float)((lo.y >> (8 * k)) & 0xffu));
      }
      f[8] = __float_as_uint((float)(nx & 0xffu));
#pragma unroll
      for (int a_ = 0; a_ < 2; ++a_) {
        const bf16x8 xa = frag_from_pairs(__builtin_amdgcn_perm(f[a_ + 1], f[a_], 0x07060302u),
                                          __builtin_amdgcn_perm(f[a_ + 3], f[a_ + 2], 0x07060302u),
                                          __builtin_amdgcn_perm(f[a_ + 5], f[a_ + 4], 0x07060302u),
                                          __builtin_amdgcn_perm(f[a_ + 7], f[a_ + 6], 0x07060302u));
        mfma_x3(xa, bh, bm, bl, big3[a_], sml3[a_]);
      }
    }
  }
  // ---- partial slab of this workgroup
  float* out = a.slab + (int64_t)blockIdx.x * SLAB;
  // dW2: C map col = kk within n-tile 2w + j, rows g*4+r -> oc = 16 mt + g*4 + r
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab_store(out + (16 * mt + g * 4 + r) * 256 + 16 * (2 * wave + j) + col, acc1[mt][j][r]);
  // dW1^T: tile a, C row g*4 + r -> ky = 4 (w & 1) + (row >> 2), kx = 4 a + (row & 3)
#pragma unroll
  for (int a_ = 0; a_ < 2; ++a_) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = g * 4 + r;
      const int ky = 4 * (wave & 1) + (row >> 2), kx = 4 * a_ + (row & 3);
      slab_store(out + SLAB_W1 + ((wave >> 1) * 64 + ky * 8 + kx) * 16 + col, __fadd_rn(big3[a_][r], sml3[a_][r]));
    }
  }
  float* red = reinterpret_cast<float*>(lds + L_RED);
  __syncthreads();
  // conv2 bias: item thread i (oc group i / 121) holds 8 channel sums; channel oc adds its group's
  // 121 cells in order
  if (tid < GI)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[tid * 8 + k] = b2a[k];
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int c = 0; c < 121; ++c) t = __fadd_rn(t, red[((tid >> 3) * 121 + c) * 8 + (tid & 7)]);
    out[SLAB_B2 + tid] = t;
  }
  __syncthreads();
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) red[(4 * g + rr) * 128 + wave * 16 + col] = b1s[rr];
  __syncthreads();
  if (tid < 16) {
    float t = 0.f;
    for (int c = 0; c < 128; ++c) t = __fadd_rn(t, red[tid * 128 + c]);
    out[SLAB_B1 + tid] = t;
  }
}

// ---------------------------------------------------------------------------
// The default form, conv_bwd_ws_kernel: 1,024 threads, 4 waves a SIMD, wave-specialised.  Waves 0-7 ("X")
// run (2) and (3), waves 8-15 ("Y") run (1) and every commit, so each SIMD's four waves issue two different
// steps at once.  Two barriers a sample s_k:
//   P_k  X: (2) of s_k (D2 -> D1), the a1 > 0 test read straight from A1 (no mask pass)
//        Y: (1) of s_k (DA, A1); screens of s_k -> XPH; loads da2 of s_{k+1} and the screens of s_{k+1}
//   Q_k  X: (3) of s_k (D1, XPH)
//        Y: a1 of s_{k+1} -> A1 by LDS-DMA (nobody reads A1 in Q), da2 of s_{k+1} -> D2 and DA; waits for
//           the DMA before the barrier
// W2 is staged once through LDS by coalesced loads (the fragment-order global loads touched one 64-byte
// segment a lane: 64 L2 requests an instruction, ~20k cycles of prologue).  Every accumulator sees the
// same products in the same order as conv_bwd_kernel (per-wave tiles unchanged), so the slabs are
// bit-identical to it (ARL_CB_WS=0 runs conv_bwd_kernel: the bitwise test arm).
namespace {
constexpr int NT2 = 1024;
constexpr int A1W = 2 * A1C * 4;                 // bytes of one Y wave's two a1 channels (3,840)
constexpr int A1W_PIECES = A1W / 16;             // 240 16-byte DMA pieces
constexpr int LW_D1 = 0;                         // da1 split planes                     47,616
constexpr int LW_XPH = LW_D1 + 3 * D1P;          // screens by column phase               32,256
constexpr int LW_D2 = LW_XPH + 4 * 84 * 4 * XR;  // da2 split grid                        24,576
constexpr int LW_A1 = LW_D2 + 3 * D2P;           // a1 f32 [16][20][A1R] + 4 zero rows     31,104
constexpr int LW_DA = LW_A1 + C1_OC * A1C * 4 + 4 * A1R * 4;   // da2 [oc][p] split planes 19,968
constexpr int LW_END = LW_DA + 3 * DAP;          // 155,520
static_assert(LW_END <= 160 * 1024, "LDS");
static_assert(LW_A1 % 16 == 0 && LW_DA % 16 == 0 && LW_XPH % 16 == 0 && LW_D2 % 16 == 0, "alignment");
static_assert(GI <= NT2 / 2, "one da2 item per Y thread");
// W2 staging in the da1 region before the first sample: (oc, ic, tap) at oc * W2S_OC + ic * W2S_IC + tap;
// the fragment reads (lanes: ic = col, oc = 8 g + j) hit 32 distinct banks (W2S_IC = 17, 8 W2S_OC = 16 mod 32)
constexpr int W2S_IC = 17, W2S_OC = 16 * W2S_IC + 2;   // 274 floats
static_assert(32 * W2S_OC * 4 <= 3 * D1P, "W2 staging fits the da1 region");
}  // namespace

__device__ inline int opaque(int x) {   // a value the compiler cannot hoist work on out of the sample loop
  asm volatile("" : "+v"(x));
  return x;
}

// Y wave wy: its two a1 channels of sample s by LDS-DMA (piece i = (channel, row, 16-byte column))
__device__ inline void dma_a1_wave(const ConvBwdArgs& a, int s, uint8_t* lds, int wy, int lane_) {
  const int lane = opaque(lane_);
  const float* g1 = a.a1 + (int64_t)s * A1 + (2 * wy) * C1_P;
  uint8_t* dst = lds + LW_A1 + wy * A1W;
#pragma unroll
  for (int ii = 0; ii < (A1W_PIECES + 63) / 64; ++ii) {
    const int i = ii * 64 + lane;
    if (i < A1W_PIECES) {   // the last instruction: 48 lanes
      const int c = i / 120, rem = i - c * 120, y = rem / 6, xq = rem - y * 6;
      __builtin_amdgcn_global_load_lds(g1 + c * C1_P + y * 20 + 4 * min(xq, 4), (lds_ptr_t)(dst + ii * 1024), 16, 0,
                                       0);
    }
  }
}

// da2 of sample s for grid item ty: 8 channels of one position
__device__ inline void load_da2(const ConvBwdArgs& a, int s, int ty, float (&d)[8]) {
  int grp, cell, p;
  bool v;
  grid_item(opaque(ty), grp, cell, v, p);
  const float* src = a.da2 + (int64_t)s * A2 + (v ? 8 * grp * C2_P + p : 0);
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = src[k * C2_P];
}

// D2 and DA of one sample (commit_a with the Y thread index): one grid item, one split
__device__ inline void commit_d2_da(const float (&r)[8], uint8_t* lds, int ty, float (&b2a)[8]) {
  int grp, cell, p;
  bool v;
  const int i = opaque(ty);
  grid_item(i, grp, cell, v, p);
  if (i >= GI) return;
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) split3_pack(v ? r[2 * k] : 0.f, v ? r[2 * k + 1] : 0.f, h[k], m[k], l[k]);
  uint8_t* dd = lds + LW_D2 + d2_slot(cell, grp);
  *reinterpret_cast<uint4*>(dd) = make_uint4(h[0], h[1], h[2], h[3]);
  *reinterpret_cast<uint4*>(dd + D2P) = make_uint4(m[0], m[1], m[2], m[3]);
  *reinterpret_cast<uint4*>(dd + 2 * D2P) = make_uint4(l[0], l[1], l[2], l[3]);
  if (!v) return;
  uint8_t* da = lds + LW_DA + (8 * grp) * DA_ROW + 2 * p;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int sh = 16 * (k & 1);
    *reinterpret_cast<uint16_t*>(da + k * DA_ROW) = (uint16_t)(h[k >> 1] >> sh);
    *reinterpret_cast<uint16_t*>(da + k * DA_ROW + DAP) = (uint16_t)(m[k >> 1] >> sh);
    *reinterpret_cast<uint16_t*>(da + k * DA_ROW + 2 * DAP) = (uint16_t)(l[k >> 1] >> sh);
    b2a[k] = __fadd_rn(b2a[k], r[k]);
  }
}

// prefetch_x with the Y thread index ty (0..511); r0 = the window's first step modulo the ring length
__device__ inline void prefetch_x_ws(const ConvBwdArgs& a, int r0, int s, int ty_, PrefetchX& r) {
  const int ty = opaque(ty_);
  const int t = s / a.n, e = s - t * a.n;
  const int rs = (r0 + t) % a.R;
  r.nv = a.nvalid[(int64_t)rs * a.n + min(e + (ty & 63), a.n - 1)];
  const int it = ty < 504 ? ty : 0;
  const int y = it / 6, q = it - 6 * (it / 6);
  const int off = y * 84 + (q < 5 ? 16 * q : 68);
#pragma unroll
  for (int c = 0; c < PX; ++c) {
    const int64_t pl = a.layout == FRAMES_STACK ? ((int64_t)rs * a.n + e) * 4 + c
                       : a.layout == FRAMES_RGB ? ((int64_t)rs * a.n + e) * 3 + (c > 0 ? c - 1 : 0)
                                                : (int64_t)((rs + a.R - 3 + c) % a.R) * a.n + e;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.frames + pl * PLANE + off);
    r.x[c] = make_uint4(src[0], src[1], src[2], src[3]);
  }
}

// screens -> phase rows (commit_x with the Y thread index ty)
__device__ inline void commit_x_ws(const PrefetchX& r, uint8_t* lds, int ty_) {
  const int ty = opaque(ty_);
  const int nv = __shfl(r.nv, 0);
  if (ty >= 504) return;
  const int y = ty / 6, q = ty - 6 * (ty / 6);
#pragma unroll
  for (int c = 0; c < PX; ++c) {
    uint4 v = r.x[c];
    if (q == 5) v = make_uint4(v.w, 0, 0, 0);
    if (c < 4 - nv) v = make_uint4(0, 0, 0, 0);
    const uint32_t lo01 = __builtin_amdgcn_perm(v.y, v.x, 0x05010400u);
    const uint32_t hi01 = __builtin_amdgcn_perm(v.y, v.x, 0x07030602u);
    const uint32_t lo23 = __builtin_amdgcn_perm(v.w, v.z, 0x05010400u);
    const uint32_t hi23 = __builtin_amdgcn_perm(v.w, v.z, 0x07030602u);
    uint8_t* d = lds + LW_XPH + (c * 84 + y) * 4 * XR + 4 * q;
    *reinterpret_cast<uint32_t*>(d) = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    *reinterpret_cast<uint32_t*>(d + XR) = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    *reinterpret_cast<uint32_t*>(d + 2 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    *reinterpret_cast<uint32_t*>(d + 3 * XR) = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
  }
}

// (1) of one sample on Y wave wy (conv_bwd_kernel's step (1) with wave -> wy).  Positions past 80 read up to
// 4 rows past the wave's second channel (the next channel's rows, or the zero rows after channel 15) times A's
// zeros.
__device__ inline void step1_wave(const uint8_t* lds, int wy, int lane_, f32x4 (&acc1)[2][2]) {
  const int lane = opaque(lane_), g = lane >> 4, col = lane & 15;
  const float* b0 = reinterpret_cast<const float*>(lds + LW_A1) + (2 * wy) * A1C + (col >> 2) * A1R + (col & 3);
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int p0 = 32 * ks + 8 * g, oy0 = p0 / 9, ox0 = p0 - 9 * oy0;
    const int off0 = 48 * oy0 + 2 * ox0, wrap = 9 - ox0;
    bf16x8 av[2][3];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int h = 0; h < 3; ++h)
        av[mt][h] = lds_load<bf16x8>(lds, LW_DA + (16 * mt + col) * DA_ROW + h * DAP + 2 * p0);
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = b0[jn * A1C + off0 + 2 * j + (j >= wrap ? 30 : 0)];
      bf16x8 bh, bm, bl;
      split3_x8(x, bh, bm, bl);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        acc1[mt][jn] = mfma_x6_acc(av[mt][0], av[mt][1], av[mt][2], bh, bm, bl, acc1[mt][jn]);
    }
  }
}

// phase stamps (diagnostic builds only: make variant DEFS=-DARL_CB_WS_STAMP, scripts/cb_ws_stamps.py):
// workgroups 0-7, wave 0 (X) and wave 8 (Y), shader clock at the start / end of each phase's work, sample
// k < 15; k = 15 the prologue
#ifdef ARL_CB_WS_STAMP
__device__ uint64_t g_cb_stamps[8][2][16][6];
#define CB_STAMP(role, k, j)                                                               \
  do {                                                                                     \
    if (b < 8 && lane == 0 && (wave & 7) == 0 && (k) < 16)                                 \
      g_cb_stamps[b][role][k][j] = __builtin_amdgcn_s_memtime();                           \
  } while (0)
extern "C" int arl_debug_cb_stamps(uint64_t* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cb_stamps), sizeof(g_cb_stamps));
}
#else
#define CB_STAMP(role, k, j) \
  do {                       \
  } while (0)
#endif

__global__ void __launch_bounds__(NT2)
conv_bwd_ws_kernel(ConvBwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LW_END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: SGPR values
  const int g = lane >> 4, col = lane & 15;
  const int b = blockIdx.x, G = a.G;
  const int n = (a.S - 1 - b) / G + 1;   // samples b, b + G, ... of this workgroup
  auto smp = [&](int k) { return b + min(k, n - 1) * G; };
  // zero once: the da2 [oc][p] planes (positions past 80 stay 0) and the 4 rows after a1 channel 15; the
  // da1 pad columns X 20..23 after the W2 staging (below)
  for (int i = tid; i < 3 * DAP / 16; i += NT2) reinterpret_cast<uint4*>(lds + LW_DA)[i] = make_uint4(0, 0, 0, 0);
  if (tid < 4 * A1R / 4)
    reinterpret_cast<uint4*>(lds + LW_A1 + C1_OC * A1C * 4)[tid] = make_uint4(0, 0, 0, 0);
  float* out = a.slab + (int64_t)b * SLAB;
  float* red = reinterpret_cast<float*>(lds + L_RED);   // after the last sample: b2a [GI][8], then b1s
  float* red1 = red + GI * 8;

  if (wave < 8) {
    // ================================================================ X: (2) and (3)
    const int wx = wave;
    const int cls = wx & 3, py = cls >> 1, px = cls & 1;
    float* w2s = reinterpret_cast<float*>(lds + LW_D1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // W2 (32 x 16 x 16 f32): 4 float4 a thread, coalesced
      const int f = tid + 512 * j, oc = f >> 6, ic = (f >> 2) & 15, t4 = (f & 3) * 4;
      const float4 w = reinterpret_cast<const float4*>(a.W2)[f];
      float* d = w2s + oc * W2S_OC + ic * W2S_IC + t4;
      d[0] = w.x;
      d[1] = w.y;
      d[2] = w.z;
      d[3] = w.w;
    }
    lds_barrier();   // #0: W2 staged
    // (2) W2 fragments of this wave's parity class: lane (ic = col, g), k-step ks = (dy, dx), k = oc = 8 g + j
    bf16x8 w2h[4], w2m[4], w2l[4];
    {
      const float* w2f = w2s + (8 * g) * W2S_OC + col * W2S_IC + py * 4 + px;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = w2f[j * W2S_OC + (ks >> 1) * 8 + 2 * (ks & 1)];
        uint32_t h[4], m[4], l[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) split3_pack(v[2 * j], v[2 * j + 1], h[j], m[j], l[j]);
        w2h[ks] = frag_from_pairs(h[0], h[1], h[2], h[3]);
        w2m[ks] = frag_from_pairs(m[0], m[1], m[2], m[3]);
        w2l[ks] = frag_from_pairs(l[0], l[1], l[2], l[3]);
      }
    }
    f32x4 big3[2], sml3[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) big3[i] = sml3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float b1s[4] = {0.f, 0.f, 0.f, 0.f};
    const int xrow3 = LW_XPH + (((wx >> 1) * 84 + 4 * (wx & 1) + (col >> 2)) * 4 + (col & 3)) * XR;
    const int mt0 = wx < 4 ? 0 : 4, mt1 = wx < 4 ? 4 : 7;
    lds_barrier();   // #0b: every X wave holds its W2 fragments: the da1 pads are zeroed over the staging
    for (int i = tid; i < 3 * 16 * 20; i += NT2 / 2) {
      const int pl = i / 320, r = i - pl * 320;
      *reinterpret_cast<uint2*>(lds + LW_D1 + pl * D1P + (r / 20) * D1_OC + (r % 20) * D1_ROW + 40) = make_uint2(0, 0);
    }
    CB_STAMP(0, 15, 0);
    lds_barrier();   // #1: zeroed pads, D2 / DA / A1 of s_0
    CB_STAMP(0, 15, 1);
    for (int k = 0; k < n; ++k) {
      // ---- P_k: (2) of s_k
      CB_STAMP(0, k, 0);
      const float* a1m = reinterpret_cast<const float*>(lds + LW_A1) + (4 * g) * A1C;
#pragma unroll 1
      for (int mt = mt0; mt < mt1; ++mt) {
        const int cell = 12 + 16 * mt + col;
        const int cy = cell / 11, cx = cell - cy * 11;
        const bool keep = cell < 121 && cx != 0;
        const int oy = keep ? 2 * (cy - 1) + py : 0, ox = keep ? 2 * (cx - 1) + px : 0;
        const float* ap = a1m + oy * A1R + ox;   // a1 of channels 4 g + rr: the > 0 test of (2)
        const float m0 = ap[0], m1 = ap[A1C], m2 = ap[2 * A1C], m3 = ap[3 * A1C];
        const uint32_t m = (m0 > 0.f ? 1u : 0u) | (m1 > 0.f ? 2u : 0u) | (m2 > 0.f ? 4u : 0u) | (m3 > 0.f ? 8u : 0u);
        f32x4 big = {0.f, 0.f, 0.f, 0.f}, sml = big;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int dcell = (ks >> 1) * 11 + (ks & 1);
          const int o = LW_D2 + d2_slot(cell < 121 ? cell - dcell : 0, g);
          const bf16x8 bh = lds_load<bf16x8>(lds, o), bm = lds_load<bf16x8>(lds, o + D2P),
                       bl = lds_load<bf16x8>(lds, o + 2 * D2P);
          mfma_x6(w2h[ks], w2m[ks], w2l[ks], bh, bm, bl, big, sml);
        }
        if (keep) {
          uint8_t* d = lds + LW_D1 + (4 * g) * D1_OC + oy * D1_ROW + ox * 2;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float v = __fadd_rn(big[rr], sml[rr]);
            if (!((m >> rr) & 1)) v = 0.f;
            b1s[rr] = __fadd_rn(b1s[rr], v);
            uint32_t h, mm, l;
            split3(v, h, mm, l);
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC) = (uint16_t)h;
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC + D1P) = (uint16_t)mm;
            *reinterpret_cast<uint16_t*>(d + rr * D1_OC + 2 * D1P) = (uint16_t)l;
          }
        }
      }
      CB_STAMP(0, k, 1);
      lds_barrier();
      // ---- Q_k: (3) of s_k
      CB_STAMP(0, k, 2);
#pragma unroll 3
      for (int ks = 0; ks < 15; ++ks) {
        const int Gk = 4 * ks + g, oy = Gk / 3, c = Gk - 3 * oy;
        const int ob = LW_D1 + col * D1_OC + oy * D1_ROW + 16 * c;
        const bf16x8 bh = lds_load<bf16x8>(lds, ob), bm = lds_load<bf16x8>(lds, ob + D1P),
                     bl = lds_load<bf16x8>(lds, ob + 2 * D1P);
        const int oa = xrow3 + oy * 16 * XR + 8 * c;
        const uint2 lo = lds_load<uint2>(lds, oa);
        const uint32_t nx = lds_load<uint32_t>(lds, oa + 8);
        uint32_t f[9];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f[q] = __float_as_uint((float)((lo.x >> (8 * q)) & 0xffu));
          f[4 + q] = __float_as_uint((float)((lo.y >> (8 * q)) & 0xffu));
        }
        f[8] = __float_as_uint((float)(nx & 0xffu));
#pragma unroll
        for (int a_ = 0; a_ < 2; ++a_) {
          const bf16x8 xa = frag_from_pairs(__builtin_amdgcn_perm(f[a_ + 1], f[a_], 0x07060302u),
                                            __builtin_amdgcn_perm(f[a_ + 3], f[a_ + 2], 0x07060302u),
                                            __builtin_amdgcn_perm(f[a_ + 5], f[a_ + 4], 0x07060302u),
                                            __builtin_amdgcn_perm(f[a_ + 7], f[a_ + 6], 0x07060302u));
          mfma_x3(xa, bh, bm, bl, big3[a_], sml3[a_]);
        }
      }
      CB_STAMP(0, k, 3);
      lds_barrier();
    }
#pragma unroll
    for (int a_ = 0; a_ < 2; ++a_) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = g * 4 + r;
        const int ky = 4 * (wx & 1) + (row >> 2), kx = 4 * a_ + (row & 3);
        slab_store(out + SLAB_W1 + ((wx >> 1) * 64 + ky * 8 + kx) * 16 + col, __fadd_rn(big3[a_][r], sml3[a_][r]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red1[(4 * g + rr) * 128 + wx * 16 + col] = b1s[rr];
  } else {
    // ================================================================ Y: (1), the commits, the a1 DMA
    const int ty = tid - NT2 / 2, wy = wave - 8;
    f32x4 acc1[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc1[0][i] = acc1[1][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float b2a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float pa[8];
    PrefetchX pxr;
    CB_STAMP(1, 15, 0);
    dma_a1_wave(a, smp(0), lds, wy, lane);
    load_da2(a, smp(0), ty, pa);
    const int r0 = (int)(a.ctl[CTL_STEP] % a.R);   // after the loads that do not need it
    prefetch_x_ws(a, r0, smp(0), ty, pxr);
    CB_STAMP(1, 15, 1);
    lds_barrier();   // #0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CB_STAMP(1, 15, 2);
    commit_d2_da(pa, lds, ty, b2a);
    CB_STAMP(1, 15, 3);
    lds_barrier();   // #0b
    lds_barrier();   // #1
    for (int k = 0; k < n; ++k) {
      // ---- P_k
      CB_STAMP(1, k, 0);
      load_da2(a, smp(k + 1), ty, pa);   // for Q_k
      commit_x_ws(pxr, lds, ty);
      step1_wave(lds, wy, lane, acc1);
      prefetch_x_ws(a, r0, smp(k + 1), ty, pxr);   // after (1): its registers are not live across it
      CB_STAMP(1, k, 1);
      lds_barrier();
      // ---- Q_k
      CB_STAMP(1, k, 2);
      if (k + 1 < n) {
        dma_a1_wave(a, smp(k + 1), lds, wy, lane);
        commit_d2_da(pa, lds, ty, b2a);
        CB_STAMP(1, k, 5);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // a1 of s_{k+1} has landed
      }
      CB_STAMP(1, k, 3);
      lds_barrier();
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          slab_store(out + (16 * mt + g * 4 + r) * 256 + 16 * (2 * wy + j) + col, acc1[mt][j][r]);
    __syncthreads();
    if (ty < GI)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[ty * 8 + k] = b2a[k];
  }
  __syncthreads();
  if (tid < 32) {   // conv2 bias: channel oc adds its group's 121 cells in order
    float t = 0.f;
    for (int c = 0; c < 121; ++c) t = __fadd_rn(t, red[((tid >> 3) * 121 + c) * 8 + (tid & 7)]);
    out[SLAB_B2 + tid] = t;
  } else if (tid >= 64 && tid < 80) {   // conv1 bias
    const int o = tid - 64;
    float t = 0.f;
    for (int c = 0; c < 128; ++c) t = __fadd_rn(t, red1[o * 128 + c]);
    out[SLAB_B1 + o] = t;
  }
}

// f64 sum of the G slabs in a fixed order: thread (o, zg) adds slabs zg,
// zg + 16, ... of output o (a wave reads 64 consecutive outputs of one slab,
// 256 contiguous bytes), then the 16 partials add in zg order
// With a NormFold (the clip norm folded into this launch, NormFold.parts !=
// null): every conv block also leaves the f64 sum of squares of the 64
// gradient values it wrote in parts[block], and rest_blocks extra blocks sum
// the squares of g[rest_begin, rest_end) -- the gradient the FC / heads / LSTM
// backward has already finished -- into parts[nconv + b]; every block of the
// update kernel then sums the partials, instead of a separate grad_sqnorm launch.
constexpr int RED_O = 64, RED_Z = 16;
constexpr int RED_BLOCKS = (SLAB + RED_O - 1) / RED_O;   // 193
__device__ inline double block_sum_f64_1024(double x, double* sh) {   // 1,024 threads, fixed order
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = x;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < RED_O * RED_Z / 64; ++i) t += sh[i];
  return t;
}
__global__ void __launch_bounds__(RED_O * RED_Z)
reduce_conv_bwd_kernel(const float* __restrict__ slab, int G, float* __restrict__ gW2, float* __restrict__ gb2,
                       float* __restrict__ gW1, float* __restrict__ gb1, int rgb, NormFold nf) {
  __shared__ double part[RED_Z][RED_O];
  __shared__ double shn[RED_O * RED_Z / 64];
  if (blockIdx.x >= RED_BLOCKS) {   // squared-norm blocks over the rest of the gradient
    const int b = blockIdx.x - RED_BLOCKS;
    double t = 0.0;
    const float4* g4 = reinterpret_cast<const float4*>(nf.g + nf.rest_begin);
    const int64_t n4 = (nf.rest_end - nf.rest_begin) >> 2;
    for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < n4; i += (int64_t)nf.rest_blocks * blockDim.x) {
      const float4 v = g4[i];
      t += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    if (b == 0 && (int64_t)threadIdx.x < ((nf.rest_end - nf.rest_begin) & 3)) {
      const float v = nf.g[nf.rest_begin + (n4 << 2) + threadIdx.x];
      t += (double)v * v;
    }
    t = block_sum_f64_1024(t, shn);
    if (threadIdx.x == 0) nf.parts[RED_BLOCKS + b] = t;
    return;
  }
  const int ol = threadIdx.x & (RED_O - 1), zg = threadIdx.x / RED_O;
  const int o = blockIdx.x * RED_O + ol;
  double t = 0.0;
  if (o < SLAB) {
    int z = zg;
    for (; z + 7 * RED_Z < G; z += 8 * RED_Z) {   // eight loads in flight
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(z + u * RED_Z) * SLAB + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) t += (double)v[u];
    }
    for (; z < G; z += RED_Z) t += (double)slab[(int64_t)z * SLAB + o];
  }
  part[zg][ol] = t;
  __syncthreads();
  double sq = 0.0;
  if (zg == 0 && o < SLAB) {
    double v = 0.0;
    for (int g = 0; g < RED_Z; ++g) v += part[g][ol];
    const float gv = conv_slab_put(o, v, gW2, gb2, gW1, gb1, rgb);
    sq = (double)gv * gv;
  }
  if (nf.parts != nullptr) {   // (block-uniform)
    sq = block_sum_f64_1024(sq, shn);
    if (threadIdx.x == 0) nf.parts[blockIdx.x] = sq;
  }
}

int conv_norm_parts(int rest_blocks) { return RED_BLOCKS + rest_blocks; }
static_assert(RED_BLOCKS + 64 <= NORM_MAX_PARTS, "the folded norm's partials fit the scratch");

// workgroups (= slab slices): one per CU on the 256-CU part, at most one per sample
int conv_bwd_blocks(int S) { return S < 256 ? S : 256; }
int64_t conv_bwd_slab_floats(int S) { return (int64_t)conv_bwd_blocks(S) * SLAB; }

hipError_t launch_conv_bwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int S,
                           const float* a1, const float* da2, const float* W2, float* slab, float* gW2, float* gb2,
                           float* gW1, float* gb1, hipStream_t s, bool reduce, int layout, const NormFold& nf) {
  if (S <= 0) return hipSuccess;
  const int G = conv_bwd_blocks(S);
  ConvBwdArgs a{frames, nvalid, ctl, n, R, a1, da2, W2, S, G, slab, layout};
  static const char* ws = getenv("ARL_CB_WS");   // "0": the 512-thread kernel (the bitwise test arm)
  if (ws != nullptr && ws[0] == '0')
    hipLaunchKernelGGL(conv_bwd_kernel, dim3(G), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL(conv_bwd_ws_kernel, dim3(G), dim3(NT2), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !reduce) return e;
  return launch_conv_reduce(slab, S, gW2, gb2, gW1, gb1, s, layout, nf);
}

hipError_t launch_conv_reduce(const float* slab, int S, float* gW2, float* gb2, float* gW1, float* gb1, hipStream_t s,
                              int layout, const NormFold& nf) {
  if (S <= 0) return hipSuccess;
  const int extra = nf.parts != nullptr ? nf.rest_blocks : 0;
  hipLaunchKernelGGL(reduce_conv_bwd_kernel, dim3(RED_BLOCKS + extra), dim3(RED_O * RED_Z), 0, s, slab,
                     conv_bwd_blocks(S), gW2, gb2, gW1, gb1, layout == FRAMES_RGB ? 1 : 0, nf);
  return hipGetLastError();
}

}  // namespace arl
