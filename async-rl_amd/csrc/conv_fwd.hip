// Fused forward of the NIPS head's two conv layers (dqn_head.py:41-42,48-52)
// for one env per workgroup, straight from the uint8 frame ring -- optionally
// with the observation itself fused in front (PHI: phi of the env's new frame
// pair, ale.py:59-89, written to the ring slot and used as conv input plane 3
// from LDS; the ring bookkeeping of phi_ring_kernel):
//   a1 = relu(conv(x/255, W1, s4) + b1)   (16 x 20 x 20)  -> LDS + HBM (kept for backward)
//   a2 = relu(conv(a1, W2, s2) + b2)      (32 x 9 x 9)    -> HBM
// Both contractions run on the bf16 matrix cores with exact bf16 splits of
// the f32 operands (bf16split.hpp): conv1 multiplies the integer pixel values
// (exact in bf16; 1/255 is applied to the sum) by W1 = h + m + l, 3 MFMAs per
// k-step; conv2 multiplies a1 = h + m + l by W2 = h + m + l, 6 MFMAs.
//
// LDS (145.5 KB, one 512-thread workgroup per CU = 2 waves per SIMD):
//   xb   4 screens as bf16 [ic][y][x]                         56,448 B
//   R1   W1 split planes [3][oc][k] (rows padded to 528 B),   25,344 B
//        then (after every wave is done with W1) the a1 split planes
//        [3][pixel][ic] with an XOR swizzle of the 16-byte slots  38,400 B
//   W2p  W2 split planes [3][oc][tap][ic] (rows 528 B)         50,688 B
//        (PHI: first the gray tap rows of the new screen [84][2][160] and the
//        resize coefficient tables, 27,720 B)
//
// PHI schedule: the bookkeeping loads, the three older ring planes and the
// weights are issued first, then the 168 x 2 source rows of the pair (161 KB,
// 24 x 16 B per thread, all in flight).  conv1's k-steps over input planes
// 0..2 (6 of 8) run on the matrix cores while the pair lands; then max +
// luminance -> gray rows, the resize -> plane 3 (ring slot + LDS), conv1's
// last two k-steps.  Each tile's k order is the unfused kernel's (bit-identical).
//
// conv1: M = 400 positions (25 tiles), N = 16 oc, K = 256 ordered (ic, ky, kx):
//   k-step s, lane quarter g -> (ic, ky) = divmod(4 s + g, 8), kx = 0..7, i.e.
//   8 contiguous bf16 pixels per lane; W1 fragments live in 96 VGPRs.
// conv2: M = 81 positions (6 tiles), N = 32 oc (2 tiles), K = 256 ordered
//   (tap = ky*4 + kx, ic): k-step s, quarter g -> tap 2 s + (g >> 1), ic
//   8 (g & 1) + 0..7 = one 16-byte read of a channel-last a1 pixel.  Wave w
//   owns n-tile w & 1 (its W2 fragments in 96 VGPRs) and m-tiles w >> 1 and
//   (w >> 1) + 4: three jobs per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "bf16split.hpp"
#include "phi_ops.hpp"

#ifndef ARL_ABLATE
#define ARL_ABLATE 0   // timing experiments only (bits: 1 conv1 MFMA, 2 conv2 MFMA, 4 staging loads
                       // (ring path), 16 epilogue /255 as a multiply; PHI: 32 pair loads, 64 max +
                       // luminance, 128 resize)
#endif

// conv1 / conv2 k-steps software-pipelined: a k-step's LDS operands are read while the previous
// k-step's MFMAs run (double-buffered registers) instead of read-then-wait inside each k-step.
// A/B knob, off: 18.6 -> 19.6 us at 512 envs, 35 -> 38 us at 1,024 (95 -> 127 VGPRs; the other
// waves of the CU already cover the LDS latency), C2 equal (profiles/r03/r3r)
#ifndef ARL_CF_PREFETCH
#define ARL_CF_PREFETCH 0
#endif

// static wave priority (A/B knob): the second-dispatched half of the workgroup's waves at s_setprio 1
// (MI355X_MICROARCH.md "Two waves per SIMD" item 4)
#ifndef ARL_CF_PRIO
#define ARL_CF_PRIO 0
#endif
// a1 global stores non-temporal (ARL_CF_NTST=2): nothing reads a1 before the window's backward, and the
// stores leave no dirty lines in the L2s for the kernel's end to write back.  a2 keeps ordinary stores: the
// next launch (fc_fwd) reads it.  0: both ordinary; 1: both non-temporal (C4 median 0.4994-0.4998 ->
// 0.4947-0.4948 ms, r4r; fc_fwd 9.5 -> 10.5 us); 2 vs 1: C4 0.4854-0.4855 -> 0.4772-0.4774 ms, C3
// 1.1142-1.1148 -> 1.1075-1.1095, C2 0.3119-0.3123 -> 0.3059-0.3064 (2 interleaved reps each, r4u)
#ifndef ARL_CF_NTST
#define ARL_CF_NTST 2
#endif
#ifndef ARL_CF_STAMP
#define ARL_CF_STAMP 0   // timing experiments only: s_memtime at phase ends into a2 (results wrong)
#endif

namespace arl {

namespace {
constexpr int NT = 512;                  // threads per workgroup (8 waves)
constexpr int XB_ROW = 84 * 2;           // bytes per bf16 screen row
constexpr int XB_PLANE = PLANE * 2;      // 14,112 bytes per bf16 screen
// bytes per oc row of a weight plane: 512 + 32, so the 16 rows a ds_read_b128 lane group reads (8 of one
// 16-byte k half, 8 of the other) land on 16 distinct bank quads (528 = 512 + 16 left a 2-way conflict)
constexpr int WROW = 544;
constexpr int W1P = 16 * WROW;           // 8,704 per W1 plane
constexpr int W2P = 32 * WROW;           // 17,408 per W2 plane
// a1 planes: 16-byte slots (8 ic bf16) of pixel (y, x), ic half h, in phase-split order -- slot
// h * A1_HALF + ((y & 1) * 2 + (x & 1)) * A1_PS + a1_pos(y >> 1, x >> 1), see a1_off
constexpr int A1_PS = 108, A1_HALF = 4 * A1_PS;
constexpr int A1P = 2 * A1_HALF * 16;    // 13,824 per a1 plane (400 pixels x 16 ic bf16 + pad)
constexpr int L_XB = 0;
constexpr int L_R1 = L_XB + 4 * XB_PLANE;   // 56,448
constexpr int L_W2 = L_R1 + 3 * A1P;        // 97,920
constexpr int L_END = L_W2 + 3 * W2P;       // 150,144
static_assert(3 * W1P <= 3 * A1P, "W1 planes fit the a1 region");
// PHI: gray tap rows + coefficient tables in the W2 region (W2 is split into it after the resize)
constexpr int G_ROWS = 2 * DST;                       // 168 (output row, tap) source rows
constexpr int L_GRAY = L_W2;                          // [84][2][160] uint8
constexpr int L_XOFS = L_GRAY + G_ROWS * SRC_W;       // int16 xofs[84], xa0[84], xa1[84], yb0[84], yb1[84]
static_assert(L_XOFS + 5 * DST * 2 <= L_END, "gray rows + tables fit the W2 region");
constexpr int PHI_TASKS = G_ROWS * 10;                // (row, 16-pixel chunk): 1680
constexpr int PHI_J = (PHI_TASKS + NT - 1) / NT;      // 4

// LDS layout by envs per workgroup (EPW).  EPW = 1 is the layout above.  EPW = 2
// (1,024 threads; waves 0-7 take env 0, waves 8-15 env 1, both share the weight
// planes): conv1 phase  [screens e0 | screens e1 | W1 planes]       139,008 B;
//          conv2 phase  [a1 planes e0 | a1 planes e1 | W2 planes]  135,168 B
// (W2 is split into the dead screen / W1 bytes after conv1's barrier).
template <int EPW>
struct Lay {
  static constexpr int XB(int el) { return el * 4 * XB_PLANE; }
  static constexpr int W1 = EPW * 4 * XB_PLANE;                      // 56,448 / 112,896
  static constexpr int A1(int el) { return EPW == 1 ? W1 : el * 3 * A1P; }
  static constexpr int W2 = EPW == 1 ? L_W2 : 2 * 3 * A1P;           // 97,920 / 82,944
  static constexpr int END = EPW == 1 ? L_END : W1 + 3 * W1P;        // 150,144 / 139,008
  // a2 > 0 mask words (81 u32 per env) in bytes dead during conv2: the screens (EPW 1), past the W2
  // planes (EPW 2)
  static constexpr int MSK(int el) { return EPW == 1 ? 0 : W2 + 3 * W2P + el * 336; }
};
static_assert(Lay<2>::MSK(1) + 336 <= Lay<2>::END && 336 <= Lay<1>::W1, "mask words");
static_assert(Lay<2>::W2 + 3 * W2P <= Lay<2>::END && Lay<2>::END <= 160 * 1024, "EPW 2 layout");
static_assert(Lay<1>::A1(0) == L_R1 && Lay<1>::END == L_END, "EPW 1 layout");
}  // namespace

// a1 plane byte offset of pixel (y, x), ic half h.  conv2's lanes read, for one tap (ky, kx), the pixels
// (2 oy + ky, 2 ox + kx) of 16 consecutive output positions r = 9 oy + ox; in the tap's phase plane
// (y & 1, x & 1) that is (Y, X) = (oy + ky / 2, ox + kx / 2), so a slot index congruent to 9 Y + X mod 16
// puts those 16 reads on 16 distinct bank quads (16 consecutive r, shifted by 9 (ky / 2) + kx / 2), and
// A1_HALF = 0 mod 16 keeps that across the lane group's two ic halves.  a1_pos: 9 Y + X for X < 9
// (0..89); the 10 pixels of column X = 9 in the free slots >= 90 of the same residue.
__device__ inline int a1_pos(int Y, int X) { return X < 9 ? 9 * Y + X : 90 + ((9 * Y + 15) & 15); }
__device__ inline int a1_off(int y, int x, int h) {
  return (h * A1_HALF + ((y & 1) * 2 + (x & 1)) * A1_PS + a1_pos(y >> 1, x >> 1)) << 4;
}

struct ConvFwdArgs {
  const uint8_t* frames;
  const uint8_t* nvalid;
  const int64_t* ctl;
  int n, R, t;          // obs step = ctl[STEP] + t; env = blockIdx.x
  const float* W1;      // (16, 4, 8, 8); RGB nets (16, 3, 8, 8) for input planes 1..3
  const float* b1;
  const float* W2;      // (32, 16, 4, 4)
  const float* b2;
  float* a1;            // (n, 16, 400), or null: not stored (the window's bootstrap slot T)
  float* a2;            // (n, 32, 81)
  int layout;           // FrameLayout: FRAMES_RGB = (R, n, 3, 84, 84), planes [0, R, G, B] of slot ks % R;
                        // FRAMES_STACK = (R, n, 4, 84, 84), the 4 planes of slot ks % R
  int e0;               // first env of this launch (env = e0 + EPW * blockIdx.x + env slot)
  RingArgs ring;        // PHI: the observation (pair pool, bookkeeping); frames / nvalid / ctl / n / R / t as above
  int e1;               // one past the last env of this launch (EPW = 2: an odd count leaves a slot idle)
  uint32_t* a2m;        // (n, 81) bits of a2 > 0 for the FC backward's ReLU mask (fc_bwd.hip job B), or null
};

// W1 (16, 4, 8, 8) f32 -> the split planes [3][oc][k] in LDS: thread tid
// stages 8 consecutive k of one oc (RGB nets: W1 (16, 3, 8, 8) on input
// planes 1..3, zeros for plane 0)
// (unconditional loads from a clamped address: a load under a per-lane branch
// is waited for at the branch's end; the RGB zero pad is applied at the split)
__device__ inline void w1_load(const float* W1, bool rgb, int tid, float4& w1a, float4& w1b) {
  const int w1oc = tid >> 5, w1k = (8 * tid) & 255;
  const float4* w1p =
      reinterpret_cast<const float4*>(rgb ? W1 + w1oc * 192 + (w1k >= 64 ? w1k - 64 : 0) : W1 + 8 * tid);
  w1a = w1p[0];
  w1b = w1p[1];
}
__device__ inline void w1_split_store(uint8_t* lds, int tid, float4 w1a, float4 w1b, bool rgb = false, int base = L_R1) {
  const int w1oc = tid >> 5, w1k = (8 * tid) & 255;
  if (rgb && w1k < 64) w1a = w1b = make_float4(0.f, 0.f, 0.f, 0.f);
  uint4 ph, pm, pl;
  split3_pack(w1a.x, w1a.y, ph.x, pm.x, pl.x);
  split3_pack(w1a.z, w1a.w, ph.y, pm.y, pl.y);
  split3_pack(w1b.x, w1b.y, ph.z, pm.z, pl.z);
  split3_pack(w1b.z, w1b.w, ph.w, pm.w, pl.w);
  uint8_t* d = lds + base + w1oc * WROW + w1k * 2;
  *reinterpret_cast<uint4*>(d) = ph;
  *reinterpret_cast<uint4*>(d + W1P) = pm;
  *reinterpret_cast<uint4*>(d + 2 * W1P) = pl;
}

// W2 slice of thread tid (oc, 4 ic, 4 taps) -> the split planes in LDS
__device__ inline void w2_load(const float* W2, int tid, float4 (&w2v)[4]) {
  const int w2oc = tid >> 4, ic4 = (tid >> 2) & 3, tg = tid & 3;
#pragma unroll
  for (int ii = 0; ii < 4; ++ii) w2v[ii] = reinterpret_cast<const float4*>(W2)[(w2oc * 16 + 4 * ic4 + ii) * 4 + tg];
}
__device__ inline void w2_split_store(uint8_t* lds, int tid, const float4 (&w2v)[4], int base = L_W2) {
  const int w2oc = tid >> 4, ic4 = (tid >> 2) & 3, tg = tid & 3;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    const float v0 = w2v[0][tt], v1 = w2v[1][tt], v2 = w2v[2][tt], v3 = w2v[3][tt];
    uint2 ph, pm, pl;
    split3_pack(v0, v1, ph.x, pm.x, pl.x);
    split3_pack(v2, v3, ph.y, pm.y, pl.y);
    uint8_t* d = lds + base + w2oc * WROW + ((4 * tg + tt) * 16 + 4 * ic4) * 2;
    *reinterpret_cast<uint2*>(d) = ph;
    *reinterpret_cast<uint2*>(d + W2P) = pm;
    *reinterpret_cast<uint2*>(d + 2 * W2P) = pl;
  }
}

// 16 uint8 pixels -> 16 bf16 in LDS (exact)
__device__ inline void px16_store(uint8_t* d, uint4 x) {
  uint4 lo, hi;
  lo.x = px_pair_bf16(x.x, 0); lo.y = px_pair_bf16(x.x, 1);
  lo.z = px_pair_bf16(x.y, 0); lo.w = px_pair_bf16(x.y, 1);
  hi.x = px_pair_bf16(x.z, 0); hi.y = px_pair_bf16(x.z, 1);
  hi.z = px_pair_bf16(x.w, 0); hi.w = px_pair_bf16(x.w, 1);
  reinterpret_cast<uint4*>(d)[0] = lo;
  reinterpret_cast<uint4*>(d)[1] = hi;
}

template <bool PHI, int EPW>
__global__ void __launch_bounds__(NT * EPW)
conv_fwd_kernel(ConvFwdArgs a) {
  static_assert(!PHI || EPW == 1, "the fused observation runs one env per workgroup");
  using LY = Lay<EPW>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LY::END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
  if (ARL_CF_PRIO && wave >= NT * EPW / 128) __builtin_amdgcn_s_setprio(1);
  // EPW = 2: waves 0-7 (threads 0-511) env slot 0, waves 8-15 slot 1; w8 / t8 index within the slot
  const int el = EPW == 1 ? 0 : wave >> 3;
  const int w8 = wave & 7, t8 = tid & (NT - 1);
  const int ev = a.e0 + EPW * blockIdx.x + el;
  const bool valid = EPW == 1 || ev < a.e1;   // an idle slot (odd env count) computes env e1 - 1, stores nothing
  const int e = valid ? ev : a.e1 - 1;
  const bool rgb = a.layout == FRAMES_RGB;
  constexpr int V = PLANE / 16;              // 441 uint4 per screen
  // the biases first: loads issued at the top land before the staging waits
  // (loaded at the epilogues they were waited for there)
#if ARL_CF_STAMP
  uint32_t stamp[8];
  int nst = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#define CF_STAMP() do { if (nst < 8) stamp[nst++] = (uint32_t)(__builtin_amdgcn_s_memtime() - t0); } while (0)
#else
#define CF_STAMP() do {} while (0)
#endif
  // conv1 runs transposed (mfma_x3_t): lane (g, col) holds oc 4g..4g+3 of position tile * 16 + col
  const float bias1[4] = {a.b1[4 * g], a.b1[4 * g + 1], a.b1[4 * g + 2], a.b1[4 * g + 3]};
  // conv2 runs transposed too (mfma_x6_t): lane (g, col) holds oc 16 nt + 4 g + r of position 16 m + col
  const float bias2[4] = {a.b2[16 * (w8 & 1) + 4 * g], a.b2[16 * (w8 & 1) + 4 * g + 1], a.b2[16 * (w8 & 1) + 4 * g + 2],
                          a.b2[16 * (w8 & 1) + 4 * g + 3]};
  const int64_t ks = a.ctl[CTL_STEP] + a.t;
  const int rs = (int)(ks % a.R);
  // conv1 tiles w, w + 8, w + 16 (and 24 on wave 0): 25 tiles over 8 waves in one
  // pass, 3-4 independent accumulator chains per wave (per-tile k order s = 0..7)
  constexpr int TJ = 4;
  // wt: the wave's conv1 tile set.  Slot 1 rotates it by one wave so its 4-tile wave (wt = 0) sits on another
  // SIMD than slot 0's (a workgroup's waves go to SIMDs in a fixed cyclic order): 13 + 13 + 12 + 12 tiles
  // over the 4 SIMDs instead of 14 + 12 + 12 + 12 (the same tiles and k order: bit-identical)
  const int wt = EPW == 2 ? (w8 + 8 - el) & 7 : w8;
  const bool has3 = wt + 24 < 25;   // wave-uniform
  int baseX[TJ], a1o[TJ];   // screen row base of the tile's position; its a1 slot (the epilogue's store)
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int tl = (j < 3 || has3) ? wt + 8 * j : wt;
    const int p = tl * 16 + col, oy = p / 20, ox = p - oy * 20;
    baseX[j] = LY::XB(el) + (4 * oy) * XB_ROW + 8 * ox;
    a1o[j] = LY::A1(el) + a1_off(oy, ox, g >> 1) + (g & 1) * 8;
  }
  f32x4 big[TJ], sml[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) big[j] = sml[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // k-step s of every tile; W1 fragments of lane (oc = col, g): k = 8 (4 s + g) + 0..7
  auto conv1_step = [&](int s, bf16x8 wh, bf16x8 wm, bf16x8 wl) {
    const int u = 4 * s + g, off = (u >> 3) * XB_PLANE + (u & 7) * XB_ROW;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const bf16x8 xa = lds_load8_a8(lds, baseX[j] + off);
      mfma_x3_t(xa, wh, wm, wl, big[j], sml[j]);
    }
    if (has3) {
      const bf16x8 xa = lds_load8_a8(lds, baseX[3] + off);
      mfma_x3_t(xa, wh, wm, wl, big[3], sml[3]);
    }
  };
  auto w1_frag = [&](int s, bf16x8& wh, bf16x8& wm, bf16x8& wl) {
    const int off = LY::W1 + col * WROW + (4 * s + g) * 16;
    wh = lds_load<bf16x8>(lds, off);
    wm = lds_load<bf16x8>(lds, off + W1P);
    wl = lds_load<bf16x8>(lds, off + 2 * W1P);
  };
  if constexpr (PHI) {
    const RingArgs& o = a.ring;
    const int64_t pidx = ks % o.pool_len;
    const uint8_t* pr = o.pair_pool + (pidx * a.n + e) * (int64_t)PAIR;
    // ---- issue: bookkeeping, older ring planes, weights, then the pair's tap rows
    const RingObs ob = ring_obs_load(o, e, ks);
    constexpr int NX = (3 * V + NT - 1) / NT;   // 3
    uint4 xv[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      const int c = i / V, oo = i - c * V;
      // loaded whatever nvalid says (planes older than the last reset are zeroed below); slots past
      // the third plane reload its last 16 bytes, so every thread issues the same number of loads
      const int cc = i < 3 * V ? c : 2, oc = i < 3 * V ? oo : V - 1;
      xv[j] = reinterpret_cast<const uint4*>(a.frames + ((int64_t)((rs + a.R - 3 + cc) % a.R) * a.n + e) * PLANE)[oc];
    }
    float4 w1a, w1b, w2v[4];
    w1_load(a.W1, false, tid, w1a, w1b);
    w2_load(a.W2, tid, w2v);
    // every wave's small loads reach the memory pipeline before any wave's pair loads (the CU
    // serves them in issue order): the staging below then waits only for these
    __builtin_amdgcn_s_barrier();
    uint4 px[PHI_J][6];
#pragma unroll
    for (int j = 0; j < PHI_J; ++j) {   // unconditional (tasks past the end reload task 0) so the load
      const int i0 = tid + NT * j;        // counter stays exact for the partial waits below
      const int i = i0 < PHI_TASKS ? i0 : 0;
      const int r = i / 10, c = i - 10 * r, dy = r >> 1, tap = r & 1;
      int so, b0, b1;
      if (o.mode & 2) resize_coeff(dy + CROP_TOP, SRC_H, CROP_H, so, b0, b1);
      else resize_coeff(dy, SRC_H, DST, so, b0, b1);
      const int sy = so + tap > SRC_H - 1 ? SRC_H - 1 : so + tap;
      const uint4* pc = reinterpret_cast<const uint4*>(pr + (size_t)sy * SRC_W * 3 + c * 48);
      const uint4* pp = reinterpret_cast<const uint4*>(pr + FRAME_BYTES + (size_t)sy * SRC_W * 3 + c * 48);
      if (ARL_ABLATE & 32) {
#pragma unroll
        for (int q = 0; q < 6; ++q) px[j][q] = make_uint4(i + q, sy, c, q);
      } else {
        px[j][0] = pc[0]; px[j][1] = pc[1]; px[j][2] = pc[2];
        px[j][3] = pp[0]; px[j][4] = pp[1]; px[j][5] = pp[2];
      }
    }
    // ---- while the pair lands: bookkeeping, coefficient tables, planes 0..2, W1 planes
    const int nv = ob.nv;
    if (tid == 0) ring_obs_store(o, e, ks, ob);
    int16_t* tab = reinterpret_cast<int16_t*>(lds + L_XOFS);
    if (tid < DST) {
      int so, a0, a1;
      resize_coeff(tid, SRC_W, DST, so, a0, a1);
      tab[tid] = (int16_t)so; tab[DST + tid] = (int16_t)a0; tab[2 * DST + tid] = (int16_t)a1;
    } else if (tid >= 128 && tid < 128 + DST) {
      const int dy = tid - 128;
      int so, b0, b1;
      if (o.mode & 2) resize_coeff(dy + CROP_TOP, SRC_H, CROP_H, so, b0, b1);
      else resize_coeff(dy, SRC_H, DST, so, b0, b1);
      tab[3 * DST + dy] = (int16_t)b0; tab[4 * DST + dy] = (int16_t)b1;
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + NT * j;
      if (i < 3 * V) {
        const int c = i / V, oo = i - c * V;
        px16_store(lds + L_XB + c * XB_PLANE + oo * 32, c >= 4 - nv ? xv[j] : make_uint4(0, 0, 0, 0));
      }
    }
    w1_split_store(lds, tid, w1a, w1b);
    __syncthreads();
    // ---- conv1 k-steps over input planes 0..2 on the matrix cores
#pragma unroll
    for (int s = 0; s < ((ARL_ABLATE & 1) ? 0 : 6); ++s) {
      bf16x8 wh, wm, wl;
      w1_frag(s, wh, wm, wl);
      conv1_step(s, wh, wm, wl);
    }
    // ---- max of the pair + luminance -> gray tap rows (row r = 2 dy + tap)
#pragma unroll
    for (int j = 0; j < PHI_J; ++j) {
      const int i = tid + NT * j;
      if (i < PHI_TASKS) {
        const int r = i / 10, c = i - 10 * r;
        *reinterpret_cast<uint4*>(lds + L_GRAY + r * SRC_W + c * 16) =
            (ARL_ABLATE & 64) ? make_uint4(px[j][0].x ^ px[j][3].x, px[j][1].y ^ px[j][4].y, px[j][2].z ^ px[j][5].z,
                                           px[j][0].w ^ px[j][5].w)
                              : max_luminance16(px[j][0], px[j][1], px[j][2], px[j][3], px[j][4], px[j][5]);
      }
    }
    __syncthreads();
    // ---- resize -> the ring slot (HBM, for later steps and the backward) and conv input plane 3 (LDS):
    // thread -> column quad q (its horizontal taps read once) x rows dy0 + 24 k
    uint8_t* dst = o.frames + ((int64_t)rs * a.n + e) * PLANE;
    constexpr int RS_ROWS = 24;                 // 21 quads x 24 row starts = 504 threads
    if (!(ARL_ABLATE & 128) && tid < (DST / 4) * RS_ROWS) {
      const int q = tid % (DST / 4), dy0 = tid / (DST / 4);
      int sx[4], sx1[4], ha0[4], ha1[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int dx = q * 4 + jj;
        sx[jj] = tab[dx];
        sx1[jj] = sx[jj] + 1 < SRC_W ? sx[jj] + 1 : SRC_W - 1;
        ha0[jj] = tab[DST + dx];
        ha1[jj] = tab[2 * DST + dx];
      }
#pragma unroll
      for (int k = 0; k < (DST + RS_ROWS - 1) / RS_ROWS; ++k) {
        const int dy = dy0 + RS_ROWS * k;
        if (dy < DST) {
          const int b0 = tab[3 * DST + dy], b1 = tab[4 * DST + dy];
          const uint8_t* g0 = lds + L_GRAY + (2 * dy) * SRC_W;
          const uint8_t* g1 = g0 + SRC_W;
          uint32_t packed = 0;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int r0 = (int)g0[sx[jj]] * ha0[jj] + (int)g0[sx1[jj]] * ha1[jj];
            const int r1 = (int)g1[sx[jj]] * ha0[jj] + (int)g1[sx1[jj]] * ha1[jj];
            packed |= (uint32_t)resize_vpass(r0, r1, b0, b1, o.mode) << (8 * jj);
          }
          *reinterpret_cast<uint32_t*>(dst + dy * DST + q * 4) = packed;
          *reinterpret_cast<uint2*>(lds + L_XB + 3 * XB_PLANE + (dy * DST + q * 4) * 2) =
              make_uint2(px_pair_bf16(packed, 0), px_pair_bf16(packed, 1));
        }
      }
    }
    __syncthreads();   // plane 3 complete, the gray rows dead
    w2_split_store(lds, tid, w2v);   // conv2 reads it after the barrier in front of conv2
    // ---- conv1's last k-steps (input plane 3)
#pragma unroll
    for (int s = 6; s < ((ARL_ABLATE & 1) ? 0 : 8); ++s) {
      bf16x8 wh, wm, wl;
      w1_frag(s, wh, wm, wl);
      conv1_step(s, wh, wm, wl);
    }
    __syncthreads();   // every wave is done with the W1 planes: the a1 planes overwrite them
  } else {
    // ---- stage: every global load in flight at once (nvalid, the weights, all
    // four ring planes whatever nvalid says), then bf16 conversion / splitting
    // into LDS; planes older than the last reset are zeroed here
    const int nv = a.nvalid[(int64_t)rs * a.n + e];
    // EPW = 2: slot 0 loads (and splits) W1 only, slot 1 W2 only (wave-uniform)
    float4 w1a, w1b, w2v[4];
    if (EPW == 1 || el == 0) w1_load(a.W1, rgb, t8, w1a, w1b);
    if (EPW == 1 || el == 1) w2_load(a.W2, t8, w2v);
    constexpr int NX = (4 * V + NT - 1) / NT;  // 4
    uint4 xv[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = t8 + NT * j;
      // past the fourth plane: reload its last 16 bytes (every thread issues NX loads)
      const int c = i < 4 * V ? i / V : 3, oo = i < 4 * V ? i - c * V : V - 1;
      // RGB: conv plane 0 is the zero pad (c - 1 < 0 reads plane 0 and is zeroed below, nvalid = 3)
      xv[j] = reinterpret_cast<const uint4*>(
          a.frames + (a.layout == FRAMES_STACK ? ((int64_t)rs * a.n + e) * 4 + c
                      : a.layout == FRAMES_RGB ? ((int64_t)rs * a.n + e) * 3 + (c > 0 ? c - 1 : 0)
                                               : (int64_t)((rs + a.R - 3 + c) % a.R) * a.n + e) * PLANE)[oo];
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = t8 + NT * j;
      if (i < 4 * V) {
        const int c = i / V, oo = i - c * V;
        px16_store(lds + LY::XB(el) + c * XB_PLANE + oo * 32,
                   (!(ARL_ABLATE & 4) && c >= 4 - nv) ? xv[j] : make_uint4(0, 0, 0, 0));
      }
    }
    if (el == 0) w1_split_store(lds, t8, w1a, w1b, rgb, LY::W1);
    if (EPW == 1) w2_split_store(lds, t8, w2v, LY::W2);   // EPW = 2: after conv1 (its bytes hold screens / W1)
    CF_STAMP();   // 0: staged
    __syncthreads();
    CF_STAMP();   // 1: barrier
    // conv1 with each k-step's W1 fragments read from LDS inside the loop (their
    // reads overlap the MFMAs instead of forming a phase of their own), then a
    // barrier: every wave is done with the W1 planes before the a1 planes overwrite them
#if ARL_CF_PREFETCH
    {
      // operands of k-step s in buffer s & 1; every lane loads a 4th tile fragment (the waves
      // without tile 24 re-read tile w's) so the loads are unconditional
      bf16x8 wh[2], wm[2], wl[2], xa[2][TJ];
      auto load = [&](int s, int b) {
        w1_frag(s, wh[b], wm[b], wl[b]);
        const int u = 4 * s + g, off = (u >> 3) * XB_PLANE + (u & 7) * XB_ROW;
#pragma unroll
        for (int j = 0; j < TJ; ++j) xa[b][j] = lds_load8_a8(lds, baseX[j] + off);
      };
      load(0, 0);
#pragma unroll
      for (int s = 0; s < ((ARL_ABLATE & 1) ? 0 : 8); ++s) {
        const int b = s & 1;
        if (s + 1 < 8) load(s + 1, b ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 3; ++j) mfma_x3_t(xa[b][j], wh[b], wm[b], wl[b], big[j], sml[j]);
        if (has3) mfma_x3_t(xa[b][3], wh[b], wm[b], wl[b], big[3], sml[3]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#else
#pragma unroll
    for (int s = 0; s < ((ARL_ABLATE & 1) ? 0 : 8); ++s) {
      bf16x8 wh, wm, wl;
      w1_frag(s, wh, wm, wl);
      conv1_step(s, wh, wm, wl);
    }
#endif
    CF_STAMP();   // 2: conv1 MFMAs issued
    __syncthreads();
    if (EPW == 2 && el == 1) w2_split_store(lds, t8, w2v, LY::W2);   // read by conv2 after the next barrier
  }
  float* a1g = a.a1 + (int64_t)e * A1;
  uint32_t* msk = reinterpret_cast<uint32_t*>(lds + LY::MSK(el));
  if (a.a2m != nullptr && t8 < A2W) msk[t8] = 0u;   // (its bytes are dead since conv1's barrier)
  {
    // C^T rows 4g + r = oc, column col -> position tile * 16 + col: the lane's 4 oc are 4 consecutive
    // ic of the a1 planes, one 8-byte LDS store per plane
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      if (j == 3 && !has3) break;
      const int p = (wt + 8 * j) * 16 + col;
      float ov[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ov[r] = (ARL_ABLATE & 16)
                    ? fmaxf(__fadd_rn(__fmul_rn(__fadd_rn(big[j][r], sml[j][r]), 1.f / 255.f), bias1[r]), 0.f)
                    : fmaxf(__fadd_rn(div255(__fadd_rn(big[j][r], sml[j][r])), bias1[r]), 0.f);
      if (valid && a.a1 != nullptr) {   // (null: the bootstrap slot, which no backward reads)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (ARL_CF_NTST) __builtin_nontemporal_store(ov[r], a1g + (4 * g + r) * C1_P + p);
          else a1g[(4 * g + r) * C1_P + p] = ov[r];
        }
      }
      uint2 ph, pm, pl;
      split3_pack(ov[0], ov[1], ph.x, pm.x, pl.x);
      split3_pack(ov[2], ov[3], ph.y, pm.y, pl.y);
      const int off = a1o[j];
      *reinterpret_cast<uint2*>(lds + off) = ph;
      *reinterpret_cast<uint2*>(lds + off + A1P) = pm;
      *reinterpret_cast<uint2*>(lds + off + 2 * A1P) = pl;
    }
  }
  CF_STAMP();   // 3: a1 epilogue
  __syncthreads();
  CF_STAMP();   // 4: barrier
  // ---- conv2: wave -> n-tile nt = w & 1 (oc = 16 nt + col), m-tiles w >> 1, (w >> 1) + 4
  {
    const int nt = w8 & 1, oc = 16 * nt + col;
    CF_STAMP();   // 5: (W2 fragments are read per k-step below)
    const int mA = w8 >> 1, mB = mA + 4;
    const bool hasB = mB < 6;
    const int posA = 16 * mA + col, posB = 16 * (hasB ? mB : mA) + col;   // A row of this lane
    // rows past the 81 positions compute (and drop) the position 16 before: 16 consecutive positions
    // whatever the tile, so the a1 reads stay on distinct banks
    const int pcA = posA < C2_P ? posA : posA - 16, pcB = posB < C2_P ? posB : posB - 16;
    const int oyA = pcA / 9, oxA = pcA - oyA * 9, oyB = pcB / 9, oxB = pcB - oyB * 9;
    // a1 offset of tap (ky, kx) = divmod(2 s + (g >> 1), 4) for this lane's position of tile A / B
    auto a1A = [&](int tap) { return LY::A1(el) + a1_off(2 * oyA + (tap >> 2), 2 * oxA + (tap & 3), g & 1); };
    auto a1B = [&](int tap) { return LY::A1(el) + a1_off(2 * oyB + (tap >> 2), 2 * oxB + (tap & 3), g & 1); };
    f32x4 bigA = {0.f, 0.f, 0.f, 0.f}, smlA = bigA, bigB = bigA, smlB = bigA;
#if ARL_CF_PREFETCH
    {
      // k-step s's W2 and a1 fragments in buffer s & 1 (tile B's re-read tile A's where absent)
      bf16x8 w2[2][3], aA[2][3], aB[2][3];
      auto load = [&](int s, int b) {
        const int off = LY::W2 + oc * WROW + (2 * s + (g >> 1)) * 32 + (g & 1) * 16;
        const int tap = 2 * s + (g >> 1);
        const int offA = a1A(tap), offB = a1B(tap);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          w2[b][k] = lds_load<bf16x8>(lds, off + k * W2P);
          aA[b][k] = lds_load<bf16x8>(lds, offA + k * A1P);
          aB[b][k] = lds_load<bf16x8>(lds, offB + k * A1P);
        }
      };
      load(0, 0);
#pragma unroll
      for (int s = 0; s < ((ARL_ABLATE & 2) ? 0 : 8); ++s) {
        const int b = s & 1;
        if (s + 1 < 8) load(s + 1, b ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_x6_t(aA[b][0], aA[b][1], aA[b][2], w2[b][0], w2[b][1], w2[b][2], bigA, smlA);
        if (hasB) mfma_x6_t(aB[b][0], aB[b][1], aB[b][2], w2[b][0], w2[b][1], w2[b][2], bigB, smlB);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#else
#pragma unroll
    for (int s = 0; s < ((ARL_ABLATE & 2) ? 0 : 8); ++s) {
      bf16x8 w2h[1], w2m[1], w2l[1];   // this k-step's W2 fragments, read inside the loop
      {
        const int off = LY::W2 + oc * WROW + (2 * s + (g >> 1)) * 32 + (g & 1) * 16;
        w2h[0] = lds_load<bf16x8>(lds, off);
        w2m[0] = lds_load<bf16x8>(lds, off + W2P);
        w2l[0] = lds_load<bf16x8>(lds, off + 2 * W2P);
      }
      const int tap = 2 * s + (g >> 1);
      const int offA = a1A(tap);
      const bf16x8 ahA = lds_load<bf16x8>(lds, offA), amA = lds_load<bf16x8>(lds, offA + A1P),
                   alA = lds_load<bf16x8>(lds, offA + 2 * A1P);
      mfma_x6_t(ahA, amA, alA, w2h[0], w2m[0], w2l[0], bigA, smlA);
      if (hasB) {
        const int offB = a1B(tap);
        const bf16x8 ahB = lds_load<bf16x8>(lds, offB), amB = lds_load<bf16x8>(lds, offB + A1P),
                     alB = lds_load<bf16x8>(lds, offB + 2 * A1P);
        mfma_x6_t(ahB, amB, alB, w2h[0], w2m[0], w2l[0], bigB, smlB);
      }
    }
#endif
    CF_STAMP();   // 6: conv2 MFMAs issued
    float* a2g = a.a2 + (int64_t)e * A2;
    // a2 > 0 -> bit k = oc * 81 + p of the env's mask words: for each r the 16 lanes of group g hold 16
    // consecutive positions of one oc, a 16-bit run of the wave's ballot, or'd into the LDS words by the
    // group's lane 0 (one or two ors, no two lanes of a wave on one word; stored after a barrier)
    const bool mk = a.a2m != nullptr;
    auto tile_out = [&](const f32x4& big, const f32x4& sml, int m) {
      const int p = 16 * m + col;
      const bool pin = p < C2_P;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 16 * nt + 4 * g + r;
        const float v = fmaxf(__fadd_rn(__fadd_rn(big[r], sml[r]), bias2[r]), 0.f);
        if (valid && pin) {
          if (ARL_CF_NTST == 1) __builtin_nontemporal_store(v, a2g + o * C2_P + p);
          else a2g[o * C2_P + p] = v;
        }
        if (mk) {   // (block-uniform)
          const unsigned long long bal = __ballot(pin && v > 0.f);
          const unsigned run = (unsigned)(bal >> (16 * g)) & 0xffffu;
          if (col == 0 && run != 0u) {
            const int k = o * C2_P + 16 * m, sh = k & 31;
            __hip_atomic_fetch_or(msk + (k >> 5), run << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (sh > 16)
              __hip_atomic_fetch_or(msk + (k >> 5) + 1, run >> (32 - sh), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    };
    tile_out(bigA, smlA, mA);
    if (hasB) tile_out(bigB, smlB, mB);
    if (mk) {   // (block-uniform)
      __syncthreads();
      if (valid && t8 < A2W) a.a2m[(int64_t)e * (A2W) + t8] = msk[t8];
    }
#if ARL_CF_STAMP
    CF_STAMP();   // 7: end
    if (lane == 0) {   // wave w's stamps -> a2[e][w * 8 ..]; wave 0 also the start time
      uint32_t* o = reinterpret_cast<uint32_t*>(a2g) + w8 * 10;
      for (int k = 0; k < 8; ++k) o[k] = stamp[k];
      o[8] = (uint32_t)t0;
      o[9] = (uint32_t)(t0 >> 32);
    }
#endif
  }
}

hipError_t launch_conv_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t,
                           const float* W1, const float* b1, const float* W2, const float* b2, float* a1, float* a2,
                           hipStream_t s, int layout, int e0, int ne, uint32_t* a2m) {
  if (n <= 0) return hipSuccess;
  if (ne < 0) ne = n;
  if (ne <= 0) return hipSuccess;
  ConvFwdArgs a{frames, nvalid, ctl, n, R, t, W1, b1, W2, b2, a1, a2, layout, e0, RingArgs{}, e0 + ne, a2m};
  // two envs a workgroup (16 waves sharing the weight planes) in nets of >= 512 envs, whether the
  // launch covers all of them or one env group's range (C4 0.513 -> 0.503 ms, C3 1.227 -> 1.212 ms at
  // two groups, profiles/r03/r3k); ARL_CONV_EPW=1 / 2 forces one form (A/B timing)
  static const char* epw = getenv("ARL_CONV_EPW");
  const int k = (epw && (epw[0] == '1' || epw[0] == '2')) ? epw[0] - '0' : (n >= 512 ? 2 : 1);
  if (k == 2) hipLaunchKernelGGL((conv_fwd_kernel<false, 2>), dim3((ne + 1) / 2), dim3(2 * NT), 0, s, a);
  else hipLaunchKernelGGL((conv_fwd_kernel<false, 1>), dim3(ne), dim3(NT), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_phi_conv_fwd(const RingArgs& ring, const float* W1, const float* b1, const float* W2,
                               const float* b2, float* a1, float* a2, hipStream_t s, uint32_t* a2m) {
  const int ne = ring.ne < 0 ? ring.n : ring.ne;
  if (ne <= 0) return hipSuccess;
  ConvFwdArgs a{ring.frames, ring.nvalid, ring.ctl, ring.n, ring.R, ring.t, W1, b1, W2, b2, a1, a2, FRAMES_RING,
                ring.e0, ring, ring.e0 + ne, a2m};
  hipLaunchKernelGGL((conv_fwd_kernel<true, 1>), dim3(ne), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace arl
