// Fused forward of the NIPS head's two conv layers (dqn_head.py:41-42,48-52)
// for one env per workgroup, straight from the uint8 frame ring:
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

template <int EPW>
__global__ void __launch_bounds__(NT * EPW)
conv_fwd_kernel(ConvFwdArgs a) {
  using LY = Lay<EPW>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LY::END];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, col = lane & 15;
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
                 c >= 4 - nv ? xv[j] : make_uint4(0, 0, 0, 0));
    }
  }
  if (el == 0) w1_split_store(lds, t8, w1a, w1b, rgb, LY::W1);
  if (EPW == 1) w2_split_store(lds, t8, w2v, LY::W2);   // EPW = 2: after conv1 (its bytes hold screens / W1)
  __syncthreads();
  // conv1 with each k-step's W1 fragments read from LDS inside the loop (their
  // reads overlap the MFMAs instead of forming a phase of their own), then a
  // barrier: every wave is done with the W1 planes before the a1 planes overwrite them
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    bf16x8 wh, wm, wl;
    w1_frag(s, wh, wm, wl);
    conv1_step(s, wh, wm, wl);
  }
  __syncthreads();
  if (EPW == 2 && el == 1) w2_split_store(lds, t8, w2v, LY::W2);   // read by conv2 after the next barrier
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
        ov[r] = fmaxf(__fadd_rn(div255(__fadd_rn(big[j][r], sml[j][r])), bias1[r]), 0.f);
      if (valid && a.a1 != nullptr) {   // (null: the bootstrap slot, which no backward reads)
#pragma unroll
        for (int r = 0; r < 4; ++r) __builtin_nontemporal_store(ov[r], a1g + (4 * g + r) * C1_P + p);
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
  __syncthreads();
  // ---- conv2: wave -> n-tile nt = w & 1 (oc = 16 nt + col), m-tiles w >> 1, (w >> 1) + 4
  {
    const int nt = w8 & 1, oc = 16 * nt + col;
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
#pragma unroll
    for (int s = 0; s < 8; ++s) {
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
        if (valid && pin) a2g[o * C2_P + p] = v;   // ordinary store: fc_fwd reads it next
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
  }
}

hipError_t launch_conv_fwd(const uint8_t* frames, const uint8_t* nvalid, const int64_t* ctl, int n, int R, int t,
                           const float* W1, const float* b1, const float* W2, const float* b2, float* a1, float* a2,
                           hipStream_t s, int layout, int e0, int ne, uint32_t* a2m) {
  if (n <= 0) return hipSuccess;
  if (ne < 0) ne = n;
  if (ne <= 0) return hipSuccess;
  ConvFwdArgs a{frames, nvalid, ctl, n, R, t, W1, b1, W2, b2, a1, a2, layout, e0, e0 + ne, a2m};
  // two envs a workgroup (16 waves sharing the weight planes) in nets of >= 512 envs, whether the
  // launch covers all of them or one env group's range (C4 0.513 -> 0.503 ms, C3 1.227 -> 1.212 ms at
  // two groups, profiles/r03/r3k); ARL_CONV_EPW=1 / 2 forces one form (A/B timing)
  static const char* epw = getenv("ARL_CONV_EPW");
  const int k = (epw && (epw[0] == '1' || epw[0] == '2')) ? epw[0] - '0' : (n >= 512 ? 2 : 1);
  if (k == 2) hipLaunchKernelGGL((conv_fwd_kernel<2>), dim3((ne + 1) / 2), dim3(2 * NT), 0, s, a);
  else hipLaunchKernelGGL((conv_fwd_kernel<1>), dim3(ne), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace arl
