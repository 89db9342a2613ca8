// Device pieces of phi shared by phi.hip and the fused observe + conv forward
// (conv_fwd.hip): ale.py:59-89 (max of the pair, float64 luminance, uint8
// truncation, cv2.resize INTER_LINEAR in OpenCV's fixed point).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

constexpr int SRC_H = 210, SRC_W = 160, DST = 84;
constexpr int FRAME_BYTES = SRC_H * SRC_W * 3;   // 100,800
constexpr int CROP_H = 110, CROP_TOP = (110 - 84) - 8;   // ale.py:75-81: resize to 110 rows, crop 18 .. 101

// OpenCV INTER_LINEAR coefficients for one axis (see oracle.resize_coeffs):
// f = (float)((d+0.5)*scale-0.5); s = floor(f); f -= s; clamps; a = rint(c*2048)
__device__ inline void resize_coeff(int d, int ssize, int dsize, int& ofs, int& a0, int& a1) {
  const double inv_scale = (double)dsize / (double)ssize;
  const double scale = 1.0 / inv_scale;
  float f = (float)__dsub_rn(__dmul_rn((double)d + 0.5, scale), 0.5);
  int s = (int)floorf(f);
  f = __fsub_rn(f, (float)s);
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
  const float c0 = __fsub_rn(1.f, f);
  ofs = s;
  a0 = (int)rintf(__fmul_rn(c0, 2048.f));
  a1 = (int)rintf(__fmul_rn(f, 2048.f));
}

__device__ inline uint32_t umax_bytes(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t x = (a >> (8 * i)) & 0xffu, y = (b >> (8 * i)) & 0xffu;
    r |= (x > y ? x : y) << (8 * i);
  }
  return r;
}

// ale.py:67-69, float64, left-to-right, explicit RN ops (no FMA contraction)
__device__ inline uint32_t luminance_f64(uint32_t r, uint32_t g, uint32_t b) {
  const double v = __dadd_rn(__dadd_rn(__dmul_rn((double)r, 0.2126), __dmul_rn((double)g, 0.0722)),
                             __dmul_rn((double)b, 0.7152));
  return (uint32_t)v;   // astype(uint8): truncation (v in [0, 255))
}

// (An integer fast path -- a 24-bit fixed-point sum with this float64 form as
// the fallback for the 3,384 triples within 64 / 2^24 of an integer, exact over
// all 2^24 triples -- measured slower inside phi_ring_kernel: 10.65 vs 9.75 us,
// the per-pixel fallback branch costs more than the float64 ops it skips.)
__device__ inline uint32_t luminance(uint32_t r, uint32_t g, uint32_t b) { return luminance_f64(r, g, b); }

// 48 RGB bytes (16 pixels) of each frame -> 16 uint8 gray values (ale.py:62-69)
__device__ inline uint4 max_luminance16(uint4 c0, uint4 c1, uint4 c2, uint4 p0, uint4 p1, uint4 p2) {
  const uint32_t w[12] = {umax_bytes(c0.x, p0.x), umax_bytes(c0.y, p0.y), umax_bytes(c0.z, p0.z),
                          umax_bytes(c0.w, p0.w), umax_bytes(c1.x, p1.x), umax_bytes(c1.y, p1.y),
                          umax_bytes(c1.z, p1.z), umax_bytes(c1.w, p1.w), umax_bytes(c2.x, p2.x),
                          umax_bytes(c2.y, p2.y), umax_bytes(c2.z, p2.z), umax_bytes(c2.w, p2.w)};
  uint32_t g[4] = {0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int b = 3 * p;
    const uint32_t R = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
    const uint32_t G = (w[(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 0xffu;
    const uint32_t B = (w[(b + 2) >> 2] >> (8 * ((b + 2) & 3))) & 0xffu;
    g[p >> 2] |= luminance(R, G, B) << (8 * (p & 3));
  }
  return make_uint4(g[0], g[1], g[2], g[3]);
}

// one output pixel of the separable fixed-point resize from the two tap rows
// r0 / r1 (horizontal pass done per row): mode bit 0 = SIMD vertical pass
__device__ inline int resize_vpass(int r0, int r1, int b0, int b1, int mode) {
  int v;
  if ((mode & 1) == 0) {   // FixedPtCast<int, uchar, 22>
    v = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22;
  } else {                 // VResizeLinearVec_32s8u (mulhi form)
    v = ((((r0 >> 4) * b0) >> 16) + (((r1 >> 4) * b1) >> 16) + 2) >> 2;
  }
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Ring bookkeeping of an observation (a3c.py:69-70,75; ale.py:135,155-158):
// nvalid[slot][e] = reset ? 1 : min(nvalid[prev slot][e] + 1, 4), the reset
// flag of step t, and the reward / done that arrived with it -> rewards[t-1],
// dones[t-1] (t >= 1).  ring_obs_load issues the loads (any thread; the fused
// kernel issues them before its bulk loads so they land first), ring_obs_store
// writes (one thread per env).
struct RingObs {
  uint8_t done;
  int nv;      // nvalid of this observation
  float r;
};
__device__ inline RingObs ring_obs_load(const RingArgs& a, int e, int64_t k) {
  const int64_t pidx = k % a.pool_len;
  const int pslot = (int)((k + a.R - 1) % a.R);
  RingObs o;
  o.done = a.done_pool ? a.done_pool[pidx * a.n + e] : 0;
  o.r = (a.t >= 1 && a.reward_pool) ? a.reward_pool[pidx * a.n + e] : 0.f;
  const int pv = (int)a.nvalid[(int64_t)pslot * a.n + e] + 1;
  o.nv = (a.force_reset || o.done != 0) ? 1 : (pv > 4 ? 4 : pv);
  return o;
}
__device__ inline void ring_obs_store(const RingArgs& a, int e, int64_t k, const RingObs& o) {
  const int slot = (int)(k % a.R);
  a.nvalid[(int64_t)slot * a.n + e] = (uint8_t)o.nv;
  a.reset_flags[(int64_t)a.t * a.n + e] = (a.force_reset || o.done != 0) ? 1 : 0;
  if (a.t >= 1) {
    a.rewards[(int64_t)(a.t - 1) * a.n + e] = o.r;
    a.dones[(int64_t)(a.t - 1) * a.n + e] = o.done;
  }
}

}  // namespace arl
