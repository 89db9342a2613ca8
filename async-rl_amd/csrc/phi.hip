// Frame preprocessing (phi) on gfx950.
//
// Reference: ale.py:59-89 (current_screen: np.maximum of the two captured RGB
// frames, float64 luminance R*0.2126 + G*0.0722 + B*0.7152, astype(uint8),
// cv2.resize(img, (84, 84), INTER_LINEAR)), ale.py:135 / :155-158 (4-plane
// deque, reset to three zero planes + the new screen), dqn_phi.py:14-16
// (f32 /= 255).  Resize mode bits: 1 = SIMD vertical pass, 2 = the 'crop'
// branch of ale.py:73-82 (resize to 84 x 110, keep rows 18..101: only the
// vertical coefficients change -- output row dy uses row dy + 18 of a
// 210 -> 110 resize).
//
// One workgroup (256 threads) = one env x one band of 12 output rows (7 bands
// per 84x84 screen).  Only the source rows the bilinear taps touch are read
// (2 per output row: for 210->84 that is 4 of every 5 rows), 48 contiguous
// bytes (16 RGB pixels) per thread per frame as three 16-byte loads, both
// frames of the pair.  Max + luminance run in registers (fp64, explicit
// round-to-nearest ops so nothing can be contracted into an FMA: bit-exact
// with NumPy), the uint8 gray rows land in LDS, and the separable fixed-point
// resize reads them back and writes 4 output pixels per thread as one u32.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "phi_ops.hpp"

namespace arl {

constexpr int BAND = 12;                   // output rows per workgroup
constexpr int NBANDS = DST / BAND;         // 7

struct PhiShared {
  uint8_t gray[BAND][2][SRC_W];   // [output row][tap][x]
  int16_t xofs[DST];
  int16_t xa0[DST], xa1[DST];
  int16_t yofs[BAND];
  int16_t yb0[BAND], yb1[BAND];
};

// the resized plane's store into the ring: an ordinary store (the next conv launch reads it; non-temporal
// measured slower, r4r)
__device__ inline void ring_store(uint32_t* p, uint32_t v) { *p = v; }

// Computes output rows [dy0, dy0+BAND) of one env's screen into `out`
// (row stride 84).  cur/prev: the env's two RGB frames (HWC, uint8).
// (non-temporal loads of the frame pairs measured slower: phi_ring 10.1 -> 13.0 us at C2, r3x)

__device__ inline void phi_band(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ prev,
                                uint8_t* __restrict__ out, int dy0, int mode, PhiShared& sh) {
  const int tid = threadIdx.x;
  // stage: task = (local row r in 0..23 -> (dy, tap), chunk c in 0..9 of 16 px).
  // Each task derives its own source row, so the loads are issued before the
  // resize coefficients are tabulated and need no barrier in front of them.
  const bool stager = tid < 2 * BAND * 10;
  const int r = tid / 10, c = tid % 10;
  const int ly = r >> 1, tap = r & 1;
  uint4 c0, c1, c2, p0, p1, p2;
  if (stager) {
    int o, b0, b1;
    if (mode & 2) resize_coeff(dy0 + ly + CROP_TOP, SRC_H, CROP_H, o, b0, b1);
    else resize_coeff(dy0 + ly, SRC_H, DST, o, b0, b1);
    int sy = o + tap;
    if (sy > SRC_H - 1) sy = SRC_H - 1;
    const uint4* pc = reinterpret_cast<const uint4*>(cur + (size_t)sy * SRC_W * 3 + c * 48);
    const uint4* pp = reinterpret_cast<const uint4*>(prev + (size_t)sy * SRC_W * 3 + c * 48);
    c0 = pc[0]; c1 = pc[1]; c2 = pc[2];
    p0 = pp[0]; p1 = pp[1]; p2 = pp[2];
  }
  if (tid < DST) {
    int o, a0, a1;
    resize_coeff(tid, SRC_W, DST, o, a0, a1);
    sh.xofs[tid] = (int16_t)o; sh.xa0[tid] = (int16_t)a0; sh.xa1[tid] = (int16_t)a1;
  } else if (tid >= 96 && tid < 96 + BAND) {
    int o, b0, b1;
    if (mode & 2) resize_coeff(dy0 + tid - 96 + CROP_TOP, SRC_H, CROP_H, o, b0, b1);
    else resize_coeff(dy0 + tid - 96, SRC_H, DST, o, b0, b1);
    sh.yofs[tid - 96] = (int16_t)o; sh.yb0[tid - 96] = (int16_t)b0; sh.yb1[tid - 96] = (int16_t)b1;
  }
  if (stager) *reinterpret_cast<uint4*>(&sh.gray[ly][tap][c * 16]) = max_luminance16(c0, c1, c2, p0, p1, p2);
  __syncthreads();
  // resize: task = (local row ly, group of 4 output columns q) -> 12*21 = 252
  if (tid < BAND * (DST / 4)) {
    const int ly = tid / (DST / 4), q = tid % (DST / 4);
    const int b0 = sh.yb0[ly], b1 = sh.yb1[ly];
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int dx = q * 4 + j;
      const int sx = sh.xofs[dx];
      const int sx1 = sx + 1 < SRC_W ? sx + 1 : SRC_W - 1;
      const int a0 = sh.xa0[dx], a1 = sh.xa1[dx];
      const int r0 = (int)sh.gray[ly][0][sx] * a0 + (int)sh.gray[ly][0][sx1] * a1;
      const int r1 = (int)sh.gray[ly][1][sx] * a0 + (int)sh.gray[ly][1][sx1] * a1;
      const int v = resize_vpass(r0, r1, b0, b1, mode);
      packed |= (uint32_t)v << (8 * j);
    }
    ring_store(reinterpret_cast<uint32_t*>(out + (size_t)(dy0 + ly) * DST + q * 4), packed);
  }
}

// ---------------------------------------------------------------- kernels
// ale.py:59-89: one 84x84 screen per env.
__global__ void __launch_bounds__(256)
current_screen_kernel(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ prev,
                      uint8_t* __restrict__ out, int mode) {
  __shared__ PhiShared sh;
  const int64_t e = blockIdx.y;
  phi_band(cur + e * FRAME_BYTES, prev + e * FRAME_BYTES, out + e * PLANE, blockIdx.x * BAND, mode, sh);
}

// Materialised 4-plane stack: out[e] = reset ? [0,0,0,new]
// : [prev[1], prev[2], prev[3], new]; pairs laid out (n, 2, 210, 160, 3).
__global__ void __launch_bounds__(256)
phi_stack_kernel(const uint8_t* __restrict__ pairs, const uint8_t* __restrict__ prev_stack,
                 const uint8_t* __restrict__ reset, uint8_t* __restrict__ out_stack, int mode) {
  __shared__ PhiShared sh;
  const int64_t e = blockIdx.y;
  const int dy0 = blockIdx.x * BAND;
  const uint8_t* pr = pairs + e * (2 * FRAME_BYTES);
  uint8_t* os = out_stack + e * (4 * PLANE);
  phi_band(pr, pr + FRAME_BYTES, os + 3 * PLANE, dy0, mode, sh);
  // shift the three older planes (rows of this band only), 16 B per thread
  const bool rs = reset != nullptr && reset[e] != 0;
  const uint8_t* ps = prev_stack + e * (4 * PLANE);
  constexpr int BAND_BYTES = BAND * DST;           // 1008 = 63 x 16
  const int tid = threadIdx.x;
  if (tid < 3 * (BAND_BYTES / 16)) {
    const int p = tid / (BAND_BYTES / 16), c = tid % (BAND_BYTES / 16);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (!rs) v = *reinterpret_cast<const uint4*>(ps + (p + 1) * PLANE + dy0 * DST + c * 16);
    *reinterpret_cast<uint4*>(os + p * PLANE + dy0 * DST + c * 16) = v;
  }
}

// In-loop ring: the new screen of obs step k = ctl[0] + t goes to slot k % R;
// nvalid[slot][e] = reset ? 1 : min(nvalid[prev slot][e] + 1, 4).  Also
// ingests the reward / done that arrived with this obs (a3c.py:69-70,75):
// rewards[t-1], dones[t-1] (t >= 1) and reset_flags[t].
__global__ void __launch_bounds__(256)
phi_ring_kernel(RingArgs a) {
  __shared__ PhiShared sh;
  const int e = a.e0 + blockIdx.y;
  const int64_t k = a.ctl[CTL_STEP] + a.t;
  const int slot = (int)(k % a.R);
  const int64_t pidx = k % a.pool_len;
  const uint8_t* pr = a.pair_pool + (pidx * a.n + e) * (int64_t)(2 * FRAME_BYTES);
  uint8_t* dst = a.frames + ((int64_t)slot * a.n + e) * PLANE;
  phi_band(pr, pr + FRAME_BYTES, dst, blockIdx.x * BAND, a.mode, sh);
  if (blockIdx.x == 0 && threadIdx.x == 0) ring_obs_store(a, e, k, ring_obs_load(a, e, k));
}

// ---------------------------------------------------------------- RGB (Doom)
// train_a3c_doom.py:21-23: phi(obs) = cv2.resize(obs.image_buffer, (84, 84))
// .transpose(2, 0, 1).astype(float32) / 255 -- the RGB24 (H, W, 3) screen of
// doom_env.py:47 resized per channel with the same fixed-point INTER_LINEAR
// as the ALE path, no max-pool, no luminance, no frame stack.  One workgroup
// = one env x one band of 6 output rows; the 12 source rows the band's taps
// touch are staged in (dynamic) LDS, W*3 bytes each, 16 bytes per load.
constexpr int RGB_BAND = 6;                  // output rows per workgroup (12 source rows of LDS)
constexpr int RGB_NBANDS = DST / RGB_BAND;   // 14
struct RgbCoef {
  int16_t xofs[DST];
  int16_t xa0[DST], xa1[DST];
  int16_t yofs[RGB_BAND];
  int16_t yb0[RGB_BAND], yb1[RGB_BAND];
};

// out(ch, dy, dx) for dy in [dy0, dy0 + 6): uint8 planes (plane stride
// `pstride` bytes) or, with OUT_F32, f32 / 255 (plane stride 84*84 floats)
template <bool OUT_F32>
__device__ inline void rgb_band(const uint8_t* __restrict__ img, int H, int W, void* __restrict__ out,
                                int64_t pstride, int dy0, int mode, RgbCoef& cf, uint8_t* rows) {
  const int tid = threadIdx.x;
  if (tid < DST) {
    int o, a0, a1;
    resize_coeff(tid, W, DST, o, a0, a1);
    cf.xofs[tid] = (int16_t)o; cf.xa0[tid] = (int16_t)a0; cf.xa1[tid] = (int16_t)a1;
  } else if (tid >= 96 && tid < 96 + RGB_BAND) {
    int o, b0, b1;
    resize_coeff(dy0 + tid - 96, H, DST, o, b0, b1);
    cf.yofs[tid - 96] = (int16_t)o; cf.yb0[tid - 96] = (int16_t)b0; cf.yb1[tid - 96] = (int16_t)b1;
  }
  __syncthreads();
  // LDS-DMA (global_load_lds_dwordx4): chunk i = (row r, 16-byte column c)
  // lands at rows + 16 i, one 1 KB wave instruction at a time, all in flight
  // before the single wait
  const int rb = W * 3, chunks = rb / 16;   // W % 16 == 0 (checked by the host)
  const int total = 2 * RGB_BAND * chunks, lane = tid & 63;
  for (int it = tid >> 6; it * 64 < total; it += 4) {
    const int i = it * 64 + lane;
    if (i < total) {
      const int r = i / chunks, c = i - r * chunks;
      int sy = cf.yofs[r >> 1] + (r & 1);
      if (sy > H - 1) sy = H - 1;
      __builtin_amdgcn_global_load_lds(img + (size_t)sy * rb + 16 * c,
                                       (__attribute__((address_space(3))) void*)(rows + 1024 * it), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int task = tid; task < 3 * RGB_BAND * (DST / 4); task += 256) {
    const int ch = task / (RGB_BAND * (DST / 4)), rem = task - ch * (RGB_BAND * (DST / 4));
    const int ly = rem / (DST / 4), q = rem - ly * (DST / 4);
    const int b0 = cf.yb0[ly], b1 = cf.yb1[ly];
    const uint8_t* s0 = rows + (2 * ly) * rb + ch;
    const uint8_t* s1 = s0 + rb;
    int v4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int dx = q * 4 + j;
      const int sx = cf.xofs[dx];
      const int sx1 = sx + 1 < W ? sx + 1 : W - 1;
      const int a0 = cf.xa0[dx], a1 = cf.xa1[dx];
      const int r0 = (int)s0[3 * sx] * a0 + (int)s0[3 * sx1] * a1;
      const int r1 = (int)s1[3 * sx] * a0 + (int)s1[3 * sx1] * a1;
      int v;
      if ((mode & 1) == 0) v = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22;
      else v = ((((r0 >> 4) * b0) >> 16) + (((r1 >> 4) * b1) >> 16) + 2) >> 2;
      v4[j] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
    const int dy = dy0 + ly;
    if (OUT_F32) {
      float4 o;
      o.x = div255((float)v4[0]);
      o.y = div255((float)v4[1]);
      o.z = div255((float)v4[2]);
      o.w = div255((float)v4[3]);
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + ch * PLANE + dy * DST + q * 4) = o;
    } else {
      const uint32_t packed = (uint32_t)v4[0] | ((uint32_t)v4[1] << 8) | ((uint32_t)v4[2] << 16) |
                              ((uint32_t)v4[3] << 24);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(out) + ch * pstride + dy * DST + q * 4) = packed;
    }
  }
}

// batched train_a3c_doom.phi: imgs (n, H, W, 3) -> out (n, 3, 84, 84) f32
__global__ void __launch_bounds__(256)
rgb_phi_kernel(const uint8_t* __restrict__ imgs, int H, int W, float* __restrict__ out, int mode) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rgb_rows[];
  __shared__ RgbCoef cf;
  const int64_t e = blockIdx.y;
  rgb_band<true>(imgs + e * H * W * 3, H, W, out + e * 3 * PLANE, 0, blockIdx.x * RGB_BAND, mode, cf, rgb_rows);
}

// In-loop ring for RGB nets: the 3 planes of obs step k go to slot k % R
// (frames (R, n, 3, 84, 84)); nvalid = 3 (conv input = [0, R, G, B]); the
// reward / done / reset bookkeeping of phi_ring_kernel.
__global__ void __launch_bounds__(256)
rgb_ring_kernel(RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rgb_rows[];
  __shared__ RgbCoef cf;
  const int e = a.e0 + blockIdx.y;
  const int64_t k = a.ctl[CTL_STEP] + a.t;
  const int slot = (int)(k % a.R);
  const int64_t pidx = k % a.pool_len;
  const uint8_t* img = a.pair_pool + (pidx * a.n + e) * (int64_t)a.H * a.W * 3;
  uint8_t* dst = a.frames + ((int64_t)slot * a.n + e) * 3 * PLANE;
  rgb_band<false>(img, a.H, a.W, dst, PLANE, blockIdx.x * RGB_BAND, a.mode, cf, rgb_rows);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint8_t d = a.done_pool ? a.done_pool[pidx * a.n + e] : 0;
    const bool rs = a.force_reset || d != 0;
    a.nvalid[(int64_t)slot * a.n + e] = 3;
    a.reset_flags[(int64_t)a.t * a.n + e] = rs ? 1 : 0;
    if (a.t >= 1) {
      float r = a.reward_pool ? a.reward_pool[pidx * a.n + e] : 0.f;
      a.rewards[(int64_t)(a.t - 1) * a.n + e] = r;
      a.dones[(int64_t)(a.t - 1) * a.n + e] = d;
    }
  }
}

// In-loop ring for ARCH_STACK nets: the env's whole 4-screen stack of obs step
// k (ale.py:91-94 ALE.state, oldest first) goes to slot k % R (frames (R, n,
// 4, 84, 84)); ARCH_STATES nets: the same with phi's f32 state (esize 4); nvalid = 4; the reward / done / reset bookkeeping of
// phi_ring_kernel.  pair_pool == null: bookkeeping only (a terminal
// observation, whose state a3c.py:72-73 never reads).  One workgroup per env,
// 16-byte copies.
__global__ void __launch_bounds__(256)
stack_ring_kernel(RingArgs a) {
  const int e = a.e0 + blockIdx.x;
  const int64_t k = a.ctl[CTL_STEP] + a.t;
  const int slot = (int)(k % a.R);
  const int64_t pidx = k % a.pool_len;
  if (a.pair_pool != nullptr) {
    const int64_t sb = (int64_t)4 * PLANE * a.esize;   // bytes per stack (uint8 screens / f32 states)
    const int V = (int)(sb / 16);                       // 1764 / 7056 uint4
    const uint4* src = reinterpret_cast<const uint4*>(a.pair_pool + (pidx * a.n + e) * sb);
    uint4* dst = reinterpret_cast<uint4*>(a.frames + ((int64_t)slot * a.n + e) * sb);
    for (int i = threadIdx.x; i < V; i += 256) dst[i] = src[i];
  }
  if (threadIdx.x == 0) {
    const uint8_t d = a.done_pool ? a.done_pool[pidx * a.n + e] : 0;
    const bool rs = a.force_reset || d != 0;
    if (a.pair_pool != nullptr) {
      a.nvalid[(int64_t)slot * a.n + e] = 4;
      a.reset_flags[(int64_t)a.t * a.n + e] = rs ? 1 : 0;
    }
    if (a.t >= 1) {
      float r = a.reward_pool ? a.reward_pool[pidx * a.n + e] : 0.f;
      a.rewards[(int64_t)(a.t - 1) * a.n + e] = r;
      a.dones[(int64_t)(a.t - 1) * a.n + e] = d;
    }
  }
}

// dqn_phi.py:14-16: float32(x) / 255.0 (IEEE correctly rounded division).
__global__ void dqn_phi_kernel(const uint8_t* __restrict__ in, float* __restrict__ out, int64_t count) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < count) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(in + i);
    float4 o;
    o.x = div255((float)(w & 0xff));
    o.y = div255((float)((w >> 8) & 0xff));
    o.z = div255((float)((w >> 16) & 0xff));
    o.w = div255((float)(w >> 24));
    *reinterpret_cast<float4*>(out + i) = o;
  } else {
    for (int64_t j = i; j < count; ++j) out[j] = div255((float)in[j]);
  }
}

// ale.py:62-69 alone (max of the pair + luminance + uint8), one pixel per
// thread; same device function as the fused path (used to verify all 2^24
// RGB triples against NumPy).
__global__ void max_luminance_kernel(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ prev,
                                     uint8_t* __restrict__ gray, int64_t npix) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t* c = cur + 3 * i;
  const uint8_t* p = prev + 3 * i;
  const uint32_t r = c[0] > p[0] ? c[0] : p[0];
  const uint32_t g = c[1] > p[1] ? c[1] : p[1];
  const uint32_t b = c[2] > p[2] ? c[2] : p[2];
  gray[i] = (uint8_t)luminance(r, g, b);
}

hipError_t launch_max_luminance(const uint8_t* cur, const uint8_t* prev, uint8_t* gray, int64_t npix,
                                hipStream_t s) {
  if (npix <= 0) return hipSuccess;
  hipLaunchKernelGGL(max_luminance_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, cur, prev, gray,
                     npix);
  return hipGetLastError();
}

hipError_t launch_current_screen(const uint8_t* cur, const uint8_t* prev, uint8_t* out, int64_t n,
                                 int mode, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(current_screen_kernel, dim3(NBANDS, (unsigned)n), dim3(256), 0, s, cur, prev, out, mode);
  return hipGetLastError();
}

hipError_t launch_phi_stack(const uint8_t* pairs, const uint8_t* prev_stack, const uint8_t* reset,
                            uint8_t* out_stack, int64_t n, int mode, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(phi_stack_kernel, dim3(NBANDS, (unsigned)n), dim3(256), 0, s, pairs, prev_stack,
                     reset, out_stack, mode);
  return hipGetLastError();
}

hipError_t launch_phi_ring(const RingArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(phi_ring_kernel, dim3(NBANDS, (unsigned)(a.ne < 0 ? a.n : a.ne)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_stack_ring(const RingArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(stack_ring_kernel, dim3((unsigned)(a.ne < 0 ? a.n : a.ne)), dim3(256), 0, s, a);
  return hipGetLastError();
}

static size_t rgb_lds(int W) { return (size_t)2 * RGB_BAND * W * 3; }

hipError_t launch_rgb_phi(const uint8_t* imgs, int64_t n, int H, int W, float* out, int mode, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rgb_phi_kernel, dim3(RGB_NBANDS, (unsigned)n), dim3(256), rgb_lds(W), s, imgs, H, W, out,
                     mode);
  return hipGetLastError();
}

hipError_t launch_rgb_ring(const RingArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(rgb_ring_kernel, dim3(RGB_NBANDS, (unsigned)(a.ne < 0 ? a.n : a.ne)), dim3(256), rgb_lds(a.W), s,
                     a);
  return hipGetLastError();
}

hipError_t launch_dqn_phi(const uint8_t* in, float* out, int64_t count, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const int64_t threads = (count + 3) / 4;
  hipLaunchKernelGGL(dqn_phi_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, in, out, count);
  return hipGetLastError();
}

}  // namespace arl
