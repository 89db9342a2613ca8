// GradientClipping(40) + RMSpropAsync over one flat parameter buffer.
//
// Reference: a3c_ale.py:224-226 (RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99)
// + GradientClipping(40) hook), rmsprop_async.py:23-29 (update_one_cpu) and
// the dormant CuPy kernel rmsprop_async.py:31-38; Chainer's GradientClipping
// (norm = sqrt(sum of per-array squared norms); if 40/norm < 1: g *= 40/norm).
//
// Two launches per update, both HBM-streaming over the padded flat buffer:
//   grad_sqnorm_kernel: per-block partial sum of g^2 (f32 per thread over a
//     grid-stride, f64 across the block) -> partials[block] (the folded form:
//     reduce_conv_bwd_kernel leaves the same partials, conv_bwd.hip), so the
//     clip rate needs no host round trip and no extra launch;
//   rmsprop_kernel: every block sums the partials in block order (their loads
//     in flight with its first p / ms / g loads; a last-arriving block of the
//     norm launch leaving one f64 instead measured 2-4 us slower a window, r4c),
//     then 4 parameters per thread per
//     iteration: g' = clip ? g*f32(rate) : g; ms = ms*alpha; ms += (c*g')*g';
//     p -= (lr*g') / sqrt(ms + eps) -- every op an explicit round-to-nearest
//     f32 op in the reference's order (NumPy f32 semantics, no FMA), so the
//     result is bit-identical to update_one_cpu.
// 20 bytes move per parameter (read p, g, ms; write p, ms) + 4 for the norm.
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "arl_internal.hpp"

namespace arl {

__device__ inline double block_sum_f64(double x, double* sh) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = x;
  __syncthreads();
  double t = 0.0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}

__global__ void __launch_bounds__(256)
grad_sqnorm_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ partials) {
  __shared__ double sh[8];
  const int64_t n4 = n >> 2;
  float acc = 0.f;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    acc = __fadd_rn(acc, __fadd_rn(__fadd_rn(__fmul_rn(v.x, v.x), __fmul_rn(v.y, v.y)),
                                   __fadd_rn(__fmul_rn(v.z, v.z), __fmul_rn(v.w, v.w))));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = g[(n4 << 2) + threadIdx.x];
    acc = __fadd_rn(acc, __fmul_rn(v, v));
  }
  const double t = block_sum_f64((double)acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

struct RmsConst {   // (AdvanceArgs is declared in arl_internal.hpp)
  float lr, alpha, one_minus_alpha, eps;
  // optional on-device lr anneal (a3c_ale.py:111-112):
  // lr = (total - global_t - 1) / total * lr0, global_t = (ctl[STEP] + t_max) * n_total
  double lr0;
  int64_t total, n_total, t_max;
  const int64_t* ctl;
  int ctl_idx;              // CTL_STEP, or CTL_STEP_SNAP when this launch also advances
};



__device__ inline void rms1(float& p, float& ms, float g, const RmsConst& c) {
  ms = __fmul_rn(ms, c.alpha);                                   // ms *= alpha
  ms = __fadd_rn(ms, __fmul_rn(__fmul_rn(c.one_minus_alpha, g), g));   // ms += (1-a)*g*g
  // sqrtf (not __fsqrt_rn = native approx sqrt) is the correctly rounded one under hipcc defaults
  p = __fsub_rn(p, __fdiv_rn(__fmul_rn(c.lr, g), sqrtf(__fadd_rn(ms, c.eps))));  // p -= lr*g/sqrt(ms+eps)
}

// one float4 of p / ms / g per thread and pass, the first pass's loads in flight with the norm's
__global__ void __launch_bounds__(256)
rmsprop_kernel(float* __restrict__ p, float* __restrict__ ms, const float* __restrict__ g, int64_t n, RmsConst c,
               const double* __restrict__ norm_sq, int nparts, float clip, AdvanceArgs adv) {
  __shared__ double sh[8];
  if (c.ctl != nullptr && c.total > 0) {
    const int64_t gt = (c.ctl[c.ctl_idx] + c.t_max) * c.n_total;
    // clamped at 0: the reference stops training once global_t passes the
    // step budget (run_a3c.py:64-68); a replay past it must not ascend
    c.lr = (float)(((double)max(c.total - gt - 1, (int64_t)0) / (double)c.total) * c.lr0);
  }
  const int64_t n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(ms);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the first pass's float4 of p / ms / g are in flight with the squared norm's loads (n4 == 0: none;
  // past the end: a clamped duplicate, never stored)
  float4 pv, mv, gv;
  if (n4 > 0) {
    const int64_t i = min(i0, n4 - 1);
    pv = p4[i];
    mv = m4[i];
    gv = g4[i];
  }
  float scale = 1.f;
  bool do_clip = false;
  if (norm_sq != nullptr) {   // re-reduce the partials [0, nparts) in block order (4 loads a thread in flight)
    double t = 0.0, v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = norm_sq[min((int)threadIdx.x + 256 * k, nparts - 1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((int)threadIdx.x + 256 * k < nparts) t += v[k];
    t = block_sum_f64(t, sh);
    const double norm = sqrt(t);
    const double rate = (double)clip / norm;
    if (norm > 0.0 && rate < 1.0) {
      do_clip = true;
      scale = (float)rate;
    }
  }
  for (int64_t ib = i0; ib < n4; ib += gsz) {
    if (ib != i0) {
      pv = p4[ib];
      mv = m4[ib];
      gv = g4[ib];
    }
    if (do_clip) {
      gv.x = __fmul_rn(gv.x, scale); gv.y = __fmul_rn(gv.y, scale);
      gv.z = __fmul_rn(gv.z, scale); gv.w = __fmul_rn(gv.w, scale);
    }
    rms1(pv.x, mv.x, gv.x, c);
    rms1(pv.y, mv.y, gv.y, c);
    rms1(pv.z, mv.z, gv.z, c);
    rms1(pv.w, mv.w, gv.w, c);
    p4[ib] = pv;
    m4[ib] = mv;
    const int64_t e = 4 * ib - adv.fc_w0;   // the FC weight's split planes follow their f32 W (fc.hip)
    if (adv.fc_planes != nullptr && e >= 0 && e < (int64_t)HID * A2) fc_planes_store(adv.fc_planes, (int)e, pv);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t j = (n4 << 2) + threadIdx.x;
    float gt = g[j];
    if (do_clip) gt = __fmul_rn(gt, scale);
    float pt = p[j], mt = ms[j];
    rms1(pt, mt, gt, c);
    p[j] = pt;
    ms[j] = mt;
  }
  if (adv.ctl == nullptr) return;   // (no window advance)
  for (int64_t i = i0; i < adv.n; i += gsz) adv.reset[i] = adv.reset[(int64_t)adv.T * adv.n + i];
  if (adv.hbuf != nullptr)
    for (int64_t i = i0; i < (int64_t)adv.n * HID; i += gsz) {
      adv.hbuf[i] = adv.hbuf[(int64_t)adv.T * adv.n * HID + i];
      adv.cbuf[i] = adv.cbuf[(int64_t)adv.T * adv.n * HID + i];
    }
  if (i0 == 0) {
    adv.ctl[CTL_STEP] += adv.T;
    adv.ctl[CTL_WINDOW] += 1;
  }
}

static int stream_blocks(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

hipError_t launch_grad_sqnorm(const float* g, int64_t n, double* partials, int blocks, hipStream_t s) {
  if (blocks < 1 || blocks > NORM_MAX_PARTS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(blocks), dim3(256), 0, s, g, n, partials);
  return hipGetLastError();
}

hipError_t launch_rmsprop(float* p, float* ms, const float* g, int64_t n, double lr, double alpha, double eps,
                          const double* norm_sq, int nparts, float clip, const int64_t* ctl,
                          int64_t total_steps, int64_t n_total, int t_max, hipStream_t s, const AdvanceArgs* adv) {
  if (norm_sq != nullptr && (nparts < 1 || nparts > NORM_MAX_PARTS)) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  // each Python-float hyperparameter meets the f32 arrays as f32(value)
  RmsConst c;
  c.lr = (float)lr;
  c.alpha = (float)alpha;
  c.one_minus_alpha = (float)(1.0 - alpha);   // (1 - self.alpha) in Python double, then f32
  c.eps = (float)eps;
  c.lr0 = lr;
  c.total = total_steps;
  c.n_total = n_total;
  c.t_max = t_max;
  c.ctl = ctl;
  c.ctl_idx = (adv != nullptr && adv->ctl != nullptr) ? CTL_STEP_SNAP : CTL_STEP;
  AdvanceArgs a{};
  if (adv != nullptr) a = *adv;
  hipLaunchKernelGGL(rmsprop_kernel, dim3(stream_blocks(n)), dim3(256), 0, s, p, ms, g, n, c, norm_sq, nparts, clip, a);
  return hipGetLastError();
}

// HBM stream-copy peak (measurement only; SURVEY 8(d) "also report vs the
// measured stream-copy peak").  Two forms, the bench keeps the faster:
//   mode 0: grid-stride, four 16-byte loads in flight per lane before the
//           first store (addresses one grid apart);
//   mode 1: each workgroup copies contiguous 64 KB blocks (block-stride over
//           the buffer), every lane 4 consecutive-in-wave 16-byte loads in
//           flight, non-temporal loads / stores (a once-read stream).
__global__ void __launch_bounds__(256)
stream_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n4; i += stride) dst[i] = src[i];
}

typedef float cp_f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256)
stream_copy_blocks_kernel(const cp_f32x4* __restrict__ src, cp_f32x4* __restrict__ dst, int64_t n4) {
  constexpr int U = 16;                         // 16-byte vectors per lane per block: 256 x 16 x 16 B = 64 KB
  const int64_t nblk = n4 / (256 * U);
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const cp_f32x4* s = src + b * (256 * U) + threadIdx.x;
    cp_f32x4* d = dst + b * (256 * U) + threadIdx.x;
    cp_f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + 256 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], d + 256 * u);
  }
  for (int64_t i = nblk * (256 * U) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    dst[i] = src[i];
}

//   mode 2 / 3: a one-shot grid, one 16-byte load and store per lane (bytes / 4 KB workgroups of 256);
//           mode 3 with non-temporal loads / stores -- the fastest form on MI355X (scripts/copy_sweep.hip:
//           6.47 TB/s non-temporal, 6.25 plain at 1 GiB; 8 loads a lane in flight ran 4.3 TB/s)
template <bool NT>
__global__ void __launch_bounds__(256)
stream_copy_chunk_kernel(const cp_f32x4* __restrict__ src, cp_f32x4* __restrict__ dst, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
  else dst[i] = src[i];
}

hipError_t launch_stream_copy(const void* src, void* dst, int64_t bytes, int blocks, int mode, hipStream_t s) {
  const float4* a = reinterpret_cast<const float4*>(src);
  float4* b = reinterpret_cast<float4*>(dst);
  if (mode >= 2) {
    const int64_t grid = (bytes / 16 + 255) / 256;
    if (grid > 0x7fffffff) return hipErrorInvalidValue;
    if (mode == 3)
      hipLaunchKernelGGL(stream_copy_chunk_kernel<true>, dim3((unsigned)grid), dim3(256), 0, s,
                         reinterpret_cast<const cp_f32x4*>(src), reinterpret_cast<cp_f32x4*>(dst), bytes / 16);
    else
      hipLaunchKernelGGL(stream_copy_chunk_kernel<false>, dim3((unsigned)grid), dim3(256), 0, s,
                         reinterpret_cast<const cp_f32x4*>(src), reinterpret_cast<cp_f32x4*>(dst), bytes / 16);
    return hipGetLastError();
  }
  if (mode == 1)
    hipLaunchKernelGGL(stream_copy_blocks_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const cp_f32x4*>(src),
                       reinterpret_cast<cp_f32x4*>(dst), bytes / 16);
  else hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, s, a, b, bytes / 16);
  return hipGetLastError();
}

}  // namespace arl
