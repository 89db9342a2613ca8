// The NIPS head (FF / LSTM) on float32 states: the drop-in for A3C's phi
// plugin (a3c.py:34,50,73 -- `phi=lambda x: x` by default; the model sees
// whatever phi returns, dqn_head.py:48-52).  An ARCH_STATES net keeps phi's
// (4, 84, 84) f32 output per obs step in its ring (frames (R, n, 4, 84, 84)
// f32, written by arl_observe_states) and runs the two convolutions on the
// generic implicit-GEMM template (gemm.hpp, exact f32 v_mfma_f32_16x16x4_f32):
//   forward   conv1  M = 400 n x 16 x K 256, im2col straight from the state ring
//             conv2  M =  81 n x 32 x K 256, im2col of a1
//   backward  conv2 dW / db (split-K over sample x position, ones column = bias)
//             da1 = stride-2 convT(da2, W2) * (a1 > 0), 4 output parity classes
//             conv1 dW / db from the state ring (no dX: the input is data)
// The FC, LSTM, heads and the rest of the learner are the NIPS path's own
// kernels (they read a1 / a2 / hfc, not the frames).  This path serves the
// one-env drop-in and any float phi; the uint8 frame paths keep the fused
// conv kernels (conv_fwd.hip / conv_bwd.hip).  Split-K slabs are summed in
// f64 in slice order (reduce_grad_kernel): deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "gemm.hpp"
#include "layers.hpp"

namespace arl {

namespace {

// conv1 im2col from the f32 state ring: sample s = tt * n + e (window step
// t0 + tt, env e), m = s * 400 + p, k = ic * 64 + ky * 8 + kx; the state of
// obs step k sits in slot k % R (k = ctl[STEP] + t).
struct StatesIm2col {
  const float* __restrict__ frames; const int64_t* __restrict__ ctl; int n, R, t0;
  __device__ const float* addr(int m, int k) const {
    const int s = m / C1_P, p = m - s * C1_P;
    const int tt = s / n, e = s - tt * n;
    const int slot = (int)((ctl[CTL_STEP] + t0 + tt) % R);
    const int ic = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
    const int oy = p / 20, ox = p - oy * 20;
    return frames + (((int64_t)slot * n + e) * 4 + ic) * PLANE + (4 * oy + ky) * 84 + 4 * ox + kx;
  }
  __device__ float load(int m, int k) const { return *addr(m, k); }
  // 4 consecutive kx (k % 4 == 0): 16-byte aligned (PLANE, 84 and 4 ox are multiples of 4 floats)
  __device__ float4 load4(int m, int k) const { return *reinterpret_cast<const float4*>(addr(m, k)); }
};

struct SPlans {
  int c2_w, c1_w;
};

SPlans states_plans(const Net& net) {
  const int64_t S = (int64_t)net.T * net.N;
  SPlans p;
  p.c2_w = effective_splits<32>((int)(S * C2_P), plan_splits(ceil_div(C1_OC * 16 + 1, 64), S * C2_P, 32));
  p.c1_w = effective_splits<32>((int)(S * C1_P), plan_splits(ceil_div(4 * 64 + 1, 64), S * C1_P, 32));
  return p;
}

#define ARL_TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

}  // namespace

int64_t states_slab_floats(const Net& net) {
  const SPlans pl = states_plans(net);
  return std::max((int64_t)pl.c2_w * C2_OC * (C1_OC * 16 + 1), (int64_t)pl.c1_w * C1_OC * (4 * 64 + 1));
}

hipError_t states_conv_fwd(const Net& net, int t, float* a1, float* a2, hipStream_t s) {
  const int n = net.N;
  const float* P = net.p;
  ARL_TRY((launch_gemm<64, 16, 32, 4, 1, GK, GS>(
      StatesIm2col{net.at<float>(net.w_frames), net.at<int64_t>(net.w_ctl), n, net.R, t}, WeightT{P + net.o_c1W, 256},
      EpiConv{a1, P + net.o_c1b, C1_OC, C1_P}, n * C1_P, C1_OC, 256, 1, s)));
  return launch_gemm<32, 32, 32, 2, 2, GS, GK>(Im2col<C1_OC, 20, 4, 2, 9>{a1}, WeightT{P + net.o_c2W, C1_OC * 16},
                                               EpiConv{a2, P + net.o_c2b, C2_OC, C2_P}, n * C2_P, C2_OC, C1_OC * 16, 1,
                                               s);
}

hipError_t states_conv_bwd(Net& net, hipStream_t s) {
  const int n = net.N, S = net.T * n;
  const SPlans pl = states_plans(net);
  const float* P = net.p;
  float* G = net.g;
  float* slab = net.at<float>(net.w_slab);
  const float* a1 = net.at<float>(net.w_a1);
  const float* da2 = net.at<float>(net.w_da2);
  float* da1 = net.at<float>(net.w_da1);
  // conv2: dW2 / db2 over (sample, position)
  ARL_TRY((launch_gemm<32, 64, 32, 2, 2, GS, GS>(ConvDyT{da2, C2_OC, C2_P},
                                                 OnesCol<Im2col<C1_OC, 20, 4, 2, 9>>{{a1}, C1_OC * 16},
                                                 EpiSlab{slab, C2_OC, C1_OC * 16 + 1}, C2_OC, C1_OC * 16 + 1, S * C2_P,
                                                 pl.c2_w, s)));
  ARL_TRY(launch_reduce_grad(slab, pl.c2_w, C2_OC, C1_OC * 16 + 1,
                             MapDense{G, net.o_c2W, net.o_c2b, -1, C1_OC * 16}, s));
  // da1 = convT(da2, W2) * (a1 > 0), one launch per output parity class
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    ARL_TRY((launch_gemm<64, 16, 32, 4, 1, GS, GS>(ConvT2ClassA<C2_OC, C1_OC>{da2, py, px},
                                                   ConvT2ClassW<C2_OC, C1_OC>{P + net.o_c2W, py, px},
                                                   EpiT2Class<C1_OC>{da1, a1, py, px}, S * 100, C1_OC, C2_OC * 4, 1,
                                                   s)));
  }
  // conv1: dW1 / db1 straight from the state ring (the window's T steps)
  const StatesIm2col ring{net.at<float>(net.w_frames), net.at<int64_t>(net.w_ctl), n, net.R, 0};
  ARL_TRY((launch_gemm<32, 64, 32, 2, 2, GK, GM>(ConvDyT{da1, C1_OC, C1_P}, OnesCol<StatesIm2col>{ring, 256},
                                                 EpiSlab{slab, C1_OC, 257}, C1_OC, 257, S * C1_P, pl.c1_w, s)));
  return launch_reduce_grad(slab, pl.c1_w, C1_OC, 257, MapDense{G, net.o_c1W, net.o_c1b, -1, 256}, s);
}

}  // namespace arl
