// A3CFF with the Nature DQN head on gfx950.
//
// Reference: dqn_head.py:6-28 (NatureDQNHead: conv 4->32 k8 s4, conv 32->64
// k4 s2, conv 64->64 k3 s1, Linear 3136->512, ReLU after each), used in place
// of NIPSDQNHead inside a3c_ale.py:28-40 (A3CFF) with FCSoftmaxPolicy(512, A)
// and FCVFunction(512); backward of the window loss as a3c.py:129-130.
//
// Every contraction is an implicit GEMM on the exact-f32 MFMA template
// (gemm.hpp, v_mfma_f32_16x16x4_f32) with an accessor that gathers its operand
// on the fly:
//   forward   conv1  M = 400 n  x 32 x K 256   im2col straight from the uint8
//                                              frame ring (dqn_phi /255 per byte)
//             conv2  M =  81 n  x 64 x K 512   im2col of a1
//             conv3  M =  49 n  x 64 x K 576   im2col of a2
//             FC     M = n x 512 x K 3136      split-K slabs + bias/ReLU reduce
//   backward  heads dW (ones column = bias), dfc = dh * (h > 0)
//             FC dW (split-K over samples), da3 = dfc W * (a3 > 0)
//             conv3 dW (split-K over sample x position), da2 = convT(da3) * (a2 > 0)
//             conv2 dW, da1 = stride-2 convT as 4 output-parity classes
//                   (K = 64 oc x 2 x 2 taps each, no structural zeros) * (a1 > 0)
//             conv1 dW from the ring (no dX: the input is data)
// Split-K slabs are summed in f64 in slice order (reduce_grad_kernel), so the
// gradient is deterministic and replicas stay bitwise identical.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"
#include "gemm.hpp"
#include "layers.hpp"

namespace arl {

namespace {

constexpr int NFC_SPLIT = 8;   // FC forward split-K (K = 3136 -> 8 slices of 416)

// dqn_phi.py:14-16: f32(byte) / 255 as an IEEE f32 division
__device__ inline float phi_scale(uint32_t b) { return div255((float)b); }

// conv1 im2col from the frame ring (ale.py:135,155-158 stack, oldest plane
// first, planes older than the env's last reset read as 0).  Sample s =
// (t - t0) * n + e (window step t, env e); m = s * 400 + p; k = ic*64 + ky*8 + kx.
struct RingIm2col {
  const uint8_t* __restrict__ frames; const uint8_t* __restrict__ nvalid; const int64_t* __restrict__ ctl;
  int n, R, t0;
  // byte address of (m, k) with k % 4 == 0 handled by the caller; null = zero plane
  __device__ const uint8_t* addr(int m, int k) const {
    const int s = m / NP1, p = m - s * NP1;
    const int tt = s / n, e = s - tt * n;
    const int rs = (int)((ctl[CTL_STEP] + t0 + tt) % R);
    const int ic = k >> 6;
    if (ic < 4 - (int)nvalid[(int64_t)rs * n + e]) return nullptr;
    const int slot = (rs + R - 3 + ic) % R;
    const int oy = p / 20, ox = p - oy * 20, ky = (k >> 3) & 7, kx = k & 7;
    return frames + ((int64_t)slot * n + e) * PLANE + (4 * oy + ky) * 84 + 4 * ox + kx;
  }
  __device__ float load(int m, int k) const {
    const uint8_t* a = addr(m, k);
    return a ? phi_scale(*a) : 0.f;
  }
  __device__ float4 load4(int m, int k) const {   // 4 consecutive kx: one aligned u32 (84 % 4 == 0)
    const uint8_t* a = addr(m, k);
    if (!a) return make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t w = *reinterpret_cast<const uint32_t*>(a);
    return make_float4(phi_scale(w & 255u), phi_scale((w >> 8) & 255u), phi_scale((w >> 16) & 255u),
                       phi_scale(w >> 24));
  }
};

// stride-1 transposed conv (conv3 backward): A(m, k) = dy[s][oc][y-ky][x-kx],
// m = s*IH*IH + y*IH + x, k = oc*KS*KS + ky*KS + kx
template <int OC, int OH, int KS, int IH>
struct ConvT1A {
  const float* __restrict__ dy;
  __device__ float load(int m, int k) const {
    constexpr int IP = IH * IH, KK = KS * KS;
    const int s = m / IP, q = m - s * IP, y = q / IH, x = q - y * IH;
    const int oc = k / KK, r = k - oc * KK, ky = r / KS, kx = r - ky * KS;
    const int oy = y - ky, ox = x - kx;
    if (oy < 0 || oy >= OH || ox < 0 || ox >= OH) return 0.f;
    return dy[((int64_t)s * OC + oc) * (OH * OH) + oy * OH + ox];
  }
};
// B(k, ic) = W[oc][ic][ky][kx] with k = oc*KK + (ky*KS + kx)
struct ConvTW {
  const float* __restrict__ w; int IC, KK;
  __device__ float load(int k, int ic) const {
    const int oc = k / KK, r = k - oc * KK;
    return w[((int64_t)oc * IC + ic) * KK + r];
  }
};

// out[s][n][p] = mask > 0 ? v : 0  (ReLU backward into a conv activation layout)
struct EpiConvMask {
  float* __restrict__ out; const float* __restrict__ mask; int OC, P;
  __device__ void store(int m, int n, float v, int) const {
    const int s = m / P, p = m - s * P;
    const int64_t i = ((int64_t)s * OC + n) * P + p;
    out[i] = mask[i] > 0.f ? v : 0.f;
  }
};
#define ARL_TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return _e; } while (0)

struct NPlans {
  int heads_w, fc_w, c3_w, c2_w, c1_w;
};

NPlans nature_plans(const Net& net) {
  const int S = net.T * net.N;
  NPlans p;
  p.heads_w = effective_splits<32>(S, plan_splits(ceil_div(net.A + 1, 16) * ceil_div(NHID + 1, 64), S, 32));
  p.fc_w = effective_splits<32>(S, plan_splits(ceil_div(NHID, 64) * ceil_div(NA3 + 1, 64), S, 32));
  const int64_t K3 = (int64_t)S * NP3, K2 = (int64_t)S * NP2, K1 = (int64_t)S * NP1;
  p.c3_w = effective_splits<32>((int)K3, plan_splits(ceil_div(64 * 9 + 1, 64), K3, 32));
  p.c2_w = effective_splits<32>((int)K2, plan_splits(ceil_div(32 * 16 + 1, 64), K2, 32));
  p.c1_w = effective_splits<32>((int)K1, plan_splits(ceil_div(4 * 64 + 1, 64), K1, 32));
  return p;
}

// ---------------------------------------------------------------- forward pieces
hipError_t conv23_fwd(const Net& net, int n, const float* a1, float* a2, float* a3, hipStream_t s) {
  const float* P = net.p;
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GS, GK>(Im2col<NC1, 20, 4, 2, 9>{a1}, WeightT{P + net.o_c2W, NC1 * 16},
                                                 EpiConv{a2, P + net.o_c2b, NC2, NP2}, n * NP2, NC2, NC1 * 16, 1, s)));
  return launch_gemm<64, 64, 32, 2, 2, GS, GK>(Im2col<NC2, 9, 3, 1, 7>{a2}, WeightT{P + net.o_c3W, NC2 * 9},
                                               EpiConv{a3, P + net.o_c3b, NC3, NP3}, n * NP3, NC3, NC2 * 9, 1, s);
}

hipError_t fc_fwd(const Net& net, int n, const float* a3, float* h, hipStream_t s) {
  const float* P = net.p;
  float* slab = net.at<float>(net.w_slab);
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GK, GK>(RowMajor{a3, NA3}, WeightT{P + net.o_fcW, NA3},
                                                 EpiSlab{slab, n, NHID}, n, NHID, NA3, NFC_SPLIT, s)));
  return launch_reduce_grad(slab, effective_splits<32>(NA3, NFC_SPLIT), n, NHID,
                            MapBiasRelu{h, P + net.o_fcb, NHID}, s);
}

hipError_t policy_at(const Net& net, int t, int n, int mode, const float* h, hipStream_t s) {
  const float* P = net.p;
  const int A = net.A;
  const int64_t o = (int64_t)t * net.N;
  const bool draw = mode != 0;
  return launch_policy(h, n, P + net.o_piW, P + net.o_pib, P + net.o_vW, P + net.o_vb, A, net.seed,
                       net.at<int64_t>(net.w_ctl), t, net.env_offset, mode, net.at<float>(net.w_logits) + o * A,
                       net.at<float>(net.w_probs) + o * A, net.at<float>(net.w_logp) + o * A,
                       net.at<float>(net.w_v) + o, net.at<float>(net.w_ent) + o,
                       draw ? net.at<int32_t>(net.w_act) + o : nullptr,
                       draw ? net.at<float>(net.w_logpa) + o : nullptr, s, NHID);
}

hipError_t conv1_fwd_ring(const Net& net, int t, float* a1, hipStream_t s) {
  const int n = net.N;
  const float* P = net.p;
  return launch_gemm<64, 32, 32, 2, 2, GK, GK>(
      RingIm2col{net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid), net.at<int64_t>(net.w_ctl), n,
                 net.R, t},
      WeightT{P + net.o_c1W, 256}, EpiConv{a1, P + net.o_c1b, NC1, NP1}, n * NP1, NC1, 256, 1, s);
}

// ---------------------------------------------------------------- backward pieces
hipError_t fc_bwd(Net& net, hipStream_t s) {
  const int S = net.T * net.N;
  const NPlans pl = nature_plans(net);
  float* slab = net.at<float>(net.w_slab);
  const float* dfc = net.at<float>(net.w_dfc);
  const float* a3 = net.at<float>(net.w_a3);
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GM, GM>(ColMajor{dfc, NHID}, OnesColB{a3, NA3}, EpiSlab{slab, NHID, NA3 + 1},
                                                 NHID, NA3 + 1, S, pl.fc_w, s)));
  ARL_TRY(launch_reduce_grad(slab, pl.fc_w, NHID, NA3 + 1, MapDense{net.g, net.o_fcW, net.o_fcb, -1, NA3}, s));
  return launch_gemm<64, 64, 32, 2, 2, GK, GM>(RowMajor{dfc, NHID}, RowMajor{net.p + net.o_fcW, NA3},
                                               EpiMask{net.at<float>(net.w_da3), a3, NA3}, S, NA3, NHID, 1, s);
}

hipError_t conv_bwd(Net& net, hipStream_t s) {
  const int n = net.N, S = net.T * n;
  const NPlans pl = nature_plans(net);
  const float* P = net.p;
  float* G = net.g;
  float* slab = net.at<float>(net.w_slab);
  const float* a1 = net.at<float>(net.w_a1);
  const float* a2 = net.at<float>(net.w_a2);
  float* da1 = net.at<float>(net.w_da1);
  float* da2 = net.at<float>(net.w_da2);
  const float* da3 = net.at<float>(net.w_da3);
  // conv3: dW3 / db3 over (sample, position), then da2 = convT(da3, W3) * (a2 > 0)
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GS, GS>(ConvDyT{da3, NC3, NP3},
                                                 OnesCol<Im2col<NC2, 9, 3, 1, 7>>{{a2}, NC2 * 9},
                                                 EpiSlab{slab, NC3, NC2 * 9 + 1}, NC3, NC2 * 9 + 1, S * NP3, pl.c3_w,
                                                 s)));
  ARL_TRY(launch_reduce_grad(slab, pl.c3_w, NC3, NC2 * 9 + 1, MapDense{G, net.o_c3W, net.o_c3b, -1, NC2 * 9}, s));
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GS, GS>(ConvT1A<NC3, 7, 3, 9>{da3}, ConvTW{P + net.o_c3W, NC2, 9},
                                                 EpiConvMask{da2, a2, NC2, NP2}, S * NP2, NC2, NC3 * 9, 1, s)));
  // conv2: dW2 / db2, then da1 = convT(da2, W2) * (a1 > 0), one launch per output parity class
  ARL_TRY((launch_gemm<64, 64, 32, 2, 2, GS, GS>(ConvDyT{da2, NC2, NP2},
                                                 OnesCol<Im2col<NC1, 20, 4, 2, 9>>{{a1}, NC1 * 16},
                                                 EpiSlab{slab, NC2, NC1 * 16 + 1}, NC2, NC1 * 16 + 1, S * NP2,
                                                 pl.c2_w, s)));
  ARL_TRY(launch_reduce_grad(slab, pl.c2_w, NC2, NC1 * 16 + 1, MapDense{G, net.o_c2W, net.o_c2b, -1, NC1 * 16}, s));
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    ARL_TRY((launch_gemm<64, 32, 32, 2, 2, GS, GS>(ConvT2ClassA<NC2, NC1>{da2, py, px}, ConvT2ClassW<NC2, NC1>{P + net.o_c2W, py, px},
                                                   EpiT2Class<NC1>{da1, a1, py, px}, S * 100, NC1, NC2 * 4, 1, s)));
  }
  // conv1: dW1 / db1 straight from the frame ring (the window's T steps)
  RingIm2col ring{net.at<uint8_t>(net.w_frames), net.at<uint8_t>(net.w_nvalid), net.at<int64_t>(net.w_ctl), n,
                  net.R, 0};
  ARL_TRY((launch_gemm<32, 64, 32, 2, 2, GK, GM>(ConvDyT{da1, NC1, NP1}, OnesCol<RingIm2col>{ring, 256},
                                                 EpiSlab{slab, NC1, 257}, NC1, 257, S * NP1, pl.c1_w, s)));
  return launch_reduce_grad(slab, pl.c1_w, NC1, 257, MapDense{G, net.o_c1W, net.o_c1b, -1, 256}, s);
}

}  // namespace

int64_t nature_slab_floats(const Net& net) {
  const NPlans pl = nature_plans(net);
  int64_t m = (int64_t)NFC_SPLIT * net.N * NHID;
  m = std::max(m, (int64_t)pl.heads_w * (net.A + 1) * (NHID + 1));
  m = std::max(m, (int64_t)pl.fc_w * NHID * (NA3 + 1));
  m = std::max(m, (int64_t)pl.c3_w * NC3 * (NC2 * 9 + 1));
  m = std::max(m, (int64_t)pl.c2_w * NC2 * (NC1 * 16 + 1));
  m = std::max(m, (int64_t)pl.c1_w * NC1 * 257);
  return m;
}

hipError_t nature_act(Net& net, int t, int mode, hipStream_t s) {
  const int n = net.N;
  float* a1 = net.at<float>(net.w_a1) + (int64_t)t * n * NA1;
  float* a2 = net.at<float>(net.w_a2) + (int64_t)t * n * NA2;
  float* a3 = net.at<float>(net.w_a3) + (int64_t)t * n * NA3;
  float* h = net.at<float>(net.w_hfc) + (int64_t)t * n * NHID;
  ARL_TRY(conv1_fwd_ring(net, t, a1, s));
  ARL_TRY(conv23_fwd(net, n, a1, a2, a3, s));
  ARL_TRY(fc_fwd(net, n, a3, h, s));
  return policy_at(net, t, n, t < net.T ? mode : 0, h, s);
}

// pi_and_v on explicit (n, 4, 84, 84) f32 states; results in slot T
hipError_t nature_forward_f32(Net& net, const float* x, int n, int mode, hipStream_t s) {
  if (n > net.N) return hipErrorInvalidValue;
  const int T = net.T, N = net.N;
  float* a1 = net.at<float>(net.w_a1) + (int64_t)T * N * NA1;
  float* a2 = net.at<float>(net.w_a2) + (int64_t)T * N * NA2;
  float* a3 = net.at<float>(net.w_a3) + (int64_t)T * N * NA3;
  float* h = net.at<float>(net.w_hfc) + (int64_t)T * N * NHID;
  const float* P = net.p;
  ARL_TRY((launch_gemm<64, 32, 32, 2, 2, GS, GK>(Im2col<4, 84, 8, 4, 20>{x}, WeightT{P + net.o_c1W, 256},
                                                 EpiConv{a1, P + net.o_c1b, NC1, NP1}, n * NP1, NC1, 256, 1, s)));
  ARL_TRY(conv23_fwd(net, n, a1, a2, a3, s));
  ARL_TRY(fc_fwd(net, n, a3, h, s));
  return launch_policy_args(h, n, states_policy_args(net, mode), s, NHID);
}

hipError_t nature_learn(Net& net, double gamma, float beta, float vcoef, int clip_reward, hipStream_t s) {
  const int n = net.N, T = net.T, A = net.A, S = T * n;
  const NPlans pl = nature_plans(net);
  float* slab = net.at<float>(net.w_slab);
  float* dl = net.at<float>(net.w_dlogits);
  float* dv = net.at<float>(net.w_dv);
  // n-step returns + loss gradient (a3c.py:82-126)
  ARL_TRY(launch_returns(net.at<float>(net.w_rewards), net.at<uint8_t>(net.w_dones), net.at<float>(net.w_v),
                         net.at<float>(net.w_probs), net.at<float>(net.w_logp), net.at<int32_t>(net.w_act), T, n, A,
                         gamma, beta, vcoef, clip_reward, dl, dv, net.at<float>(net.w_loss), s,
                         net.at<int64_t>(net.w_ctl), net.pi_coef, net.keep_scale));
  const float* h = net.at<float>(net.w_hfc);
  // heads: weight grads (ones column = bias) and dfc = dh * (h > 0)
  ARL_TRY((launch_gemm<16, 64, 32, 1, 4, GS, GM>(HeadsGA{dl, dv, A}, OnesColB{h, NHID},
                                                 EpiSlab{slab, A + 1, NHID + 1}, A + 1, NHID + 1, S, pl.heads_w, s)));
  ARL_TRY(launch_reduce_grad(slab, pl.heads_w, A + 1, NHID + 1,
                             MapHeads{net.g, net.o_piW, net.o_pib, net.o_vW, net.o_vb, A, NHID}, s));
  ARL_TRY(launch_heads_bwd(dl, dv, net.p + net.o_piW, net.p + net.o_vW, A, NHID, h, net.at<float>(net.w_dfc), S, s));
  ARL_TRY(fc_bwd(net, s));
  return conv_bwd(net, s);
}

hipError_t nature_stage(Net& net, int stage, int t, hipStream_t s) {
  const int n = net.N;
  float* a1 = net.at<float>(net.w_a1) + (int64_t)t * n * NA1;
  float* a2 = net.at<float>(net.w_a2) + (int64_t)t * n * NA2;
  float* a3 = net.at<float>(net.w_a3) + (int64_t)t * n * NA3;
  float* h = net.at<float>(net.w_hfc) + (int64_t)t * n * NHID;
  switch (stage) {
    case STAGE_CONV_FWD:
      ARL_TRY(conv1_fwd_ring(net, t, a1, s));
      return conv23_fwd(net, n, a1, a2, a3, s);
    case STAGE_FC_FWD:
      return fc_fwd(net, n, a3, h, s);
    case STAGE_POLICY:
      return policy_at(net, t, n, 0, h, s);
    case STAGE_FC_BWD:
      return fc_bwd(net, s);
    case STAGE_CONV_BWD:
      return conv_bwd(net, s);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace arl
