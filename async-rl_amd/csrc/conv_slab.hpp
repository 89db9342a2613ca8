// Layout of the per-workgroup partial slab of conv_bwd_kernel (conv_bwd.hip)
// and the map from a reduced slab entry to the flat gradient; shared by
// reduce_conv_bwd_kernel and the learner's single reduce (net.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

constexpr int SLAB_W2 = C2_OC * 256;       // 8192: dW2 [oc][ic*16 + ky*4 + kx]
constexpr int SLAB_B2 = SLAB_W2;           // +32
constexpr int SLAB_W1 = SLAB_B2 + C2_OC;   // 8224: D1^T[k][oc], 4096 (integer pixels: /255 on the way out)
constexpr int SLAB_B1 = SLAB_W1 + 256 * 16;
constexpr int SLAB = SLAB_B1 + 16;         // 12336 floats per block

// returns the f32 gradient value written (for the fused squared norm)
// (RGB nets: dW1 rows of the zero pad plane ic = 0 are dropped, W1 is (16, 3, 8, 8))
__device__ inline float conv_slab_put(int o, double v, float* gW2, float* gb2, float* gW1, float* gb1, int rgb) {
  float g;
  if (o < SLAB_B2) { g = (float)v; gW2[o] = g; }
  else if (o < SLAB_W1) { g = (float)v; gb2[o - SLAB_B2] = g; }
  else if (o < SLAB_B1) {
    const int kk = o - SLAB_W1, k = kk >> 4, oc = kk & 15;
    g = (float)(v / 255.0);
    if (!rgb) gW1[oc * 256 + k] = g;
    else if (k >= 64) gW1[oc * 192 + k - 64] = g;
    else g = 0.f;
  } else { g = (float)v; gb1[o - SLAB_B1] = g; }
  return g;
}

}  // namespace arl
