// Microbenchmark of the FC-backward GEMM shapes (N = 256 envs x T = 5):
//   da2 = (dfc . W) * (a2 > 0)        M = 1280, N = 2592, K = 256
//   dW  = dfc^T . [a2 | 1] (split-K)  M = 256,  N = 2593, K = 1280
// for the exact-f32 and bf16x6 GEMM variants.  Timing only (hipEvents, 50
// back-to-back launches); outputs are checked against each other.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I async-rl_amd/csrc scripts/gemm_bench.hip -o /tmp/gemm_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "layers.hpp"

using namespace arl;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct EpiPlain {
  float* __restrict__ out; int ld;
  __device__ void store(int m, int n, float v, int) const { out[(int64_t)m * ld + n] = v; }
};

template <class F>
static float timeit(F f, int reps = 50) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1e3f * ms / reps;
}

static void fill(std::vector<float>& v, unsigned seed, float lo = -1.f, float hi = 1.f) {
  srand(seed);
  for (auto& x : v) x = lo + (hi - lo) * (rand() / (float)RAND_MAX);
}

static double maxrel(const std::vector<float>& a, const std::vector<float>& b) {
  double m = 0, s = 0;
  for (size_t i = 0; i < a.size(); ++i) { m = fmax(m, fabs((double)a[i] - b[i])); s = fmax(s, fabs((double)b[i])); }
  return m / (s > 0 ? s : 1);
}

int main() {
  const int S = 1280, H = 256, K2 = 2592;
  std::vector<float> dfc(S * H), a2(S * K2), W(H * K2);
  fill(dfc, 1); fill(a2, 2, -0.5f, 1.f); fill(W, 3);
  float *d_dfc, *d_a2, *d_W, *d_out, *d_out2, *d_slab;
  CK(hipMalloc(&d_dfc, dfc.size() * 4)); CK(hipMalloc(&d_a2, a2.size() * 4)); CK(hipMalloc(&d_W, W.size() * 4));
  CK(hipMalloc(&d_out, (size_t)S * K2 * 4)); CK(hipMalloc(&d_out2, (size_t)S * K2 * 4));
  CK(hipMalloc(&d_slab, (size_t)16 * H * (K2 + 1) * 4));
  CK(hipMemcpy(d_dfc, dfc.data(), dfc.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_a2, a2.data(), a2.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_W, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  hipStream_t s = 0;
  std::vector<float> r1((size_t)S * K2), r2((size_t)S * K2);

  printf("== da2: M=%d N=%d K=%d\n", S, K2, H);
  float t;
  t = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GK, GM>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_out, d_a2, K2}, S, K2, H, 1, s); });
  printf("f32 64x64 GK/GM EpiMask       %8.2f us\n", t);
  CK(hipMemcpy(r1.data(), d_out, r1.size() * 4, hipMemcpyDeviceToHost));
  t = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GK, GM>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiPlain{d_out2, K2}, S, K2, H, 1, s); });
  printf("f32 64x64 GK/GM plain store   %8.2f us\n", t);
  t = timeit([&] { launch_gemm_x6<64, 128, 32, 2, 2, GK, GS>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_out2, d_a2, K2}, S, K2, H, 1, s); });
  CK(hipMemcpy(r2.data(), d_out2, r2.size() * 4, hipMemcpyDeviceToHost));
  printf("x6 64x128 GK/GS EpiMask       %8.2f us   maxrel vs f32 %.2e\n", t, maxrel(r2, r1));
  t = timeit([&] { launch_gemm_x6<64, 64, 32, 2, 2, GK, GS>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_out2, d_a2, K2}, S, K2, H, 1, s); });
  printf("x6 64x64 GK/GS EpiMask        %8.2f us\n", t);
  t = timeit([&] { launch_gemm_x6<64, 64, 64, 2, 2, GK, GS>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_out2, d_a2, K2}, S, K2, H, 1, s); });
  printf("x6 64x64 BK64 GK/GS EpiMask   %8.2f us\n", t);
  t = timeit([&] { launch_gemm_x6<128, 64, 32, 2, 2, GK, GS>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_out2, d_a2, K2}, S, K2, H, 1, s); });
  printf("x6 128x64 GK/GS EpiMask       %8.2f us\n", t);
  t = timeit([&] { launch_gemm_x6<64, 128, 32, 2, 2, GK, GS>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiPlain{d_out2, K2}, S, K2, H, 1, s); });
  printf("x6 64x128 GK/GS plain store   %8.2f us\n", t);

  printf("== dW: M=%d N=%d K=%d (split-K slabs)\n", H, K2 + 1, S);
  for (int sp : {1, 2, 4, 6, 8, 12}) {
    t = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GM, GM>(ColMajor{d_dfc, H}, OnesColB{d_a2, K2}, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    float t2 = timeit([&] { launch_gemm_x6<64, 128, 32, 2, 2, GS, GS>(ColMajor{d_dfc, H}, OnesColB{d_a2, K2}, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    float t3 = timeit([&] { launch_gemm_x6<64, 64, 64, 2, 2, GS, GS>(ColMajor{d_dfc, H}, OnesColB{d_a2, K2}, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    printf("splits %2d: f32 64x64 %8.2f us   x6 64x128 %8.2f us   x6 64x64 BK64 %8.2f us\n", sp, t, t2, t3);
  }
  return 0;
}
