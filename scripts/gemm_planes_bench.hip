// Microbenchmark + check of gemm_planes_kernel (pre-split bf16 planes) on the
// FC shapes of the NIPS head at N = 256 envs, T = 5 (S = 1280 samples):
//   fc fwd  C[e][j]  = sum_c a2[e][c] W[j][c]      M = 256,  N = 256,  K = 2592 (split-K)
//   da2     C[s][c]  = sum_j dfc[s][j] W[j][c]     M = 1280, N = 2592, K = 256
//   dW      C[j][c]  = sum_s dfc[s][j] a2[s][c]    M = 256,  N = 2593 (ones column), K = 1280 (split-K)
// against the exact-f32 gemm_kernel on the same data.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I async-rl_amd/csrc scripts/gemm_planes_bench.hip -o scripts/gemm_planes_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm_planes.hpp"
#include "layers.hpp"

using namespace arl;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct EpiPlain {
  static constexpr bool kRow4 = false;
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

static void fill(std::vector<float>& v, unsigned seed, float lo, float hi) {
  srand(seed);
  for (auto& x : v) x = lo + (hi - lo) * (rand() / (float)RAND_MAX);
}

static void cmp(const char* what, float* d_a, float* d_b, size_t n) {
  std::vector<float> a(n), b(n);
  CK(hipMemcpy(a.data(), d_a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), d_b, n * 4, hipMemcpyDeviceToHost));
  double m = 0, s = 0;
  for (size_t i = 0; i < n; ++i) { m = fmax(m, fabs((double)a[i] - b[i])); s = fmax(s, fabs((double)b[i])); }
  printf("   %s: max |planes - f32| / max |f32| = %.2e\n", what, m / (s > 0 ? s : 1));
}

int main() {
  const int S = 1280, H = 256, K2 = 2592, LD2 = 2600, NE = 256;
  std::vector<float> dfc(S * H), a2(S * K2), W(H * K2);
  fill(dfc, 1, -1.f, 1.f); fill(a2, 2, -0.5f, 1.f); fill(W, 3, -0.02f, 0.02f);
  for (auto& x : a2) x = x > 0.f ? x : 0.f;
  float *d_dfc, *d_a2, *d_W, *d_o1, *d_o2, *d_slab;
  uint16_t *p_dfc, *p_a2, *p_W;
  CK(hipMalloc(&d_dfc, dfc.size() * 4)); CK(hipMalloc(&d_a2, a2.size() * 4)); CK(hipMalloc(&d_W, W.size() * 4));
  CK(hipMalloc(&d_o1, (size_t)S * K2 * 4 + 64)); CK(hipMalloc(&d_o2, (size_t)S * K2 * 4 + 64));
  CK(hipMalloc(&d_slab, (size_t)64 * H * (K2 + 1) * 4));
  const int64_t sd = (int64_t)S * H, sa = (int64_t)S * LD2, sw = (int64_t)H * K2;
  CK(hipMalloc(&p_dfc, 3 * sd * 2)); CK(hipMalloc(&p_a2, 3 * sa * 2)); CK(hipMalloc(&p_W, 3 * sw * 2));
  CK(hipMemcpy(d_dfc, dfc.data(), dfc.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_a2, a2.data(), a2.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_W, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(p_a2, 0, 3 * sa * 2));
  CK(launch_split_planes(d_dfc, S, H, H, p_dfc, H, sd, 0));
  CK(launch_split_planes(d_a2, S, K2, K2, p_a2, LD2, sa, 0));
  CK(launch_split_planes(d_W, H, K2, K2, p_W, K2, sw, 0));
  {  // ones column of a2 (bias gradient): h-plane col 2592 = bf16 1.0
    std::vector<uint16_t> one(S, 0x3F80);
    CK(hipMemcpy2D(p_a2 + K2, LD2 * 2, one.data(), 2, 2, S, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  const Planes Pdfc{p_dfc, sd, H}, Pa2{p_a2, sa, LD2}, PW{p_W, sw, K2};
  hipStream_t s = 0;
  float t1, t2;

  printf("== fc fwd  M=%d N=%d K=%d (split-K 8, slab only)\n", NE, H, K2);
  t1 = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GK, GK>(RowMajor{d_a2, K2}, WeightT{d_W, K2}, EpiSlab{d_o1, NE, H}, NE, H, K2, 8, s); });
  t2 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, false, false>(Pa2, PW, EpiSlab{d_o2, NE, H}, NE, H, K2, 8, s); });
  printf("f32 %8.2f us   planes 64x64x64 %8.2f us\n", t1, t2);
  launch_gemm<64, 64, 32, 2, 2, GK, GK>(RowMajor{d_a2, K2}, WeightT{d_W, K2}, EpiSlab{d_o1, NE, H}, NE, H, K2, 1, s);
  launch_gemm_planes<64, 64, 64, 2, 2, false, false>(Pa2, PW, EpiSlab{d_o2, NE, H}, NE, H, K2, 1, s);
  cmp("fc fwd", d_o2, d_o1, (size_t)NE * H);
  for (int sp : {4, 16}) {
    t2 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, false, false>(Pa2, PW, EpiSlab{d_o2, NE, H}, NE, H, K2, sp, s); });
    float t3 = timeit([&] { launch_gemm_planes<32, 64, 64, 2, 2, false, false>(Pa2, PW, EpiSlab{d_o2, NE, H}, NE, H, K2, sp, s); });
    printf("splits %2d: planes 64x64 %8.2f us  32x64 %8.2f us\n", sp, t2, t3);
  }

  printf("== da2  M=%d N=%d K=%d\n", S, K2, H);
  t1 = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GK, GM>(RowMajor{d_dfc, H}, RowMajor{d_W, K2}, EpiMask{d_o1, d_a2, K2}, S, K2, H, 1, s); });
  t2 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, false, true>(Pdfc, PW, EpiMask{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  printf("f32 %8.2f us   planes 64x64x64 %8.2f us\n", t1, t2);
  cmp("da2", d_o2, d_o1, (size_t)S * K2);
  t2 = timeit([&] { launch_gemm_planes<64, 128, 64, 2, 2, false, true>(Pdfc, PW, EpiMask{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  float t3 = timeit([&] { launch_gemm_planes<128, 64, 64, 2, 2, false, true>(Pdfc, PW, EpiMask{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  float t4 = timeit([&] { launch_gemm_planes<64, 64, 32, 2, 2, false, true>(Pdfc, PW, EpiMask{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  printf("planes 64x128x64 %8.2f us  128x64x64 %8.2f us  64x64x32 %8.2f us\n", t2, t3, t4);
  t2 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, false, true>(Pdfc, PW, EpiMask4{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  t3 = timeit([&] { launch_gemm_planes<64, 128, 64, 2, 2, false, true>(Pdfc, PW, EpiMask4{d_o2, d_a2, K2}, S, K2, H, 1, s); });
  t4 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, false, true>(Pdfc, PW, EpiPlain{d_o2, K2}, S, K2, H, 1, s); });
  printf("row epilogue: planes 64x64x64 %8.2f us  64x128x64 %8.2f us;  plain MFMA-layout store %8.2f us\n", t2, t3, t4);
  launch_gemm_planes<64, 64, 64, 2, 2, false, true>(Pdfc, PW, EpiMask4{d_o2, d_a2, K2}, S, K2, H, 1, s);
  cmp("da2 (row epilogue)", d_o2, d_o1, (size_t)S * K2);

  printf("== dW  M=%d N=%d K=%d (split-K, slab only)\n", H, K2 + 1, S);
  for (int sp : {2, 4, 6, 8, 10, 16}) {
    t1 = timeit([&] { launch_gemm<64, 64, 32, 2, 2, GM, GM>(ColMajor{d_dfc, H}, OnesColB{d_a2, K2}, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    t2 = timeit([&] { launch_gemm_planes<64, 64, 64, 2, 2, true, true>(Pdfc, Pa2, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    t3 = timeit([&] { launch_gemm_planes<64, 128, 64, 2, 2, true, true>(Pdfc, Pa2, EpiSlab{d_slab, H, K2 + 1}, H, K2 + 1, S, sp, s); });
    printf("splits %2d: f32 %8.2f us   planes 64x64x64 %8.2f us  64x128x64 %8.2f us\n", sp, t1, t2, t3);
  }
  launch_gemm<64, 64, 32, 2, 2, GM, GM>(ColMajor{d_dfc, H}, OnesColB{d_a2, K2}, EpiSlab{d_o1, H, K2 + 1}, H, K2 + 1, S, 1, s);
  launch_gemm_planes<64, 64, 64, 2, 2, true, true>(Pdfc, Pa2, EpiSlab{d_o2, H, K2 + 1}, H, K2 + 1, S, 1, s);
  cmp("dW (+bias column)", d_o2, d_o1, (size_t)H * (K2 + 1));
  CK(hipDeviceSynchronize());
  return 0;
}
