// Do independent branches of a captured HIP graph run concurrently on gfx950?
// Two chains of K latency-bound kernels (1 workgroup spinning ~5 us each),
// captured (a) on one stream, (b) on two streams forked / joined by events.
// If the graph runs branches concurrently, (b) takes about half of (a).
//   hipcc --offload-arch=gfx950 -O3 scripts/graph_branches.hip -o scripts/graph_branches
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin_kernel(long long cycles, float* out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) out[blockIdx.x] = 1.f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  float* buf;
  CK(hipMalloc(&buf, 1 << 20));
  hipEvent_t a, b, fork, join;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  int wclk = 0;
  CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));   // kHz
  const long long cyc = (long long)wclk * 5 / 1000;                          // ~5 us
  const int K = 50;
  for (int grid : {1, 128}) {
    for (int mode = 0; mode < 2; ++mode) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
      if (mode == 0) {
        for (int i = 0; i < 2 * K; ++i) hipLaunchKernelGGL(spin_kernel, dim3(grid), dim3(64), 0, s0, cyc, buf);
      } else {
        CK(hipEventRecord(fork, s0));
        CK(hipStreamWaitEvent(s1, fork, 0));
        for (int i = 0; i < K; ++i) {
          hipLaunchKernelGGL(spin_kernel, dim3(grid), dim3(64), 0, s0, cyc, buf);
          hipLaunchKernelGGL(spin_kernel, dim3(grid), dim3(64), 0, s1, cyc, buf + 4096);
        }
        CK(hipEventRecord(join, s1));
        CK(hipStreamWaitEvent(s0, join, 0));
      }
      CK(hipStreamEndCapture(s0, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 2; ++w) CK(hipGraphLaunch(ge, s0));
      CK(hipEventRecord(a, s0));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s0));
      CK(hipEventRecord(b, s0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"grid\": %d, \"branches\": %d, \"kernels\": %d, \"us_per_kernel\": %.3f}\n", grid, mode + 1, 2 * K,
             1e3 * ms / (5 * 2 * K));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
