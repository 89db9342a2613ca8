// Launch-floor microbenchmark: back-to-back tiny kernels captured in a HIP
// graph on one stream, timed with HIP events (per-kernel cost of the kernel
// boundary on gfx950, as a function of grid size and of whether the kernel
// writes memory).
//   hipcc --offload-arch=gfx950 -O3 scripts/launch_floor.hip -o scripts/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_kernel() {}
__global__ void write_kernel(float* p) { p[blockIdx.x * blockDim.x + threadIdx.x] = 1.f; }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* buf;
  CK(hipMalloc(&buf, 1 << 26));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int K = 200;
  const int grids[] = {1, 16, 256, 1024, 4096};
  for (int mode = 0; mode < 2; ++mode)
    for (int gi = 0; gi < 5; ++gi) {
      const int G = grids[gi];
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < K; ++i) {
        if (mode == 0) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), 0, s);
        else hipLaunchKernelGGL(write_kernel, dim3(G), dim3(256), 0, s, buf);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(a, s));
      for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"kernel\": \"%s\", \"grid\": %d, \"block\": 256, \"us_per_kernel\": %.3f}\n",
             mode ? "write" : "empty", G, 1e3 * ms / (10 * K));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  return 0;
}
