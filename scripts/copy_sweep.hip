// HBM stream-copy sweep (measurement only): which copy form reaches the chip's achievable HBM rate
// (MI355X_MICROARCH.md: float4 copy 6.29 TB/s).  hipcc --offload-arch=gfx950 -O3 copy_sweep.hip -o copy_sweep
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

// U float4 per lane, lane-linear (wave instruction = 1 KB contiguous), one-shot grid
template <int U, bool NT>
__global__ void copy_u(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * blockDim.x;
    if (i < n4) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * blockDim.x;
    if (i < n4) {
      if (NT) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

// persistent grid-stride, U in flight
template <int U, bool NT>
__global__ void copy_gs(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n4; base += step) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n4) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n4) {
        if (NT) __builtin_nontemporal_store(v[u], d + i);
        else d[i] = v[u];
      }
    }
  }
}

__global__ void read_only(const f4* __restrict__ s, float* __restrict__ out, int64_t n4) {
  f4 a = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    a += s[i];
  if (a.x + a.y + a.z + a.w == 1234.5f) out[0] = a.x;
}

template <class F>
static double timeit(F f, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  for (int64_t mib : {1024, 4096}) {
    const int64_t bytes = mib << 20, n4 = bytes / 16;
    f4 *s, *d;
    float* o;
    hipMalloc(&s, bytes);
    hipMalloc(&d, bytes);
    hipMalloc(&o, 64);
    hipMemset(s, 1, bytes);
    hipMemset(d, 0, bytes);
    auto rep = [&](const char* name, double ms, double traffic) {
      printf("%5lld MiB %-28s %8.3f ms  %7.1f GB/s\n", (long long)mib, name, ms, traffic / (ms * 1e-3) / 1e9);
    };
#define ONESHOT(U, NT, B)                                                                                        \
  rep("oneshot U" #U " nt" #NT " b" #B,                                                                          \
      timeit([&] { hipLaunchKernelGGL((copy_u<U, NT>), dim3((n4 + (int64_t)B * U - 1) / ((int64_t)B * U)), dim3(B), 0, 0, s, d, n4); }, 20), \
      2.0 * bytes);
    ONESHOT(1, false, 256); ONESHOT(1, false, 512); ONESHOT(1, false, 1024); ONESHOT(2, false, 256); ONESHOT(4, false, 256);
    ONESHOT(8, false, 256); ONESHOT(1, true, 256); ONESHOT(4, true, 256); ONESHOT(8, true, 256); ONESHOT(4, false, 512);
#define GS(U, NT, G, B)                                                                                           \
  rep("gridstride U" #U " nt" #NT " g" #G " b" #B,                                                               \
      timeit([&] { hipLaunchKernelGGL((copy_gs<U, NT>), dim3(G), dim3(B), 0, 0, s, d, n4); }, 20), 2.0 * bytes)
    GS(4, false, 2048, 256); GS(4, false, 4096, 256); GS(8, false, 2048, 256); GS(8, true, 2048, 256); GS(4, true, 4096, 256);
    GS(2, false, 8192, 256); GS(4, false, 1024, 1024); GS(8, false, 1024, 512);
    rep("read-only g8192 b256", timeit([&] { hipLaunchKernelGGL(read_only, dim3(8192), dim3(256), 0, 0, s, o, n4); }, 20),
        1.0 * bytes);
    rep("hipMemcpyDtoD", timeit([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 20), 2.0 * bytes);
    hipFree(s);
    hipFree(d);
    hipFree(o);
  }
  return 0;
}
