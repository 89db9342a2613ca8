// How many workgroups with a given static LDS size and thread count share a CU?
// Each workgroup spins ~20 us; the launch time of 256 / 512 / 768 workgroups
// tells the residency (equal times = co-resident).
//   hipcc --offload-arch=gfx950 -O3 scripts/lds_occupancy.hip -o scripts/lds_occupancy && ./scripts/lds_occupancy
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int LDS, int NT>
__global__ void __launch_bounds__(NT) spin(float* out, long cycles) {
  __shared__ float lds[LDS / 4];
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  const long t0 = clock64();
  float acc = 0.f;
  while (clock64() - t0 < cycles) acc += lds[(threadIdx.x * 7) % NT];
  if (acc == -1.f) out[blockIdx.x] = acc;
}

template <int LDS, int NT>
void probe(const char* name, float* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int g : {256, 512, 768, 1024}) {
    spin<LDS, NT><<<g, NT>>>(d, 40000);
    hipEventRecord(a);
    spin<LDS, NT><<<g, NT>>>(d, 40000);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%s workgroups=%d: %.1f us\n", name, g, ms * 1000.f);
  }
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * 4);
  probe<79104, 256>("lds=79104 nt=256", d);
  probe<65536, 256>("lds=65536 nt=256", d);
  probe<40960, 256>("lds=40960 nt=256", d);
  probe<140416, 512>("lds=140416 nt=512", d);
  hipFree(d);
  return 0;
}
