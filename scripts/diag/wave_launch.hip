// Wave-launch microbenchmark (diagnostic, not product code): 2-wave workgroups whose waves spin
// for a fixed number of VALU iterations, on N waves, 72 VGPRs-class occupancy (7 waves/SIMD via
// launch bounds). Compares the kernel time with N * T_wave / slots: a gap means the launch rate
// (or slot turnaround), not the work, bounds short waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(128, 7) spin(float* out, int iters) {
  // s_sleep: the waves wait without competing for issue, so a wave lasts the same alone or with
  // 6 others on its SIMD
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(16);
  if (iters < 0) out[blockIdx.x] = 1.0f;
}

// the same with 1 KB of scratch per lane and 6 KB of LDS per workgroup (the render kernel's)
__global__ void __launch_bounds__(128, 7) spin_scratch(float* out, int iters) {
  __shared__ float4 tab[128 * 3];
  float stack[256];
  const int t = threadIdx.x;
  tab[t] = make_float4(float(t), 0.f, 0.f, 0.f);
  stack[(iters * 7 + t) & 255] = float(t);   // one scratch store: the allocation, not traffic
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(16);
  if (iters < 0) out[blockIdx.x] = stack[(t * 3) & 255] + tab[t].x;
}

template <typename K>
void run(const char* name, K kern, float* d, hipEvent_t a, hipEvent_t b) {
  for (int iters : {20, 80}) {
    for (int wgs : {16200, 64800}) {
      kern<<<wgs, 128>>>(d, iters);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) kern<<<wgs, 128>>>(d, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 5;
      printf("%-13s sleep iters %3d  wgs %6d: %.4f ms = %.2f us per round of 7168 waves\n", name, iters, wgs, ms,
             ms * 1e3 / (2.0 * wgs / 7168.0));
    }
  }
}

int main(int argc, char** argv) {
  float* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int wgs_list[] = {3584, 16200, 64800};
  const int iters_list[] = {5, 20, 80};
  for (int iters : iters_list) {
    // one workgroup alone: the wave's own duration
    spin<<<1, 128>>>(d, iters);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) spin<<<1, 128>>>(d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float alone;
    hipEventElapsedTime(&alone, a, b);
    alone /= 5;
    for (int wgs : wgs_list) {
      spin<<<wgs, 128>>>(d, iters);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) spin<<<wgs, 128>>>(d, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 5;
      // ideal with 7168 slots: waves / 7168 rounds of the lone wave's duration
      const double waves = 2.0 * wgs, ideal = alone * waves / 7168.0;
      printf("sleep iters %3d  wgs %6d (waves/slot %5.2f)  kernel %.4f ms  lone wave %.4f ms  ideal %.4f ms"
             "  -> per-wave overhead %.2f us\n", iters, wgs, waves / 7168.0, ms, alone, ideal,
             (ms - ideal) * 1e3 / (waves / 7168.0));
    }
  }
  run("plain", spin, d, a, b);
  run("scratch+lds", spin_scratch, d, a, b);
  return 0;
}
