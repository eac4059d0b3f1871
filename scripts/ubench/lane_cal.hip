// Microbenchmark (not part of the product): calibrates the SQ "VALU lane utilisation" figure that
// bench.py and the round records quote (SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)) against kernels
// whose active-lane fraction is known by construction.  Each kernel runs 8 independent v_fma_f32 chains per
// lane with `active` of the wave's 64 lanes enabled (the others skip the loop), every CU busy; kernel k<A>
// is named by its active-lane count so rocprofv3 rows identify it.  The FMAs are inline asm, so nothing is
// folded away.  hipcc --offload-arch=gfx950 -O3 scripts/ubench/lane_cal.hip -o scripts/ubench/lane_cal
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int ACTIVE, int CHAINS>
__global__ __launch_bounds__(256) void lanes(float* out, uint32_t seed, int iters) {
  float acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (float)(threadIdx.x + i) * 1e-3f;
  const float f0 = (float)((seed ^ threadIdx.x) & 255) * 1e-3f, x = 0.999f;
  if ((int)(threadIdx.x & 63u) < ACTIVE) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < CHAINS; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(f0), "v"(x));
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int A, int C>
static void run(float* out, const char* what) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4000, blocks = 256 * 16;
  hipEventRecord(a);
  hipLaunchKernelGGL((lanes<A, C>), dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double inst = (double)blocks * 4 * iters * C;  // wave-level v_fma_f32 issued
  printf("%-28s active %2d/64 chains %d: %.3f ms, %.1f G wave-instr/s\n", what, A, C, ms, inst / ms * 1e-6);
  hipEventDestroy(a);
  hipEventDestroy(b);
}
int main() {
  float* out;
  if (hipMalloc(&out, 256 * 256 * 16 * sizeof(float)) != hipSuccess) return 1;
  run<64, 8>(out, "full lanes, 8 chains");
  run<48, 8>(out, "3/4 lanes, 8 chains");
  run<32, 8>(out, "half lanes, 8 chains");
  run<16, 8>(out, "1/4 lanes, 8 chains");
  run<64, 1>(out, "full lanes, 1 chain");
  run<32, 1>(out, "half lanes, 1 chain");
  hipFree(out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
