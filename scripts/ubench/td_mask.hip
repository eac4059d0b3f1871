// Microbenchmark (not part of the product): does a wave's 16-B-per-lane vector load cost the texture data
// path (TD) the same whatever the exec mask, or do inactive lanes / 4-lane groups skip their L1 accesses?
// Each kernel issues 8 independent global_load_dwordx4 per loop trip from an 8-KB L1-resident table with
// `mask` selecting the lanes that run the loop; the time per wave-load separates the cases:
//   all 64 lanes | lanes 0-31 | even lanes (32, every 4-lane group half on) | lanes 0-15 | every 4th lane.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench/td_mask.hip -o scripts/ubench/td_mask
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int PAT>
__device__ __forceinline__ bool on(uint32_t l) {
  if (PAT == 0) return true;
  if (PAT == 1) return l < 32;
  if (PAT == 2) return (l & 1) == 0;
  if (PAT == 3) return l < 16;
  return (l & 3) == 0;
}
template <int PAT>
__global__ __launch_bounds__(256) void loads(const uint4* __restrict__ tab, uint32_t* out, int iters) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0;
  if (on<PAT>(lane)) {
    uint32_t h = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
    for (int it = 0; it < iters; ++it) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = tab[(h + (uint32_t)k * 977u) & 511u];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
      h = h * 1664525u + 1013904223u;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int PAT>
static void run(const uint4* tab, uint32_t* out, const char* what, int active) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000, blocks = 256 * 8;
  hipLaunchKernelGGL((loads<PAT>), dim3(blocks), dim3(256), 0, 0, tab, out, 10);  // warm
  hipEventRecord(a);
  hipLaunchKernelGGL((loads<PAT>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double wl = (double)blocks * 4 * iters * 8;  // wave-level dwordx4 loads
  printf("%-34s %2d lanes: %.3f ms, %.2f G wave-loads/s, %.2f ns per wave-load per CU\n", what, active, ms,
         wl / ms * 1e-6, ms * 1e6 / (wl / 256));
  hipEventDestroy(a);
  hipEventDestroy(b);
}
int main() {
  uint4* tab;
  uint32_t* out;
  if (hipMalloc(&tab, 512 * sizeof(uint4)) != hipSuccess) return 1;
  if (hipMemset(tab, 1, 512 * sizeof(uint4)) != hipSuccess) return 1;
  if (hipMalloc(&out, 256 * 8 * 256 * sizeof(uint32_t)) != hipSuccess) return 1;
  run<0>(tab, out, "all lanes", 64);
  run<1>(tab, out, "lanes 0-31 (8 groups of 4 off)", 32);
  run<2>(tab, out, "even lanes (every group half on)", 32);
  run<3>(tab, out, "lanes 0-15 (12 groups off)", 16);
  run<4>(tab, out, "every 4th lane (every group on)", 16);
  run<0>(tab, out, "all lanes (again)", 64);
  hipFree(tab);
  hipFree(out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
