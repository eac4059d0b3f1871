// Microbenchmark (not part of the product): issue rate of v_fma_mix_f32 (f16 operand, f32 math) vs
// v_fma_f32 on gfx950, 8 independent chains per lane, every CU busy.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, uint32_t seed, int iters) {
  float acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (float)(threadIdx.x + i) * 1e-3f;
  const uint32_t hv = seed ^ threadIdx.x;
  const h2 h = __builtin_bit_cast(h2, hv & 0x3bff3bffu);
  const float f0 = (float)(hv & 255) * 1e-3f, f1 = f0 * 0.5f;
  const float x = 0.999f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(f0), "v"(x));
      else if (MODE == 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc[i]) : "v"(hv), "v"(x));
      else asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(acc[i]) : "v"(hv));
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * 32 * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 20000, blocks = 256 * 32;
  for (int mode = 0; mode < 3; ++mode)
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
      else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
      else hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double ops = (double)blocks * 256 / 64 * iters * 8;  // wave-level instructions
      printf("%s: %.3f ms, %.1f G wave-instr/s\n", mode == 0 ? "v_fma_f32" : mode == 1 ? "v_fma_mix_f32" : "v_cvt_f32_f16", ms, ops / ms / 1e6);
    }
  return 0;
}
