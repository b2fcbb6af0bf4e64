// Issue cost of packed vs single f32 FMA for ONE wave per SIMD (the step kernel's regime at
// 65 536 envs): each lane runs `iters` rounds of 16 independent FMAs, either as 16 v_fma_f32
// or as 8 v_pk_fma_f32 (float2 ext-vector ops). Timed with wall-clock events over a grid of
// 1024 waves (one per SIMD); cycles per FMA-pair follow from the clock.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/pk_probe.hip -o /tmp/pk_probe && /tmp/pk_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_single(int iters, float* out, float a, float b) {
  float x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = threadIdx.x * 0.001f + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = __builtin_fmaf(x[j], a, b);
  }
  float s = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += x[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_packed(int iters, float* out, float a, float b) {
  f2 x[8];
  const f2 av = {a, a}, bv = {b, b};
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (f2){threadIdx.x * 0.001f + 2 * j, threadIdx.x * 0.001f + 2 * j + 1};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = __builtin_elementwise_fma(x[j], av, bv);
  }
  float s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 1024 * 256 * 4 * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int blocks : {256, 512}) {  // 256 blocks x 4 waves = one wave per SIMD; 512 = two
    for (int rep = 0; rep < 2; ++rep) {
      float ms[2];
      for (int v = 0; v < 2; ++v) {
        hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(k_single, dim3(blocks), dim3(256), 0, 0, iters, out, 0.999f, 0.001f);
        else hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(256), 0, 0, iters, out, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[v], e0, e1);
      }
      // at ~2.4 GHz: cycles per round of 16 FMAs per wave
      printf("blocks %d: single %.3f ms (%.1f cyc/16 fma)  packed %.3f ms (%.1f cyc/16 fma)\n", blocks, ms[0],
             ms[0] * 1e-3 * 2.4e9 / iters, ms[1], ms[1] * 1e-3 * 2.4e9 / iters);
    }
  }
  hipFree(out);
  return 0;
}
