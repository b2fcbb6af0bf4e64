// Does an XCD's L2 keep lines across a dependent kernel boundary? Kernel W writes a 16 MB
// buffer, kernel R then reads it back. Work chunks are mapped to blocks by the block's own
// XCD (HW_REG_XCC_ID): "stable" gives chunk c to the same XCD in W and R, "shifted" to the
// next XCD in R. If R(stable) is faster than R(shifted), the L2 kept the written lines.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/l2_keep_probe.hip -o tools/probes/l2_keep_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
__device__ __forceinline__ int chunk_of(int mode) {
  const int b = blockIdx.x;
  if (mode == 0) return b;  // plain
  const int x = (xcc_id() + (mode == 2 ? 1 : 0)) & 7;
  return (b & ~7) | x;
}
constexpr int PER = 16;  // float4 per thread
__global__ __launch_bounds__(256) void kw(float4* buf, int mode, float v) {
  const int c = chunk_of(mode);
  float4* p = buf + (size_t)c * 256 * PER + threadIdx.x;
#pragma unroll
  for (int i = 0; i < PER; ++i) p[i * 256] = make_float4(v, v + i, v, v);
}
__global__ __launch_bounds__(256) void kr(const float4* buf, int mode, float* out) {
  const int c = chunk_of(mode);
  const float4* p = buf + (size_t)c * 256 * PER + threadIdx.x;
  float s = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) { const float4 q = p[i * 256]; s += q.x + q.y + q.z + q.w; }
  out[c * 256 + threadIdx.x] = s;
}
__global__ void kflush(float4* junk, size_t n) {  // evict: stream 256 MB
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) junk[i].x += 1.0f;
}

int main() {
  const int blocks = 256;  // one block per CU: 2 MB per XCD
  float4 *buf, *junk;
  float* out;
  const size_t n4 = (size_t)blocks * 256 * PER;
  hipMalloc(&buf, n4 * 16);
  hipMalloc(&out, blocks * 256 * 4);
  const size_t nj = (256u << 20) / 16;
  hipMalloc(&junk, nj * 16);
  hipMemset(junk, 0, nj * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("buffer %.1f MB, %d blocks\n", n4 * 16 / 1e6, blocks);
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode : {1, 2, 0}) {
      float tw = 0, tr = 0;
      const int it = 20;
      for (int i = 0; i < it; ++i) {
        hipLaunchKernelGGL(kflush, dim3(1024), dim3(256), 0, 0, junk, nj);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kw, dim3(blocks), dim3(256), 0, 0, buf, mode == 0 ? 0 : 1, (float)i);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        tw += ms;
        hipEventRecord(e0);
        hipLaunchKernelGGL(kr, dim3(blocks), dim3(256), 0, 0, buf, mode, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        tr += ms;
      }
      printf("rep %d mode %s: write %.2f us, read %.2f us\n", rep, mode == 1 ? "stable " : (mode == 2 ? "shifted" : "plain  "),
             tw / it * 1e3, tr / it * 1e3);
    }
  }
  return 0;
}
