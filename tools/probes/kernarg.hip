// Where the empty kernel's ~1 µs per launch of "LDS" goes (round 6): profiles/r06_floors_lds_sweep.json
// split it -- an argument-free kernel given 46 KB of LDS costs what the empty kernel does, the
// kernel that reads one pointer argument and has no LDS costs the extra ~1 µs. This probe times,
// back to back at the step's grid (256 x 256 threads, 300 launches), kernels whose first memory
// access is:
//   empty          none
//   arg            the kernel argument segment (one pointer, used in a never-taken branch)
//   arg_big        the same pointer at the end of a 640 B argument struct (the step's size class)
//   arg_load       a pointer argument, then a 16 B load per lane through it (1 MiB, cold-ish)
//   glob_load      the same load from a __device__ array (address by relocation, no argument)
//   globptr_load   a pointer read from a __device__ variable, then the load through it
// Built twice, without and with -mllvm -amdgpu-kernarg-preload-count=8 (the step's build flag):
// with preload the argument SGPRs are filled before the wave starts and "arg" needs no s_load.
// Every kernel's only store is a vector store in a never-taken branch (no scalar stores).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/kernarg.hip -o tools/probes/kernarg_p0
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 \
//         tools/probes/kernarg.hip -o tools/probes/kernarg_p8
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static constexpr int BLOCK = 256;
static constexpr int N = 65536;

__device__ float4 g_state[N];
__device__ float4* g_ptr;
__device__ float g_sink[N];

struct Big {
  float pad[158];
  float* out;
};

__global__ __launch_bounds__(BLOCK, 1) void k_empty() {}
__global__ __launch_bounds__(BLOCK, 1) void k_arg(float* out) {
  if (out && blockIdx.x == 0x7fffffff) out[threadIdx.x] = 1.0f;
}
__global__ __launch_bounds__(BLOCK, 1) void k_arg_big(Big b) {
  if (b.out && blockIdx.x == 0x7fffffff) b.out[threadIdx.x] = 1.0f;
}
__global__ __launch_bounds__(BLOCK, 1) void k_arg_load(const float4* in, float* out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  const float4 v = in[i];
  if (v.x == 12345.0f) out[i] = v.y;
}
__global__ __launch_bounds__(BLOCK, 1) void k_glob_load() {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  const float4 v = g_state[i];
  if (v.x == 12345.0f) g_sink[i] = v.y;
}
__global__ __launch_bounds__(BLOCK, 1) void k_globptr_load() {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  const float4 v = g_ptr[i];
  if (v.x == 12345.0f) g_sink[i] = v.y;
}

// the step's prologue chain: 16 state columns per lane (n x 16 B apart) whose addresses come
//   chain_arg   from the kernel arguments (the step today: arguments, then the state loads)
//   chain_glob  from a __device__ variable, the arguments read after the loads are in flight
// on a rotation of NBUF state buffers (NBUF x 16 MiB: beyond the L2s, as the step's 43 MB)
static constexpr int NBUF = 8;
__device__ const float4* g_states[NBUF];
__device__ int64_t g_n;

__global__ __launch_bounds__(BLOCK, 1) void k_chain_arg(const float4* st, int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  float acc = 0.0f;
  const float4* p = st + i;
  float4 c[16];
#pragma unroll
  for (int j = 0; j < 16; ++j, p += n) c[j] = *p;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc += c[j].x + c[j].w;
  if (acc == 12345.0f) out[i] = acc;
}
__global__ __launch_bounds__(BLOCK, 1) void k_chain_glob(int buf, float* out) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int64_t n = g_n;
  float acc = 0.0f;
  const float4* p = g_states[0] + i;
  float4 c[16];
#pragma unroll
  for (int j = 0; j < 16; ++j, p += n) c[j] = *p;
  // the argument only now: its latency under the state loads'
  if (buf < 0) acc = 1.0f;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc += c[j].x + c[j].w;
  if (acc == 12345.0f) out[i] = acc;
}

// the step's real pattern: the action pointer is an argument too; chain_glob_act issues the
// state loads from the __device__ address, then reads the action pointer argument and loads
// through it (the argument round trip under the state loads'); chain_arg_act reads everything
// from the arguments first
__global__ __launch_bounds__(BLOCK, 1) void k_chain_arg_act(const float4* st, const float4* act, int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  float acc = 0.0f;
  const float4* p = st + i;
  float4 c[16];
#pragma unroll
  for (int j = 0; j < 16; ++j, p += n) c[j] = *p;
  const float4 a = act[i];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc += c[j].x + c[j].w;
  acc += a.y;
  if (acc == 12345.0f) out[i] = acc;
}
__global__ __launch_bounds__(BLOCK, 1) void k_chain_glob_act(const float4* act, float* out) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int64_t n = g_n;
  float acc = 0.0f;
  const float4* p = g_states[0] + i;
  float4 c[16];
#pragma unroll
  for (int j = 0; j < 16; ++j, p += n) c[j] = *p;
  const float4 a = act[i];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc += c[j].x + c[j].w;
  acc += a.y;
  if (acc == 12345.0f) out[i] = acc;
}

template <class F>
static void timed(const char* name, int launches, F launch) {
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0.0f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(s, 0));
    for (int i = 0; i < launches; ++i) launch();
    CK(hipEventRecord(e, 0));
    CK(hipEventSynchronize(e));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, s, e));
    best = ms < best ? ms : best;
    sum += ms;
  }
  printf("{\"probe\": \"%s\", \"launches\": %d, \"region_us_per_launch_best\": %.3f, "
         "\"region_us_per_launch_mean\": %.3f}\n",
         name, launches, 1e3 * best / launches, 1e3 * sum / 5 / launches);
  CK(hipEventDestroy(s));
  CK(hipEventDestroy(e));
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 300;
  const char* tag = argc > 2 ? argv[2] : "";
  float4* in;
  float* out;
  CK(hipMalloc(&in, sizeof(float4) * N));
  CK(hipMalloc(&out, sizeof(float) * N));
  CK(hipMemset(in, 0, sizeof(float4) * N));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ptr), &in, sizeof(in)));
  const dim3 grid(N / BLOCK), blk(BLOCK);
  Big big{};
  big.out = out;
  printf("{\"build\": \"%s\", \"grid\": %d, \"block\": %d}\n", tag, N / BLOCK, BLOCK);
  timed("empty", launches, [&] { hipLaunchKernelGGL(k_empty, grid, blk, 0, 0); });
  timed("arg", launches, [&] { hipLaunchKernelGGL(k_arg, grid, blk, 0, 0, out); });
  timed("arg_big", launches, [&] { hipLaunchKernelGGL(k_arg_big, grid, blk, 0, 0, big); });
  timed("arg_load", launches, [&] { hipLaunchKernelGGL(k_arg_load, grid, blk, 0, 0, (const float4*)in, out); });
  timed("glob_load", launches, [&] { hipLaunchKernelGGL(k_glob_load, grid, blk, 0, 0); });
  timed("globptr_load", launches, [&] { hipLaunchKernelGGL(k_globptr_load, grid, blk, 0, 0); });
  {
    float4* bufs[NBUF];
    for (int b = 0; b < NBUF; ++b) {
      CK(hipMalloc(&bufs[b], sizeof(float4) * 16 * (size_t)N));
      CK(hipMemset(bufs[b], 0, sizeof(float4) * 16 * (size_t)N));
    }
    const int64_t n = N;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_n), &n, sizeof(n)));
    int it = 0;
    timed("chain_arg_rot", launches, [&] {
      hipLaunchKernelGGL(k_chain_arg, grid, blk, 0, 0, (const float4*)bufs[it++ % NBUF], n, out);
    });
    timed("chain_arg_same", launches, [&] {
      hipLaunchKernelGGL(k_chain_arg, grid, blk, 0, 0, (const float4*)bufs[0], n, out);
    });
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_states), &bufs[0], sizeof(float4*)));
    timed("chain_glob_same", launches, [&] { hipLaunchKernelGGL(k_chain_glob, grid, blk, 0, 0, 0, out); });
    // interleaved A B A B ..., 6 pairs: the action-pointer chain both ways
    for (int r = 0; r < 6; ++r) {
      timed("chain_arg_act", launches, [&] {
        hipLaunchKernelGGL(k_chain_arg_act, grid, blk, 0, 0, (const float4*)bufs[0], (const float4*)in, n, out);
      });
      timed("chain_glob_act", launches, [&] {
        hipLaunchKernelGGL(k_chain_glob_act, grid, blk, 0, 0, (const float4*)in, out);
      });
    }
    for (int b = 0; b < NBUF; ++b) CK(hipFree(bufs[b]));
  }
  timed("empty_again", launches, [&] { hipLaunchKernelGGL(k_empty, grid, blk, 0, 0); });
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
