// The persistent-step hand-off without the command processor: what does a stream-ordered
// step cost when a resident kernel P does the work and a one-workgroup "gate" kernel G on the
// caller's stream hands each step over?
//   G(t), launched on the caller's stream behind whatever produced the actions: stores go = t
//   (release, agent scope), then waits until every P workgroup has published flag[b] >= t
//   (acquire), and exits -- so the caller's next kernel on that stream sees the step's outputs.
//   P (blocks workgroups of 64 lanes, resident over all steps): polls go, does `work_us` of
//   (sleep) work, publishes flag[b] = t (release; one plain store per workgroup: no RMW on a
//   shared counter, which cost cp_pingpong ~10 ns per workgroup).
// Both sides give up after 2 s without progress (error flag set, every wait released), so a
// hand-off that never arrives cannot hang the box; P always reaches its exit.
// Reference lines: back-to-back launches of a `blocks`-workgroup kernel doing the same work.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/kernel_handoff.hip -o tools/probes/kernel_handoff
#include <hip/hip_runtime.h>
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

static constexpr uint64_t GIVE_UP_TICKS = 200000000ull;  // 2 s of the 100 MHz real-time clock
static constexpr uint32_t STOP = 0x7fffffffu;

// polling loads are relaxed (a coherent load, no cache invalidation per poll); the waiter
// issues ONE acquire fence once the condition holds (an acquire per poll invalidated the L2
// on every iteration: 43 / 165 us per step at 256 / 1024 workgroups, gpurun r03h)
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void work(int work_ticks) {
  if (work_ticks > 0) {  // the step's work, as a wait of work_ticks x 10 ns
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - w0 < (uint64_t)work_ticks) __builtin_amdgcn_s_sleep(2);
  }
}

__global__ __launch_bounds__(64) void p_kernel(uint32_t* go, uint32_t* flags, uint32_t* err, int steps, int work_ticks) {
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (int t = 1; t <= steps; ++t) {
    int tt = t;
    if (threadIdx.x == 0) {
      for (;;) {
        const uint32_t v = ld_rlx(go);
        if (v >= (uint32_t)t) {
          if (v == STOP) tt = steps + 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t_last > GIVE_UP_TICKS) {
          st_rel(err, 1u);
          tt = steps + 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    tt = __shfl(tt, 0);
    if (tt > steps) break;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    work(work_ticks);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, (uint32_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  // whatever happened, publish "past the end" so a waiting gate is released
  if (threadIdx.x == 0) st_rel(flags + blockIdx.x, STOP);
}

__global__ __launch_bounds__(256) void g_kernel(uint32_t* go, const uint32_t* flags, uint32_t* err, int blocks, uint32_t t) {
  if (threadIdx.x == 0) st_rel(go, t);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
    for (int b = threadIdx.x; b < blocks; b += blockDim.x) ok = ok && ld_rlx(flags + b) >= t;
    if (__syncthreads_and(ok)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      break;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > GIVE_UP_TICKS) {
      if (threadIdx.x == 0) st_rel(err, 2u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ __launch_bounds__(64) void step_like_kernel(int work_ticks) { work(work_ticks); }
__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1000000) *p = 0;
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t sP, sC;
  CK(hipStreamCreateWithFlags(&sP, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  const int blocks_list[2] = {256, 1024};
  const int warm = 20;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int bi = 0; bi < 2; ++bi) {
    for (int work_us = 0; work_us <= 10; work_us += 10) {
      for (int consumer = 0; consumer < 2; ++consumer) {
        const int blocks = blocks_list[bi];
        uint32_t *go = nullptr, *flags = nullptr, *err = nullptr;
        CK(hipMalloc((void**)&go, 4));
        CK(hipMalloc((void**)&flags, 4 * blocks));
        CK(hipMalloc((void**)&err, 4));
        CK(hipMemset(go, 0, 4));
        CK(hipMemset(flags, 0, 4 * blocks));
        CK(hipMemset(err, 0, 4));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(p_kernel, dim3(blocks), dim3(64), 0, sP, go, flags, err, steps, work_us * 100);
        CK(hipGetLastError());
        for (int t = 1; t <= steps; ++t) {
          if (t == warm + 1) CK(hipEventRecord(e0, sC));
          hipLaunchKernelGGL(g_kernel, dim3(1), dim3(256), 0, sC, go, flags, err, blocks, (uint32_t)t);
          if (consumer) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, sC, (int*)nullptr);
        }
        CK(hipEventRecord(e1, sC));
        CK(hipStreamSynchronize(sC));
        CK(hipStreamSynchronize(sP));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        uint32_t e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        printf("gate  blocks %4d work %2d us consumer %d: %.3f us per step%s\n", blocks, work_us, consumer,
               ms * 1e3 / (steps - warm), e ? "  [TIMEOUT]" : "");
        fflush(stdout);
        hipFree(go);
        hipFree(flags);
        hipFree(err);
        if (e) return 2;
      }
      // reference: the launch-per-step structure with the same work
      const int blocks = blocks_list[bi];
      for (int i = 0; i < warm; ++i) hipLaunchKernelGGL(step_like_kernel, dim3(blocks), dim3(64), 0, sC, work_us * 100);
      CK(hipEventRecord(e0, sC));
      for (int i = 0; i < steps - warm; ++i) hipLaunchKernelGGL(step_like_kernel, dim3(blocks), dim3(64), 0, sC, work_us * 100);
      CK(hipEventRecord(e1, sC));
      CK(hipStreamSynchronize(sC));
      float ms = 0.0f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("launch blocks %4d work %2d us: %.3f us per step\n", blocks, work_us, ms * 1e3 / (steps - warm));
      fflush(stdout);
    }
  }
  return 0;
}
