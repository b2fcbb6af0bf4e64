// What does a per-step hand-off between a host stream and a resident (persistent) kernel cost?
// The stream advances a "go" counter with hipStreamWriteValue32 (the command processor writes
// it once everything earlier on the stream is done); every workgroup of the resident kernel
// polls it, does its step, and adds 1 to a "done" counter; the stream's next command is a
// hipStreamWaitValue64 on done >= t * blocks. The loop time per step is the round trip
// stream -> kernel -> stream, with `work_us` of (sleep) work per step inside the kernel.
// The kernel gives up after 2 s without progress (releases the waits, sets an error flag), so
// a hand-off that never arrives cannot hang the box.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/cp_pingpong.hip -o tools/probes/cp_pingpong
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

__global__ __launch_bounds__(64) void pp_kernel(uint32_t* go, uint64_t* done, uint32_t* err, int steps,
                                                int work_ticks, int sys) {
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  uint64_t t_last = t_start;
  for (int t = 1; t <= steps; ++t) {
    if (threadIdx.x == 0) {
      for (;;) {
        const uint32_t v = sys ? __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= (uint32_t)t) break;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - t_last > 200000000ull) {  // 2 s at 100 MHz: give up, release every wait
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(done, 1ull << 62, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // no later add wraps it
          t = steps + 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    t = __shfl(t, 0);
    if (t > steps) break;
    if (work_ticks > 0) {  // the step's work, as a wait of work_ticks x 10 ns
      const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - w0 < (uint64_t)work_ticks) __builtin_amdgcn_s_sleep(2);
    }
    if (threadIdx.x == 0) {
      if (sys)
        __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    t_last = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1000000) *p = 0;
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 2000;
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("CanUseStreamWaitValue %d\n", can);
  hipStream_t sK, sC;
  CK(hipStreamCreateWithFlags(&sK, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  const char* kinds[3] = {"signal", "uncached", "device"};
  const unsigned flags[3] = {hipMallocSignalMemory, hipDeviceMallocUncached, hipDeviceMallocDefault};
  const int blocks_list[2] = {256, 1024};
  for (int kind = 0; kind < 3; ++kind) {
    for (int bi = 0; bi < 2; ++bi) {
      for (int work_us = 0; work_us <= 10; work_us += 10) {
        for (int consumer = 0; consumer < 2; ++consumer) {
          const int blocks = blocks_list[bi];
          uint32_t *go = nullptr, *err = nullptr;
          uint64_t* done = nullptr;
          if (hipExtMallocWithFlags((void**)&go, 8, flags[kind]) != hipSuccess ||
              hipExtMallocWithFlags((void**)&done, 8, flags[kind]) != hipSuccess) {
            (void)hipGetLastError();
            printf("%s: alloc failed\n", kinds[kind]);
            continue;
          }
          CK(hipMalloc((void**)&err, 8));
          CK(hipMemset(go, 0, 4));
          CK(hipMemset(done, 0, 8));
          CK(hipMemset(err, 0, 4));
          CK(hipDeviceSynchronize());
          const int sys = kind < 2 ? 1 : 0;
          hipLaunchKernelGGL(pp_kernel, dim3(blocks), dim3(64), 0, sK, go, done, err, steps, work_us * 100, sys);
          CK(hipGetLastError());
          hipEvent_t e0, e1;
          CK(hipEventCreate(&e0));
          CK(hipEventCreate(&e1));
          const int warm = 20;
          for (int t = 1; t <= steps; ++t) {
            if (t == warm + 1) CK(hipEventRecord(e0, sC));
            CK(hipStreamWriteValue32(sC, go, (uint32_t)t, 0));
            CK(hipStreamWaitValue64(sC, done, (uint64_t)t * blocks, hipStreamWaitValueGte, ~0ull));
            if (consumer) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, sC, (int*)nullptr);
          }
          CK(hipEventRecord(e1, sC));
          CK(hipStreamSynchronize(sC));
          CK(hipStreamSynchronize(sK));
          float ms = 0.0f;
          CK(hipEventElapsedTime(&ms, e0, e1));
          uint32_t e = 0;
          CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
          printf("%-8s blocks %4d work %2d us consumer %d: %.3f us per step%s\n", kinds[kind], blocks, work_us, consumer,
                 ms * 1e3 / (steps - warm), e ? "  [TIMEOUT]" : "");
          fflush(stdout);
          hipEventDestroy(e0);
          hipEventDestroy(e1);
          hipFree(go);
          hipFree(done);
          hipFree(err);
          if (e) return 2;
        }
      }
    }
  }
  // reference: back-to-back launches of an empty kernel, and of a 10 us kernel-like wait
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(64), 0, sC, (int*)nullptr);
  CK(hipEventRecord(e0, sC));
  for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(64), 0, sC, (int*)nullptr);
  CK(hipEventRecord(e1, sC));
  CK(hipStreamSynchronize(sC));
  float ms = 0.0f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("empty kernel launches back to back: %.3f us each\n", ms * 1e3 / steps);
  return 0;
}
