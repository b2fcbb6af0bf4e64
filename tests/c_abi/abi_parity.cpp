// The drop-in boundary used from C/C++ alone -- no Python, no torch: a host program links
// libf16env.so (include/f16env.h) and the CPU oracle (oracle/f16ref.h, test infrastructure),
// owns its device buffers with the HIP runtime, and steps the reference's own configuration
// (f16env_config_default: K = 10, down_sample 4, max 1200 steps; jsbsim_gym.py:58,157,159) on
// both, with the oracle's Philox random actions, through every call a C host binding would make:
// config, create, reset, step (contiguous layout), get_state, nonfinite_count, last_error,
// destroy. Checked: done flags and episode bookkeeping bit-exact, frames within
// tests/test_gpu_parity.py's 30-step random-action tolerance, rewards within 2e-3, and the
// error path (a NULL handle returns < 0 with a message).
//
//   make -C tests/c_abi      (hipcc; links f16_jsb_amd/libf16env.so and oracle/_build/libf16ref.so)
//   tests/c_abi/abi_parity [n_envs] [steps]      (exit 0 = parity)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "f16env.h"
#include "f16ref.h"

#define HCK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                        \
    }                                                                                  \
  } while (0)
#define FCK(x)                                                                     \
  do {                                                                             \
    int r_ = (x);                                                                  \
    if (r_ != 0) {                                                                 \
      fprintf(stderr, "%s:%d %s = %d: %s\n", __FILE__, __LINE__, #x, r_, f16env_last_error()); \
      return 2;                                                                    \
    }                                                                              \
  } while (0)

// tests/test_gpu_parity.py TOL_RAND30 (x, y, h, mach, alpha, beta, p, q, r, phi, theta, psi,
// goal x, y, z); angles compared modulo 2 pi
static const double TOL[15] = {5e-3, 5e-3, 5e-3, 2e-5, 5e-5, 5e-5, 5e-4, 5e-4, 5e-4, 5e-5, 5e-5, 5e-5, 0, 0, 0};

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2048;
  const int steps = argc > 2 ? atoi(argv[2]) : 30;
  if (n <= 0 || steps <= 0) return 2;

  // the error path first: a NULL handle is rejected with a message, nothing is launched
  if (f16env_step(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                  nullptr, nullptr) >= 0 ||
      f16env_last_error()[0] == '\0') {
    fprintf(stderr, "NULL handle not rejected\n");
    return 1;
  }
  printf("NULL handle rejected: %s\n", f16env_last_error());

  f16env_config cfg;
  FCK(f16env_config_default(&cfg));
  cfg.n_envs = n;
  cfg.seed = 2024;
  cfg.max_steps = 12;  // every lane truncates and auto-resets inside the run
  const int K = cfg.stack_k, KC = K * 15;

  f16env_t h = nullptr;
  FCK(f16env_create(&cfg, 0, &h));
  f16ref* ref = f16ref_create(&cfg);
  if (!ref) return 2;

  hipStream_t st;
  HCK(hipStreamCreate(&st));
  float *d_obs[2], *d_act, *d_rew;
  uint8_t *d_term, *d_trunc;
  double* d_ret;
  int32_t* d_len;
  HCK(hipMalloc((void**)&d_obs[0], sizeof(float) * n * KC));
  HCK(hipMalloc((void**)&d_obs[1], sizeof(float) * n * KC));
  HCK(hipMalloc((void**)&d_act, sizeof(float) * n * 4));
  HCK(hipMalloc((void**)&d_rew, sizeof(float) * n));
  HCK(hipMalloc((void**)&d_term, n));
  HCK(hipMalloc((void**)&d_trunc, n));
  HCK(hipMalloc((void**)&d_ret, sizeof(double) * n));
  HCK(hipMalloc((void**)&d_len, sizeof(int32_t) * n));

  std::vector<float> o_ref(n * KC), o_gpu(n * KC), act(n * 4), r_ref(n), r_gpu(n);
  std::vector<uint8_t> te_ref(n), tr_ref(n), te_gpu(n), tr_gpu(n);
  std::vector<double> ret_ref(n), ret_gpu(n);
  std::vector<int32_t> len_ref(n), len_gpu(n);

  FCK(f16env_reset(h, st, nullptr, nullptr, nullptr, d_obs[0]));
  if (f16ref_reset(ref, nullptr, nullptr, nullptr, o_ref.data()) != 0) return 2;
  double worst[15] = {0};
  auto compare_frames = [&]() {
    for (int i = 0; i < n; ++i)
      for (int r = 0; r < K; ++r)
        for (int c = 0; c < 15; ++c) {
          double d = std::fabs((double)o_gpu[i * KC + r * 15 + c] - (double)o_ref[i * KC + r * 15 + c]);
          if (c >= 9 && c <= 11) d = std::fabs(std::remainder(d, 2.0 * M_PI));
          if (!(d <= worst[c])) worst[c] = d;  // NaN propagates as a failure below
        }
  };
  HCK(hipMemcpyAsync(o_gpu.data(), d_obs[0], sizeof(float) * n * KC, hipMemcpyDeviceToHost, st));
  HCK(hipStreamSynchronize(st));
  compare_frames();  // the reset observation (K copies of frame 0)

  long done_total = 0, mismatches = 0, reward_bad = 0;
  for (int t = 0; t < steps; ++t) {
    if (f16ref_sample_actions(ref, 77, (uint64_t)t, act.data()) != 0) return 2;
    HCK(hipMemcpyAsync(d_act, act.data(), sizeof(float) * n * 4, hipMemcpyHostToDevice, st));
    float* prev = d_obs[t & 1];
    float* next = d_obs[(t + 1) & 1];
    FCK(f16env_step(h, st, d_act, prev, next, d_rew, d_term, d_trunc, nullptr, d_ret, d_len, nullptr, nullptr));
    if (f16ref_step(ref, act.data(), o_ref.data(), r_ref.data(), te_ref.data(), tr_ref.data(), nullptr,
                    ret_ref.data(), len_ref.data()) != 0)
      return 2;
    HCK(hipMemcpyAsync(o_gpu.data(), next, sizeof(float) * n * KC, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(r_gpu.data(), d_rew, sizeof(float) * n, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(te_gpu.data(), d_term, n, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(tr_gpu.data(), d_trunc, n, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(ret_gpu.data(), d_ret, sizeof(double) * n, hipMemcpyDeviceToHost, st));
    HCK(hipMemcpyAsync(len_gpu.data(), d_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    HCK(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) {
      if (te_gpu[i] != te_ref[i] || tr_gpu[i] != tr_ref[i]) ++mismatches;
      const bool done = te_ref[i] || tr_ref[i];
      if (done) {
        ++done_total;
        if (len_gpu[i] != len_ref[i] || std::fabs(ret_gpu[i] - ret_ref[i]) > 1e-3) ++mismatches;
      }
      if (!(std::fabs((double)r_gpu[i] - (double)r_ref[i]) <= 2e-3)) ++reward_bad;
    }
    compare_frames();
  }
  uint64_t nonfinite = 0;
  FCK(f16env_nonfinite_count(h, st, &nonfinite));
  // canonical state export (a device buffer, like every array argument of the ABI): the step
  // counters must say every lane is inside its (12-step) episode
  double* d_canon = nullptr;
  HCK(hipMalloc((void**)&d_canon, sizeof(double) * n * F16C_N));
  FCK(f16env_get_state(h, st, d_canon));
  std::vector<double> canon((size_t)n * F16C_N);
  HCK(hipMemcpyAsync(canon.data(), d_canon, sizeof(double) * n * F16C_N, hipMemcpyDeviceToHost, st));
  HCK(hipStreamSynchronize(st));
  HCK(hipFree(d_canon));
  for (int i = 0; i < n; ++i) {
    const double s = canon[(size_t)i * F16C_N + F16C_STEP];
    if (!(s >= 0.0 && s < cfg.max_steps)) ++mismatches;
  }

  bool ok = mismatches == 0 && reward_bad == 0 && done_total >= n && nonfinite == 0;
  printf("kernel %s  n %d  K %d  steps %d  dones %ld  flag/episode mismatches %ld  rewards off %ld\n",
         f16env_step_kernel_name(h), n, K, steps, done_total, mismatches, reward_bad);
  printf("max |gpu - oracle| per frame component:");
  for (int c = 0; c < 15; ++c) {
    printf(" %.3g", worst[c]);
    if (!(worst[c] <= TOL[c])) ok = false;
  }
  printf("\n%s\n", ok ? "ABI PARITY OK" : "ABI PARITY FAILED");

  f16ref_destroy(ref);
  FCK(f16env_destroy(h));
  for (void* p : {(void*)d_obs[0], (void*)d_obs[1], (void*)d_act, (void*)d_rew, (void*)d_term, (void*)d_trunc,
                  (void*)d_ret, (void*)d_len})
    HCK(hipFree(p));
  HCK(hipStreamDestroy(st));
  return ok ? 0 : 1;
}
