// Static VALU cost of the per-frame sections a lane-pair split could divide (VERDICT r03
// item 3). Not a product kernel and never launched: tools/pair_bound.py compiles this file to
// gfx950 assembly and counts the VALU instructions of each kernel. Each kernel reads its inputs
// per lane from global memory (so nothing constant-folds) and stores its outputs; k_base is that
// load/store frame alone, subtracted from the others.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -fno-slp-vectorize --cuda-device-only -S
#include "../../f16_jsb_amd/csrc/f16_device.h"

using namespace f16;

__device__ __forceinline__ void stage(float* sT) {
  for (int i = threadIdx.x; i < F16_BLOB_FLOATS; i += blockDim.x) sT[i] = F16_BLOB_INIT[i];
  __syncthreads();
}
#define LANE_IN(j) in[(int64_t)(j) * n + k]

// the load / store frame every probe shares
__global__ void k_base(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += LANE_IN(j);
  out[k] = s;
}

// the four breakpoint brackets of aero() (alpha, elevator, beta13 -> beta7, mach)
__global__ void k_brackets(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  __shared__ float sT[F16_BLOB_FLOATS];
  stage(sT);
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const Seg sa = bracket(BP_alpha_bp, sT + OFF_pair_alpha, LANE_IN(0));
  const Seg se = bracket(BP_de_bp, sT + OFF_pair_de, LANE_IN(1));
  const Seg sb = bracket(BP_beta13_bp, sT + OFF_pair_beta13, LANE_IN(2));
  const Seg sm = bracket(BP_machu, sT + OFF_pair_machu, LANE_IN(3));
  out[k] = sa.f + se.f + sb.f + sm.f + (float)(sa.i + se.i + sb.i + sm.i);
}

// brackets + every table value aero() blends (34 coefficients), summed so all stay live
__global__ void k_blends(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  __shared__ float sT[F16_BLOB_FLOATS];
  stage(sT);
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // aero() with every input zero except the bracket arguments and unit factors: the sums then
  // reduce to the blended values (same blends, same LDS reads); the force/moment sums are
  // counted by k_aero minus this kernel
  AeroIn a = {};
  a.alpha = LANE_IN(0); a.de = LANE_IN(1); a.beta = LANE_IN(2); a.mach = LANE_IN(3);
  const Seg sa = bracket(BP_alpha_bp, sT + OFF_pair_alpha, a.alpha);
  float acc = 0.0f;
  {
    const float* r0 = sT + OFF_alpha1d + (sa.i - 1) * (2 * F16_N_A1D);
#pragma unroll
    for (int q = 0; q < F16_N_A1D / 2; ++q) {
      const f2v r = blend2(sa.f, ld2(r0 + 2 * q), ld2(r0 + F16_N_A1D + 2 * q));
      acc += r.x * LANE_IN(4 + (q & 3)) + r.y;
    }
  }
  const Seg se = bracket(BP_de_bp, sT + OFF_pair_de, a.de);
  {
    const float* p0 = sT + OFF_ade + ((sa.i - 1) * F16_N_DE + se.i - 1) * 6;
    const float* p1 = p0 + 6;
    const f2v c1 = blend2(sa.f, ld2(p0), ld2(p0 + 2)), c2 = blend2(sa.f, ld2(p1), ld2(p1 + 2));
    const f2v r = blend2(se.f, c1, c2 - c1);
    const float d1 = blend(sa.f, p0[4], p0[5]), d2 = blend(sa.f, p1[4], p1[5]);
    acc += r.x + r.y + (d1 + se.f * (d2 - d1));
  }
  const Seg sb13 = bracket(BP_beta13_bp, sT + OFF_pair_beta13, a.beta);
  {
    const float* p0 = sT + OFF_ab13 + ((sa.i - 1) * F16_N_B13 + sb13.i - 1) * 4;
    const float* p1 = p0 + 4;
    const f2v c1 = blend2(sa.f, ld2(p0), ld2(p0 + 2)), c2 = blend2(sa.f, ld2(p1), ld2(p1 + 2));
    const f2v r = blend2(sb13.f, c1, c2 - c1);
    acc += r.x + r.y;
  }
  Seg sb7;
  sb7.i = 1 + ((sb13.i - 1) >> 1);
  {
    const float2 p = reinterpret_cast<const float2*>(sT + OFF_pair_beta7)[sb7.i - 1];
    sb7.f = __builtin_amdgcn_fmed3f((a.beta - p.x) * p.y, 0.0f, 1.0f);
    const float* p0 = sT + OFF_ab7 + ((sa.i - 1) * F16_N_B7 + sb7.i - 1) * 8;
    const float* p1 = p0 + 8;
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      const f2v c1 = blend2(sa.f, ld2(p0 + q), ld2(p0 + q + 4)), c2 = blend2(sa.f, ld2(p1 + q), ld2(p1 + q + 4));
      const f2v r = blend2(sb7.f, c1, c2 - c1);
      acc += r.x + r.y;
    }
  }
  const Seg sm = bracket(BP_machu, sT + OFF_pair_machu, a.mach);
  {
    const float* r0 = sT + OFF_machu_v + (sm.i - 1) * (2 * MACHU_NT);
#pragma unroll
    for (int q = 0; q + 1 < MACHU_NT; q += 2) {
      const f2v r = blend2(sm.f, ld2(r0 + 2 * q), ld2(r0 + 2 * q + 2));
      acc += r.x + r.y;
    }
    if (MACHU_NT & 1) acc += blend(sm.f, r0[2 * MACHU_NT - 2], r0[2 * MACHU_NT - 1]);
  }
  out[k] = acc;
}

// the whole of aero(): brackets, blends, force and moment sums
__global__ void k_aero(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  __shared__ float sT[F16_BLOB_FLOATS];
  stage(sT);
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  AeroIn a;
  a.qbar = LANE_IN(0); a.alpha = LANE_IN(1); a.beta = LANE_IN(2); a.mach = LANE_IN(3);
  a.p = LANE_IN(4); a.q = LANE_IN(5); a.r = LANE_IN(6); a.bi2vel = LANE_IN(7); a.ci2vel = LANE_IN(8);
  a.kclge = LANE_IN(9); a.de = LANE_IN(10); a.da = LANE_IN(11); a.dr = LANE_IN(12); a.dlef = LANE_IN(13);
  a.flap = LANE_IN(14); a.dsb = LANE_IN(15);
  float F6[6];
  aero(a, sT, F6);
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 6; ++j) s += F6[j];
  out[k] = s;
}

// one polynomial atan2 (alpha and beta each take one per frame); k_io2 is its load / store
__global__ void k_io2(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  out[k] = LANE_IN(0) + LANE_IN(1);
}
__global__ void k_fatan2(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  out[k] = fatan2(LANE_IN(0), LANE_IN(1));
}

// one whole FDM frame of the reference task (frame<false, false>, as the headline kernel runs
// it), the lane loaded from / stored to its 16 state columns; k_frame_io is that load / store
__global__ void k_frame(SoA s, const float* __restrict__ act, ModelConsts C, double ce, double se) {
  __shared__ float sT[F16_BLOB_FLOATS];
  stage(sT);
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Lane L;
  lane_load<false>(s, k, L);
  const float cmd[4] = {act[4 * k], act[4 * k + 1], act[4 * k + 2], act[4 * k + 3]};
  const AltRef A = alt_ref(L, ce, se);
  frame<false, false>(L, cmd, ce, se, A, sT, C, false);
  lane_store<false>(s, k, L);
}
__global__ void k_frame_io(SoA s, const float* __restrict__ act, ModelConsts C, double ce, double se) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Lane L;
  lane_load<false>(s, k, L);
  const AltRef A = alt_ref(L, ce, se);
  L.rI[0] += A.h0 + act[4 * k];
  lane_store<false>(s, k, L);
}
