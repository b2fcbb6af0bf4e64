#!/usr/bin/env bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each step has its own time limit; a step that faults / aborts / times out ends the session
# (pytest's "tests failed" exit 1 does not). Output lands in gpurun_out/.
#   usage: tools/gpu_session.sh [tag] [steps...]
#   steps: tests prodtests smoke bench driver profdrv bench5 dist2 soak gap probe handoff jsbsim
#          stamps iccsweep variants div sweep report prof sq pmc   (default: tests smoke bench prof)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
STEPS=${*:-"tests smoke bench prof"}
OUT=gpurun_out
mkdir -p "$OUT"

run() {  # run <name> <timeout> <cmd...>
  local name=$1 lim=$2
  shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[session] stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}

run_abs() {  # run_abs <name> <timeout> <cmd...>: as run, from any working directory
  local name=$1 lim=$2
  shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$lim" "$@" > "$R/$OUT/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc"
  tail -5 "$R/$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[session] stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}
R=$(pwd)

python -c "from f16_jsb_amd.build import build; build()" || exit 3
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu_$TAG 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    prodtests) run pytest_prod 600 python -u -m pytest tests/test_gpu_production.py -m gpu -v -s --timeout 300 --timeout-method thread ;;
    smoke) run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 1000 --warmup 50 ;;
    driver) run bench_driver_$TAG 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    profdrv)  # rocprofv3 summary of the driver's exact command (the per-dispatch trace is dropped:
              # gpurun copies back at most 64 MiB of gpurun_out)
      (cd /tmp && run_abs prof_drv_$TAG 600 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof_drv_$TAG" -o run --output-format csv -- \
        python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5) || exit $?
      rm -f "$OUT/prof_drv_$TAG/run_kernel_trace.csv" ;;
    dist2)  # the bench's N > 1 code path with 2 ranks sharing this box's GPU (gloo: rehearsal only)
      run bench_dist2_$TAG 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo ;;
    soak)  # long runs at the bench's sizes: product build, then the bounds-checked debug build
      run soak_$TAG 600 python tools/soak.py
      F16ENV_LIB=f16_jsb_amd/libf16env_debug.so run soak_debug_$TAG 900 python tools/soak.py --steps3 5000 --steps5 3000 ;;
    gap) run driver_gap_$TAG 300 python tools/driver_gap.py --json "$OUT/driver_gap_$TAG.json" ;;
    probe) run cp_pingpong_$TAG 120 tools/probes/cp_pingpong 2000 ;;
    handoff) run kernel_handoff_$TAG 120 tools/probes/kernel_handoff 2000 ;;
    jsbsim)  # is a JSBSim binding present on the box? (probe only; never installed)
      python -c "import jsbsim, sys; print('jsbsim', jsbsim.__version__)" > "$OUT/jsbsim_probe_$TAG.log" 2>&1
      echo "[session] jsbsim probe rc=$?"; tail -2 "$OUT/jsbsim_probe_$TAG.log" ;;
    stamps) run stamp_profile_$TAG 600 python tools/stamp_profile.py ;;
    floors)  # empty / copy / issue-cost floors, then the step's own (ds 4 / 0 / 1 / 2)
      run floors_$TAG 120 tools/probes/floors 65536 300
      run floors_step_$TAG 300 python tools/floors_step.py --json "$OUT/floors_step_$TAG.json" ;;
    ab)  # same-box A/B of f16_jsb_amd/libf16env_ab_*.so against the product: bit identity + kernel time
      run ab_$TAG 900 python tools/ab_builds.py run --rounds ${AB_ROUNDS:-2} --json "$OUT/ab_$TAG.json" ;;
    launch2)  # bench.py --gpus 2 with no external launcher (gloo: 2 ranks share the box's GPU)
      run bench_launch2_$TAG 600 python bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo ;;
    iccsweep)  # cfg5 reset-cache refill period, same box
      for P in ${ICC_PERIODS:-8 16 32 64 128}; do
        F16ENV_ICC_PERIOD=$P run bench_cfg5_icc${P}_$TAG 300 python bench.py --workload cfg5 --steps ${ICC_STEPS:-300} --warmup 20 --no-cpu-baseline
      done ;;
    bench5) run bench_cfg5_$TAG 600 python bench.py --workload cfg5 --steps 300 --warmup 20 --cpu-seconds 5 ;;
    variants) run variant_sweep 900 python tools/variant_sweep.py run --json "$OUT/variants_$TAG.json" ;;
    div) run cfg5_divergence_$TAG 900 python tests/cfg5_divergence.py --n 4096 --json "$OUT/cfg5_divergence_$TAG.json" ;;
    sweep) run kernel_sweep 600 python tools/kernel_sweep.py --json "$OUT/sweep_$TAG.json" ;;
    report) run parity_report 600 python tests/parity_report.py --n 256 --steps 300 --json "$OUT/parity_$TAG.json" ;;
    prof)
      run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- \
        python bench.py --steps 300 --warmup 20 --no-cpu-baseline --rollout-envs 0
      rm -f "$OUT/prof_$TAG/run_kernel_trace.csv" ;;
    sq)  # summarised on the box (pmc_valu_$TAG.json), the raw rows compressed
      run pmc_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/pmc_sq_$TAG" -o run --output-format csv -- \
        python bench.py --steps 50 --warmup 5 --no-cpu-baseline --rollout-envs 0
      run pmc_sq2 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES -d "$OUT/pmc_sq2_$TAG" -o run --output-format csv -- \
        python bench.py --steps 50 --warmup 5 --no-cpu-baseline --rollout-envs 0
      run pmc_sq3 600 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 -d "$OUT/pmc_sq3_$TAG" -o run --output-format csv -- \
        python bench.py --steps 50 --warmup 5 --no-cpu-baseline --rollout-envs 0
      python tools/pmc_valu.py "$OUT/pmc_sq_$TAG" "$OUT/pmc_sq2_$TAG" "$OUT/pmc_sq3_$TAG" --kernel f16_step_win_nt_kernel \
        --out "$OUT/pmc_valu_$TAG.json" > /dev/null
      for d in pmc_sq_$TAG pmc_sq2_$TAG pmc_sq3_$TAG; do tar cJf "$OUT/$d.tar.xz" -C "$OUT" $d && rm -rf "$OUT/$d"; done ;;
    pmc5)  # HBM traffic of the cfg5 step kernel (summary: tools/pmc_traffic.py ... --envs 131072 --extra-bytes 24)
      run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc5_fetch_$TAG" -o run --output-format csv -- \
        python bench.py --workload cfg5 --steps 50 --warmup 5 --no-cpu-baseline
      run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc5_write_$TAG" -o run --output-format csv -- \
        python bench.py --workload cfg5 --steps 50 --warmup 5 --no-cpu-baseline ;;
    pmc)
      run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$TAG" -o run --output-format csv -- \
        python bench.py --steps 50 --warmup 5 --no-cpu-baseline --rollout-envs 0
      run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$TAG" -o run --output-format csv -- \
        python bench.py --steps 50 --warmup 5 --no-cpu-baseline --rollout-envs 0
      python tools/pmc_traffic.py "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG" --envs 65536 --stack 4 \
        --kernel f16_step_win_nt_kernel --out "$OUT/pmc_traffic_$TAG.json" > /dev/null
      for d in pmc_fetch_$TAG pmc_write_$TAG; do tar cJf "$OUT/$d.tar.xz" -C "$OUT" $d && rm -rf "$OUT/$d"; done ;;
  esac
done
echo "[session] done"
