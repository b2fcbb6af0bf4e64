#!/usr/bin/env bash
# variant-sweep A/B on the GPU box: tools/variant_sweep.py run, twice (same box), each under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sweep}
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 500 python tools/variant_sweep.py run --json gpurun_out/${TAG}_$r.json > gpurun_out/${TAG}_$r.log 2>&1
  rc=$?; echo "sweep $r rc=$rc"; tail -4 gpurun_out/${TAG}_$r.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
