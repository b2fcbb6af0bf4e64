set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_window.log 2>&1
rc=$?; echo "window tests rc=$rc"; tail -15 gpurun_out/pytest_window.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
F16_AB_HISTORY=${F16_AB_HISTORY:-0} timeout -k 10 600 python -u tools/layout_ab.py --json gpurun_out/layout_ab.json > gpurun_out/layout_ab.log 2>&1
rc=$?; echo "layout ab rc=$rc"; cat gpurun_out/layout_ab.log
