# GPU tests (one process, per-test timeout) then a short bench without the CPU baseline.
# usage: bash scripts/gpu_check.sh [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; grep '^{' gpurun_out/bench_quick.log | cut -c1-420
exit $rc
