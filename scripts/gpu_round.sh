# One GPU call: gpu tests, smoke, default bench (with cpu_baseline), rocprof kernel stats and a
# FETCH_SIZE pass on the dominant kernel. Every GPU step has its own time limit; steps chain with &&.
set -o pipefail
R=${1:-r01}
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$R -o bench -f csv -- python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/prof_bench_$R.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gemm_wstream -d $ROOTD/gpurun_out/pmc_$R -o fetch -f csv -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/pmc_bench_$R.log 2>&1
rc=$?
echo EXIT $rc >> $ROOTD/gpurun_out/round.log
exit $rc
