# Round-end measurement in one call: GPU tests, smoke, default bench (cpu_baseline + single user), duplex
# bench, rocprofv3 kernel stats of the bench, a FETCH_SIZE pass on the dominant kernel, and the kernel trace
# of the AR decode step alone.  Every GPU step has its own time limit; the steps chain with &&.
# usage: bash scripts/gpu_final.sh r02s
set -o pipefail
R=${1:-rNN}
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--config real --steps 2 --warmup 1 --no-cpu-baseline --no-single-user"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --out gpurun_out/bench_default_$R.json > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 python -u bench.py --scenario duplex --out gpurun_out/bench_duplex_$R.json > gpurun_out/bench_duplex.log 2>&1 && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$R -o bench -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/prof_bench_$R.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gemm_xs -d $ROOTD/gpurun_out/pmc_$R -o fetch -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/pmc_bench_$R.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_tts_$R -o tts -f csv -- python3 $ROOTD/scripts/tts_step_time.py 8 multi > $ROOTD/gpurun_out/prof_tts_$R.log 2>&1
rc=$?
cd $ROOTD
echo "EXIT $rc" >> gpurun_out/final_$R.log
tail -1 gpurun_out/pytest_gpu.log >> gpurun_out/final_$R.log
grep -h '^{' gpurun_out/bench_default.log gpurun_out/bench_duplex.log | cut -c1-300 >> gpurun_out/final_$R.log
cat gpurun_out/final_$R.log
exit $rc
