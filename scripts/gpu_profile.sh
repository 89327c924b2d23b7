# rocprofv3 kernel-trace stats of the bench command, then a separate FETCH_SIZE pass on the
# dominant kernel (FETCH_RE, default k_gemm_xs) -- counters never share a pass with other trace domains.
set -o pipefail
R=${1:-r01}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ROOTD=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARGS="--config real --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$R -o bench -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/prof_bench_$R.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ${FETCH_RE:-k_gemm_xs} -d $ROOTD/gpurun_out/pmc_$R -o fetch -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/pmc_bench_$R.log 2>&1
echo EXIT $? >> $ROOTD/gpurun_out/pmc_bench_$R.log
