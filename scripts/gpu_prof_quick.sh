# kernel-trace of a short bench (1 warmup + 1 step) -> gpurun_out/prof_quick (+ trace table)
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_quick -o bench -f csv -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $ROOTD/gpurun_out/prof_quick.log 2>&1
rc=$?
cd $ROOTD && python scripts/trace_table.py gpurun_out/prof_quick 30 > gpurun_out/prof_quick_table.txt; grep '^{' gpurun_out/prof_quick.log | cut -c1-300
exit $rc
