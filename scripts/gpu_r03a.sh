# Round-3 first call: box facts (CPU share), the default bench as it stands, the text-step split
# (wall + rocprof kernel stats) and the gate/up partial Infinity-Cache residency probe.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; lscpu | grep -E 'Model name|Socket|Core|Thread|NUMA node\(s\)'; } > gpurun_out/r03a_box.txt 2>&1
timeout -k 10 200 python -u scripts/gu_mall_probe.py > gpurun_out/r03a_gu_mall.txt 2>&1 && \
timeout -k 10 200 python -u scripts/text_step_time.py 8 40 > gpurun_out/r03a_text_step.txt 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_r03a_text -o text -f csv -- python3 $ROOTD/scripts/text_step_time.py 8 40 > $ROOTD/gpurun_out/r03a_text_prof.log 2>&1 && \
cd $ROOTD && timeout -k 10 400 python -u bench.py --no-cpu-baseline --out gpurun_out/r03a_bench.json > gpurun_out/r03a_bench.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
