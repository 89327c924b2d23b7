set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --config real --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo EXIT $? >> gpurun_out/prof_bench.log
