set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --config tiny --steps 1 --warmup 1 --users 2 --input-sec 2 --codec-tokens 100 --no-cpu-baseline > gpurun_out/bench_tiny.log 2>&1 && \
timeout -k 10 600 python bench.py --config real --steps 1 --warmup 1 --users 8 --no-cpu-baseline > gpurun_out/bench_real.log 2>&1
echo EXIT $? >> gpurun_out/bench_real.log
