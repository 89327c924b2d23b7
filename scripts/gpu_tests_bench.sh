set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --config real --steps 2 --warmup 1 > gpurun_out/bench_real.log 2>&1
echo EXIT $? >> gpurun_out/bench_real.log
