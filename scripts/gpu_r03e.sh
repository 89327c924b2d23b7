# Round-3 call e: the whole GPU suite (prefix cache, broadcast-row sampler, encoder facade fixes), the turn
# bench with high-priority speech streams, then the profile passes of gpu_r03d.sh.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03e_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --out gpurun_out/r03e_bench.json > gpurun_out/r03e_bench.log 2>&1 && \
bash scripts/gpu_r03d.sh r03e
