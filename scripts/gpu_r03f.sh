# Round-3 call f: the down-projection sweep checked against a torch fp32 reference (which (tiles, K split)
# configurations are wrong, and where), and the k-steps-in-flight sweep of the small Qwen2 / TTS projections.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/down_sweep.py > gpurun_out/r03f_down_sweep.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gemm_u_sweep.py > gpurun_out/r03f_u_sweep.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
