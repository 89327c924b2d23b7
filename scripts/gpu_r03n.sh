# Round-3 call n: listen-stage CU partition probe; merged split for the Qwen2 down (FO_GEMM_MERGE=1) A/B.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/cu_partition_probe.py > gpurun_out/r03n_cu_partition.txt 2>&1 && \
timeout -k 10 200 python -u scripts/llm_stage_time.py > gpurun_out/r03n_stage.txt 2>&1 && \
FO_GEMM_MERGE=1 timeout -k 10 200 python -u scripts/llm_stage_time.py > gpurun_out/r03n_stage_merge1.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
