# Alternate two environment settings (ENV_A / ENV_B, e.g. 'FO_GEMM_MERGE=1') on the listen-stage probe
# (scripts/llm_stage_time.py: Qwen2 stage alone, encoder alone, both overlapped), twice each, on one box.
#   usage on the GPU box: ENV_A='' ENV_B='FO_GEMM_MERGE=1' bash scripts/ab_env_stage.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/$1
: > ${O}_stage_ab.txt
for i in 1 2; do for AB in A B; do
  E=ENV_$AB
  timeout -k 10 200 env ${!E} python -u scripts/llm_stage_time.py > ${O}_stage_$AB$i.log 2>&1 || { tail -20 ${O}_stage_$AB$i.log; exit 1; }
  echo "$AB$i [${!E}] $(grep -E 'alone|overlapped' ${O}_stage_$AB$i.log | grep -v tiny | tr -s ' ' | tr '\n' '|')" >> ${O}_stage_ab.txt
done; done
cat ${O}_stage_ab.txt
