# Same-box A/B of two builds of libfo_hip.so (in-tree = cur, fo/libfo_hip_ab.so = ab) on the text-decode step
# (scripts/text_step_time.py) and the 16..64-row Qwen2 GEMMs (scripts/gemm_mid_probe.py), alternated twice.
#   usage on the GPU box: bash scripts/ab_lib_text_mid.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/$1
: > ${O}_lib_ab.txt
for i in 1 2; do for v in cur ab; do
  if [ $v = ab ]; then export FO_LIB_PATH=$GRAFT_REPO_ROOT/freeze-omni_amd/fo/libfo_hip_ab.so; else unset FO_LIB_PATH; fi
  timeout -k 10 200 python -u scripts/text_step_time.py 8 > ${O}_text_$v$i.log 2>&1 || { tail -5 ${O}_text_$v$i.log; exit 1; }
  timeout -k 10 200 python -u scripts/gemm_mid_probe.py > ${O}_mid_$v$i.log 2>&1 || { tail -5 ${O}_mid_$v$i.log; exit 1; }
  unset FO_LIB_PATH
  echo "$v$i: $(grep -v amdgpu ${O}_text_$v$i.log | tail -2 | tr '\n' ' ')" >> ${O}_lib_ab.txt
  grep -E "qwen_gu|qwen_down" ${O}_mid_$v$i.log | sed "s/^/   $v$i /" >> ${O}_lib_ab.txt
done; done
cat ${O}_lib_ab.txt
