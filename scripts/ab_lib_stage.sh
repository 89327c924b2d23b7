# Same-box A/B of two builds of libfo_hip.so (the in-tree one vs fo/libfo_hip_ab.so) on the AR decode step
# (scripts/tts_step_time.py, graph replay) and the listen stage (scripts/llm_stage_time.py), alternated twice.
#   usage on the GPU box: bash scripts/ab_lib_stage.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/$1
: > ${O}_lib_ab.txt
for i in 1 2; do for v in cur ab; do
  if [ $v = ab ]; then export FO_LIB_PATH=$GRAFT_REPO_ROOT/freeze-omni_amd/fo/libfo_hip_ab.so; else unset FO_LIB_PATH; fi
  timeout -k 10 200 python -u scripts/tts_step_time.py 8 multi > ${O}_tts_$v$i.log 2>&1 || { tail -5 ${O}_tts_$v$i.log; exit 1; }
  timeout -k 10 200 python -u scripts/llm_stage_time.py > ${O}_stage_$v$i.log 2>&1 || { tail -5 ${O}_stage_$v$i.log; exit 1; }
  unset FO_LIB_PATH
  echo "$v$i: $(grep 'graph replay only' ${O}_tts_$v$i.log | tail -1) | $(grep -E 'alone|overlapped' ${O}_stage_$v$i.log | grep -v tiny | tr -s ' ' | tr '\n' '|')" >> ${O}_lib_ab.txt
done; done
cat ${O}_lib_ab.txt
