# Round-3 call za: the Qwen2 down's K split merged inside its launch by all splits of a group (FO_DOWN_DMERGE=1)
# vs the reduce launch: bit-exactness test, the GPU suite with it on, the down sweep, the listen-stage probe, bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03za
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -k "down_split_merged or split_merge" > gpurun_out/${R}_test.log 2>&1 || { tail -40 gpurun_out/${R}_test.log; exit 1; }
tail -1 gpurun_out/${R}_test.log >> $O
FO_DOWN_DMERGE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
echo -n "suite with FO_DOWN_DMERGE=1: " >> $O; tail -1 gpurun_out/${R}_pytest_gpu.log >> $O
for E in "FO_DOWN_DMERGE=0" "FO_DOWN_DMERGE=1"; do
  echo "== $E down sweep" >> $O
  env $E DOWN_CFGS="2,8,7,8" timeout -k 10 200 python -u scripts/down_sweep.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  echo "== $E stage probe" >> $O
  env $E timeout -k 10 200 python -u scripts/llm_stage_time.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for i in 1 2; do
  for E in "FO_DOWN_DMERGE=0" "FO_DOWN_DMERGE=1"; do
    echo -n "$i [$E] " >> $O
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text')})" >> $O
  done
done
cat $O
