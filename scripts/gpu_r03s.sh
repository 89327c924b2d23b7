# Round-3 call s (new container, rebuilt library): the Qwen2 down over all 256 CUs -- 7 tiles x 8-way split (256
# workgroups) or 8 tiles x 9-way split (252) vs the 224-workgroup default: down sweep, listen-stage probe, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03s
O=gpurun_out/${R}.txt
: > $O
DOWN_CFGS="2,8,8,8;2,8,8,9;2,8,7,8;2,8,7,9;2,8,8,10" timeout -k 10 200 python -u scripts/down_sweep.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
for E in "FO_DOWN_S=8" "FO_DOWN_NT=7" "FO_DOWN_S=9"; do
  echo "== $E stage probe" >> $O
  env $E timeout -k 10 200 python -u scripts/llm_stage_time.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for i in 1 2; do
  for E in "FO_DOWN_S=8" "FO_DOWN_NT=7" "FO_DOWN_S=9"; do
    echo -n "$i $E " >> $O
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || exit 1
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text')})" >> $O
  done
done
cat $O
