# Round-3 call zf: default (two sentence workers) vs the hardened lane (+ its tail worker), four times each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zf
O=gpurun_out/${R}.txt
: > $O
for i in 1 2 3 4; do
  for A in "" "--tts-lane"; do
    echo -n "$i [$A] " >> $O
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 $A > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text')})" >> $O
  done
done
cat $O
