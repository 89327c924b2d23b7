# Round-3 call zh: lane (default) vs --no-tts-lane once more, on another box, with the sentence waits.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zh
O=gpurun_out/${R}.txt
: > $O
for i in 1 2 3; do
  for A in "" "--no-tts-lane"; do
    echo -n "$i [$A] " >> $O
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 $A > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text') or k.endswith('_wait')})" >> $O
  done
done
cat $O
