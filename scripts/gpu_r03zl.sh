# Round-3 call zl: the lane's join window (steps launched ahead while a group's prefill runs): 4 (default) vs 2 vs 8.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zl
O=gpurun_out/${R}.txt
: > $O
for i in 1 2; do
  for W in 4 2 8; do
    echo -n "$i [FO_LANE_JOIN_WINDOW=$W] " >> $O
    FO_LANE_JOIN_WINDOW=$W timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text') or k.startswith('sentence')})" >> $O
  done
done
cat $O
