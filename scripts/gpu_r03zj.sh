# Round-3 call zj: a lane whose rows all launched out no longer drains inside the pump (the next sentence is
# taken in while the last steps are read) vs the old drain (FO_AB_OLD=1, a temporary switch): lane tests + 3 runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zj
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engines_gpu.py -m gpu -k "lane or silence_cut or two_workers" > gpurun_out/${R}_t.log 2>&1 || { tail -40 gpurun_out/${R}_t.log; exit 1; }
tail -1 gpurun_out/${R}_t.log >> $O
for i in 1 2 3; do
  for D in "" 1; do
    echo -n "$i [FO_AB_OLD=$D] " >> $O
    FO_AB_OLD=$D timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text') or k.startswith('sentence')})" >> $O
  done
done
cat $O
