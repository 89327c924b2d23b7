# Round-3 call v: SpeechLane rows that launched their last token leave the batch on the device (no drain, no
# host round trip), parity tests; then the bench A/B with the text step queued ahead: two sentence workers vs
# the lane, twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03v
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -x -v --timeout 120 --timeout-method thread -k "lane" > gpurun_out/${R}_lane_test.log 2>&1 || { tail -40 gpurun_out/${R}_lane_test.log; exit 1; }
tail -1 gpurun_out/${R}_lane_test.log >> $O
for i in 1 2; do
  for A in "--text-ahead" "--tts-lane --text-ahead"; do
    echo -n "$i [$A] " >> $O
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 $A > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k.startswith(('listen','text','speak','sentence'))})" >> $O
  done
done
cat $O
