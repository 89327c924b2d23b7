# Round-3 call u: SpeechLane with device-side joins and a prefill stream, the batched silence cut, the text step
# queued ahead (parity tests), the full GPU suite with the 8-wave attention as the default, then the bench A/B:
# two sentence workers vs the lane vs the lane + text launch-ahead, three times each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03u
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_graphs_gpu.py -x -v --timeout 120 --timeout-method thread -k "lane or two_workers or silence_cut or launch_ahead" > gpurun_out/${R}_lane_test.log 2>&1 || { tail -40 gpurun_out/${R}_lane_test.log; exit 1; }
tail -1 gpurun_out/${R}_lane_test.log >> $O
echo "== attention, ping-pong tile prefetch (kps 256: two tiles per split, no merge up to 256 keys)" >> $O
ATTN_KPS=128,256 timeout -k 10 120 python -u scripts/attn_kps_sweep.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${R}_pytest_gpu.log >> $O
for i in 1 2; do
  for A in "" "--tts-lane" "--tts-lane --text-ahead" "--tts-lane --text-ahead FO_ATTN_KPS=256"; do
    echo -n "$i [$A] " >> $O
    EV=$(echo "$A" | tr ' ' '\n' | grep = | tr '\n' ' '); ARGS=$(echo "$A" | tr ' ' '\n' | grep -v = | tr '\n' ' ')
    env $EV timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 $ARGS > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k.startswith(('listen','text','speak','sentence'))})" >> $O
  done
done
cat $O
