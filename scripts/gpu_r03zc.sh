# Round-3 call zc: vocoder convolutions with the next Cin chunk's activations prefetched into registers while the
# current chunk computes (CONV_XPF): codec / speech tests, the vocoder call time base (-DFO_CONV_XPF=0) vs new,
# the bench twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zc
O=gpurun_out/${R}.txt
BASE=$GRAFT_REPO_ROOT/freeze-omni_amd/fo/libfo_hip_base.so
: > $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "codec or vocoder or speak or silence or lane or tts" > gpurun_out/${R}_test.log 2>&1 || { tail -40 gpurun_out/${R}_test.log; exit 1; }
tail -1 gpurun_out/${R}_test.log >> $O
for i in 1 2; do
  echo -n "base " >> $O; FO_LIB_PATH=$BASE timeout -k 10 200 python -u scripts/vocoder_time.py 8 20 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  echo -n "new  " >> $O; timeout -k 10 200 python -u scripts/vocoder_time.py 8 20 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${R}_pytest_gpu.log >> $O
for i in 1 2; do
  for L in base new; do
    echo -n "$i [$L] " >> $O
    if [ $L = base ]; then export FO_LIB_PATH=$BASE; else unset FO_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text')})" >> $O
  done
done
unset FO_LIB_PATH
cat $O
