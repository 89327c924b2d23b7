# Round-3 call zb: BatchMeta filled vectorised for long entries (the sentence prefills): GPU suite, bench x3.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zb
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${R}_pytest_gpu.log >> $O
for i in 1 2 3; do
  echo -n "$i " >> $O
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
  grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k.startswith(('listen','text','speak','sentence3'))})" >> $O
done
cat $O
