# A/B: the same bench twice in one call, with ENV_A and ENV_B (e.g. 'FO_X=0'); prints both lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
  env $ENV_A timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_A$i.log 2>&1 || exit 1
  env $ENV_B timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/ab_B$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log; do
  echo -n "$f "; grep '^{' $f | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], d['rtf_per_user_p50'])"
done
