# A/B of two environment settings in one call (same library): GPU tests, the listen-stage contention probe
# (scripts/llm_stage_time.py) under each, then the default bench alternating A / B twice.
# usage: ENV_A='FO_X=0' ENV_B='FO_X=1' [PYTEST_K=expr] bash scripts/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/ab_env.txt
: > $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log >> $O
for E in "$ENV_A" "$ENV_B"; do
  echo "== $E stage probe" >> $O
  env $E timeout -k 10 200 python -u scripts/llm_stage_time.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  echo "== $E AR decode step" >> $O
  env $E timeout -k 10 120 python -u scripts/tts_step_time.py 8 multi 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for i in 1 2; do
  env $ENV_A timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/ab_A$i.log 2>&1 || exit 1
  env $ENV_B timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/ab_B$i.log 2>&1 || exit 1
done
for f in A1 B1 A2 B2; do
  echo -n "$f " >> $O; grep '^{' gpurun_out/ab_$f.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], d['rtf_per_user_p50'])" >> $O
done
cat $O
