# A/B of two builds of libfo_hip in one call: GPU tests on the new build, the TTS step rate and the
# per-workgroup GEMM trace on both, then the default bench alternating base / new twice.
# BASE = in-tree libfo_hip_base.so (built from the previous commit), NEW = libfo_hip.so.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/freeze-omni_amd/fo/libfo_hip_base.so
O=gpurun_out/ab_lib.txt
: > $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log >> $O
for L in base new; do
  if [ $L = base ]; then export FO_LIB_PATH=$BASE FO_ATTN_DENSE=${BASE_ATTN_DENSE:-1}; else unset FO_LIB_PATH FO_ATTN_DENSE; fi
  echo "== $L tts step" >> $O
  timeout -k 10 120 python -u scripts/tts_step_time.py 8 multi >> $O 2>&1 || exit 1
  echo "== $L gemm trace" >> $O
  timeout -k 10 200 python -u scripts/gemm_trace.py >> $O 2>&1 || exit 1
done
unset FO_LIB_PATH FO_ATTN_DENSE
for i in 1 2; do
  FO_LIB_PATH=$BASE FO_ATTN_DENSE=${BASE_ATTN_DENSE:-1} timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/ab_base$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/ab_new$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_base1.log gpurun_out/ab_new1.log gpurun_out/ab_base2.log gpurun_out/ab_new2.log; do
  echo -n "$f " >> $O; grep '^{' $f | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], d['rtf_per_user_p50'])" >> $O
done
cat $O
