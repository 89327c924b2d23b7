# GPU tests + one default-config bench line (no cpu baseline); each GPU step time-limited, && chained.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; grep '^{' gpurun_out/bench_quick.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k: d[k] for k in ('value','ms_per_step','p50_first_audio_ms','p50_first_emit_gated_ms','rtf_per_user_p50')}, d['roofline']['achieved'], d['roofline']['avg_launch_us'])"
exit $rc
