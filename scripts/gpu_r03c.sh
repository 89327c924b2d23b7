# Round-3 call c: new tests (real-geometry Qwen2 vs the reference, sampler NaN errors, reference-signature
# constructors, pool replicas), the whole GPU suite, the text-step timing (split arg-max), then the reshaped
# turn bench (32 text tokens, 4 sentences, speech per sentence beside the text decode; cpu_baseline = config 1
# end to end), its serial A/B and the attention keys-per-split sweep.
# A test FAILURE (pytest rc 1) does not stop the measurements; any other status (fault, abort, time limit) does.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_real_qwen2_gpu.py tests/test_sampler_errors_gpu.py tests/test_facades_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r03c_new_tests.log 2>&1
rc=$?; echo "new tests rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03c_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/text_step_time.py 8 40 > gpurun_out/r03c_text_step.txt 2>&1 && \
timeout -k 10 500 python -u bench.py --out gpurun_out/r03c_bench.json > gpurun_out/r03c_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-concurrent-tts --no-cpu-baseline --no-single-user --out gpurun_out/r03c_bench_serial.json > gpurun_out/r03c_bench_serial.log 2>&1 && \
timeout -k 10 200 python -u scripts/attn_kps_sweep.py > gpurun_out/r03c_attn_kps.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
