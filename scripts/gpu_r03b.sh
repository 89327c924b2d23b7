# Round-3 call b: the new real-geometry Qwen2 / sampler-error tests first, then the whole GPU suite and the
# text-step timing (split arg-max sampler).
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_real_qwen2_gpu.py tests/test_sampler_errors_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b_new_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u scripts/text_step_time.py 8 40 > gpurun_out/r03b_text_step.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
