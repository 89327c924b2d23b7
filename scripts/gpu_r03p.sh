# Round-3 call p: two sentence-speech workers (sentence k on worker k % 2, each with its own streams and graph
# caches) vs one, in one call; the speech GPU tests first.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --no-single-user"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03p_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --tts-workers 2 --out gpurun_out/r03p_w2.json > gpurun_out/r03p_w2.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03p_w1.json > gpurun_out/r03p_w1.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --tts-workers 2 --out gpurun_out/r03p_w2b.json > gpurun_out/r03p_w2b.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --tts-workers 4 --out gpurun_out/r03p_w4.json > gpurun_out/r03p_w4.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
