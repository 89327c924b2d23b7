# Round-3 call o: turn-bench A/B in one call: default; Python switch interval 0.5 ms (the sentence-speech worker
# thread beside the text loop) and 0.2 ms; default again.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --no-single-user"
timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03o_base.json > gpurun_out/r03o_base.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --switch-interval 0.0005 --out gpurun_out/r03o_sw.json > gpurun_out/r03o_sw.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --switch-interval 0.0002 --out gpurun_out/r03o_sw2.json > gpurun_out/r03o_sw2.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03o_base2.json > gpurun_out/r03o_base2.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
