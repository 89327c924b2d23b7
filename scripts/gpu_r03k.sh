# Round-3 call k: the default bench line (cpu_baseline at 64 BLAS threads = one socket, config 2 leg), then
# kernel traces of the AR step and the text step alone.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --out gpurun_out/r03k_bench.json > gpurun_out/r03k_bench.log 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_tts_r03k -o tts -f csv -- python3 $ROOTD/scripts/tts_step_time.py 8 multi > $ROOTD/gpurun_out/prof_tts_r03k.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_text_r03k -o text -f csv -- python3 $ROOTD/scripts/text_step_time.py 8 20 > $ROOTD/gpurun_out/prof_text_r03k.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
