# Round-3 call j: grouped vocoder launches (polyphase components in one launch, the resblock chains side by
# side, their last convs summed: 7 launches a stage) -- the codec tests, call time grouped vs one launch per conv
# (x 32/64-channel chunks), its kernel trace, then the GPU suite and the turn bench.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_parity_r02_gpu.py tests/test_replica_gpu.py -q -x -k "codec or vocoder or generator or speak" --timeout 120 --timeout-method thread > gpurun_out/r03j_codec_tests.log 2>&1 && \
timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03j_voc_grouped.txt 2>&1 && \
FO_CODEC_GROUPED=0 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03j_voc_single.txt 2>&1 && \
FO_CONV_CK=64 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03j_voc_grouped_ck64.txt 2>&1 && \
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/voc_t_r03j -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_t_r03j.log 2>&1 && cd $ROOTD && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03j_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --out gpurun_out/r03j_bench.json > gpurun_out/r03j_bench.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
