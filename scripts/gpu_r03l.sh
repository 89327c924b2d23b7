# Round-3 call l: the fused ResBlock1 step kernel (fo_conv_pair_multi) -- codec tests, call time pair vs two
# launches per step, the half-time-tile probe, a kernel trace; then the GPU suite and the default bench line.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_parity_r02_gpu.py tests/test_replica_gpu.py -q -x -k "codec or vocoder or generator or speak" --timeout 120 --timeout-method thread > gpurun_out/r03l_codec_tests.log 2>&1
rc=$?; echo "codec tests rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03l_voc_pair.txt 2>&1 && \
FO_CODEC_PAIR=0 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03l_voc_nopair.txt 2>&1 && \
FO_CODEC_PAIR=0 FO_CONV_HALFT=1 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03l_voc_nopair_halft.txt 2>&1 && \
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/voc_t_r03l -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_t_r03l.log 2>&1 && cd $ROOTD && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03l_pytest_gpu.log 2>&1
rc=$?; echo "suite rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u bench.py --out gpurun_out/r03l_bench.json > gpurun_out/r03l_bench.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
