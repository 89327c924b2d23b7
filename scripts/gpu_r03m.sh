# Round-3 call m: the vocoder as it ships (grouped launches, 32-channel chunks, the pair kernel on the 16/32-channel
# stages): call time, kernel trace, and the MFMA counter passes (separate --pmc runs, no trace domains with them).
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03m
timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/${R}_voc.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_parity_r02_gpu.py -q -x -k "codec or vocoder or generator" --timeout 120 --timeout-method thread > gpurun_out/${R}_codec_tests.log 2>&1 && \
cd /tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/voc_t_$R -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_t_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-include-regex "k_conv|k_codec" -d $ROOTD/gpurun_out/voc_p1_$R -o p1 -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_p1_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_conv|k_codec" -d $ROOTD/gpurun_out/voc_p2_$R -o p2 -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_p2_$R.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
