# config-5 duplex bench line, the vocoder call timing, the counter list, and two --pmc passes on the
# vocoder's MFMA kernels (one pass per counter block, each its own run: MI355X_MICROARCH.md rocprofv3 PMC slots)
set -o pipefail
R=${1:-r02}
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --scenario duplex --no-cpu-baseline > gpurun_out/${R}_duplex.log 2>&1 && \
timeout -k 10 120 python scripts/vocoder_time.py 8 20 > gpurun_out/${R}_vocoder.log 2>&1 && \
(timeout -k 10 60 rocprofv3 -L > gpurun_out/${R}_counters.txt 2>&1 || true) && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-include-regex k_conv_cl -d $ROOTD/gpurun_out/pmc_voc1_$R -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/${R}_pmc_voc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex k_conv_cl -d $ROOTD/gpurun_out/pmc_voc2_$R -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/${R}_pmc_voc2.log 2>&1
rc=$?
echo EXIT $rc >> $ROOTD/gpurun_out/${R}_vocoder.log
exit $rc
