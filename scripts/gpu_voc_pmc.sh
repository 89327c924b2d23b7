#!/bin/bash
# Stall-reason counters on the vocoder convs (k_conv_cl), one rocprofv3 --pmc pass per counter group
# (guide limits: <= 8 SQ, <= 2 GRBM per pass), csv output summarised by scripts/pmc_summary.py.
set -e
tag=${1:-vpmc}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_IFETCH" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "${2:-k_conv_cl}" --output-format csv -d $out/p$i -o p$i -- python3 $GRAFT_REPO_ROOT/scripts/vocoder_time.py 8 3 > $out/p$i.log 2>&1
done
cd $GRAFT_REPO_ROOT
python scripts/pmc_summary.py $out > $out/summary.txt
cat $out/summary.txt
