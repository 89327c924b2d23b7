#!/bin/bash
# Kernel trace of the listen-chunk stages (scripts/llm_stage_time.py: LLM stage alone, encoder alone, both),
# summarised per kernel and grid by scripts/rocpd_summary.py.
set -e
tag=${1:-lt}
mkdir -p gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$tag/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/llm_stage_time.py > $GRAFT_REPO_ROOT/gpurun_out/$tag/run.log 2>&1
cd $GRAFT_REPO_ROOT
python scripts/rocpd_summary.py $(find gpurun_out/$tag/trace -name "*.db" | head -1) "" > gpurun_out/$tag/summary.txt
tail -4 gpurun_out/$tag/run.log; head -40 gpurun_out/$tag/summary.txt
