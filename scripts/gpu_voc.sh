#!/bin/bash
# vocoder parity tests, event timing and a kernel trace (summarised by scripts/rocpd_summary.py)
set -e
tag=${1:-vp}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engines_gpu.py tests/test_parity_r02_gpu.py tests/test_checkpoint_gpu.py > gpurun_out/$tag/tests.log 2>&1
timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/$tag/time.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$tag/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/vocoder_time.py 8 5 > $GRAFT_REPO_ROOT/gpurun_out/$tag/trace.log 2>&1
cd $GRAFT_REPO_ROOT
python scripts/rocpd_summary.py $(find gpurun_out/$tag/trace -name "*.db" | head -1) "conv|codec|post" 1 > gpurun_out/$tag/summary.txt
tail -2 gpurun_out/$tag/tests.log; cat gpurun_out/$tag/time.log; head -20 gpurun_out/$tag/summary.txt
