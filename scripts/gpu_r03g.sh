# Round-3 call g: stream-priority A/B on the turn bench (default; the encoder side stream at the device's least
# priority; the engine stream at its greatest), then the listen stage-overlap probe.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --no-single-user"
timeout -k 10 300 python -u -c "
import ctypes, sys; sys.path.insert(0, 'freeze-omni_amd')
from fo import _lib
lo, hi = ctypes.c_int(), ctypes.c_int()
_lib.call('fo_stream_priority_range', ctypes.byref(lo), ctypes.byref(hi)); print('priority range least', lo.value, 'greatest', hi.value)
" > gpurun_out/r03g_prio_range.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03g_bench_base.json > gpurun_out/r03g_bench_base.log 2>&1 && \
FO_SIDE_PRIORITY=-1 timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03g_bench_sidelow.json > gpurun_out/r03g_bench_sidelow.log 2>&1 && \
FO_MAIN_PRIORITY=1 timeout -k 10 300 python -u bench.py $A --out gpurun_out/r03g_bench_mainhigh.json > gpurun_out/r03g_bench_mainhigh.log 2>&1 && \
timeout -k 10 200 python -u scripts/llm_stage_time.py > gpurun_out/r03g_stage_overlap.txt 2>&1 && \
timeout -k 10 300 python -u scripts/down_sweep.py > gpurun_out/r03g_down_sweep.txt 2>&1 && \
FO_SIDE_PRIORITY=-1 timeout -k 10 200 python -u scripts/llm_stage_time.py > gpurun_out/r03g_stage_overlap_sidelow.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
