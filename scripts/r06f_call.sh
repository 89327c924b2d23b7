# round 6: grouped-listen tolerances + the isolated grouped-encoder check, C = 8 stage probe, C 4 vs 8 bench sweep
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_graphs_gpu.py tests/test_parity_r02_gpu.py -k "group or grouped" -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06f_pytest.log 2>&1; rc=$?
grep -E "grouped encoder|listen group|passed|failed" gpurun_out/r06f_pytest.log
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/group_stage_time.py 4 8 > gpurun_out/r06f_group.log 2>&1; rc=$?
tail -4 gpurun_out/r06f_group.log
[ $rc -eq 0 ] || exit $rc
SWEEP='FO_LISTEN_CHUNKS=4|FO_LISTEN_CHUNKS=8' bash scripts/gpu_call.sh r06f sweep
