cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/r06a_pytest.log
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/group_stage_time.py 1 2 3 4 > gpurun_out/r06a_group.log 2>&1; rc=$?
cat gpurun_out/r06a_group.log | tail -8
[ $rc -eq 0 ] || exit $rc
SWEEP='FO_LISTEN_CHUNKS=1|FO_LISTEN_CHUNKS=2|FO_LISTEN_CHUNKS=4' bash scripts/gpu_call.sh r06a sweep
