# round 6: k_gemm_rows default for 65..128 rows -- GEMM + listen-group tests, stage probe C 4 / 8, bench C 4 vs 8
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_graphs_gpu.py -q -x -s -k "65_to_128 or group" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_pytest.log 2>&1; rc=$?
grep -E "listen group|passed|failed|Error" gpurun_out/r06n_pytest.log | tail -8; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 128 > gpurun_out/r06n_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06n_probe.log; echo "probe rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/group_stage_time.py 4 8 > gpurun_out/r06n_group.log 2>&1; rc=$?
tail -4 gpurun_out/r06n_group.log
[ $rc -eq 0 ] || exit $rc
SWEEP='FO_LISTEN_CHUNKS=4|FO_LISTEN_CHUNKS=8' bash scripts/gpu_call.sh r06n sweep
