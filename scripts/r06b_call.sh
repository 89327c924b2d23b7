# round 6: the grouped listen (encoder + Qwen2 stages over C chunks) -- parity tests, stage probe, bench sweep
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_graphs_gpu.py tests/test_serve_gpu.py tests/test_parity_r02_gpu.py tests/test_api_gpu.py tests/test_attn_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06b_pytest.log 2>&1; rc=$?
tail -25 gpurun_out/r06b_pytest.log
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/group_stage_time.py 1 2 4 > gpurun_out/r06b_group.log 2>&1; rc=$?
tail -8 gpurun_out/r06b_group.log
[ $rc -eq 0 ] || exit $rc
SWEEP='FO_LISTEN_CHUNKS=2|FO_LISTEN_CHUNKS=4' bash scripts/gpu_call.sh r06b sweep
