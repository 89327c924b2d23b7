# round 6: parallel chunk attention -- parity, grouped stage probe, A/B, duplex line
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_parity_r02_gpu.py tests/test_graphs_gpu.py tests/test_serve_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06d_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/group_stage_time.py 4 > gpurun_out/r06d_group.log 2>&1 || exit $?
grep "C=" gpurun_out/r06d_group.log
SWEEP='FO_ENC_CHUNK_ATTN=0|' bash scripts/gpu_call.sh r06d sweep duplex
