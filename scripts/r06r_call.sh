# round 6: k_gemm_rows with K-thirds gate/up -- tests, probe, rocprof table of the 8-chunk stage, quick bench
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_graphs_gpu.py -q -x -s -k "65_to_128 or group or qkv_rope" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r_pytest.log 2>&1; rc=$?
grep -E "listen group|passed|failed|Error" gpurun_out/r06r_pytest.log | tail -8; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 128 > gpurun_out/r06r_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06r_probe.log; echo "probe rc=$rc"
[ $rc -eq 0 ] || exit $rc
GROUP_C=8 bash scripts/gpu_call.sh r06r profgroup quick
