# round 6: k_gemm_rows with equal weight / X leads (the in-order vmcnt caps the weights' depth at X's lead)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x -k "65_to_128 or rope" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06x_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06x_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 72 128 > gpurun_out/r06x_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06x_probe.log; echo "probe rc=$rc"
[ $rc -eq 0 ] || exit $rc
GROUP_C=8 bash scripts/gpu_call.sh r06x profgroup quick
