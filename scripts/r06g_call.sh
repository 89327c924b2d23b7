# round 6: k_gemm_rows (65..128-row weight streams) -- its GEMM tests, then the probe against the row halves
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x -k "65_to_128 or mid_rows" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06g_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r06g_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 64 72 96 128 > gpurun_out/r06g_probe.log 2>&1; rc=$?
cat gpurun_out/r06g_probe.log | grep -v amdgpu.ids; echo "probe rc=$rc"
