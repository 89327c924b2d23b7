# round 6: k_gemm_wrow (one tile per wave, X staged once per workgroup) -- GEMM tests, probe against k_gemm_rows / halves
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x -k "65_to_128" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06m_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r06m_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 72 128 > gpurun_out/r06m_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06m_probe.log; echo "probe rc=$rc"
