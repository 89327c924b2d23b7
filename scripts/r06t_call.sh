# round 6: k_gemm_reduce prefetching 16 slabs -- GEMM tests, 8-chunk stage table, quick bench
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06t_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06t_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
GROUP_C=8 bash scripts/gpu_call.sh r06t profgroup quick
