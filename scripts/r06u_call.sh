# round 6: reduce prefetch templated; attention keys per split sweep on the quick bench (text steps graph-replayed)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x -k "65_to_128 or mid_rows or rope" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06u_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06u_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
SWEEP='FO_ATTN_KPS=0|FO_ATTN_KPS=64' bash scripts/gpu_call.sh r06u sweep
