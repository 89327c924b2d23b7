# round 6: k_gemm_rows weight-ring depth probe (no X loads: 7 vs 11 k-steps of weights in flight)
cd $GRAFT_REPO_ROOT
ROWS_DEPTH=1 timeout -k 10 300 python -u scripts/gemm_rows_probe.py 128 > gpurun_out/r06w_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06w_probe.log; echo "probe rc=$rc"
