# round 6: k_gemm_rows with twice the tiles per workgroup and K split further (probe 3) against the default
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 72 128 > gpurun_out/r06p_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06p_probe.log; echo "probe rc=$rc"
