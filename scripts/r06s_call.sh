# round 6: k_gemm_rows at 33..64 rows (probe 4) against k_gemm_xsk
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 40 48 64 > gpurun_out/r06s_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06s_probe.log; echo "probe rc=$rc"
