# round 6: k_gemm_rows variants (nt weight loads, ring depths) against the row halves
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/gemm_rows_probe.py 72 128 > gpurun_out/r06k_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r06k_probe.log; echo "probe rc=$rc"
