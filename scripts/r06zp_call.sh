# round 6: the attention's per-workgroup clocks, first pass vs the same code run a second time in the workgroup
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/attn_trace.py > gpurun_out/r06zp_attn_reps.txt 2>&1 || { tail -20 gpurun_out/r06zp_attn_reps.txt; exit 1; }
FO_ATTN_TRACE_REPS=2 timeout -k 10 200 python -u scripts/attn_trace.py >> gpurun_out/r06zp_attn_reps.txt 2>&1 || { tail -20 gpurun_out/r06zp_attn_reps.txt; exit 1; }
FO_ATTN_TRACE_REPS=3 timeout -k 10 200 python -u scripts/attn_trace.py >> gpurun_out/r06zp_attn_reps.txt 2>&1 || { tail -20 gpurun_out/r06zp_attn_reps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06zp_attn_reps.txt
