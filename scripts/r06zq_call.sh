# round 6: the attention tile's phases per workgroup (K split, each wave's arrival at the max exchange, barriers, PV)
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/attn_trace.py > gpurun_out/r06zq_attn_phases.txt 2>&1 || { tail -20 gpurun_out/r06zq_attn_phases.txt; exit 1; }
FO_ATTN_TRACE_REPS=2 timeout -k 10 200 python -u scripts/attn_trace.py >> gpurun_out/r06zq_attn_phases.txt 2>&1 || { tail -20 gpurun_out/r06zq_attn_phases.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06zq_attn_phases.txt
