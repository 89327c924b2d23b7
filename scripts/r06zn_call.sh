# round 6: the text-step attention's per-workgroup clocks with a loads-landed stamp, warm and cold caches
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/attn_trace.py > gpurun_out/r06zn_attn_trace.txt 2>&1 || { tail -20 gpurun_out/r06zn_attn_trace.txt; exit 1; }
ATTN_TRACE_COLD=1 timeout -k 10 200 python -u scripts/attn_trace.py >> gpurun_out/r06zn_attn_trace.txt 2>&1 || { tail -20 gpurun_out/r06zn_attn_trace.txt; exit 1; }
cat gpurun_out/r06zn_attn_trace.txt
