# round 6: the text step alone under rocprofv3 (per-kernel split of the turn's largest stage)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_call.sh r06zd text && python3 scripts/trace_table.py gpurun_out/r06zd_prof_text 30 text > gpurun_out/r06zd_text_table.txt 2>&1; head -34 gpurun_out/r06zd_text_table.txt; grep -v amdgpu gpurun_out/r06zd_prof_text.log | tail -3
