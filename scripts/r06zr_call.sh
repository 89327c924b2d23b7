# round 6: the 8-wave attention's split merge without fences (sc1 partials): parity, text-step kernel time, bench
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_gpu.py tests/test_real_qwen2_gpu.py tests/test_full_depth_gpu.py tests/test_graphs_gpu.py tests/test_parity_r02_gpu.py > gpurun_out/r06zr_pytest.log 2>&1 || { tail -30 gpurun_out/r06zr_pytest.log; exit 1; }
tail -1 gpurun_out/r06zr_pytest.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r06zr_prof -o run -- python -u scripts/text_step_time.py > gpurun_out/r06zr_text.log 2>&1 || exit 1
grep 'text step' gpurun_out/r06zr_text.log
python scripts/rocpd_table.py /tmp/r06zr_prof 8 | tee gpurun_out/r06zr_text_table.txt
timeout -k 10 200 python -u scripts/attn_trace.py > gpurun_out/r06zr_attn_trace.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r06zr_attn_trace.txt | cut -c1-420
SWEEP='FO_ATTN_KPS=0|FO_ATTN_KPS=0 ' bash scripts/gpu_call.sh r06zr sweep
