# round 6: 2-wave attention (32-key tiles) on 32-key splits for the text step vs the default
cd $GRAFT_REPO_ROOT
FO_ATTN_KPS=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_gpu.py tests/test_real_qwen2_gpu.py tests/test_full_depth_gpu.py > gpurun_out/r06zm_pytest.log 2>&1 || { tail -30 gpurun_out/r06zm_pytest.log; exit 1; }
tail -2 gpurun_out/r06zm_pytest.log
for cfg in "FO_ATTN_KPS=0" "FO_ATTN_KPS=32"; do
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06zm_prof_${cfg#FO_ATTN_KPS=} -o run -- python -u scripts/text_step_time.py > gpurun_out/r06zm_text.log 2>&1 || exit 1
  echo "$cfg: $(grep 'text step' gpurun_out/r06zm_text.log)"
  f=$(find gpurun_out/r06zm_prof_${cfg#FO_ATTN_KPS=} -name '*kernel_stats.csv' | head -1); grep -i "attn" $f | cut -c1-160
done
SWEEP='FO_ATTN_KPS=0|FO_ATTN_KPS=32' bash scripts/gpu_call.sh r06zm sweep
