# round 6: empty attention split slots leave before their loads -- attention tests, the text step's attention under
# rocprofv3, quick bench
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_attn_gpu.py tests/test_real_qwen2_gpu.py tests/test_graphs_gpu.py tests/test_full_depth_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zi_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06zi_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06zi_text -o text -f csv -- python3 $GRAFT_REPO_ROOT/scripts/text_step_time.py) > gpurun_out/r06zi_text.log 2>&1 || exit 1
python3 scripts/trace_table.py gpurun_out/r06zi_text 40 text 2>&1 | grep -E "attn|total" | head -4; grep "text step" gpurun_out/r06zi_text.log
bash scripts/gpu_call.sh r06zi quick
