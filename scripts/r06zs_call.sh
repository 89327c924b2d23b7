# round 6: attention with the fence-free split merge + DPP row reductions: the full GPU suite, smoke, text-step kernel
# time, the default bench line and a quick sweep
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zs_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06zs_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r06zs_prof -o run -- python -u scripts/text_step_time.py > gpurun_out/r06zs_text.log 2>&1 || exit 1
grep 'text step' gpurun_out/r06zs_text.log
python scripts/rocpd_table.py /tmp/r06zs_prof 8 | tee gpurun_out/r06zs_text_table.txt
bash scripts/gpu_call.sh r06zs smoke bench
