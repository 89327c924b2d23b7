# round 6: wave reductions by lane swaps / DPP instead of ds_bpermute (same operands, same order): the full GPU suite,
# the AR decode step and text step kernel tables, a quick bench
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zu_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06zu_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r06zu_pytest.log | head -20; exit 1; }
bash scripts/gpu_call.sh r06zu tts text quick
