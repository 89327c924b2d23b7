# round 6 final set: full GPU suite, smoke, the default bench line (cpu_baseline + config 2), rocprof stats + FETCH pass
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06v_pytest.log 2>&1; rc=$?
tail -6 gpurun_out/r06v_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_call.sh r06v smoke bench prof fetch
