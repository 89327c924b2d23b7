# round 6 final-tree check: full GPU suite, smoke, the default bench line, rocprof + FETCH, duplex line, N = 2 rehearsal
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zb_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06zb_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_call.sh r06zb smoke bench prof fetch duplex rehearsal
