# round 6 last tree check: the full GPU suite, smoke, the default bench line
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zj_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06zj_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_call.sh r06zj smoke bench
