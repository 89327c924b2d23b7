# round 6: full GPU suite, smoke, then the round's profile set (rocprof stats + FETCH pass) and a quick line
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_pytest.log 2>&1; rc=$?
tail -6 gpurun_out/r06e_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_call.sh r06e smoke quick prof fetch
