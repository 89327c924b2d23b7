# round 6: stream priorities under the grouped listen (the encoder pass on the side stream beside the Qwen2 stage)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x -k "65_to_128" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ze_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/r06ze_pytest.log; [ $rc -eq 0 ] || exit $rc
SWEEP='FO_SIDE_PRIORITY=0|FO_SIDE_PRIORITY=-1|FO_MAIN_PRIORITY=1' bash scripts/gpu_call.sh r06ze sweep
