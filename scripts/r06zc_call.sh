# round 6: vocoder chunk loop with the next chunk's window prefetched (FO_CONV_PREFETCH=1) vs staged (0)
cd $GRAFT_REPO_ROOT
FO_CONV_PREFETCH=1 timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "codec or vocoder or tts or speak or llm2tts" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zc_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06zc_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for pf in 0 1; do
  FO_CONV_PREFETCH=$pf timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r06zc_voc_${pf}_${r}.log 2>&1 || exit 1
  echo "FO_CONV_PREFETCH=$pf: $(grep -v amdgpu gpurun_out/r06zc_voc_${pf}_${r}.log | tail -1)"
done; done
SWEEP='FO_CONV_PREFETCH=0|FO_CONV_PREFETCH=1' bash scripts/gpu_call.sh r06zc sweep
