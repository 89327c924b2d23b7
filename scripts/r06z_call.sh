# round 6: bf16 paged-KV A/B (verdict r05 item 6) -- the full-depth drift test and the real-geometry goldens with the
# appended K / V rounded to bf16 (FO_KV_BF16=1) against the fp32 default, then the quick bench both ways
cd $GRAFT_REPO_ROOT
for kv in 0 1; do
  FO_KV_BF16=$kv timeout -k 10 500 python -u -m pytest tests/test_full_depth_gpu.py tests/test_real_qwen2_gpu.py tests/test_parity_r02_gpu.py tests/test_real_geometry_gpu.py -q -s --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z_kv${kv}_pytest.log 2>&1; rc=$?
  echo "== FO_KV_BF16=$kv rc=$rc"; grep -E "full depth|passed|failed|FAILED|drift" gpurun_out/r06z_kv${kv}_pytest.log | tail -12
  [ $rc -le 1 ] || exit $rc
done
SWEEP='FO_KV_BF16=0|FO_KV_BF16=1' bash scripts/gpu_call.sh r06z sweep
