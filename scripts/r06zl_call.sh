# round 6: 4-wave attention (64-key tiles) with 64-key splits vs the default (8 waves, 128-key tiles and splits)
cd $GRAFT_REPO_ROOT
for cfg in "FO_ATTN_NW=8" "FO_ATTN_NW=4 FO_ATTN_KPS=64" "FO_ATTN_NW=4"; do
  env $cfg timeout -k 10 200 python -u scripts/text_step_time.py > gpurun_out/r06zl_text.log 2>&1 || exit 1
  echo "$cfg: $(grep 'text step' gpurun_out/r06zl_text.log)"
done
SWEEP='FO_ATTN_NW=8|FO_ATTN_NW=4 FO_ATTN_KPS=64' bash scripts/gpu_call.sh r06zl sweep
