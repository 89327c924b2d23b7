# round 6: the <= 8-row o (and layer-0 q|k|v) projections with K split 2 / 4 ways (FO_SMALL_SPLIT) -- text step alone
# and the quick bench
cd $GRAFT_REPO_ROOT
for sp in 0 2 4; do
  FO_SMALL_SPLIT=$sp timeout -k 10 200 python -u scripts/text_step_time.py > gpurun_out/r06zk_text_$sp.log 2>&1 || exit 1
  echo "FO_SMALL_SPLIT=$sp: $(grep 'text step' gpurun_out/r06zk_text_$sp.log)"
done
SWEEP='FO_SMALL_SPLIT=0|FO_SMALL_SPLIT=2|FO_SMALL_SPLIT=4' bash scripts/gpu_call.sh r06zk sweep
