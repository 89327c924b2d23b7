# round 6: the text step's attention kernel vs keys per split (rocprofv3 of scripts/text_step_time.py per setting)
cd $GRAFT_REPO_ROOT
for k in 64 256 512; do
  (cd /tmp && FO_ATTN_KPS=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06zh_kps$k -o text -f csv -- python3 $GRAFT_REPO_ROOT/scripts/text_step_time.py) > gpurun_out/r06zh_kps$k.log 2>&1 || exit 1
  echo "== FO_ATTN_KPS=$k"; python3 scripts/trace_table.py gpurun_out/r06zh_kps$k 40 text 2>&1 | grep -E "attn|total" | head -4
  grep -v amdgpu gpurun_out/r06zh_kps$k.log | grep -iE "step|ms" | grep -v rocprofv3 | tail -1
done
