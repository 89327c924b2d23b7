# Same-box A/B of two builds of libfo_hip.so on the AR decode step (profiles/r05v_sampler_ab.txt): the candidate in
# freeze-omni_amd/fo/libfo_hip.so against a build of the previous commit placed at fo/libfo_hip_ab.so (git worktree
# + make OUT=...), each under rocprofv3 --kernel-trace, alternated twice.  Run on the GPU box: bash scripts/ab_sampler_r05v.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
 for v in old new; do
  if [ $v = old ]; then export FO_LIB_PATH=$GRAFT_REPO_ROOT/freeze-omni_amd/fo/libfo_hip_ab.so; else unset FO_LIB_PATH; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r05v_${v}$i -o tts -f csv -- \
     python3 $GRAFT_REPO_ROOT/scripts/tts_step_time.py 8 multi) > gpurun_out/r05v_${v}$i.log 2>&1 || exit 1
  unset FO_LIB_PATH
  python3 scripts/step_timeline.py gpurun_out/r05v_${v}$i > gpurun_out/r05v_${v}$i.txt 2>&1 || exit 1
  echo "$v$i: $(tail -1 gpurun_out/r05v_${v}$i.txt) | $(grep k_sample gpurun_out/r05v_${v}$i.txt) | $(grep 'us per step' gpurun_out/r05v_${v}$i.log | tr '\n' ' ')"
 done
done
