# Round-3 call x: the Qwen2 attention inside the q|k|v projection's launch (fo_gemm_qkv_rope_attn): the fused vs
# two-launch bit-exactness tests first, the full GPU suite, the listen-stage probe and the bench, fused vs not.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03x
O=gpurun_out/${R}.txt
: > $O
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_qkv" > gpurun_out/${R}_fuse_test.log 2>&1 || { tail -40 gpurun_out/${R}_fuse_test.log; exit 1; }
tail -1 gpurun_out/${R}_fuse_test.log >> $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${R}_pytest_gpu.log >> $O
for E in "FO_ATTN_FUSE=0" "FO_ATTN_FUSE=1"; do
  echo "== $E stage probe" >> $O
  env $E timeout -k 10 200 python -u scripts/llm_stage_time.py 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for i in 1 2; do
  for E in "FO_ATTN_FUSE=0" "FO_ATTN_FUSE=1"; do
    echo -n "$i [$E] " >> $O
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
    grep '^{' gpurun_out/${R}_b.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['p50_first_audio_ms'], {k: round(v,1) for k, v in d['stage_ms'].items() if k in ('listen','text','speak_after_text')})" >> $O
  done
done
cat $O
