# Round-3 call h: GPU suite on the 8-tile x 8-way Qwen2 down; the encoder stage's GEMM shape beside the Qwen2
# stage (FO_ENC_TUNE: fewer, wider workgroups re-read the 32 activation rows less often); the graph-replayed
# small-GEMM sweep (o / q|k|v / TTS shapes, with the in-launch split merge); the turn bench.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03h_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc $rc"; [ $rc -le 1 ] || exit $rc
for t in "" "16,2" "8,2" "8,1" "4,2"; do
  FO_ENC_TUNE=$t timeout -k 10 200 python -u scripts/llm_stage_time.py > gpurun_out/r03h_stage_enc_${t/,/_}.txt 2>&1 || exit $?
done
timeout -k 10 400 python -u scripts/gemm_graph_sweep.py > gpurun_out/r03h_gemm_graph_sweep.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --out gpurun_out/r03h_bench.json > gpurun_out/r03h_bench.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
