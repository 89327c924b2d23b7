set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for k in 256 128 512; do
  timeout -k 10 300 env FO_ATTN_KPS=$k python -u bench.py --scenario duplex --out gpurun_out/r04zd_dup_kps$k.json > gpurun_out/r04zd_dup_kps$k.log 2>&1 || { echo "fail kps $k"; tail -5 gpurun_out/r04zd_dup_kps$k.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04zd_dup_kps$k.json')); print('kps $k', d['value'], d['p50_decision_ms'], d.get('p90_decision_ms'), d.get('tick_stage_ms',{}).get('qwen2'))"
done
