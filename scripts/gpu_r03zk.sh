# Round-3 call zk: the final tree (lane without the launched-out drain) -- GPU suite, smoke(), the full default
# bench line (cpu_baseline, config-2 leg), the N = 2 rehearsal (receive-only replica, two ranks on one GPU over gloo).
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zk
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/${R}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 && tail -1 gpurun_out/${R}_smoke.log && \
timeout -k 10 900 python -u bench.py --out gpurun_out/${R}_bench.json > gpurun_out/${R}_bench.log 2>&1 && \
FO_DIST_REHEARSAL=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline --no-single-user --out gpurun_out/${R}_rehearsal_n2.json > gpurun_out/${R}_rehearsal_n2.log 2>&1
rc=$?
grep '^{' gpurun_out/${R}_bench.log | cut -c1-200
echo "EXIT $rc"
exit $rc
