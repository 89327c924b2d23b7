# Round-3 call r: the round-end paths on the current code -- smoke(), the duplex bench line (config 5, one
# replica), and the N = 2 rehearsal (two ranks on one GPU over gloo: receive-only replica, weight broadcast).
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --scenario duplex --out gpurun_out/${R}_duplex.json > gpurun_out/${R}_duplex.log 2>&1 && \
FO_DIST_REHEARSAL=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline --no-single-user --out gpurun_out/${R}_rehearsal_n2.json > gpurun_out/${R}_rehearsal_n2.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
