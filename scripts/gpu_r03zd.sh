# Round-3 call zd: the committed tree as the round ends -- GPU suite, smoke(), the default bench line (short).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zd
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/${R}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 && tail -1 gpurun_out/${R}_smoke.log && \
timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 3 --out gpurun_out/${R}_bench.json > gpurun_out/${R}_bench.log 2>&1
rc=$?
grep '^{' gpurun_out/${R}_bench.log | cut -c1-300
echo "EXIT $rc"
exit $rc
