# Round-3 call zz: the final profile set (7-tile down, 8-wave attention with two tiles in flight, vocoder streams at the default priority,
# text steps queued ahead, batched silence cut) -- the GPU suite, the default bench line (cpu_baseline, config-2
# leg), rocprofv3 kernel stats of the bench, the FETCH_SIZE pass of the dominant kernel, the AR step's kernel
# trace, the duplex line.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03zz
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1
rc=$?; echo "suite rc $rc"; tail -1 gpurun_out/${R}_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u bench.py --out gpurun_out/${R}_bench.json > gpurun_out/${R}_bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$R -o bench -f csv -- python3 $ROOTD/bench.py --config real --steps 2 --warmup 1 --no-cpu-baseline --no-single-user > $ROOTD/gpurun_out/prof_bench_$R.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gemm_xs -d $ROOTD/gpurun_out/pmc_$R -o fetch -f csv -- python3 $ROOTD/bench.py --config real --steps 2 --warmup 1 --no-cpu-baseline --no-single-user > $ROOTD/gpurun_out/pmc_bench_$R.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_tts_$R -o tts -f csv -- python3 $ROOTD/scripts/tts_step_time.py 8 multi > $ROOTD/gpurun_out/prof_tts_$R.log 2>&1 && \
cd $ROOTD && timeout -k 10 400 python -u bench.py --scenario duplex --out gpurun_out/${R}_duplex.json > gpurun_out/${R}_duplex.log 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1
rc=$?
[ $rc -eq 0 ] && FO_DIST_REHEARSAL=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline --no-single-user --out gpurun_out/${R}_rehearsal_n2.json > gpurun_out/${R}_rehearsal_n2.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
