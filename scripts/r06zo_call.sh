# round 6: instruction-fetch counters of the text step's kernels (is the attention's one-shot 62 KB body fetch-bound?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=/tmp/r06zo
mkdir -p $P
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_WAVES -d $P/p1 -o run -- python -u scripts/text_step_time.py 8 5 > gpurun_out/r06zo_p1.log 2>&1 || { tail -5 gpurun_out/r06zo_p1.log; exit 1; }
python scripts/rocpd_pmc.py $P/p1 12 > gpurun_out/r06zo_pmc.txt 2>&1; cat gpurun_out/r06zo_pmc.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $P/p2 -o run -- python -u scripts/text_step_time.py 8 5 > gpurun_out/r06zo_p2.log 2>&1 || { tail -5 gpurun_out/r06zo_p2.log; exit 1; }
python scripts/rocpd_pmc.py $P/p2 12 >> gpurun_out/r06zo_pmc.txt 2>&1; tail -13 gpurun_out/r06zo_pmc.txt
