# Round-3 call d: measurement passes for the committed profiles -- rocprofv3 kernel stats of the bench, a
# FETCH_SIZE pass on the dominant kernel, the vocoder's MFMA counter passes (current k_conv_cl kernels), the
# MFMA / busy counters of the Qwen2 weight-stream GEMMs, the AR step's kernel trace, and the down sweep.
# Each pass has its own time limit; counters never share a pass with trace domains (guide).
set -o pipefail
R=${1:-r03d}
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--config real --steps 2 --warmup 1 --no-cpu-baseline --no-single-user"
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$R -o bench -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/prof_bench_$R.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gemm_xs -d $ROOTD/gpurun_out/pmc_$R -o fetch -f csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/pmc_bench_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-include-regex "k_conv|k_codec" -d $ROOTD/gpurun_out/voc_p1_$R -o p1 -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_p1_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_conv|k_codec" -d $ROOTD/gpurun_out/voc_p2_$R -o p2 -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_p2_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/voc_t_$R -o voc -f csv -- python3 $ROOTD/scripts/vocoder_time.py 8 5 > $ROOTD/gpurun_out/voc_t_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-include-regex "k_gemm" -d $ROOTD/gpurun_out/llm_p1_$R -o p1 -f csv -- python3 $ROOTD/scripts/text_step_time.py 8 10 > $ROOTD/gpurun_out/llm_p1_$R.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_gemm" -d $ROOTD/gpurun_out/llm_p2_$R -o p2 -f csv -- python3 $ROOTD/scripts/text_step_time.py 8 10 > $ROOTD/gpurun_out/llm_p2_$R.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_tts_$R -o tts -f csv -- python3 $ROOTD/scripts/tts_step_time.py 8 multi > $ROOTD/gpurun_out/prof_tts_$R.log 2>&1 && \
cd $ROOTD && timeout -k 10 300 python -u scripts/down_sweep.py > gpurun_out/${R}_down_sweep.txt 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
