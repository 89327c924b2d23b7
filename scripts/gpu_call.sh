# One parameterised GPU call (replaces the per-call scripts of rounds 1-3).
#   usage: bash scripts/gpu_call.sh <tag> <step> [<step> ...]
# Steps run in order, each under its own time limit, and the call stops at the first failing step (no GPU step is
# started after a fault, abort or time-out). Outputs go to gpurun_out/<tag>_*.
#   tests      pytest -m gpu (PYTEST_K=expr narrows it)
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (cpu_baseline + config-2 leg)      -> <tag>_bench.json
#   quick      bench without the CPU baseline / config-2 leg, 3 turns    -> <tag>_quick.json
#   prof       rocprofv3 --kernel-trace --stats of the bench (2 turns)   -> <tag>_prof/
#   fetch      FETCH_SIZE pass on the dominant kernel                    -> <tag>_pmc/
#   fetchdup   FETCH_SIZE pass on the duplex line's split-K / encoder kernels  -> <tag>_fetchdup.txt
#   tts        rocprofv3 kernel stats of the AR decode step alone        -> <tag>_prof_tts/
#   text       rocprofv3 kernel stats of the text step alone             -> <tag>_prof_text/
#   steptrace  per-node timeline of the AR decode step (kernel trace)   -> <tag>_step_timeline.txt
#   duplex     the config-5 duplex line                                  -> <tag>_duplex.json
#   profdup    rocprofv3 kernel trace + stats of a 20 s duplex run       -> <tag>_profdup/, <tag>_profdup_table.txt
#   profstage  rocprofv3 kernel trace of scripts/llm_stage_time.py (LLM / encoder stage replays) -> <tag>_profstage_table.txt
#   profgroup  rocprofv3 kernel trace of scripts/group_stage_time.py $GROUP_C (grouped listen stages) -> <tag>_profgroup_table.txt
#   rehearsal  the N = 2 path on one GPU (FO_DIST_REHEARSAL, gloo)      -> <tag>_rehearsal_n2.json
#   vocpmc     vocoder: MFMA counter passes + FETCH_SIZE + kernel trace of one 8-user call -> <tag>_vocoder_mfma.json
#   ddp1       bench.py as one torch.distributed.run rank (world 1: RCCL init, broadcast, checksum) -> <tag>_ddp1.json
#   n2guard    bench.py --gpus 2 on this 1-GPU box must refuse without touching the GPU
#   ab         ENV_A / ENV_B (e.g. 'FO_X=0') alternated twice on the quick bench -> <tag>_ab.txt
#   abdup      DUP_SET='A=1|B=2|' settings, two rounds on a 30 s duplex line -> <tag>_abdup.txt
#   sweep      SWEEP='A=1|B=2|' settings ('|'-separated, empty = default), two rounds on the quick bench -> <tag>_sweep.txt
#   py:<script args>   any scripts/ probe, e.g. 'py:llm_stage_time.py' (200 s limit)
set -o pipefail
R=$1; shift
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${R}
line() {   # the JSON line's headline fields
  grep '^{' "$1" | tail -1 | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('ms_per_step'), d.get('p50_first_audio_ms'), d.get('p50_decision_ms'),
 {k: round(v,1) for k, v in (d.get('stage_ms') or {}).items() if k in ('listen','text','speak_after_text')})"
}
for S in "$@"; do
  echo "== step $S" >&2
  case $S in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
             ${PYTEST_K:+-k "$PYTEST_K"} > ${O}_pytest_gpu.log 2>&1; rc=$?; tail -3 ${O}_pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1
           rc=$?; tail -1 ${O}_smoke.log ;;
    bench) timeout -k 10 900 python -u bench.py --out ${O}_bench.json > ${O}_bench.log 2>&1; rc=$?
           [ $rc -eq 0 ] && line ${O}_bench.log ;;
    quick) timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 --out ${O}_quick.json \
             > ${O}_quick.log 2>&1; rc=$?; [ $rc -eq 0 ] && line ${O}_quick.log ;;
    prof)  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_prof -o bench -f csv -- \
             python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-user) > ${O}_prof.log 2>&1; rc=$? ;;
    fetch) (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gemm_xs|k_gemm_rows" -d $ROOTD/${O}_pmc \
             -o fetch -f csv -- python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-user) \
             > ${O}_pmc.log 2>&1; rc=$? ;;
    fetchdup) (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gemm_xsk|k_subsample|k_enc" \
             -d $ROOTD/${O}_pmcdup -o fetch -f csv -- python3 $ROOTD/bench.py --scenario duplex --duplex-sec 6 --steps 1 \
             --warmup 1) > ${O}_pmcdup.log 2>&1 && python3 scripts/fetch_table.py ${O}_pmcdup > ${O}_fetchdup.txt 2>&1; rc=$?
             cat ${O}_fetchdup.txt | head -30 ;;
    tts)   (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_prof_tts -o tts -f csv -- \
             python3 $ROOTD/scripts/tts_step_time.py 8 multi) > ${O}_prof_tts.log 2>&1; rc=$? ;;
    steptrace) (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $ROOTD/${O}_steptrace -o tts -f csv -- \
             python3 $ROOTD/scripts/tts_step_time.py 8 multi) > ${O}_steptrace.log 2>&1 && \
             python3 scripts/step_timeline.py ${O}_steptrace > ${O}_step_timeline.txt 2>&1; rc=$?; cat ${O}_step_timeline.txt ;;
    profdup) (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_profdup -o duplex -f csv -- \
             python3 $ROOTD/bench.py --scenario duplex --duplex-sec 20 --steps 1 --warmup 1) > ${O}_profdup.log 2>&1; rc=$?
             [ $rc -eq 0 ] && python3 scripts/trace_table.py ${O}_profdup 40 duplex > ${O}_profdup_table.txt 2>&1; cat ${O}_profdup_table.txt | head -45 ;;
    profstage) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_profstage -o stage -f csv -- \
             python3 $ROOTD/scripts/llm_stage_time.py) > ${O}_profstage.log 2>&1; rc=$?
             [ $rc -eq 0 ] && python3 scripts/trace_table.py ${O}_profstage 45 stage > ${O}_profstage_table.txt 2>&1; head -48 ${O}_profstage_table.txt ;;
    profgroup) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_profgroup -o stage -f csv -- \
             python3 $ROOTD/scripts/group_stage_time.py ${GROUP_C:-4}) > ${O}_profgroup.log 2>&1; rc=$?
             [ $rc -eq 0 ] && python3 scripts/trace_table.py ${O}_profgroup 60 stage > ${O}_profgroup_table.txt 2>&1; head -62 ${O}_profgroup_table.txt ;;
    text)  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOTD/${O}_prof_text -o text -f csv -- \
             python3 $ROOTD/scripts/text_step_time.py) > ${O}_prof_text.log 2>&1; rc=$? ;;
    duplex) timeout -k 10 400 python -u bench.py --scenario duplex --out ${O}_duplex.json > ${O}_duplex.log 2>&1; rc=$?
            [ $rc -eq 0 ] && line ${O}_duplex.log ;;
    rehearsal) FO_DIST_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline \
             --no-single-user --out ${O}_rehearsal_n2.json > ${O}_rehearsal_n2.log 2>&1; rc=$? ;;
    vocpmc) V="python3 $ROOTD/scripts/vocoder_time.py 8 3"
           (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
             SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-include-regex "k_conv|k_codec|k_silence" -d $ROOTD/${O}_voc_p1 -o p1 \
             -f csv -- $V) > ${O}_voc_p1.log 2>&1 && \
           (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex \
             "k_conv|k_codec|k_silence" -d $ROOTD/${O}_voc_p2 -o p2 -f csv -- $V) > ${O}_voc_p2.log 2>&1 && \
           (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_conv|k_codec|k_silence" \
             -d $ROOTD/${O}_voc_p3 -o p3 -f csv -- $V) > ${O}_voc_p3.log 2>&1 && \
           (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $ROOTD/${O}_voc_t -o t -f csv -- $V) \
             > ${O}_voc_t.log 2>&1 && timeout -k 10 120 python3 -u scripts/vocoder_time.py 8 20 > ${O}_voc_time.log 2>&1 && \
           python3 scripts/pmc_json.py ${O}_vocoder_mfma.json ${O}_voc_p1 ${O}_voc_p2 ${O}_voc_t --pass3 ${O}_voc_p3 \
             --note "$(tail -1 ${O}_voc_time.log)" > ${O}_voc_pmc.txt 2>&1; rc=$?; cat ${O}_voc_time.log; head -30 ${O}_voc_pmc.txt ;;
    ddp1)  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
             --master-port 29517 bench.py --gpus 1 --steps 1 --warmup 1 --no-cpu-baseline --no-single-user \
             --out ${O}_ddp1.json > ${O}_ddp1.log 2>&1; rc=$?; [ $rc -eq 0 ] && line ${O}_ddp1.log ;;
    n2guard) timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > ${O}_n2guard.log 2>&1; rc=$?
             if [ $rc -eq 2 ] && grep -q refusing ${O}_n2guard.log; then echo "n2guard ok: $(tail -1 ${O}_n2guard.log)"; rc=0
             else echo "n2guard: expected a refusal, got rc $rc"; tail -5 ${O}_n2guard.log; [ $rc -eq 0 ] && rc=1; fi ;;
    ab)    : > ${O}_ab.txt
           for i in 1 2; do for AB in A B; do
             E=ENV_$AB; timeout -k 10 300 env ${!E} python -u bench.py --no-cpu-baseline --no-single-user --steps 3 \
               > ${O}_ab_$AB$i.log 2>&1 || { rc=$?; tail -20 ${O}_ab_$AB$i.log; break 2; }
             echo "$AB$i [${!E}] $(line ${O}_ab_$AB$i.log)" >> ${O}_ab.txt; rc=0
           done; done; cat ${O}_ab.txt ;;
    abdup) : > ${O}_abdup.txt   # the same alternation on the duplex line (SWEEP-style settings in DUP_SET='A|B|C')
           IFS='|' read -ra SET <<< "$DUP_SET"; rc=0
           for i in 1 2; do for k in "${!SET[@]}"; do
             timeout -k 10 300 env ${SET[$k]} python -u bench.py --scenario duplex --duplex-sec 30 \
               > ${O}_abdup_$k$i.log 2>&1 || { rc=$?; tail -20 ${O}_abdup_$k$i.log; break 2; }
             echo "$i [${SET[$k]:-default}] $(line ${O}_abdup_$k$i.log)" >> ${O}_abdup.txt
           done; done; cat ${O}_abdup.txt ;;
    sweep) : > ${O}_sweep.txt   # SWEEP='A=1|B=2 C=3|' : each setting (empty = default) on the quick bench, two rounds
           IFS='|' read -ra SET <<< "$SWEEP"; rc=0
           for i in 1 2; do for k in "${!SET[@]}"; do
             timeout -k 10 300 env ${SET[$k]} python -u bench.py --no-cpu-baseline --no-single-user --steps 3 \
               > ${O}_sweep_$k$i.log 2>&1 || { rc=$?; tail -20 ${O}_sweep_$k$i.log; break 2; }
             echo "$i [${SET[$k]:-default}] $(line ${O}_sweep_$k$i.log)" >> ${O}_sweep.txt
           done; done; cat ${O}_sweep.txt ;;
    py:*)  P=${S#py:}; L=${O}_$(basename ${P%% *} .py).log
           timeout -k 10 200 python -u scripts/$P > $L 2>&1; rc=$?; tail -40 $L ;;
    *) echo "unknown step $S"; rc=1 ;;
  esac
  echo "step $S rc $rc" >&2
  [ $rc -eq 0 ] || { echo "EXIT $rc at $S"; exit $rc; }
done
echo "EXIT 0"
