# Round-3 call ze: SpeechLane after the graph-reuse hardening: lane parity tests, then the bench in lane mode once.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=r03ze
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -x -v --timeout 120 --timeout-method thread -k "lane or two_workers or speak" > gpurun_out/${R}_test.log 2>&1 || { tail -40 gpurun_out/${R}_test.log; exit 1; }
tail -1 gpurun_out/${R}_test.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single-user --steps 3 --tts-lane > gpurun_out/${R}_b.log 2>&1 || { tail -30 gpurun_out/${R}_b.log; exit 1; }
grep '^{' gpurun_out/${R}_b.log | cut -c1-240
