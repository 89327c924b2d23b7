# Round-3 call i: the whole GPU suite (8-tile row statistics fix), then the vocoder's channel chunk A/B
# (FO_CONV_CK=32: half the LDS per workgroup, 2-3 workgroups per CU) -- call time and the codec tests under it.
set -o pipefail
ROOTD=$GRAFT_REPO_ROOT
cd $ROOTD; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03i_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03i_voc_ck64.txt 2>&1 && \
FO_CONV_CK=32 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03i_voc_ck32.txt 2>&1 && \
FO_CONV_CK=16 timeout -k 10 120 python -u scripts/vocoder_time.py 8 20 > gpurun_out/r03i_voc_ck16.txt 2>&1 && \
FO_CONV_CK=32 timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_parity_r02_gpu.py -q -k "codec or vocoder or generator" --timeout 120 --timeout-method thread > gpurun_out/r03i_codec_ck32.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
