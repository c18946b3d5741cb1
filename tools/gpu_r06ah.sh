set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06ah_hash.txt 2> gpurun_out/r06ah_hash.err && \
STZS_UPS_BT=64 timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06ah_hash64.txt 2> gpurun_out/r06ah_hash64.err && \
for bt in 128 0 64; do STZS_UPS_BT=$bt timeout -k 10 300 python -u tools/back_launches.py > gpurun_out/r06ah_back_$bt.txt 2>/dev/null || exit 1; done && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "ups or noise or convt" > gpurun_out/r06ah_tests.log 2>&1
