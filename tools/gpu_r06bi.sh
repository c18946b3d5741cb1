set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OLD=$GRAFT_REPO_ROOT/tools/variants/libstzs_prepair.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "pair or trio" > gpurun_out/r06bi_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06bi_hash.txt 2> gpurun_out/r06bi_hash.err && \
timeout -k 10 200 python -u tools/lat_probe.py > gpurun_out/r06bi_lat.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 python -u tools/front_ab.py >> gpurun_out/r06bi_front.log 2>&1 && \
  STZS_LIB=$OLD timeout -k 10 200 python -u tools/front_ab.py >> gpurun_out/r06bi_front.log 2>&1 || exit 1
done
