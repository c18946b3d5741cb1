set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "pair or trio" > gpurun_out/r06bh_pair_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06bh_hash.txt 2> gpurun_out/r06bh_hash.err && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_abi_generic.py > gpurun_out/r06bh_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/lat_probe.py > gpurun_out/r06bh_lat.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r06bh_bench.log 2>&1 && tail -1 gpurun_out/r06bh_bench.log > gpurun_out/r06bh_bench.json
