set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06bm_hash.txt 2> gpurun_out/r06bm_hash.err && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_fp8.py tests/test_gpu_precise.py tests/test_gpu_golden.py tests/test_gpu_stages.py tests/test_gpu_stream.py tests/test_gpu_scheduler.py tests/test_gpu_abi_generic.py > gpurun_out/r06bm_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/lat_probe.py > gpurun_out/r06bm_lat.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r06bm_bench.log 2>&1 && tail -1 gpurun_out/r06bm_bench.log > gpurun_out/r06bm_bench.json
