set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --no-cpu --no-longform --no-stages --no-latency > gpurun_out/r06x_pipe.json 2> gpurun_out/r06x_pipe.err && \
timeout -k 10 500 python -u bench.py --no-cpu --no-longform --no-stages --no-latency --schedule shards --precise-schedule shards > gpurun_out/r06x_shards.json 2> gpurun_out/r06x_shards.err && \
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "runner" > gpurun_out/r06x_tests.log 2>&1
