set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --steps 10 > gpurun_out/r06bc_s10.json 2>/dev/null && \
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --steps 30 > gpurun_out/r06bc_s30.json 2>/dev/null && \
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --steps 30 --schedule shards > gpurun_out/r06bc_s30_shards.json 2>/dev/null
