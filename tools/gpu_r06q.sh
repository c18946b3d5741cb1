set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06q_trace -o trace -- python3 -u bench.py --steps 4 --warmup 2 --no-cpu --no-latency --no-longform --no-precise --no-stages > gpurun_out/r06q_bench.log 2>&1
