set -o pipefail
cd $GRAFT_REPO_ROOT
for nb in 1 2 4; do
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --schedule pipe --pipe-backs $nb > gpurun_out/r06w_pipe_b$nb.json 2> gpurun_out/r06w_pipe_b$nb.err || exit 1
done
