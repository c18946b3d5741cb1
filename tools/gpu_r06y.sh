set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do for pr in 0 -1; do
STZS_PIPE_FRONT_PRIO=$pr timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency > gpurun_out/r06y_fprio$pr.$i.json 2> gpurun_out/r06y_fprio$pr.$i.err || exit 1
done; done
