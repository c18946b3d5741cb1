set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do for b in 0 src; do
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --branch-streams $b > gpurun_out/r06ag_$b$i.json 2> gpurun_out/r06ag_$b$i.err || exit 1
done; done
