set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do for c in dec src; do
timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency --pipe-cut $c > gpurun_out/r06z_$c$i.json 2> gpurun_out/r06z_$c$i.err || exit 1
done; done
