set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --no-cpu --no-longform --no-precise --no-stages > gpurun_out/r06v_bench.json 2> gpurun_out/r06v_bench.err && \
timeout -k 10 200 python -u tools/lat_probe.py > gpurun_out/r06v_lat.log 2>&1
