set -o pipefail
cd $GRAFT_REPO_ROOT
for st in 0 4 2 8; do
STZS_PIPE_FRONT_CU_STRIDE=$st timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency > gpurun_out/r06af_s$st.json 2> gpurun_out/r06af_s$st.err || exit 1
done
