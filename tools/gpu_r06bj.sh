set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/r06_round.sh r06bj && \
N=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06bj_lat -o run -- python3 -u tools/lat_probe.py > gpurun_out/r06bj_latprof.log 2>&1
