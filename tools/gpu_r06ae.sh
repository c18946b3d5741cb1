set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06ae_lat -o run -- python3 -u tools/lat_probe.py > gpurun_out/r06ae_lat.log 2>&1
