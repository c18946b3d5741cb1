set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/sc_bench.py > gpurun_out/r06ab_sc.log 2>&1
