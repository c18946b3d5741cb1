set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u tools/mrfv_bench.py > gpurun_out/r06p_t128.log 2>&1 && \
STZS_MRFV_T64_SNAKE=100000 timeout -k 10 240 python -u tools/mrfv_bench.py > gpurun_out/r06p_t64.log 2>&1
