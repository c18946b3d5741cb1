set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
CASES=0,1 timeout -k 10 200 python -u tools/mrfv_bench.py > gpurun_out/r06s_base$i.log 2>&1 || exit 1
STZS_LIB=$PWD/tools/variants/libstzs_o4.so CASES=0,1 timeout -k 10 200 python -u tools/mrfv_bench.py > gpurun_out/r06s_o4_$i.log 2>&1 || exit 1
done
