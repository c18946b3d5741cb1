set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 4 8; do
STZS_MRFV_RUN=$r CASES=0,1,2,3 timeout -k 10 200 python -u tools/mrfv_bench.py > gpurun_out/r06r_run$r.log 2>&1 || exit 1
done
