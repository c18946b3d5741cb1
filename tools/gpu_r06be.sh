set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for st in 0 1; do for d in 1 5; do
  B=1 D=$d STAGE=$st GRAPH=1 REPS=10 timeout -k 10 180 python3 -u tools/mrf_cosched.py >> gpurun_out/r06be_trio.log 2>&1 || exit 1
done; done
