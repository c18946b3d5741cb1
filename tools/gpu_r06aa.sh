set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/back_launches.py > gpurun_out/r06aa_back.txt 2> gpurun_out/r06aa_back.err
