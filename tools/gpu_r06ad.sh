set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/synth_hash.py > gpurun_out/r06ad_hash.txt 2> gpurun_out/r06ad_hash.err && \
timeout -k 10 300 python -u tools/back_launches.py > gpurun_out/r06ad_back.txt 2> gpurun_out/r06ad_back.err && \
STZS_NARROW_RING=1 timeout -k 10 300 python -u tools/back_launches.py > gpurun_out/r06ad_back_ring.txt 2> gpurun_out/r06ad_back_ring.err
