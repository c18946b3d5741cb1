set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do for g in 16 32 64; do
STZS_LSTM_GROUP=$g timeout -k 10 300 python -u bench.py --no-cpu --no-longform --no-precise --no-stages --no-latency > gpurun_out/r06bb_g$g.$i.json 2> gpurun_out/r06bb_g$g.$i.err || exit 1
done; done
