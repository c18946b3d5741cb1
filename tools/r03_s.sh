#!/bin/bash
# round-3 final GPU round: every GPU parity test, smoke, default bench line, rocprofv3 kernel trace + roofline
# cross-check, PMC traffic of the MRF convs, PMC per kernel family, and a configs[1] latency trace (fused engine)
set -o pipefail
tag=${1:-r03_s}
bash tools/gpu_round.sh $tag || exit $?
bash tools/pmc_bench.sh $tag || exit $?
bash tools/pmc_families.sh $tag > /dev/null || exit $?
echo PMC families done
export TMPDIR=/tmp
mkdir -p gpurun_out/lat_$tag
N=5 STZS_FUSE_ROWS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_$tag -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/lat_$tag.log 2>&1 || exit $?
python3 tools/lat_trace.py gpurun_out/lat_$tag/run_kernel_trace.csv --list > gpurun_out/${tag}_lat_trace.txt && head -30 gpurun_out/${tag}_lat_trace.txt
