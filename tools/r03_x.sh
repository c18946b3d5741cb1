#!/bin/bash
# conv_mfma split-K for the latency engine's text-encoder convs: GPU tests (split-K conv, latency-engine configs[1]
# vs the oracle), then configs[1] p50 A/B (te split-K 0 / 2 / 4) and a latency kernel trace
set -o pipefail
tag=${1:-r03_x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_xcd.py tests/test_gpu_configs.py tests/test_gpu_splitk.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error|split-K" gpurun_out/t_$tag.log | tail -10
[ $rc -ne 0 ] && exit $rc
for te in 0 4 2 0 4; do
  STZS_TE_SPLITK=$te timeout -k 10 200 python tools/lat_probe.py >> gpurun_out/${tag}_lat_ab.log 2>&1 || exit $?
done
grep latency gpurun_out/${tag}_lat_ab.log
export TMPDIR=/tmp
mkdir -p gpurun_out/lat_$tag
N=5 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_$tag -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/lat_$tag.log 2>&1 || exit $?
python3 tools/lat_trace.py gpurun_out/lat_$tag/run_kernel_trace.csv --list > gpurun_out/${tag}_lat_trace.txt && head -40 gpurun_out/${tag}_lat_trace.txt
