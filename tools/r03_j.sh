#!/bin/bash
# LN-prologue linears: unit tests, configs[1] oracle tests, latency A/B, batch-1 kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_configs.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_j.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_j.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/lat_probe.py > gpurun_out/lat_r03_j.log 2>&1 || exit $?
STZS_DN_LN_FUSE=0 timeout -k 10 200 python tools/lat_probe.py >> gpurun_out/lat_r03_j.log 2>&1 || exit $?
timeout -k 10 200 python tools/lat_probe.py >> gpurun_out/lat_r03_j.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/lat_r03_j.log
export TMPDIR=/tmp
N=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/lat_prof_r03_j -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/lat_prof_r03_j.log 2>&1 || exit $?
python3 tools/lat_trace.py gpurun_out/lat_prof_r03_j/run_kernel_trace.csv > gpurun_out/lat_trace_r03_j.txt && cat gpurun_out/lat_trace_r03_j.txt
