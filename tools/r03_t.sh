#!/bin/bash
# fused small-M linears: parity of the fused forms, then configs[1] p50 per fused consumer set, and a kernel trace
set -o pipefail
tag=${1:-r03_t}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_rows.py -q -m gpu -k "fused" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; tail -2 gpurun_out/t_$tag.log; [ $rc -ne 0 ] && exit $rc
for m in none ln attn cfg ln,attn,cfg none ln,attn,cfg; do
  if [ $m = none ]; then f=0; else f=1; fi
  echo -n "modes=$m " >> gpurun_out/lat_$tag.log
  STZS_FUSE_ROWS=$f STZS_FUSE_MODES=$m timeout -k 10 120 python tools/lat_probe.py >> gpurun_out/lat_$tag.log 2>&1 || exit $?
done
grep latency gpurun_out/lat_$tag.log
export TMPDIR=/tmp
mkdir -p gpurun_out/tr_$tag
N=5 STZS_FUSE_ROWS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr_$tag -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/tr_$tag.log 2>&1 || exit $?
python3 tools/lat_trace.py gpurun_out/tr_$tag/run_kernel_trace.csv --list > gpurun_out/${tag}_lat_trace.txt && head -30 gpurun_out/${tag}_lat_trace.txt
