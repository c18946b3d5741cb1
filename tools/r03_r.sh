#!/bin/bash
# round 3, r: wide register-direct stage-0 MRF convs + fused small-M denoiser linears (LayerNorm / attention in
# the linear's launch): parity tests of both, the latency A/B, then the default bench line
set -o pipefail
tag=${1:-r03_r}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_ops.py tests/test_gpu_configs.py -v -m gpu -k "rows or mrf or configs1 or latency or fused or sample_style or denoiser" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_$tag.log | tail -12
[ $rc -ne 0 ] && exit $rc
for f in 0 1 0 1; do STZS_FUSE_ROWS=$f timeout -k 10 120 python tools/lat_probe.py >> gpurun_out/lat_$tag.log 2>&1 || exit $?; done
cat gpurun_out/lat_$tag.log | grep latency
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log | cut -c1-400
