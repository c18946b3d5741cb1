#!/bin/bash
# XCD-aware conv_mfma tile order: bit-identity tests + A/B on the decoder_pre / predictor conv shapes
set -o pipefail
tag=${1:-r03_v}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_xcd.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error|xcd" gpurun_out/t_$tag.log | tail -14
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/convm_bench.py > gpurun_out/${tag}_convm.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${tag}_convm.log
