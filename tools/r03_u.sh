#!/bin/bash
# XCD-aware gemm_glds tile order: bit-identity test, linear-GEMM A/B (flags 0 = remap, 128 = linear order) at the
# batch-64 row counts, then the default bench line
set -o pipefail
tag=${1:-r03_u}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_xcd.py tests/test_gpu_splitk.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_$tag.log | tail -8
[ $rc -ne 0 ] && exit $rc
for M in 3200 6400; do
  M=$M FLAGS=0,128 CASES=ffn1,qkv,out,ffn2,kv,lstm timeout -k 10 200 python tools/gemm_bench.py >> gpurun_out/${tag}_gemm.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/${tag}_gemm.log
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log | cut -c1-400
