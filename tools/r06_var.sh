#!/bin/bash
# mrfv_bench on the in-tree library and on each variant library (tools/variants/libstzs_<v>.so)
tag=$1; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
REPS=10 timeout -k 10 300 python tools/mrfv_bench.py > gpurun_out/${tag}_base.log 2>&1 || exit 1
for v in "$@"; do
  STZS_LIB=tools/variants/libstzs_$v.so REPS=10 timeout -k 10 300 python tools/mrfv_bench.py > gpurun_out/${tag}_$v.log 2>&1 || exit 1
done
