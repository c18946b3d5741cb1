#!/bin/bash
# staggered-start sweep of the mrfv kernel (STZS_MRFV_STAG) on the stage-1 / stage-0 generator shapes
tag=$1; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for st in "$@"; do
  STZS_MRFV_STAG=$st REPS=10 timeout -k 10 300 python tools/mrfv_bench.py > gpurun_out/${tag}_stag$st.log 2>&1 || exit 1
done
for st in "$@"; do echo "STAG $st"; grep " mrfv \| mrfvN " gpurun_out/${tag}_stag$st.log | cut -c1-60; done
