#!/bin/bash
# mrfv ablation (FLAGS 0 / 1 / 4 / 5: full, no staging, no epilogue, K loop alone) + SQ passes on one stage-1 shape
tag=$1; cases=${2:-0,3}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for f in 0 1 4 5; do
  CASES=$cases FLAGS=$f REPS=5 timeout -k 10 200 python tools/mrfv_bench.py > gpurun_out/${tag}_flags$f.log 2>&1 || exit 1
done
bash tools/sq_pmc.sh ${tag}_full 3 0 && python tools/sq_summary.py gpurun_out/sq_${tag}_full > gpurun_out/${tag}_sq_full.json &&
bash tools/sq_pmc.sh ${tag}_k3 0 0 && python tools/sq_summary.py gpurun_out/sq_${tag}_k3 > gpurun_out/${tag}_sq_k3.json
