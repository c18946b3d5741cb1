#!/bin/bash
# SQ stall / issue counters of the stage-1 MRF conv (tools/mrfv_bench.py CASES, FLAGS: 0 full, 5 K loop alone) in two
# PMC passes (8 SQ counters each; kernel-trace only).   usage: tools/sq_pmc.sh <tag> <CASES> <FLAGS>
tag=${1:-sq}; cases=${2:-3}; flags=${3:-0}
export TMPDIR=/tmp
out=gpurun_out/sq_$tag
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for p in "$P1" "$P2"; do
  i=$((i+1))
  mkdir -p $out/p$i
  CASES=$cases FLAGS=$flags REPS=3 timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d $GRAFT_REPO_ROOT/$out/p$i -o run --output-format csv -- \
    python3 tools/mrfv_bench.py > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
echo done
