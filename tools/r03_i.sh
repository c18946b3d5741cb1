#!/bin/bash
# round-3 GPU round trip on the current tree + the gfx950 counter list (for the MFMA-utilisation passes)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_round.sh ${1:-r03_i} || exit $?
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_gfx950.txt 2>&1; echo LIST $?
grep -i -E "mfma|FETCH_SIZE|WRITE_SIZE|GRBM_GUI|SQ_BUSY_CU" gpurun_out/counters_gfx950.txt | head -40
