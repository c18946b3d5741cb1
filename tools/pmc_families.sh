#!/bin/bash
# HBM traffic + MFMA utilisation per kernel family of one eager batch-64 bench pass: one rocprofv3 run per counter
# group (kernel-trace only, MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE in separate passes), summarised by
# tools/pmc_families.py into gpurun_out/pmcf_<tag>/<tag>_pmc_families.json.   usage: tools/pmc_families.sh <tag>
tag=${1:-r03}
export TMPDIR=/tmp
out=gpurun_out/pmcf_$tag
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  mkdir -p $out/p$i
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $GRAFT_REPO_ROOT/$out/p$i -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-latency --no-longform --no-precise --no-graph --no-stages \
    > $out/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_families.py $out > $out/${tag}_pmc_families.json && head -c 3000 $out/${tag}_pmc_families.json
