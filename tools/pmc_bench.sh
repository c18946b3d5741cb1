#!/bin/bash
# HBM traffic of the dominant kernel on the bench workload: two separate PMC passes (kernel-trace only)
# over the eager bench command, summarised into profiles/<tag>_pmc_mrf.json.   usage: tools/pmc_bench.sh <tag>
tag=${1:-r01}
export TMPDIR=/tmp
out=gpurun_out/pmcb_$tag
for c in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $out/$c
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d $GRAFT_REPO_ROOT/$out/$c -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu --no-latency --no-longform --no-precise --no-graph > $out/$c.log 2>&1 || { echo "PMC $c failed"; tail -5 $out/$c.log; exit 1; }
done
# written under gpurun_out/ so it travels back; copy it into profiles/ to publish it to bench.py
# the 36 MRF resblock convs of a step (mrfv_conv, Snake prologue), per shape against their algorithmic bytes
python3 tools/pmc_traffic.py $out "mrfv_conv<2" > $out/${tag}_pmc_mrf.json && cat $out/${tag}_pmc_mrf.json
