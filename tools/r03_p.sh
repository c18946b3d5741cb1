#!/bin/bash
# round-3 full GPU round on the current tree: parity tests, smoke, default bench line (CPU baseline, precise,
# long-form), rocprofv3 kernel trace + roofline cross-check, PMC traffic of the MRF convs, PMC per kernel family
set -o pipefail
tag=${1:-r03_p}
bash tools/gpu_round.sh $tag || exit $?
bash tools/pmc_bench.sh $tag || exit $?
bash tools/pmc_families.sh $tag > /dev/null || exit $?
echo PMC families done
