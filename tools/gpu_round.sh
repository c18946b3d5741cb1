#!/bin/bash
# full GPU round trip (tag = $1): gpu parity tests, default bench (with CPU baseline), kernel-trace profile
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -x -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_$tag.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log
bash tools/prof.sh prof_$tag
python3 tools/roofline_check.py gpurun_out/prof_$tag/run_kernel_trace.csv gpurun_out/prof_$tag.log > gpurun_out/roofline_check_$tag.json && cat gpurun_out/roofline_check_$tag.json
[ -n "$PMC" ] && bash tools/pmc_bench.sh $tag
exit 0
