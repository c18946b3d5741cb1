#!/bin/bash
# one GPU round trip: parity tests, a bench line, a kernel-trace profile (tag = $1)
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/ -q -s -m gpu -p no:cacheprovider > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED" gpurun_out/t_$tag.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'roof', d['roofline']['achieved'], d['roofline']['avg_launch_us'])"
bash tools/prof.sh prof_$tag
