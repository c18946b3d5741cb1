#!/bin/bash
# bench variance: three default bench runs (no CPU baseline / precise) on one box
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu --no-precise --no-longform --steps 20 > gpurun_out/bench_r03_n$i.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_r03_n$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['avg_launch_us'], 'h2h', d['host_to_host']['value'])"
done
