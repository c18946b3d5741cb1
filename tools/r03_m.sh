#!/bin/bash
# AdaIN-block convs on mrfv, faster iSTFT / harmonic source: full GPU suite, bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_m.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_m.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --no-cpu --no-precise > gpurun_out/bench_r03_m.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r03_m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=r['stages']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['time_frac'], r['avg_launch_us'], 'lf', d['longform']['p50_total_ms'], d['longform']['chunked']['p50_first_chunk_ms']); print(s['total']); [print(k, v['t_meas_us'], v['frac']) for k, v in s['stages'].items()]; [print(k, v) for k, v in s['families'].items()]"
