#!/bin/bash
# one full GPU round: every GPU test (-s: measured errors kept), smoke(), a full bench line, a kernel-trace profile.
#   bash tools/r06_round.sh TAG [BENCH_ARGS...]
tag=$1; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/${tag}_gpu_tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['avg_launch_us'], 'precise', (d.get('precise') or {}).get('audio_s_per_s'), 'cpu', (d.get('cpu_baseline') or {}).get('latency_ms'))"
