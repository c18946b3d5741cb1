#!/bin/bash
# register-direct GEMM epilogue (csrc/gemm.hip), AdaIN-block convs on mrfv: full GPU suite, GEMM microbench, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_l.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_l.log | tail -8; [ $rc -ne 0 ] && exit $rc
M=3200 FLAGS=0,0x10002,0x10004 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_r03_l.log 2>&1 || exit $?
CASES=kv,lstm M=8300 FLAGS=0,0x10000,0x20000 timeout -k 10 200 python tools/gemm_bench.py >> gpurun_out/gemm_r03_l.log 2>&1 || exit $?
M=100 timeout -k 10 200 python tools/gemm_bench.py >> gpurun_out/gemm_r03_l.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/gemm_r03_l.log
timeout -k 10 500 python bench.py --no-cpu --no-precise > gpurun_out/bench_r03_l.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r03_l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=r['stages']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['time_frac'], r['avg_launch_us']); print(s['total']); [print(k, v['t_meas_us'], v['frac']) for k, v in s['stages'].items()]; [print(k, v) for k, v in s['families'].items()]"
