#!/bin/bash
# fused noise-conv ConvT + mrfv k3 c1 at 4 workgroups per CU: targeted tests, microbenches, then the full suite + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "convtranspose" -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_o_ups.log 2>&1
rc=$?; echo UPS TEST $rc; grep -E "passed|failed|FAILED|Error|fused noise" gpurun_out/t_r03_o_ups.log | tail -8; [ $rc -ne 0 ] && exit $rc
CASES=0,1 timeout -k 10 200 python tools/mrfv_bench.py > gpurun_out/mrfv_r03_o.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/mrfv_r03_o.log | grep -E "c1 |MISMATCH|mrfv4"
timeout -k 10 400 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_o.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_o.log | tail -8; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  STZS_UPS_NOISE=$v timeout -k 10 400 python bench.py --no-cpu --no-precise --no-longform --steps 20 > gpurun_out/bench_r03_o$v.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_r03_o$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; f=r['stages']['families']; print('UPS_NOISE=$v BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], 'ups1', f['ConvT ups1'], 'gen', r['stages']['stages']['generator']['t_meas_us'])"
done
