#!/bin/bash
# stage-0 per-shape MRF forms: full GPU suite, bench line, PMC families, batch-1 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_k.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_k.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --no-cpu --no-precise > gpurun_out/bench_r03_k.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r03_k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['time_frac'], r['avg_launch_us']); [print(k, v) for k, v in r['stages']['families'].items() if k.startswith('mrf')]"
M=3200 FLAGS=0,0x10000,0x20000,0x10002,0x10004,0x40000,0x40002,0x40004 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_r03_k.log 2>&1 || exit $?
CASES=kv,lstm M=8300 FLAGS=0,0x10000,0x20000,0x10002,0x10004,0x20002,0x20004,0x50000 timeout -k 10 200 python tools/gemm_bench.py >> gpurun_out/gemm_r03_k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/gemm_r03_k.log
timeout -k 10 100 python tools/ups_bench.py > gpurun_out/ups_r03_k.log 2>&1 || exit $?
RES=0 timeout -k 10 100 python tools/ups_bench.py >> gpurun_out/ups_r03_k.log 2>&1 || exit $?
FLAGS=4 timeout -k 10 100 python tools/ups_bench.py >> gpurun_out/ups_r03_k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ups_r03_k.log
timeout -k 10 200 python tools/blk_bench.py > gpurun_out/blk_r03_k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/blk_r03_k.log
bash tools/pmc_families.sh r03_k || exit $?
export TMPDIR=/tmp
N=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/lat_prof_r03_k -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/lat_prof_r03_k.log 2>&1 || exit $?
python3 tools/lat_trace.py gpurun_out/lat_prof_r03_k/run_kernel_trace.csv > gpurun_out/lat_trace_r03_k.txt && head -12 gpurun_out/lat_trace_r03_k.txt
