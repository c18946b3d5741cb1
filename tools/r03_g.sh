set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "convtranspose" -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_g.log 2>&1
rc=$?; echo OPS $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_g.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/ups_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/ups_r03_g.log || exit $?
cat gpurun_out/ups_r03_g.log
timeout -k 10 500 python bench.py --no-cpu --no-precise --no-longform > gpurun_out/bench_r03_g.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r03_g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'roof', d['roofline']['achieved'], d['roofline']['avg_launch_us'], d['roofline']['time_frac'])"
