set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_b_rows.log 2>&1
rc=$?; echo ROWS $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_b_rows.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 env M=100 ROWS=0,1,2,4 FLAGS=0 python tools/gemm_bench.py > gpurun_out/gemm_r03_b.log 2>&1 || exit $?
cat gpurun_out/gemm_r03_b.log
timeout -k 10 200 python tools/lat_probe.py > gpurun_out/lat_r03_b.log 2>&1 || exit $?
STZS_DN_ROWS=0 timeout -k 10 200 python tools/lat_probe.py >> gpurun_out/lat_r03_b.log 2>&1 || exit $?
cat gpurun_out/lat_r03_b.log
bash tools/gpu_tests.sh r03_b tests/test_gpu_status.py tests/test_gpu_abi_generic.py tests/test_gpu_configs.py tests/test_gpu_precise.py tests/test_gpu_stream.py tests/test_gpu_torch_ops.py
