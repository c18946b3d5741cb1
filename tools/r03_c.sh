set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_c_rows.log 2>&1
rc=$?; echo ROWS $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_r03_c_rows.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 env M=100 ROWS=0,1,2,4 FLAGS=0 python tools/gemm_bench.py > gpurun_out/gemm_r03_c.log 2>&1 || exit $?
cat gpurun_out/gemm_r03_c.log | grep -v amdgpu.ids
timeout -k 10 200 python tools/lat_probe.py > gpurun_out/lat_r03_c.log 2>&1 || exit $?
STZS_DN_ROWS=0 timeout -k 10 200 python tools/lat_probe.py >> gpurun_out/lat_r03_c.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/lat_r03_c.log
