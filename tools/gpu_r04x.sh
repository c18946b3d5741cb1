# r04_x: rows16 with K slices (batch-1 ffn2): rows / lnrows tests, configs[1] parity, batch-1 latency A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lnrows.py tests/test_gpu_rows.py > gpurun_out/r04_x_rows.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "configs1" -s > gpurun_out/r04_x_c1.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_SPLIT=0 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_x_lat.log 2>&1 || exit $?
