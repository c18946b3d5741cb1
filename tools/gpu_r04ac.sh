# r04_ac: attention fused into the output projection (stzs_attn_linear): tests, configs[1] parity, latency A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lnrows.py > gpurun_out/r04_ac_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "configs1" -s > gpurun_out/r04_ac_c1.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && STZS_ATTN_FUSE=0 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_ac_lat.log 2>&1 || exit $?
