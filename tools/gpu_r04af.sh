# r04_af: rows16 with 32-row workgroups (STZS_ROWS16_WPG=2) vs 16: rows tests under both, batch-1 latency A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_lnrows.py > gpurun_out/r04_af_tests.log 2>&1 || exit $?
STZS_ROWS16_WPG=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/r04_af_tests_mt2.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_WPG=2 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_WPG=2 timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_af_lat.log 2>&1 || exit $?
