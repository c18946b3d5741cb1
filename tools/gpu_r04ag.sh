# r04_ag: rows16 waves per workgroup 2 (default) vs 1 vs 4: rows tests under 1, batch-1 latency A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_lnrows.py > gpurun_out/r04_ag_tests.log 2>&1 || exit $?
STZS_ROWS16_WPG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/r04_ag_tests_wpg1.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_WPG=1 timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_WPG=4 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py && STZS_ROWS16_WPG=1 timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_ag_lat.log 2>&1 || exit $?
