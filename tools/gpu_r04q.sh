# r04_q: fused LayerNorm linear with batched row statistics: tests, batch-1 latency fused vs unfused
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lnrows.py > gpurun_out/r04_q_lnrows.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && STZS_LN_FUSE=0 timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_q_lat.log 2>&1 || exit $?
