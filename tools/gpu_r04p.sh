# r04_p: LayerNorm-fed rows linear (csrc/lnrows.hip) tests, configs[1] parity, batch-1 latency, GEMM tile sweep
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lnrows.py > gpurun_out/r04_p_lnrows.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "configs1" -s > gpurun_out/r04_p_c1.log 2>&1 || exit $?
(for i in 1 2; do timeout -k 10 100 python tools/lat_probe.py || exit $?; done) > gpurun_out/r04_p_lat.log 2>&1 || exit $?
STZS_LN_FUSE=0 timeout -k 10 100 python tools/lat_probe.py >> gpurun_out/r04_p_lat.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_tile.py > gpurun_out/r04_p_tile.log 2>&1
