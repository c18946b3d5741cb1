# r04_n: gemm_glds 64-row tiles at three workgroups per CU, tile height by wave quantisation: GEMM tests, tile sweep
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_xcd.py tests/test_gpu_splitk.py tests/test_gpu_ops.py -k "gemm or splitk or linear or flat" > gpurun_out/r04_n_gemm_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_tile.py > gpurun_out/r04_n_tile.log 2>&1 || exit $?
(for i in 1 2; do timeout -k 10 100 python tools/lat_probe.py || exit $?; done) > gpurun_out/r04_n_lat.log 2>&1
