# r04_m: split TUs, deferred epilogue stores: phases, GEMM / conv tests, then the full round
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/gemm_phase.py > gpurun_out/r04_m_gemm_phase.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_xcd.py tests/test_gpu_splitk.py tests/test_gpu_ops.py -k "gemm or splitk or linear or flat or conv" > gpurun_out/r04_m_gemm_tests.log 2>&1 || exit $?
(for i in 1 2; do timeout -k 10 100 python tools/lat_probe.py || exit $?; done) > gpurun_out/r04_m_lat.log 2>&1 || exit $?
bash tools/gpu_round.sh r04_m
