# r04_k: gemm_glds phases after the 64-bit row division fix, latency p50, then the full round (tests, smoke, bench, prof)
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/gemm_phase.py > gpurun_out/r04_k_gemm_phase.log 2>&1 || exit $?
(for i in 1 2 3; do timeout -k 10 100 python tools/lat_probe.py || exit $?; done) > gpurun_out/r04_k_lat.log 2>&1 || exit $?
bash tools/gpu_round.sh r04_k
