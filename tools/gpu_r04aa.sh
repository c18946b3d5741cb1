# r04_aa: attention with 128-key chunks when Lk > 64: attention / configs tests, batch-1 latency, throughput main leg
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_abi_generic.py tests/test_gpu_torch_ops.py -k "attn or attention or denoiser" > gpurun_out/r04_aa_attn.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -s > gpurun_out/r04_aa_cfg.log 2>&1 || exit $?
(timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_aa_lat.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu --no-latency --no-longform --no-precise --no-stages > gpurun_out/r04_aa_bench.log 2>&1
