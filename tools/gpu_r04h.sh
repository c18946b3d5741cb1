mkdir -p gpurun_out
bash tools/gpu_round.sh r04_h || exit $?
timeout -k 10 120 python -u tools/gemm_phase.py > gpurun_out/r04_h_gemm_phase.log 2>&1 || exit $?
(STZS_BLK_SPLITK=0 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_h_blk_ab.log 2>&1 || exit $?
export TMPDIR=/tmp; N=5 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_r04_h -o run --output-format csv -- python tools/lat_probe.py > gpurun_out/lat_r04_h.log 2>&1 || exit $?
python3 tools/lat_trace.py $(ls gpurun_out/lat_r04_h/*/run_kernel_trace.csv gpurun_out/lat_r04_h/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/r04_h_lat_trace.txt 2>&1; echo LAT $?
