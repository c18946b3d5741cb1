# r04_i: gemm_glds phase stamps, batch-1 block split-K A/B, configs[1] latency kernel trace
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/gemm_phase.py > gpurun_out/r04_i_gemm_phase.log 2>&1 || exit $?
(STZS_BLK_SPLITK=0 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py && STZS_BLK_SPLITK=0 timeout -k 10 100 python tools/lat_probe.py && timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_i_blk_ab.log 2>&1 || exit $?
export TMPDIR=/tmp
N=5 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_r04_i -o run --output-format csv -- python tools/lat_probe.py > gpurun_out/lat_r04_i.log 2>&1 || exit $?
f=$(find gpurun_out/lat_r04_i -name run_kernel_trace.csv | head -1)
python3 tools/lat_trace.py $f > gpurun_out/r04_i_lat_trace.txt 2>&1; echo LAT $?
