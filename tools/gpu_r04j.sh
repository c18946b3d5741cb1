# r04_j (part 2): latency engine block split-K 0 / 4 / 8, gemm_glds epilogue stamps, latency trace
mkdir -p gpurun_out
(for v in 0 4 8 0 4 8; do STZS_BLK_SPLITK=$v timeout -k 10 100 python tools/lat_probe.py || exit $?; done) > gpurun_out/r04_j_blk_ab.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/gemm_phase.py > gpurun_out/r04_j_gemm_phase.log 2>&1 || exit $?
export TMPDIR=/tmp
N=5 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_r04_j -o run --output-format csv -- python tools/lat_probe.py > gpurun_out/lat_r04_j.log 2>&1 || exit $?
f=$(find gpurun_out/lat_r04_j -name run_kernel_trace.csv | head -1)
python3 tools/lat_trace.py $f --list > gpurun_out/r04_j_lat_trace.txt 2>&1; echo LAT $?
