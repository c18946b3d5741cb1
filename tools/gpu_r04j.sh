# r04_j (part 2): LSTM K-split A/B + LSTM / latency tests, block split-K 0 / 4 / 8 and branch streams, gemm_glds
# epilogue stamps, latency trace
mkdir -p gpurun_out
(for b in 1 64; do B=$b LSTM_PROF_SO=liblstmprof_b1.so timeout -k 10 60 python -u tools/probe/lstm_prof.py && B=$b LSTM_PROF_SO=liblstmprof_ks2.so LSTM_REF_SO=liblstmprof_b1.so timeout -k 10 60 python -u tools/probe/lstm_prof.py || exit $?; done) > gpurun_out/r04_j_lstm_ks2.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_abi_generic.py tests/test_gpu_torch_ops.py tests/test_gpu_precise.py -k "lstm or latency or configs1 or bilstm or configs2" > gpurun_out/r04_j_tests2.log 2>&1 || exit $?
(for v in 0 4 8 0 4 8; do STZS_BLK_SPLITK=$v timeout -k 10 100 python tools/lat_probe.py || exit $?; done; STZS_BRANCH_STREAMS=1 timeout -k 10 100 python tools/lat_probe.py; STZS_BRANCH_STREAMS=1 timeout -k 10 100 python tools/lat_probe.py) > gpurun_out/r04_j_blk_ab.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/gemm_phase.py > gpurun_out/r04_j_gemm_phase.log 2>&1 || exit $?
export TMPDIR=/tmp
N=5 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/lat_r04_j -o run --output-format csv -- python tools/lat_probe.py > gpurun_out/lat_r04_j.log 2>&1 || exit $?
f=$(find gpurun_out/lat_r04_j -name run_kernel_trace.csv | head -1)
python3 tools/lat_trace.py $f --list > gpurun_out/r04_j_lat_trace.txt 2>&1; echo LAT $?
