# r04_o: graph-timed tile sweep of the linear GEMM
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_tile.py > gpurun_out/r04_o_tile.log 2>&1
