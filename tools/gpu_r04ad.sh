# r04_ad: kernel trace of the batch-1 latency replay (phase / family summary)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lat_r04_ad -o run --output-format csv -- python3 tools/lat_probe.py > gpurun_out/lat_r04_ad.log 2>&1 || exit $?
f=$(find gpurun_out/lat_r04_ad -name "run_kernel_trace.csv" | head -1)
python3 tools/lat_trace.py "$f" > gpurun_out/r04_ad_lat_trace.txt
