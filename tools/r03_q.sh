#!/bin/bash
# how often does the branch-streams two-shard replay differ from eager?  (3 runs of the one test)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -k "two_shard_streams_match_eager" -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_r03_q$i.log 2>&1
  echo RUN $i rc $?; grep -E "^concurrent|PASSED|FAILED" gpurun_out/t_r03_q$i.log | tail -6
done
