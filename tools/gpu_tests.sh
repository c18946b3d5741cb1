#!/bin/bash
# GPU parity tests on a subset (or all, no args) -> gpurun_out/t_<tag>.log.   usage: tools/gpu_tests.sh <tag> [test paths...]
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests/} -v -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_$tag.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_$tag.log | tail -12
exit $rc
