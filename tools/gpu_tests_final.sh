# GPU parity suite + smoke on the current tree (tag = $1), the -s output kept
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -x -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$1.log 2>&1
rc=$?; echo TEST $rc; grep -E "passed|failed|FAILED|Error" gpurun_out/t_$1.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$1.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$1.log
