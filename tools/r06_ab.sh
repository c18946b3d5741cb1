#!/bin/bash
# A/B of a library variant against the in-tree library: mrfv / ups microbenches + one bench line each.
#   bash tools/r06_ab.sh TAG VARIANT_SO [BENCH_ARGS...]
tag=$1; var=$2; shift 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { echo "== $*"; "$@"; }
run timeout -k 10 300 python tools/mrfv_bench.py > gpurun_out/${tag}_mrfv_new.log 2>&1 &&
STZS_LIB=$var timeout -k 10 300 python tools/mrfv_bench.py > gpurun_out/${tag}_mrfv_old.log 2>&1 &&
run timeout -k 10 200 python tools/ups_bench.py > gpurun_out/${tag}_ups_new.log 2>&1 &&
STZS_LIB=$var timeout -k 10 200 python tools/ups_bench.py > gpurun_out/${tag}_ups_old.log 2>&1 &&
run timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --no-longform --no-precise "$@" > gpurun_out/${tag}_bench_new.log 2>&1 &&
STZS_LIB=$var timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --no-longform --no-precise "$@" > gpurun_out/${tag}_bench_old.log 2>&1 &&
run timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --no-longform --no-precise "$@" > gpurun_out/${tag}_bench_new2.log 2>&1
rc=$?
for f in gpurun_out/${tag}_bench_*.log; do echo $f; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], 'p50', d['p50_latency_ms'], 'frac', r['frac'], r['avg_launch_us'], {k: (v['t_meas_us'], v['frac']) for k, v in list(r['stages']['families'].items())[:8]})" || true; done
exit $rc
