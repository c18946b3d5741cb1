# r04_z: throughput bench with the text-encoder / AdaIN-block split-K knobs (A/B, main leg only)
mkdir -p gpurun_out
for v in "" "STZS_TE_SPLITK=2" "STZS_TE_SPLITK=4" "STZS_BLK_SPLITK=2" ""; do
  echo "== $v" >> gpurun_out/r04_z_ab.log
  env $v timeout -k 10 200 python bench.py --no-cpu --no-latency --no-longform --no-precise --no-stages >> gpurun_out/r04_z_ab.log 2>&1 || exit $?
done
