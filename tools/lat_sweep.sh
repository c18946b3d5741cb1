# configs[1] p50 over denoiser linear tables (STZS_DN_ROWS / STZS_DN_SPLITK), one lat_probe run each
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/lat_sweep_$1.log; shift
: > $out
for cfg in "$@"; do
  rows=${cfg%%|*}; sk=${cfg##*|}
  STZS_DN_ROWS="$rows" STZS_DN_SPLITK="$sk" timeout -k 10 200 python tools/lat_probe.py 2>&1 | grep -v amdgpu.ids >> $out || exit $?
done
cat $out
