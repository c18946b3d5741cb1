#!/bin/bash
# Per-kernel register / LDS / spill figures of one csrc/*.hip file (device-only compile, code-object metadata).
# usage: tools/kstats.sh gemm.hip [name-filter]
set -e
SRC=${1:?source}
FILT=${2:-.}
D=$(mktemp -d)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=fast -I"$ROOT/include" \
    -Xclang -target-feature -Xclang -packed-fp32-ops --cuda-device-only --no-gpu-bundle-output -c "$ROOT/styletts-zs_amd/csrc/$SRC" \
    -o "$D/dev.o" 2>/dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$D/dev.o" |
    grep -E "^\s+\.(name|vgpr_count|agpr_count|group_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):" |
    awk '/\.agpr_count/{ag=$2} /\.group_segment/{lds=$2} /\.name:/{nm=$2} /\.sgpr_spill/{ss=$2}
         /\.vgpr_count/{vg=$2} /\.vgpr_spill/{vs=$2; if (nm!="") {printf "%-90s v%-4s a%-4s spill %s/%s lds %s\n", substr(nm,1,90), vg, ag, vs, ss, lds}}' |
    grep -E "$FILT" || true
rm -rf "$D"
