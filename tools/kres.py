"""Per-kernel resource usage of one csrc/*.hip file (hipcc -Rpass-analysis=kernel-resource-usage), one line per
kernel: VGPRs, spills, occupancy.   usage: python tools/kres.py styletts-zs_amd/csrc/mrfx.hip [name filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=fast", "-Iinclude",
       "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"remark: (.*) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for n, r in rows.items():
    dn = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    if flt and flt not in dn:
        continue
    dn = re.sub(r"\(anonymous namespace\)::", "", dn).replace("(stzs_conv_args)", "")
    print(f"{dn:60s} vgpr {r.get('VGPRs', '?'):>4} spill {r.get('VGPRs Spill', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?')}")
