"""Fast A/B variant: recompile ONE source with extra definitions and relink it with the in-tree objects of every other
source (styletts-zs_amd/build/*.o) into tools/variants/libstzs_<tag>.so (STZS_LIB=... selects it at run time).

    python tools/variant_one.py TAG FILE.hip -DSTZS_MRFV_PRIO=1 [...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "styletts-zs_amd"))
import build as B  # noqa: E402

tag, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = os.path.join("/tmp", "variant1_" + tag)
os.makedirs(tmp, exist_ok=True)
out = os.path.join(ROOT, "tools", "variants", f"libstzs_{tag}.so")
os.makedirs(os.path.dirname(out), exist_ok=True)
path = os.path.join(B.CSRC, src)
obj = os.path.join(tmp, src + ".o")
subprocess.check_call([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get(src, []) + defs + ["-c", path, "-o", obj])
objs = [obj if os.path.basename(s) == src else os.path.join(B.BUILD, os.path.basename(s).replace(".hip", ".o"))
        for s in B.sources()]
subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"])
os.replace(out + ".tmp", out)
print(out)
