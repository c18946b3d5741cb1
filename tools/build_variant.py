"""Build a variant of the whole library with extra compile definitions into tools/variants/libstzs_<tag>.so (A/B runs:
STZS_LIB=tools/variants/libstzs_<tag>.so python tools/mrfv_bench.py).  Objects in /tmp/variant_<tag>.

    python tools/build_variant.py TAG -DSTZS_MRFV_PD=3 [...]
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "styletts-zs_amd"))
import build as B  # noqa: E402

tag, defs = sys.argv[1], sys.argv[2:]
tmp = os.path.join("/tmp", "variant_" + tag)
os.makedirs(tmp, exist_ok=True)
out = os.path.join(ROOT, "tools", "variants", f"libstzs_{tag}.so")


def one(f):
    o = os.path.join(tmp, os.path.basename(f) + ".o")
    subprocess.check_call([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get(os.path.basename(f), []) + defs + ["-c", f, "-o", o],
                          stderr=subprocess.DEVNULL)
    return o


with cf.ThreadPoolExecutor(max_workers=8) as ex:
    objs = list(ex.map(one, B.sources()))
subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"])
os.replace(out + ".tmp", out)
print(out)
