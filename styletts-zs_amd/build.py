"""Build libstzs_hip.so in-tree for gfx950 (explicit hipcc, no JIT cache, no cmake).

    python styletts-zs_amd/build.py [-v] [--force]

Objects go to styletts-zs_amd/build/, the shared library to styletts-zs_amd/stzs/libstzs_hip.so
(git-ignored, but shipped to the GPU box by gpurun with the rest of the tree).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "stzs", "libstzs_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=fast", "-Wall",
         "-Wno-unused-result", f"-I{INCLUDE}"]
# per-file extra flags (the host compile ignores the gfx950 target feature with a warning).  source.hip: no packed
# fp32 VALU ops -- its STFT tail, compiled to v_pk_fma_f32 with op_sel / neg modifiers, stored wrong imaginary bins
# for 16-lane groups in ~1 of 3 two-shard concurrent replays (timing-dependent: never in a sequential replay);
# without packed ops, 0 of 120 (tools/two_shard_stress.py)
FILE_FLAGS = {"source.hip": ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _includes(path, seen):
    """the quoted #include files of `path`, recursively (csrc/ headers and include/stzs.h)"""
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("#include") and '"' in line:
                name = line.split('"')[1]
                for d in (os.path.dirname(path), CSRC, INCLUDE):
                    q = os.path.join(d, name)
                    if os.path.exists(q):
                        if q not in seen:
                            seen.add(q)
                            _includes(q, seen)
                        break
    return seen


def _deps_mtime(src):
    return max(os.path.getmtime(p) for p in [src] + sorted(_includes(src, set())))


def _compile(src, force, verbose):
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime(src):
        return obj
    cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.force, a.verbose))
