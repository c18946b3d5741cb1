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
# per-file extra flags (the host compile ignores the gfx950 target feature with a warning): no packed-fp32 VALU ops
# where hipcc emits packed ops that SWAP a source's 32-bit halves (op_sel 1 + op_sel_hi 0 on one operand).  On MI355X
# such an op intermittently writes wrong values for lanes 48-63 of a wave while other kernels share the CU: the
# harmonic-source STFT built with them failed 104 of 512 swept two-shard passes, the same code with only its 7 swapped
# operands pre-swapped by two v_mov_b32 (everything else still packed) 0 of 512 (tools/pk_bisect.py,
# profiles/r04_*_pk_bisect*.log).  tests/test_isa_audit.py fails the build if any kernel of the
# library contains the pattern; the conv / GEMM epilogues and prologues (conv.hip, gemm.hip, convx.hip: one file until r04)
# and source.hip's STFT sums are where hipcc made it
# (and the r04 warp-specialised MRF conv's staging transform, since removed).
NO_PK = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
FILE_FLAGS = {"source.hip": NO_PK, "conv.hip": NO_PK, "gemm.hip": NO_PK, "convx.hip": NO_PK,
              # (r06, for speed, not the hazard: the stage-1 MRF convs' staging VALU beside MFMAs, csrc/mrfv_n1.hip)
              "mrfv_n1.hip": NO_PK}


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
    """compile one source unless its object is newer than every dependency AND was built by the same command:
    the exact command line is kept in a stamp file beside the object, so a change of FLAGS / FILE_FLAGS / HIPCC
    rebuilds it (an object from before a codegen flag existed is never reused)"""
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    stamp = obj + ".cmd"
    cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    key = " ".join(cmd)
    fresh = (os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime(src) and os.path.exists(stamp) and
             open(stamp).read() == key)
    if not force and fresh:
        return obj
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    with open(stamp, "w") as f:
        f.write(key)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"  # linked aside and renamed: a reader (a copy of the tree) never sees a partial library
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.force, a.verbose))
