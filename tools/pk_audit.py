"""Audit packed-fp32 VALU usage per kernel in libstzs_hip.so (or any offload bundle / code object).

    python tools/pk_audit.py [path/to/libstzs_hip.so] [--json out.json]

Unbundles the gfx950 code objects into a temp dir, disassembles every kernel and classifies its
v_pk_{fma,mul,add}_f32 / v_pk_mov_b32 instructions by operand modifiers:
  plain   -- no op_sel / neg modifiers (lane-wise pair arithmetic)
  opsel   -- op_sel:[..1..] (a source's HIGH half feeds the low lane: cross-half select)
  opselhi -- op_sel_hi with a 0 (a source's LOW half feeds the high lane: broadcast)
  swap    -- one source with op_sel 1 AND op_sel_hi 0: its halves exchanged (the two-shard fault pattern)
  neg     -- neg_lo / neg_hi
  pkmov   -- v_pk_mov_b32 (half shuffles)
Used for the DESIGN.md §5 two-shard root-cause audit.
"""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, tmp):
    """unbundle the gfx950 code objects of `lib` into `tmp` (llvm-objdump --offloading writes next to its input)"""
    import shutil
    local = os.path.join(tmp, "lib.so")
    shutil.copy(lib, local)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], cwd=tmp, capture_output=True)
    return sorted(glob.glob(os.path.join(tmp, "lib.so.*gfx950")))


def classify(line):
    m = re.search(r"\b(v_pk_(?:fma|mul|add)_f32|v_pk_mov_b32)\b(.*)", line)
    if not m:
        return None
    op, rest = m.groups()
    cls = []
    if op == "v_pk_mov_b32":
        cls.append("pkmov")
    else:
        os_ = re.search(r"op_sel:\[([0-9,]+)\]", rest)
        osv = [int(x) for x in os_.group(1).split(",")] if os_ else [0, 0, 0]
        oh = re.search(r"op_sel_hi:\[([0-9,]+)\]", rest)
        ohv = [int(x) for x in oh.group(1).split(",")] if oh else [1, 1, 1]
        if any(osv):
            cls.append("opsel")
        if not all(ohv):
            cls.append("opselhi")
        # a source whose halves are exchanged: its HIGH dword feeds the low lane and its LOW dword the high lane
        if any(o == 1 and h == 0 for o, h in zip(osv, ohv)):
            cls.append("swap")
        if "neg_lo" in rest or "neg_hi" in rest:
            cls.append("neg")
        if not cls:
            cls.append("plain")
    return op, cls


def audit(lib):
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn", co],
                                 capture_output=True, text=True).stdout
            kern = None
            for line in dis.splitlines():
                h = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if h:
                    kern = h.group(1)
                    continue
                c = classify(line)
                if c and kern:
                    k = res.setdefault(kern, collections.Counter())
                    k["total"] += 1
                    for x in c[1]:
                        k[x] += 1
    return res


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?")
    ap.add_argument("--json")
    a = ap.parse_args()
    lib = a.lib if a.lib else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "styletts-zs_amd", "stzs", "libstzs_hip.so")
    res = audit(lib)
    names = sorted(res)
    dem = demangle(names)
    rows = []
    for n, d in sorted(zip(names, dem), key=lambda x: -res[x[0]]["total"]):
        c = res[n]
        rows.append(dict(kernel=d[:110], **{k: c.get(k, 0) for k in ("total", "plain", "opsel", "opselhi", "swap", "neg", "pkmov")}))
    print(f"{'kernel':110s} total plain opsel opselhi swap neg pkmov")
    for r in rows:
        print(f"{r['kernel']:110s} {r['total']:5d} {r['plain']:5d} {r['opsel']:5d} {r['opselhi']:7d} {r['swap']:4d} "
              f"{r['neg']:3d} {r['pkmov']:5d}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
