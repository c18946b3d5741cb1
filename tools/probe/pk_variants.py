"""Build code-object variants of csrc/source.hip for the two-shard root-cause bisection.

    python tools/probe/pk_variants.py        -> tools/probe/pk_<variant>.hsaco

Variants of source_stft_kernel<20> (the harmonic-source STFT; phase_prefix_kernel is unchanged in all):
  pk         packed-fp32 VALU ops, as hipcc emits them (the build before round 3's workaround)
  pk_nop     pk + `s_nop 4` in front of every packed op that SWAPS a source's halves (op_sel 1 + op_sel_hi 0)
  pk_nopa    pk + `s_nop 4` right after every such op (a wait state between it and whatever reads its result)
  pk_unswap  pk with every swapped source replaced by a pre-swapped copy in two fresh VGPRs (two v_mov_b32
             ahead of the op, default op_sel / op_sel_hi for that source): the same arithmetic, no swap
  nopk       built with -packed-fp32-ops (the current library's form)
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(ROOT, "styletts-zs_amd", "csrc", "source.hip")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_ZN12_GLOBAL__N_118source_stft_kernelILi20EEEv16stzs_source_args"
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast", f"-I{ROOT}/include",
         "--cuda-device-only", "-S"]
NOPK = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]

PK = re.compile(r"^(\s*)(v_pk_(?:fma|mul|add)_f32)\s+(.*)$")


def device_asm(extra, out):
    subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + [SRC, "-o", out], check=True, capture_output=True)
    with open(out) as f:
        return f.read().splitlines()


def swap_info(rest):
    """-> (operands, op_sel list, op_sel_hi list, modifier text) of a VOP3P packed-fp32 op"""
    body = rest.split("//")[0].strip()
    mods = re.findall(r"(op_sel(?:_hi)?|neg_lo|neg_hi):\[([0-9,]+)\]", body)
    ops_txt = re.split(r"\s+(?=op_sel|neg_)", body, maxsplit=1)[0]
    ops = [o.strip() for o in ops_txt.split(",")]
    nsrc = len(ops) - 1
    osel = [0] * nsrc
    ohi = [1] * nsrc
    other = []
    for k, v in mods:
        vals = [int(x) for x in v.split(",")]
        if k == "op_sel":
            osel = vals
        elif k == "op_sel_hi":
            ohi = vals
        else:
            other.append(f"{k}:[{v}]")
    return ops, osel, ohi, other


def fmt(op, ops, osel, ohi, other):
    mods = []
    if any(osel):
        mods.append("op_sel:[" + ",".join(map(str, osel)) + "]")
    if not all(ohi):
        mods.append("op_sel_hi:[" + ",".join(map(str, ohi)) + "]")
    return f"\t{op} " + ", ".join(ops) + ("" if not mods + other else " " + " ".join(mods + other))


def transform(lines, mode):
    out, inside, nsw = [], False, 0
    for ln in lines:
        if ln.startswith(KERNEL + ":"):
            inside = True
        elif inside and ln.startswith(".Lfunc_end") :
            inside = False
        m = PK.match(ln) if inside else None
        if m:
            ops, osel, ohi, other = swap_info(m.group(3))
            sw = [i for i in range(len(osel)) if osel[i] == 1 and ohi[i] == 0]
            if sw:
                nsw += 1
                if mode == "pk_nop":
                    out.append("\ts_nop 4")
                elif mode == "pk_nopa":
                    out.append(ln)
                    out.append("\ts_nop 4")
                    continue
                elif mode == "pk_unswap":
                    assert len(sw) == 1, ln
                    i = sw[0]
                    r = re.fullmatch(r"v\[(\d+):(\d+)\]", ops[1 + i])
                    assert r, ln
                    lo = int(r.group(1))
                    out.append(f"\tv_mov_b32_e32 v132, v{lo + 1}")
                    out.append(f"\tv_mov_b32_e32 v133, v{lo}")
                    ops = list(ops)
                    ops[1 + i] = "v[132:133]"
                    osel = list(osel)
                    ohi = list(ohi)
                    osel[i], ohi[i] = 0, 1
                    out.append(fmt(m.group(2), ops, osel, ohi, other))
                    continue
        if mode == "pk_unswap" and inside is False and ln.strip().startswith(".amdhsa_kernel " + KERNEL):
            pass
        out.append(ln)
    if mode == "pk_unswap":  # two more VGPRs for the pre-swapped copies (132 -> 136 with the accum offset)
        txt = "\n".join(out)
        blk = txt.index(".amdhsa_kernel " + KERNEL)
        end = txt.index(".end_amdhsa_kernel", blk)
        seg = txt[blk:end]
        seg = re.sub(r"\.amdhsa_next_free_vgpr \d+", ".amdhsa_next_free_vgpr 136", seg)
        seg = re.sub(r"\.amdhsa_accum_offset \d+", ".amdhsa_accum_offset 136", seg)
        txt = txt[:blk] + seg + txt[end:]
        md = txt.index(".name:           " + KERNEL)
        vc = txt.index(".vgpr_count:", md)
        eol = txt.index("\n", vc)
        txt = txt[:vc] + ".vgpr_count:     136" + txt[eol:]
        out = txt.split("\n")
    return out, nsw


def assemble(lines, name):
    s = os.path.join("/tmp", f"pk_{name}.s")
    o = os.path.join("/tmp", f"pk_{name}.o")
    co = os.path.join(HERE, f"pk_{name}.hsaco")
    with open(s, "w") as f:
        f.write("\n".join(lines) + "\n")
    subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s, "-o", o],
                   check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", o, "-o", co], check=True)
    return co


if __name__ == "__main__":
    pk = device_asm([], "/tmp/pk_src.s")
    nopk = device_asm(NOPK, "/tmp/nopk_src.s")
    for mode in ("pk", "pk_nop", "pk_nopa", "pk_unswap"):
        lines, nsw = transform(pk, mode)
        print(mode, "swapped-source packed ops in the STFT kernel:", nsw, "->", assemble(lines, mode))
    print("nopk ->", assemble(nopk, "nopk"))
