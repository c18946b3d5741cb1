"""Static instruction mix of one kernel in a hipcc -S listing: counts per class and the summed ISSUE cycles of a
wave's stream, with the costs measured in /opt/skills/guides/MI355X_MICROARCH.md (constants table): plain VALU 4,
transcendental 8, v_cvt_pk_bf16_f32 4, 16x16x32 MFMA 8 of issue (16 of pipe).  Straight-line kernels only
(loops are counted once).

    python tools/isa_count.py listing.s <kernel-symbol-substring>
"""
import re
import sys
from collections import Counter

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def body(path, sym):
    out, on = [], False
    for ln in open(path):
        if not on and re.match(rf"^\S*{re.escape(sym)}\S*:", ln):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            s = ln.strip()
            if s and not s.startswith((";", ".")) and not s.endswith(":"):
                out.append(s.split()[0])
    return out


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(TRANS):
        return "valu_trans"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_write"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith(("global_load", "buffer_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


if __name__ == "__main__":
    ops = body(sys.argv[1], sys.argv[2])
    c = Counter(classify(o) for o in ops)
    cyc = 4 * (c["valu"] + c["valu_pk"]) + 8 * c["valu_trans"] + 8 * c["mfma"]
    print(f"{len(ops)} instructions: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    print(f"vector issue cycles per wave: VALU {4 * (c['valu'] + c['valu_pk']) + 8 * c['valu_trans']}, "
          f"MFMA {8 * c['mfma']} (pipe {16 * c['mfma']}), total issue {cyc}")
    top = Counter(o for o in ops if o.startswith("v_") and not o.startswith("v_mfma"))
    print("top VALU:", ", ".join(f"{k} {v}" for k, v in top.most_common(25)))
