"""Static check of LDS-load waits in a straight-line stretch of gfx950 assembly.

    python tools/lgkm_check.py file.s START_LINE END_LINE

Models LDS loads (ds_read*) as an in-order FIFO against `s_waitcnt lgkmcnt(N)` and reports every
instruction that reads or overwrites a VGPR whose ds_read may still be outstanding (RAW / WAW).
Scalar-memory loads also count in lgkmcnt (out of order): if one is outstanding the checker assumes
the worst and says so.  Used for the source_stft_kernel root-cause study.
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def operands(line):
    body = line.split("//")[0].split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    ops = [o.strip().lstrip("-|").rstrip("|") for o in re.split(r",\s*", parts[1])]
    ops = [o.split()[0] if o else o for o in ops]
    return parts[0], ops


def check(lines):
    fifo = []  # outstanding LDS loads: (line_no, set(vregs))
    smem = 0
    issues = []
    for no, line in lines:
        op, ops = operands(line)
        if not op or op.startswith(".") or op.endswith(":"):
            continue
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", line)
            if m:
                n = int(m.group(1))
                if smem and n == 0:
                    smem = 0
                while len(fifo) > n:
                    fifo.pop(0)
            continue
        if op.startswith("s_load") or op.startswith("s_buffer_load"):
            smem += 1
            continue
        if not op.startswith(("v_", "ds_", "global_", "buffer_")):
            continue
        all_regs = [regs(o) for o in ops]
        if op.startswith("ds_read") or op.startswith("ds_load"):
            dst, srcs = all_regs[0], all_regs[1:]
        elif op.startswith(("ds_write", "ds_store", "global_store", "buffer_store")):
            dst, srcs = set(), all_regs
        else:
            dst, srcs = (all_regs[0] if all_regs else set()), all_regs[1:]
        used = set().union(*srcs) if srcs else set()
        for lno, d in fifo:
            if used & d:
                issues.append((no, "RAW", lno, sorted(used & d), line.strip()))
            if dst & d:
                issues.append((no, "WAW", lno, sorted(dst & d), line.strip()))
        if op.startswith("ds_read") or op.startswith("ds_load"):
            fifo.append((no, dst))
    return issues, smem


if __name__ == "__main__":
    path, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    with open(path) as f:
        src = f.read().splitlines()
    iss, smem = check([(i + 1, src[i]) for i in range(a - 1, min(b, len(src)))])
    print(f"{path}:{a}-{b}: {len(iss)} possible LDS-wait hazards; scalar loads outstanding at end: {smem}")
    for x in iss:
        print(f"  line {x[0]} {x[1]} on v{x[3]} of ds_read at line {x[2]}: {x[4]}")
