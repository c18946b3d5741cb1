"""Phase summary of a configs[1] latency trace: rocprofv3 --kernel-trace over tools/lat_probe.py (N graph replays).

    python tools/lat_trace.py gpurun_out/<dir>/run_kernel_trace.csv > profiles/<name>.txt

Takes the last graph replay (each synth() opens with the token embedding kernel), splits it at the kernels that open each
stage of synth() (state_init: sampler; pr_prep: durations; align_kernel: prosody; phase_prefix / source_stft:
decoder) and prints, per phase, the span, the summed kernel time and the launch count, then the per-kernel-family
totals of the replay."""
import collections
import csv
import re
import sys


def name(r):
    m = re.search(r"::(\w+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"].split("(")[0][:40]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    reps = [[]]
    for r in rows:  # a synth() opens with the token embedding
        if name(r) in ("embed_kernel", "embed_f32_kernel") and reps[-1]:
            reps.append([])
        reps[-1].append(r)
    last = reps[-1]
    names = [name(r) for r in last]
    t0 = lambda r: int(r["Start_Timestamp"])
    t1 = lambda r: int(r["End_Timestamp"])
    marks = [("front (text + prompt)", 0)]
    for label, key in (("sampler (NFE x CFG)", "state_init_kernel"), ("durations (BiLSTMs + dur LSTM)", "pr_prep"),
                       ("prosody (align -> F0/N)", "align_kernel"), ("decoder (source -> iSTFT)", "phase_prefix_kernel")):
        idx = next((i for i, n in enumerate(names) if n == key), None)
        if idx is None and key == "phase_prefix_kernel":
            idx = next((i for i, n in enumerate(names) if n == "source_stft_kernel"), None)
        if idx is not None:
            marks.append((label, idx))
    marks.append(("end", len(last)))
    span = (t1(last[-1]) - t0(last[0])) / 1e3
    busy = sum(t1(r) - t0(r) for r in last) / 1e3
    print(f"last replay: {len(last)} kernels, span {span:.1f} us, kernel-busy {busy:.1f} us")
    print(f"{'phase':34s} {'span us':>9s} {'busy us':>9s} {'kernels':>8s}")
    for (label, i), (_, j) in zip(marks, marks[1:]):
        seg = last[i:j]
        if not seg:
            continue
        print(f"{label:34s} {(t1(seg[-1]) - t0(seg[0])) / 1e3:9.1f} {sum(t1(r) - t0(r) for r in seg) / 1e3:9.1f} "
              f"{len(seg):8d}")
    c, t = collections.Counter(), collections.Counter()
    for r, n in zip(last, names):
        c[n] += 1
        t[n] += (t1(r) - t0(r)) / 1e3
    print(f"\n{'kernel family':30s} {'calls':>6s} {'total us':>9s} {'avg us':>8s}")
    for n, _ in t.most_common(20):
        print(f"{n:30s} {c[n]:6d} {t[n]:9.1f} {t[n] / c[n]:8.2f}")
    if "--list" in sys.argv:  # every kernel of the replay in order: duration and the gap before it
        print(f"\n{'#':>4s} {'kernel':34s} {'us':>7s} {'gap us':>7s}")
        prev = None
        for k, (r, n) in enumerate(zip(last, names)):
            gap = (t0(r) - t1(prev)) / 1e3 if prev is not None else 0.0
            print(f"{k:4d} {n[:34]:34s} {(t1(r) - t0(r)) / 1e3:7.2f} {gap:7.2f}")
            prev = r


if __name__ == "__main__":
    main(sys.argv[1])
