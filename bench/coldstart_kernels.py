#!/usr/bin/env python3
"""Per-kernel durations by step window from a rocprofv3 kernel trace of
``bench/step_trace.py``: answers whether the cold-start gap (first steps slower than
the steady state) sits in one kernel or in all of them, and in the gaps between them.

    python bench/coldstart_kernels.py <rocprof dir> <steps traced> [out.md]

Windows: steps 0-4, 5-24 (the driver's 5 warmup + 20 timed), 100-149, last 50.  Per
kernel: mean duration (us); per window also the mean step span (first kernel start to
the next step's first kernel start) and the idle share of it (span - kernel sum).
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    count, first = {}, {}
    for r in rows:
        n = r["Kernel_Name"]
        count[n] = count.get(n, 0) + 1
        first.setdefault(n, int(r["Start_Timestamp"]))
    # the step's first kernel: the earliest-starting kernel that runs exactly once per traced
    # step (prewarm kernels of another kind run before the first boundary)
    once = [n for n, c in count.items() if c >= steps]
    k0 = min(once, key=lambda n: first[n])
    bounds = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"] == k0][-steps:]
    bounds.append(max(int(r["End_Timestamp"]) for r in rows))
    per_step = [dict() for _ in range(steps)]
    j = 0
    for r in rows:
        s = int(r["Start_Timestamp"])
        if s < bounds[0]:
            continue
        while j + 1 < steps and s >= bounds[j + 1]:
            j += 1
        n = short(r["Kernel_Name"])
        per_step[j][n] = per_step[j].get(n, 0) + (int(r["End_Timestamp"]) - s)
    wins = [("0-4", 0, 5), ("5-24", 5, 25), ("100-149", 100, 150), (f"last 50", steps - 50, steps)]
    wins = [w for w in wins if w[2] <= steps and w[1] >= 0]
    names = sorted({n for ps in per_step for n in ps}, key=lambda n: -sum(ps.get(n, 0) for ps in per_step))
    lines = ["| kernel | " + " | ".join(f"steps {w[0]} (us)" for w in wins) + " |",
             "|---|" + "---|" * len(wins)]
    for n in names:
        vals = [sum(per_step[i].get(n, 0) for i in range(a, b)) / (b - a) / 1e3 for _, a, b in wins]
        lines.append(f"| `{n}` | " + " | ".join(f"{v:.1f}" for v in vals) + " |")
    spans, sums = [], []
    for _, a, b in wins:
        sp = [(bounds[i + 1] - bounds[i]) / 1e3 for i in range(a, b)]
        ks = [sum(per_step[i].values()) / 1e3 for i in range(a, b)]
        spans.append(sum(sp) / len(sp))
        sums.append(sum(ks) / len(ks))
    lines.append("| **kernel sum / step** | " + " | ".join(f"**{v:.1f}**" for v in sums) + " |")
    lines.append("| _step span (boundary to boundary)_ | " + " | ".join(f"_{v:.1f}_" for v in spans) + " |")
    lines.append("| _idle in the span_ | " + " | ".join(f"_{s - k:.1f}_" for s, k in zip(spans, sums)) + " |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if out:
        open(out, "w").write(txt)


if __name__ == "__main__":
    main()
