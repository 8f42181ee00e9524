#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace --stats`` CSV directory: per-kernel
time per training step, sorted.  Usage: prof_summary.py <dir> <steps> [out.md] [skip]

``steps`` = every step the traced command ran (warmup included); the first ``skip`` step
windows (warmup: clock ramp, first touches) are left out of the table, and the table ends
with the traced wall span per kept step (first kept step's first kernel start to the last
kernel's end), which is what the kernel sum is reconciled against."""
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"mnistx::", "", name)
    m = re.match(r"(?:void )?([\w:]+)(<.*>)?\(", name)
    base = m.group(1) if m else name[:60]
    tmpl = ""
    if m and m.group(2):
        t = m.group(2)
        t = re.sub(r"Geo<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", r"Geo<ci\1,co\2,k\3,p\4,\5x\6>", t)
        tmpl = t[:90]
    return base + tmpl


def step_windows(d: str, steps: int, skip: int = 0):
    """Per-kernel (calls, total ns) inside the training steps, from the kernel trace:
    the step boundaries are the launches of the earliest kernel that runs exactly once per
    step; everything before the first boundary (dataset upload, buffer fills, clock
    prewarm) is setup.  The last step runs to the trace's end."""
    tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not tr:
        return None
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    count: dict = {}
    first: dict = {}
    for r in rows:
        n = r["Kernel_Name"]
        count[n] = count.get(n, 0) + 1
        first.setdefault(n, int(r["Start_Timestamp"]))
    once = [n for n, c in count.items() if c == steps]
    if not once:
        return None
    k0 = min(once, key=lambda n: first[n])
    bounds = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"] == k0]
    t0 = bounds[min(skip, len(bounds) - 1)]
    agg: dict = {}
    setup_ns = 0
    end = t0
    for r in rows:
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if int(r["Start_Timestamp"]) < t0:
            setup_ns += dur
            continue
        end = max(end, int(r["End_Timestamp"]))
        c, t = agg.get(r["Kernel_Name"], (0, 0))
        agg[r["Kernel_Name"]] = (c + 1, t + dur)
    step_wall_ns = (end - t0) / max(1, steps - skip)
    return agg, setup_ns, step_wall_ns


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    win = step_windows(d, steps, skip)
    wall_ns = None
    if win is not None:
        agg, setup_ns, wall_ns = win
        rows = [{"Name": n, "Calls": str(c), "TotalDurationNs": str(t), "AverageNs": str(t / c)} for n, (c, t) in agg.items()]
        steps -= skip
    else:
        f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
        rows, setup_ns = list(csv.DictReader(open(f))), 0
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = ["| kernel | calls | avg us | per-step us | share |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if t / tot < 0.002:
            continue
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{t/1e3/steps:.1f} | {100*t/tot:.1f}% |")
    lines.append(f"| **total GPU time / step** | | | **{tot/1e3/steps:.1f}** | |")
    if wall_ns:
        lines.append(f"| _traced wall span / step ({steps} steps after {skip} warmup; kernel sum / span "
                     f"{tot / steps / wall_ns:.3f})_ | | | _{wall_ns/1e3:.1f}_ | |")
    if setup_ns:
        lines.append(f"| _setup before the first step (dataset upload, fills, prewarm): not in the total_ | | | "
                     f"_{setup_ns/1e3:.1f} us in all_ | |")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out + "\n")


if __name__ == "__main__":
    main()
