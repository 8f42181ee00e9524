#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace --stats`` CSV directory: per-kernel
time per training step, sorted.  Usage: prof_summary.py <dir> <steps> [out.md]"""
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


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = ["| kernel | calls | avg us | per-step us | share |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if t / tot < 0.002:
            continue
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{t/1e3/steps:.1f} | {100*t/tot:.1f}% |")
    lines.append(f"| **total GPU time / step** | | | **{tot/1e3/steps:.1f}** | |")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out + "\n")


if __name__ == "__main__":
    main()
