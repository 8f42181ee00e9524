"""Summarise a rocprofv3 kernel_trace.csv as a per-step timeline: for the last
complete training step (delimited by the first kernel of the step, given by a
name substring), print each kernel's start/end relative to the step start, its
duration, and mark collectives (RCCL kernels) so it is visible which compute
kernels they run next to.  Usage: trace_timeline.py CSV STEP_FIRST_KERNEL [N_STEPS_BACK]"""
import csv
import sys


def main():
    path, first = sys.argv[1], sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    if len(starts) < back + 1:
        print("not enough steps in trace", len(starts))
        return 1
    i0, i1 = starts[-back - 1], starts[-back]
    step = rows[i0:i1]
    t0 = step[0][0]
    print(f"# step window: {len(step)} kernels, {(step[-1][1] - t0) / 1e3:.1f} us from first start to last end")
    print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8}  kernel")
    coll_us = 0.0
    busy = []
    for s, e, n in step:
        tag = "  <== COLLECTIVE" if ("ncclDevKernel" in n or "nccl" in n.lower() or "rccl" in n.lower()) else ""
        if tag:
            coll_us += (e - s) / 1e3
        else:
            busy.append((s, e))
        short = n.split("(")[0][:90]
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {short}{tag}")
    # collective time overlapped by some compute kernel
    ov = 0.0
    for s, e, n in step:
        if "nccl" not in n.lower() and "rccl" not in n.lower():
            continue
        for bs, be in busy:
            lo, hi = max(s, bs), min(e, be)
            if hi > lo:
                ov += (hi - lo) / 1e3
    print(f"# collective kernel time {coll_us:.1f} us, of which concurrent with compute kernels {min(ov, coll_us):.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
