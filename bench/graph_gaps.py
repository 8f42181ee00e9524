"""Per-step kernel durations and inter-kernel gaps of a graph-replayed bench run
(rocprofv3 --kernel-trace CSV).  usage: python bench/graph_gaps.py RUN_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# steps start at the input-gather kernel
starts = [i for i, r in enumerate(rows) if "prep_images" in r["Kernel_Name"] or "perm_positions" in r["Kernel_Name"]]
steps = [(a, b) for a, b in zip(starts, starts[1:])][-10:]
tot_busy = tot_wall = 0
for a, b in steps:
    seg = rows[a:b]
    wall = int(rows[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    tot_busy += busy
    tot_wall += wall
n = len(steps)
print(f"steps {n}: wall {tot_wall / n / 1e3:.1f} us/step, kernel busy {tot_busy / n / 1e3:.1f} us, "
      f"gaps {(tot_wall - tot_busy) / n / 1e3:.1f} us over {steps[-1][1] - steps[-1][0]} kernels")
a, b = steps[-1]
for i in range(a, b):
    r = rows[i]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    g = (int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
    print(f"{d:8.1f} us  gap {g:6.1f}  {r['Kernel_Name'][:80]}")
