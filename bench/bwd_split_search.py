#!/usr/bin/env python3
"""Work-split candidates for the fused LeNet-5 conv backward (lenet_bwd.hip), timed as separate
processes (MNISTX_BWD_SPLIT, bench/micro_lenet_bwd_quick.py), rounds interleaved.  The parent
never touches the GPU.

    python bench/bwd_split_search.py [rounds]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the round-4 split (the searches below start from it; the kernel's default is now round 5's "duD_c1_44444422")
DU = [2, 10, 0, -1, 6, 5, 3, 8, 7, 11, -1, 1, 12, 13, 9, 4]
K20 = [0, 1, 8, 23, 0, 8, 16, 23, 0, 7, 15, 22, 0, 7, 14, 22]
K21 = [1, 8, 23, 30, 8, 16, 23, 30, 7, 15, 22, 30, 7, 14, 22, 30]
K10 = [0, 4, 8, 12, 16, 19, 22, 25]
K11 = [4, 8, 12, 16, 19, 22, 25, 28]


def cfg(du=DU, k20=K20, k21=K21, k10=K10, k11=K11):
    return ",".join(str(v) for v in list(du) + list(k20) + list(k21) + list(k10) + list(k11))


def swap(du, a, b):
    d = list(du)
    d[a], d[b] = d[b], d[a]
    return d


def group_ranges(k20, k21, G, cuts):
    """tile group G's 30 k-steps cut at `cuts` (3 increasing values) in wave order"""
    a, b = list(k20), list(k21)
    edges = [0] + list(cuts) + [30]
    for t in range(4):
        a[4 * G + t], b[4 * G + t] = edges[t], edges[t + 1]
    return a, b


def c1_ranges(steps):
    a, b, k = [], [], 0
    for n in steps:
        a.append(k)
        b.append(k + n)
        k += n
    assert k == 28
    return a, b


def candidates():
    """round 3 (round 2: base2 + conv1 ranks 3,3,4,4,4,4,3,3 gave 201.0 -> 197.0 us)"""
    c = {"default": cfg()}   # the round-4 split
    d = swap(swap(DU, 15, 3), 14, 10)
    a0, b0 = group_ranges(K20, K21, 0, (6, 13, 23))
    a1, b1 = c1_ranges([3, 3, 4, 4, 4, 4, 3, 3])
    c["best2"] = cfg(du=d, k20=a0, k21=b0, k10=a1, k11=b1)   # round 3 winner
    for name, steps in (("c1_3444_4433", [3, 4, 4, 4, 4, 4, 3, 2]), ("c1_2344_4444", [2, 3, 4, 4, 4, 4, 4, 3]),
                        ("c1_3344_4442", [3, 3, 4, 4, 4, 4, 4, 2])):
        a, b = c1_ranges(steps)
        c["best2_" + name] = cfg(du=d, k20=a0, k21=b0, k10=a, k11=b)
    for name, cuts in (("g0_5_12_22", (5, 12, 22)), ("g0_7_14_23", (7, 14, 23)), ("g0_6_14_22", (6, 14, 22))):
        a, b = group_ranges(K20, K21, 0, cuts)
        c["best2_" + name] = cfg(du=d, k20=a, k21=b, k10=a1, k11=b1)
    a, b = group_ranges(a0, b0, 1, (7, 15, 23))
    c["best2_g1_7_15_23"] = cfg(du=d, k20=a, k21=b, k10=a1, k11=b1)
    return c


def candidates4():
    """round 4, from the per-wave clocks of best2 (profiles/r5/lenet/bwd_split/): on each SIMD
    (waves s, s+4, s+8, s+12) the oldest wave finishes phase 1 first and the youngest last, so
    move dgrad taps (unit cost: rows 0/6 2 taps, 1/5 4, 2-4 5) and conv1 k-steps to older waves"""
    d0 = swap(swap(DU, 15, 3), 14, 10)
    a0, b0 = group_ranges(K20, K21, 0, (6, 13, 23))
    a1, b1 = c1_ranges([3, 3, 4, 4, 4, 4, 3, 3])
    c = {"best2": cfg(du=d0, k20=a0, k21=b0, k10=a1, k11=b1)}
    dB = swap(d0, 2, 10)
    dC = swap(dB, 0, 8)
    dD = swap(dC, 1, 5)
    c["du_2_10"] = cfg(du=dB, k20=a0, k21=b0, k10=a1, k11=b1)
    c["du_2_10_0_8"] = cfg(du=dC, k20=a0, k21=b0, k10=a1, k11=b1)
    c["du_2_10_0_8_1_5"] = cfg(du=dD, k20=a0, k21=b0, k10=a1, k11=b1)
    for name, steps in (("c1_4444_3333", [4, 4, 4, 4, 3, 3, 3, 3]), ("c1_4344_4432", [4, 3, 4, 4, 4, 4, 3, 2]),
                        ("c1_4444_4422", [4, 4, 4, 4, 4, 4, 2, 2])):
        a, b = c1_ranges(steps)
        c["best2_" + name] = cfg(du=d0, k20=a0, k21=b0, k10=a, k11=b)
        c["du_2_10_0_8_" + name] = cfg(du=dC, k20=a0, k21=b0, k10=a, k11=b)
    return c


def candidates5():
    """round 5: round 4 found conv1 ranks 4,4,4,4,4,4,2,2 (193.2 vs 195.2 us); push further"""
    d0 = swap(swap(DU, 15, 3), 14, 10)
    dD = swap(swap(swap(d0, 2, 10), 0, 8), 1, 5)
    a0, b0 = group_ranges(K20, K21, 0, (6, 13, 23))
    c = {}
    for steps in ([4, 4, 4, 4, 4, 4, 2, 2], [4, 4, 4, 4, 4, 4, 3, 1], [5, 5, 4, 4, 4, 4, 1, 1], [4, 4, 5, 5, 4, 4, 1, 1],
                  [4, 4, 4, 4, 5, 5, 1, 1], [4, 4, 4, 4, 4, 4, 4, 0], [5, 5, 5, 5, 4, 4, 0, 0]):
        a, b = c1_ranges(steps)
        tag = "".join(map(str, steps))
        c["best2_c1_" + tag] = cfg(du=d0, k20=a0, k21=b0, k10=a, k11=b)
        if tag in ("44444422", "55444411", "44554411"):
            c["duD_c1_" + tag] = cfg(du=dD, k20=a0, k21=b0, k10=a, k11=b)
    return c


def candidates_ab():
    """confirmation A/B of round 5's leaders against the default"""
    c5 = candidates5()
    c4 = candidates4()
    return {"best2": c4["best2"], "best2_c1_44444422": c5["best2_c1_44444422"], "duD_c1_44444422": c5["duD_c1_44444422"]}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cands = {"3": candidates, "4": candidates4, "5": candidates5, "ab": candidates_ab}[os.environ.get("SEARCH_ROUND", "5")]()
    res = {k: [] for k in cands}
    for _ in range(rounds):
        for name, split in cands.items():
            env = dict(os.environ, MNISTX_BWD_SPLIT=split)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "micro_lenet_bwd_quick.py")], env=env,
                                 capture_output=True, text=True, timeout=120)
            if out.returncode != 0:
                res[name].append(None)
                print(name, "failed", out.stderr[-300:], flush=True)
                continue
            res[name].append(json.loads(out.stdout.strip().splitlines()[-1])["lenet_bwd_us"])
            print(name, res[name][-1], flush=True)
    summary = {k: sorted(v for v in vs if v is not None) for k, vs in res.items()}
    print(json.dumps({k: (v[len(v) // 2] if v else None) for k, v in summary.items()}), flush=True)


if __name__ == "__main__":
    main()
