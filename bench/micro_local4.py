#!/usr/bin/env python3
"""The reference CNN's local4 GEMMs at B = 16384 (16384 x 1024 -> 192: forward + bias + ReLU,
data gradient with local3's ReLU mask, split-K weight gradient with the bias row) on every
candidate gemm.hip tile, interleaved rounds in one process; median us.

    python bench/micro_local4.py [B]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops import functional as Fk  # noqa: E402
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402

# gemm.hip TileCode values
CODES = {"256x16": 0, "256x32": 1, "128x64": 2, "64x128": 3, "128x128": 4, "64x16": 5, "64x32": 6, "64x64": 7,
         "256x128": 8, "32x192": 9, "64x192": 10, "128x192": 11}


def main():
    K = kernels()
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    din, dout = 1024, 192
    torch.manual_seed(0)
    x = torch.randn(B, din, device=dev).to(torch.bfloat16)
    w = (torch.randn(din, dout, device=dev) / din ** 0.5).to(torch.bfloat16)
    b = torch.randn(dout, device=dev) * 0.1
    dy = torch.randn(B, dout, device=dev).to(torch.bfloat16)
    y = torch.empty(B, dout, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, din, device=dev, dtype=torch.bfloat16)
    slab = torch.empty(64 * (din + 1) * dout, device=dev)

    def fwd(code):
        return lambda: K.dense_fwd(x, w, y, B, dout, din, din, dout, dout, b, dout, True, None, 0, code)

    def dgrad(code):
        return lambda: K.dense_dgrad(dy, w, dx, B, din, dout, dout, dout, din, x, din, code)

    def wgrad(code, bm, bn):
        S = Fk.pick_splits(din + 1, dout, B, dense=True) if code < 0 else None

        def f():
            s = S
            if s is None:   # the split rule for this tile
                tiles = -(-(din + 1) // bm) * -(-dout // bn)
                s = Fk.eff_splits(B, min(max(1, -(-1000 // tiles)), 64, max(1, B // 256)))
            K.dense_wgrad(x, dy, slab, din, dout, B, din, dout, True, s, code)
        return f

    cases = {"fwd_auto": fwd(-1), "dgrad_auto": dgrad(-1), "wgrad_auto": wgrad(-1, 0, 0)}
    for t in ("64x128", "32x192", "64x192", "128x192"):
        cases[f"fwd_{t}"] = fwd(CODES[t])
    for t in ("64x128", "128x128", "256x128"):
        cases[f"dgrad_{t}"] = dgrad(CODES[t])
    for t in ("64x64", "128x128", "128x192"):
        bm, bn = (int(v) for v in t.split("x"))
        cases[f"wgrad_{t}"] = wgrad(CODES[t], bm, bn)
    res = {k: [] for k in cases}
    for f in cases.values():
        f()
    for _ in range(7):
        for name, f in cases.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(json.dumps({"B": B, **{k: round(statistics.median(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
