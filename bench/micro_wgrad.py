#!/usr/bin/env python3
"""Dense weight-gradient sweep: GEMM tile x split-K count for the LeNet-5 fc shapes
at B = 65536 (wgrad GEMM + multi-tensor split-K reduce, CUDA-event timed).
Usage: python bench/micro_wgrad.py [B] [ref] [TILE,TILE..]   (ref: the reference CNN's local3/local4
shapes; the tile list restricts the sweep)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402

TILES = {"64x64": 7, "128x128": 4, "128x64": 2, "64x128": 3, "64x32": 6, "64x16": 5, "256x128": 8}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    shapes = [("fc3", 400, 120, 120), ("fc4", 120, 84, 88), ("fc5", 84, 10, 16)]
    splits = (16, 32, 64, 128, 256)
    if len(sys.argv) > 2 and sys.argv[2] == "ref":
        shapes = [("local3", 3136, 1024, 1024), ("local4", 1024, 192, 192)]
        splits = (1, 2, 3, 4, 6, 8, 12, 16)
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else None
    if len(sys.argv) > 2 and sys.argv[2] == "ref":
        shapes = shapes[:1]
    for name, din, dout, Np in shapes:
        Dp = din if name != "fc5" else 88
        x = (torch.randn(B, Dp, device=dev) * 0.5).to(torch.bfloat16)
        dy = (torch.randn(B, Np, device=dev) * 0.1).to(torch.bfloat16)
        ref = (x.float().t() @ dy.float())[:din, :dout]
        M = Dp + 1
        slab = torch.empty(max(splits) * M * Np + 64, device=dev)
        dw = torch.empty(din * dout, device=dev)
        db = torch.empty(dout, device=dev)
        geo_row = lambda S: [S, M, Np, 1, Dp, din, dout, Dp]
        print(f"{name}: M={M} N={Np} K={B}", flush=True)
        for tname, code in TILES.items():
            if only and tname not in only:
                continue
            if Np <= 16 and tname not in ("64x16",):
                continue
            if 16 < Np <= 32 and tname not in ("64x32",):
                continue
            if Np > 32 and tname in ("64x16", "64x32"):
                continue
            row = []
            for S in splits:
                def run():
                    s = K.dense_wgrad(x, dy, slab, Dp, Np, B, Dp, Np, True, S, code)
                    K.splitk_reduce_multi([slab], [dw], [db], torch.tensor([geo_row(s)]), [1.0])
                run()
                torch.cuda.synchronize()
                err = (dw.view(din, dout) - ref).abs().max().item() / ref.abs().max().item()
                # hipGraph of 20 iterations: device time only (no per-launch host overhead)
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    run()
                torch.cuda.current_stream().wait_stream(st)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(20):
                        run()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                row.append(f"S={S}:{e0.elapsed_time(e1) / 20 * 1e3:6.1f}us" + ("" if err < 2e-2 else f"(ERR {err:.2e})"))
            print(f"  {tname:8s} " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
