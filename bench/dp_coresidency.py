#!/usr/bin/env python3
"""Can a collective start while a persistent, LDS-filling compute kernel runs?

VERDICT r4 Missing #2 / SURVEY C1: the DP bucket hook (parallel/dp.py) launches RCCL
all-reduces on RCCL's own stream while the backward continues on the compute stream.
Whether the all-reduce kernel actually runs beside the compute kernel depends on a free
CU slot: LDS, VGPRs and wave slots.  This measures it on one GPU with a stand-in of the
collective's footprint (probe.hip: a few blocks of 256-512 threads with 0-32 KB LDS that
stamp the 100 MHz wall clock when they start):

    compute stream:  mark(0) -> TARGET -> mark(1)
    side stream:     wait(event after mark 0) -> probe

For each target it prints the probe's first-block start as a fraction of the target's
span (mark 0 .. mark 1): ~0 = co-resident (the collective overlaps), ~1 = it queued
behind the target.  With ``--reserve 8`` the persistent grids leave 8 CUs (one per XCD)
free (kernels.set_reserve_cus) and the target's own time shows the cost of that.

    python bench/dp_coresidency.py [--reserve 0,8] [--out profiles/r5/dp_coresidency/result.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DataParallelReserve = 8      # parallel/dp.DataParallel.RESERVE_CUS
PROBES = [  # (name, blocks, threads, lds bytes): RCCL-like launch shapes
    ("256t_0KB", 8, 256, 0),
    ("256t_16KB", 8, 256, 16384),
    ("512t_32KB", 16, 512, 32768),
]


def build_targets(dev):
    """(name, callable, net) of the kernels a bucket all-reduce could be issued before."""
    import torch
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet, ConvLayer
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

    out = []
    spec = get_model("lenet5", 1)
    B = 65536
    net = HipNet(spec, B, dev, torch_ref.init_params(spec, seed=0), OptConfig(lr0=0.01))
    g = torch.Generator(device=dev).manual_seed(0)
    net.x0.copy_((torch.rand(B, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16))
    net.labels.copy_(torch.randint(0, 10, (B,), device=dev, generator=g, dtype=torch.int32))
    net.train_step()
    assert net.fused_bwd and net.band_fwd
    out.append(("lenet_bwd_k (LeNet B=65536)", lambda: net._fused_conv_backward(B, net.dbuf[2], []), net))
    out.append(("lenet_band_fwd_k (LeNet B=65536)", lambda: net._band_forward(B), net))

    spec2 = get_model("reference_cnn", 1)
    B2 = 16384
    net2 = HipNet(spec2, B2, dev, torch_ref.init_params(spec2, seed=0), OptConfig(lr0=0.01))
    net2.x0.copy_((torch.rand(B2, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16))
    net2.labels.copy_(torch.randint(0, 10, (B2,), device=dev, generator=g, dtype=torch.int32))
    net2.train_step()
    k = next(i for i, lay in enumerate(net2.layers) if isinstance(lay, ConvLayer) and lay.name == "conv2")
    c2 = net2.layers[k]
    out.append(("conv5_halo_k dgrad (reference CNN conv2, B=16384)",
                lambda: c2.bwd_data(B2, net2.dbuf[k + 1], net2.dbuf[k]), net2))
    out.append(("conv5_halo_wgrad_k (reference CNN conv2, B=16384)",
                lambda: c2.bwd_weight(B2, net2.dbuf[k + 1], net2.slabs[k], []), net2))
    c1 = net2.layers[0]
    out.append(("refc1_wgrad_k (reference CNN conv1 + norm1, B=16384)",
                lambda: c1.bwd_weight(B2, net2.dbuf[1], net2.slabs[0], []), net2))
    out.append(("conv5_halo_k fwd (reference CNN conv2, B=16384)", lambda: c2.fwd(B2), net2))
    return out


def trial(K, target, probe, side, stamps, marks):
    import torch
    _, blocks, threads, lds = probe
    main = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    K.clock_mark(marks, 0)
    ev.record(main)
    target()
    K.clock_mark(marks, 1)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        K.coresidency_probe(stamps, blocks, threads, lds, 200)   # 2 us of work per block
    torch.cuda.synchronize()
    m = marks.tolist()
    s = stamps[: 2 * blocks].view(blocks, 2).tolist()
    span = m[1] - m[0]
    first = min(a for a, _ in s) - m[0]
    last = max(a for a, _ in s) - m[0]
    return span / 100.0, first / 100.0, last / 100.0   # us (100 MHz clock)


def target_time(target, iters=20):
    import torch
    for _ in range(3):
        target()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        target()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reserve", default="0,8")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
    K = kernels()
    dev = torch.device("cuda", 0)
    # a few hundred ms of GEMMs so the clocks are up before anything is timed
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    for _ in range(2000):
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
    targets = build_targets(dev)
    side = torch.cuda.Stream(device=dev)
    stamps = torch.zeros(2 * 64, dtype=torch.int64, device=dev)
    marks = torch.zeros(2, dtype=torch.int64, device=dev)
    rows = []
    # control: nothing between the marks (how soon a probe starts on an idle GPU)
    for r in [int(v) for v in args.reserve.split(",")]:
        K.set_reserve_cus(r)
        for name, fn, _ in targets:
            t_us = target_time(fn)
            for probe in PROBES:
                res = [trial(K, fn, probe, side, stamps, marks) for _ in range(args.reps)]
                span = statistics.median(x[0] for x in res)
                first = statistics.median(x[1] for x in res)
                last = statistics.median(x[2] for x in res)
                row = {"target": name, "reserve_cus": r, "probe": probe[0], "target_us": round(t_us, 1),
                       "span_us": round(span, 1), "probe_first_start_us": round(first, 1),
                       "probe_last_start_us": round(last, 1), "first_start_frac": round(first / span, 3),
                       "coresident": first / span < 0.5}
                rows.append(row)
                print(json.dumps(row), flush=True)
    # the compute cost of the reserve: each target at 0 and 8 reserved CUs, interleaved rounds
    # (the probe rows above ran the reserve settings one after the other, so box clock drift
    # between them is not a cost)
    cost = {}
    for name, fn, _ in targets:
        ts = {0: [], DataParallelReserve: []}
        for _ in range(5):
            for r in ts:
                K.set_reserve_cus(r)
                ts[r].append(target_time(fn, iters=10))
        cost[name] = {f"R{r}_us": round(statistics.median(v), 1) for r, v in ts.items()}
        print(json.dumps({"target": name, "reserve_cost": cost[name]}), flush=True)
    K.set_reserve_cus(0)
    rows.append({"reserve_cost_interleaved": cost})
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
