#!/usr/bin/env python3
"""Per-step GPU time of the first N training steps on the bench.py configuration (HIP
events around each step), after an optional prewarm of a chosen KIND: shows how long the
step takes to reach steady state on a fresh box and what kind of load gets it there.

    python bench/step_trace.py [--steps 300] [--pre none|gemm|copy|steps] [--pre_ms 300]

--pre gemm  : bench.py's clock prewarm (bf16 4096^3 GEMMs: compute-bound, L2-resident)
--pre copy  : HBM streaming (1 GiB device-to-device copies: memory / fabric bound)
--pre steps : --pre_steps real training steps (what bench.py --prewarm_steps does)

Prints the per-step times in rows of 10, the means over the driver's window (steps 5..24:
5 warmup + 20 timed) and over the last 50 steps, and the DPM clock levels the box exposes
(sysfs pp_dpm_*; "n/a" where it does not) before and after.
"""
import argparse
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dpm_levels():
    """Current DPM level of every clock domain sysfs exposes for the first GPU card
    (the line marked '*' of pp_dpm_sclk / mclk / fclk / socclk)."""
    out = {}
    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        for dom in ("sclk", "mclk", "fclk", "socclk"):
            p = os.path.join(card, f"pp_dpm_{dom}")
            try:
                lines = open(p).read().splitlines()
            except OSError:
                continue
            cur = [ln.strip() for ln in lines if ln.strip().endswith("*")]
            out[dom] = cur[0] if cur else "?"
        if out:
            out["card"] = card
            break
    return out or {"dpm": "n/a"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--pre", default="none", choices=["none", "gemm", "copy", "steps"])
    ap.add_argument("--pre_ms", type=float, default=300.0)
    ap.add_argument("--pre_steps", type=int, default=200)
    ap.add_argument("--idle_ms", type=float, default=0.0, help="host sleep between the prewarm and the traced steps")
    ap.add_argument("--json", default="", help="also write the per-step times here")
    a = ap.parse_args()
    import torch
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = get_model(a.model, 1)
    net = HipNet(spec, a.batch, dev, init_params(spec, seed=0),
                 OptConfig(lr0=0.01, decay_rate=0.1, decay_steps=0, momentum=0.9, use_momentum=True, ema_max=0.9999))
    imgs, labs = make_synthetic(60000, seed=0, channels=1, device=dev)
    ds = DeviceDataset(imgs, labs, dev, hw=784, channels=1)
    fused = net.can_gather_input() and net.bind_u8_input(ds.bf16_images(), bwd_images=ds.images)
    loader = DeviceLoader(ds, net.x0, net.labels, idx_out=net.idx_buf if fused else None)
    if fused:
        net.next_input_job = loader.lookahead_job

    def step():
        loader.next()
        net.train_step()

    torch.cuda.synchronize()
    before = dpm_levels()
    t_pre = time.perf_counter()
    if a.pre == "gemm":
        x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        y = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        while (time.perf_counter() - t_pre) * 1e3 < a.pre_ms:
            for _ in range(8):
                z = x @ y
            torch.cuda.synchronize()
        del x, y, z
    elif a.pre == "copy":
        src = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)
        while (time.perf_counter() - t_pre) * 1e3 < a.pre_ms:
            for _ in range(4):
                dst.copy_(src)
            torch.cuda.synchronize()
        del src, dst
    elif a.pre == "steps":
        for _ in range(a.pre_steps):
            step()
        torch.cuda.synchronize()
    pre_s = time.perf_counter() - t_pre
    mid = dpm_levels()
    if a.idle_ms > 0:
        time.sleep(a.idle_ms / 1e3)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record()
    for i in range(a.steps):
        step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    after = dpm_levels()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
    print(f"pre={a.pre} ({pre_s * 1e3:.0f} ms)  dpm before {before}  after pre {mid}  after {after}")
    for i in range(0, a.steps, 10):
        print(f"steps {i:3d}-{i + 9:3d}: " + " ".join(f"{m:.3f}" for m in ms[i:i + 10]))
    drv = sum(ms[5:25]) / 20
    last = sum(ms[-50:]) / 50
    print(f"mean 5..24 (driver window) {drv:.4f}  mean last 50 {last:.4f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"pre": a.pre, "pre_ms": pre_s * 1e3, "ms": ms, "driver_window": drv, "last50": last,
                       "dpm": [before, mid, after]}, f)


if __name__ == "__main__":
    main()
