#!/usr/bin/env python3
"""Per-step GPU time of the first N training steps (HIP events around each
replay): shows how long the step takes to reach steady state on a fresh box
(clock ramp, first-touch) -- the driver times only 20 steps after 5 warmups.

    python bench/step_trace.py [--model lenet5] [--batch 65536] [--steps 120] [--graph 1]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--idle_ms", type=float, default=0.0, help="host sleep before the traced steps")
    a = ap.parse_args()
    import torch
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader
    from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph

    dev = torch.device("cuda", 0)
    spec = get_model(a.model, 1)
    net = HipNet(spec, a.batch, dev, init_params(spec, seed=0),
                 OptConfig(lr0=0.01, use_momentum=True, momentum=0.9))
    imgs, labs = make_synthetic(60000, seed=0, channels=1, device=dev)
    loader = DeviceLoader(DeviceDataset(imgs, labs, dev), net.x0, net.labels)
    g = StepGraph(net.train_step) if a.graph else None
    torch.cuda.synchronize()
    if a.idle_ms > 0:
        time.sleep(a.idle_ms / 1e3)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record()
    for i in range(a.steps):
        loader.next()
        g.replay() if g is not None else net.train_step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
    for i in range(0, a.steps, 10):
        print(f"steps {i:3d}-{i + 9:3d}: " + " ".join(f"{m:.3f}" for m in ms[i:i + 10]))
    print(f"mean 5..25 {sum(ms[5:25]) / 20:.4f}  mean last 50 {sum(ms[-50:]) / 50:.4f}")


if __name__ == "__main__":
    main()
