#!/usr/bin/env python3
"""Second BASELINE metric: steps to 99% train accuracy (MNIST LeNet-5).

Trains from random init on synthetic 28x28x1 data and, every ``--eval_every``
steps, measures top-1 accuracy on a fixed probe of ``--probe`` TRAINING images
(forward only, same kernels).  Reports the first global step at which the probe
accuracy reaches ``--target`` (default 0.99), plus wall time and images seen.

    python bench/steps_to_acc.py [--batch 128] [--lr 0.01] [--optimizer momentum]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        bench/steps_to_acc.py ...          (data parallel: global batch = N x batch)
    python bench/steps_to_acc.py --cpu --impl torch --model mlp     (CPU plumbing)

Defaults follow the reference's training hyperparameters where it has them
(batch 128) and BASELINE's model (LeNet-5).  Rank 0 prints one
JSON line; ``value`` is the step count (lower is better), null if the target
was not reached within ``--max_steps``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LABEL = {"lenet5": "LeNet-5", "reference_cnn": "reference CNN (mnist_input.inference)", "mlp": "MLP 784-128-10"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet5", choices=sorted(LABEL))
    ap.add_argument("--in_channels", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128, help="per-rank batch")
    ap.add_argument("--optimizer", default="momentum", choices=["sgd", "momentum", "nesterov"])
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--target", type=float, default=0.99)
    ap.add_argument("--eval_every", type=int, default=50)
    ap.add_argument("--probe", type=int, default=10000, help="training images in the accuracy probe")
    ap.add_argument("--max_steps", type=int, default=20000)
    ap.add_argument("--dataset_size", type=int, default=60000)
    ap.add_argument("--noise", type=float, default=0.25, help="synthetic-data noise amplitude")
    ap.add_argument("--style", default="hand", choices=["hand", "glyph"],
                    help="synthetic generator: hand = per-sample re-drawn strokes (default), glyph = shifted templates")
    ap.add_argument("--impl", default="hip", choices=["hip", "torch"])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fused_input", type=int, default=0, help="first conv reads the uint8 dataset directly")
    return ap.parse_args(argv)


def run(args) -> dict:
    import torch
    import torch.distributed as dist

    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader, eval_batches
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
    spec = get_model(args.model, args.in_channels)
    opt = OptConfig(lr0=args.lr, decay_rate=0.1, decay_steps=0, momentum=0.9 if args.optimizer != "sgd" else 0.0,
                    nesterov=args.optimizer == "nesterov", use_momentum=args.optimizer != "sgd", ema_max=0.9999)
    init = init_params(spec, seed=args.seed)
    if args.impl == "hip":
        from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
        net = HipNet(spec, args.batch, dev, init, opt)
    else:
        from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
        net = TorchNet(spec, args.batch, dev, init, opt)
    dp = DataParallel(net)
    dp.broadcast_state()

    imgs, labs = make_synthetic(args.dataset_size, seed=args.seed, channels=args.in_channels, noise=args.noise,
                                device=dev, style=args.style)
    ds = DeviceDataset(imgs, labs, dev, hw=784, channels=args.in_channels)
    n_probe = min(args.probe, args.dataset_size)
    probe = DeviceDataset(imgs[:n_probe], labs[:n_probe], dev, hw=784, channels=args.in_channels)
    # --fused_input: the first fused conv reads the uint8 dataset through the batch index
    # (K10 fused).  Off by default: measured ~25 us/step slower on LeNet-5 at 65536 than
    # prep_images + bf16 (profiles/r1_u8_input/).
    fused_in = args.impl == "hip" and args.fused_input and net.bind_u8_input(ds.images)
    loader = DeviceLoader(ds, net.x0, net.labels, rank=rank, world=world, seed=args.seed,
                          idx_out=net.idx_buf if fused_in else None)

    graph = None
    if args.graph and args.impl == "hip" and world == 1 and dev.type == "cuda":
        from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph
        loader.next()                               # StepGraph's warmup replays train on a real batch
        graph = StepGraph(dp.train_step)

    def probe_accuracy() -> float:
        st = net.eval_stats
        st.zero_()
        n = 0
        for nb in eval_batches(probe, net.x0, net.labels):
            net.eval_batch(nb, st)
            n += nb
        return float(st[1].item()) / max(n, 1)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    sync()
    t0 = time.perf_counter()
    start_step = int(net.fp.step.item())
    reached, acc, step = None, 0.0, start_step
    history = []
    while step - start_step < args.max_steps:
        loader.next()
        if graph is not None:
            graph.replay()
        else:
            dp.train_step()
        step += 1
        if (step - start_step) % args.eval_every == 0:
            acc = probe_accuracy()
            history.append((step, round(acc, 5)))
            if acc >= args.target:
                reached = step
                break
    sync()
    el = time.perf_counter() - t0
    global_batch = args.batch * world
    out = {
        "metric": f"steps-to-{args.target * 100:g}%-train-acc MNIST {LABEL[args.model]}",
        "value": reached,
        "unit": "steps",
        "higher_is_better": False,
        "n_gpus": world if dev.type == "cuda" else 0,
        "seconds": round(el, 3),
        "images_seen": (reached or step) * global_batch,
        "final_probe_accuracy": round(acc, 5),
        "dtype": "bf16" if dev.type == "cuda" else "fp32",
        "data": f"synthetic 28x28x{args.in_channels} (style {args.style}, noise {args.noise}), random-init weights; "
                f"probe = first {n_probe} training images",
        "config": {"model": LABEL[args.model], "global_batch": global_batch, "optimizer": args.optimizer,
                   "lr": args.lr, "eval_every": args.eval_every, "impl": args.impl, "hip_graph": graph is not None,
                   "parallelism": f"dp{world}"},
        "history": history[-20:],
    }
    if world > 1:
        dist.destroy_process_group()
    return out if rank == 0 else {}


def main() -> int:
    out = run(parse())
    if out:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
