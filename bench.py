#!/usr/bin/env python3
"""Headline benchmark: training images/sec (whole node), MNIST LeNet-5, bf16.

BASELINE.json metric: "images/sec (whole node) MNIST LeNet-5 at 1/2/4/8 MI355X"
on synthetic 28x28x1 data with random-init weights; the per-GPU batch defaults
to the BASELINE stress config (65536 / GPU, weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model lenet5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Each timed step is the complete training step: on-device batch gather +
normalise (K10), forward, softmax-CE, backward, RCCL all-reduce of the gradient
buckets (N > 1), fused SGD + weight-EMA update, loss-EMA/step finalisation.
K steps are bracketed by barrier + device synchronize on both sides; the
reported time is the MAX over ranks; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODEL_LABEL = {"lenet5": "LeNet-5", "reference_cnn": "reference CNN (mnist_input.inference)", "mlp": "MLP 784-128-10"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm_steps", type=int, default=200,
                    help="steady-state ramp before the W warmup steps: this many steps of the real step on the "
                         "real buffers, then the model, optimizer, loss and loader state is restored bitwise, so "
                         "the W + K steps start from the state they would have had without it (0 = off)")
    ap.add_argument("--prewarm_ms", type=float, default=300.0,
                    help="before the warmup steps: this long of plain bf16 GEMMs on the device (no model "
                         "state touched) so the GPU leaves its idle clock state; 0 = off")
    ap.add_argument("--model", default="lenet5", choices=sorted(MODEL_LABEL))
    ap.add_argument("--batch", type=int, default=65536, help="per-GPU batch (BASELINE stress config: 65536)")
    ap.add_argument("--in_channels", type=int, default=1)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="HIP compute precision: bf16 (headline) | fp32 (the reference's tf.float32, fp32 MFMA)")
    ap.add_argument("--impl", default="hip", choices=["hip", "torch"],
                    help="hip = our CDNA4 kernels; torch = PyTorch-ROCm baseline (MIOpen/hipBLASLt, bf16 autocast)")
    ap.add_argument("--bucket_mb", type=float, default=0.125,
                    help="gradient bucket cap (MB); every bucket but the last overlaps backward")
    ap.add_argument("--graph", type=int, default=-1,
                    help="hipGraph capture of the step: 1 on (N > 1: with its RCCL all-reduces -- UNVERIFIED on a real "
                         "multi-GPU node, rehearsed only with one-rank RCCL / gloo ranks), 0 off, -1 auto = "
                         "on for one GPU at per-GPU batch <= 8192 (launch-bound); at the BASELINE batch eager "
                         "launches measure as fast (profiles/r2/graph_vs_eager.md), so 1..8 GPUs run one mode")
    ap.add_argument("--force_collectives", type=int, default=0,
                    help="issue the bucket all-reduces even at N=1 (one-rank RCCL rehearsal of the DP path)")
    ap.add_argument("--optimizer", default="momentum", choices=["sgd", "momentum", "nesterov"])
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fused_input", type=int, default=0, help="alias of --input u8")
    ap.add_argument("--input", default="bf16", choices=["prep", "u8", "bf16"],
                    help="HIP input path: bf16 (default: the first conv gathers the resident dataset, normalised "
                         "once to bf16) | u8 (same, uint8 normalised in the kernels) | prep (a per-step "
                         "gather+normalise kernel writes the batch buffer)")
    ap.add_argument("--overlap", default="none", choices=["none", "dense", "all"],
                    help="weight gradients on a side stream: none / dense layers only / every layer")
    ap.add_argument("--dataset_size", type=int, default=60000)
    ap.add_argument("--dist_backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo = host-staged rehearsal of the DP "
                         "path with several ranks sharing one GPU (ranks map to device LOCAL_RANK %% count)")
    ap.add_argument("--mode", default="dp", choices=["dp", "ps"],
                    help="dp = synchronous data parallel (headline); ps = asynchronous parameter server: "
                         "rank 0 is the PS, ranks 1..N-1 are workers (BASELINE config '1 PS + 7 workers')")
    ap.add_argument("--bwd_u8", type=int, default=1,
                    help="--input bf16: the fused LeNet conv backward reads the uint8 twin of the dataset (half "
                         "the bytes, normalised in the kernel) instead of the bf16 copy")
    ap.add_argument("--input_lookahead", type=int, default=1,
                    help="--input u8/bf16, eager: the next batch's shuffle rows + labels are computed by extra "
                         "blocks of the optimizer launch (DeviceLoader.lookahead_job) instead of a launch of their own")
    ap.add_argument("--ps_no_compute", type=int, default=0,
                    help="PS mode: workers push the same gradient back to back without computing a step -- "
                         "the PS data plane's own capacity (ms per applied update), e.g. 7 workers on one GPU")
    ap.add_argument("--ps_transport", default="", choices=["", "shm", "ipc", "host"],
                    help="PS data plane: '' = the CLI's default (parallel/ps.default_transport: shm up to 1 M "
                         "parameters per shard, ipc above); shm = CPU PS on pinned shared memory; ipc = xGMI peer "
                         "copies into a GPU PS; host = gloo, host-staged")
    ap.add_argument("--eager_steps", type=int, default=-1,
                    help="N=1 with a hipGraph: also time this many EAGER steps after the timed region "
                         "(ms_per_step_eager, comparable with N>1 runs); -1 = --steps")
    ap.add_argument("--comm_probe", type=int, default=1,
                    help="N>1 (or --force_collectives 1): after the timed steps, time each gradient bucket's "
                         "all-reduce alone (us, bus GB/s) and the exposed communication of an eager step")
    ap.add_argument("--lenet_bwd", default="fused", choices=["fused", "split"],
                    help="LeNet-5 conv-stack backward: fused = one kernel (lenet_bwd.hip); split = the three "
                         "per-layer convpool kernels (conv2 dgrad, conv2 / conv1 weight gradients)")
    ap.add_argument("--phases", type=int, default=3,
                    help="extra eager steps AFTER the timed region, timed per phase with HIP events (0 = off)")
    return ap.parse_args()


def prewarm(dev, ms: float) -> None:
    """Clock ramp, outside every timed region: an idle MI355X starts the first
    steps at a lower clock (same box, LeNet-5 B=65536, 20 timed steps: 0.625 /
    0.632 ms after 5 warmup steps, 0.594 / 0.609 ms after 300;
    profiles/r2/lenet/head_s5/).  The GEMMs touch no model, optimizer or loader
    state, so the timed steps are exactly the steps the driver asked for."""
    import torch
    if ms <= 0:
        return
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            c = a @ b
        torch.cuda.synchronize(dev)
    del a, b, c


def prewarm_steps(net, loader, step, n: int) -> int:
    """Run ``n`` real steps, then restore every piece of state a step changes (flat params,
    gradients, momentum, EMA, bf16 weight copies, step counter, weight-decay partials, loss
    stats and EMAs, loader position), so the driver's W warmup + K timed steps are exactly the
    steps it asked for.  A fixed count (not a time), so every rank runs the same collectives.
    Short runs after setup measured 5-8 % slower than the steady state the real step reaches
    (profiles/r5/prewarm/)."""
    import torch
    fp = getattr(net, "fp", None)
    if n <= 0 or fp is None or not hasattr(loader, "pos"):
        return 0
    keep = [getattr(fp, k, None) for k in ("params", "grads", "mom", "ema", "bf16", "step", "l2")]
    keep += [getattr(net, "stats", None), getattr(net, "loss_ema", None)]
    keep = [t for t in keep if isinstance(t, torch.Tensor)]
    saved = [t.clone() for t in keep]
    pos = loader.pos
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    for t, v in zip(keep, saved):
        t.copy_(v)
    loader.pos = pos
    loader._ahead = None       # the next next() gathers its batch itself
    torch.cuda.synchronize()
    return n


def pg_block(dev, t_local: float):
    """The process group as the ranks see it (not the environment): backend, size, each
    rank's device identity (index, PCI bus / UUID where torch exposes them, host), the
    RCCL version and the min / max per-rank timed seconds.  ``shared`` lists ranks that
    sit on the same physical device (the caller exits non-zero for that under nccl)."""
    import socket

    import torch
    import torch.distributed as dist
    props = torch.cuda.get_device_properties(dev)
    pci = tuple(getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    uuid = str(getattr(props, "uuid", "") or "")
    me = {"rank": dist.get_rank(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": dev.index,
          "pci": "%04x:%02x:%02x" % tuple(v or 0 for v in pci) if any(v is not None for v in pci) else None,
          "uuid": uuid or None, "host": socket.gethostname(), "name": props.name, "timed_s": t_local}
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    seen, shared = {}, []
    for r in ranks:
        key = (r["host"], r["uuid"] or r["pci"] or f"dev{r['device']}")
        if key in seen:
            shared.append([seen[key], r["rank"]])
        else:
            seen[key] = r["rank"]
    try:
        ver = torch.cuda.nccl.version()
        rccl = ".".join(str(v) for v in ver) if isinstance(ver, tuple) else str(ver)
    except Exception:              # noqa: BLE001 -- no RCCL in this build
        rccl = None
    ts = [r["timed_s"] for r in ranks]
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "rccl_version": rccl,
            "ranks": [{k: v for k, v in r.items() if k != "timed_s"} for r in ranks],
            "distinct_devices": len(seen), "shared": shared,
            "timed_s_min": round(min(ts), 6), "timed_s_max": round(max(ts), 6)}


def run_ps(args) -> int:
    """1 PS + (N-1) asynchronous workers.  The PS clock is the
    authoritative one: it marks the wall time when the shared global step passes
    warmup*(N-1) and (warmup+steps)*(N-1) applied updates (device synchronised at
    both marks), so value = steps*(N-1)*batch / that interval -- the aggregate
    images/sec of updates applied to the model."""
    import torch
    import torch.distributed as dist

    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import ParameterServer, PSClient, weight_l2_into
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader

    # one hardware queue per PS/worker process (before HIP starts): co-located tasks
    # otherwise oversubscribe the GPU's queue scheduler (profiles/r3/ps/ps_hwq_ab.txt);
    # a value set in the environment is kept
    if "GPU_MAX_HW_QUEUES" not in os.environ:
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MNISTX_PS_HW_QUEUES", "1")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world < 2:
        print("[bench] --mode ps needs >= 2 ranks (torchrun --nproc-per-node N)", file=sys.stderr)
        return 2
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import default_transport, max_shard_params
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs as _pspecs
    # the same resolution as the CLI (main.py --ps_backend ''), on every rank
    args.ps_transport = args.ps_transport or default_transport(
        torch.device("cuda"), max_shard_params(_pspecs(get_model(args.model, args.in_channels)), 1))
    if rank == 0 and args.ps_transport == "shm":
        dev = torch.device("cpu")             # the shm PS is a CPU task: it never opens the GPU
    else:
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
    dist.init_process_group("gloo")          # control plane; data moves on the PS transport
    spec = get_model(args.model, args.in_channels)
    init = init_params(spec, seed=args.seed)
    opt = OptConfig(lr0=args.lr, decay_rate=0.1, decay_steps=0, momentum=0.9 if args.optimizer != "sgd" else 0.0,
                    nesterov=args.optimizer == "nesterov", use_momentum=args.optimizer != "sgd", ema_max=0.9999)
    nw = world - 1
    m0, m1 = args.warmup * nw, (args.warmup + args.steps) * nw
    if rank == 0:
        ps = ParameterServer(0, 1, nw, param_specs(spec), init, opt, dev, m1, log=lambda *a: None,
                             transport=args.ps_transport)
        ps.marks = {m0: 0.0, m1: 0.0} if m0 > 0 else {m1: 0.0}
        t_start = time.perf_counter()
        res = ps.serve()
        t0 = ps.marks.get(m0, t_start) if m0 > 0 else t_start
        el = ps.marks[m1] - t0
        value = args.steps * nw * args.batch / el
        out = {
            "metric": f"images/sec (whole node) MNIST {MODEL_LABEL[args.model]} parameter-server mode",
            "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_update": round(el / (args.steps * nw) * 1e3, 4),
            "ms_per_worker_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic 28x28x1 (on-device generated MNIST-like glyphs), random-init weights",
            "config": {"model": MODEL_LABEL[args.model], "per_worker_batch": args.batch,
                       "parallelism": f"ps1+w{nw}", "ps_transport": args.ps_transport,
                       "gpus_visible": torch.cuda.device_count(), "optimizer": args.optimizer,
                       "ps_device": ps.device.type},
            "applied_per_worker": res["per_worker"], "global_step": res["global_step"],
            # PS host time per served message, by phase (whole run incl. warmup): idle = waiting
            # for a worker, apply = optimizer launch, reply = stage + sync + control answer
            "ps_us_per_msg": {k: round(v / max(1, res["applied"]) * 1e6, 1) for k, v in res["phase_s"].items()},
            "param_checksum": float(ps.fp.params.double().sum().item()),
            "transport_used": ps.tx.name,
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        }
        comms = [None] * world
        dist.gather_object(None, comms, dst=0)
        # per GRAD message, per worker: push (stage + copy + announce) host us and GB/s, the
        # wait for the PS reply, the pull copy's device us and GB/s
        out["ps_comm"] = comms[1:]
        print(json.dumps(out), flush=True)
    else:
        from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
        net = HipNet(spec, args.batch, dev, init, opt)
        imgs, labs = make_synthetic(args.dataset_size, seed=args.seed, channels=args.in_channels, device=dev)
        loader = DeviceLoader(DeviceDataset(imgs, labs, dev, hw=784, channels=args.in_channels), net.x0, net.labels,
                              rank=0, world=1, seed=args.seed + 7919 * rank, shard=False)
        client = PSClient(net, 1, nw, rank - 1, transport=args.ps_transport)
        client.hello()

        def compute():   # no communication inside: one hipGraph per worker step (--graph != 0)
            net.forward(defer_head=True)
            net.loss_and_grad()
            net.backward()
            weight_l2_into(net.fp)
            net.finalize(net.B, increment=False)

        graph = None
        evs = []       # device time of the worker's own step (input + fwd/bwd), shared GPU included
        if args.ps_no_compute:            # one real step: the gradient every push then re-sends
            compute()
        while not client.stop:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            if not args.ps_no_compute:
                loader.next()
                if args.graph == 0:
                    compute()
                elif graph is None:
                    from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph
                    graph = StepGraph(compute, warmup=1)     # the warm-up computes this step
                else:
                    graph.replay()
            ev[1].record()
            if (graph is not None or args.graph == 0) and len(evs) < 4096:
                evs.append(ev)
            client.push_pull()
        client.done()
        summary = client.comm_summary()
        torch.cuda.synchronize()
        summary["compute_us"] = round(sum(a.elapsed_time(b) for a, b in evs) / max(1, len(evs)) * 1e3, 1)
        dist.gather_object(summary, None, dst=0)
    dist.destroy_process_group()
    return 0


def main() -> int:
    args = parse()
    if args.mode == "ps":
        return run_ps(args)
    import torch
    import torch.distributed as dist

    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.force_collectives and world == 1:      # one-rank process group: the RCCL path on one GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1 or args.force_collectives:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    spec = get_model(args.model, args.in_channels)
    init = init_params(spec, seed=args.seed)
    opt = OptConfig(lr0=args.lr, decay_rate=0.1, decay_steps=0, momentum=0.9 if args.optimizer != "sgd" else 0.0,
                    nesterov=args.optimizer == "nesterov", use_momentum=args.optimizer != "sgd", ema_max=0.9999)
    if args.impl == "hip" and args.precision == "fp32":
        from distributed_tensorflow_ibm_mnist_amd.runtime.executor_f32 import HipNetF32
        net = HipNetF32(spec, args.batch, dev, init, opt)
    elif args.impl == "hip":
        from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
        net = HipNet(spec, args.batch, dev, init, opt,
                     overlap_backward={"none": False, "dense": "dense", "all": True}[args.overlap],
                     fused_lenet_bwd=args.lenet_bwd == "fused")
    else:
        from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
        net = TorchNet(spec, args.batch, dev, init, opt)
    dp = DataParallel(net, bucket_cap_mb=args.bucket_mb, force_collectives=bool(args.force_collectives))
    dp.broadcast_state()

    # --in_channels 3: 3-channel records (the glyphs replicated to RGB, as the reference's DLI
    # import stored MNIST: /root/reference/mnist_input.py:13-15), gathered by the first conv
    imgs, labs = make_synthetic(args.dataset_size, seed=args.seed, channels=args.in_channels, device=dev)
    ds = DeviceDataset(imgs, labs, dev, hw=784, channels=args.in_channels)
    # --input u8 / bf16: the first fused conv gathers the resident dataset through the
    # batch index (K10 fused into its staging); prep: one gather+normalise kernel per step
    mode = "u8" if args.fused_input else args.input
    fused_in = (args.impl == "hip" and mode != "prep" and getattr(net, "can_gather_input", lambda: True)()
                and net.bind_u8_input(ds.images if mode == "u8" else ds.bf16_images(),
                                       bwd_images=None if (mode == "u8" or not args.bwd_u8) else ds.images))
    loader = DeviceLoader(ds, net.x0, net.labels, rank=rank, world=world, seed=args.seed,
                          idx_out=net.idx_buf if fused_in else None)

    collectives = world > 1 or bool(args.force_collectives)
    if args.graph < 0:
        use_graph = args.impl == "hip" and not collectives and args.batch <= 8192
    else:
        use_graph = bool(args.graph) and args.impl == "hip" and (not collectives or args.dist_backend == "nccl")
    graph = None

    def step_body():
        dp.train_step()

    if use_graph:
        from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph
        graph = StepGraph(step_body)
    elif fused_in and args.input_lookahead:
        net.next_input_job = loader.lookahead_job   # a captured launch would replay one fixed batch

    def step():
        loader.next()
        if graph is not None:
            graph.replay()
        else:
            step_body()

    prewarm(dev, args.prewarm_ms)
    n_pre = prewarm_steps(net, loader, step, args.prewarm_steps)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter()   # host time to issue the K steps (== t1 - t0 when host-bound)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    el = float(elapsed.item())
    # N > 1 (or the one-rank RCCL rehearsal): what the process group itself saw
    pg = pg_block(dev, t1 - t0) if dist.is_initialized() else None
    eager_ms = None
    n_eager = args.steps if args.eager_steps < 0 else args.eager_steps
    if graph is not None and n_eager > 0:   # outside the timed region: the same step, eager
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(n_eager):
            loader.next()
            step_body()
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - te) / n_eager * 1e3
    stats = net.read_stats()
    in_sync = None
    if world > 1:                           # outside the timed region: replicas must hold identical weights
        ck = net.fp.params.double().sum().reshape(1)
        lo, hi = ck.clone(), ck.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool((hi - lo).abs().item() == 0.0)
    comm = None
    if collectives and args.comm_probe:     # outside the timed region, after the replica check
        #  each bucket's all-reduce alone, then the exposed communication:
        # eager steps with the collectives on vs off (the off steps let replicas drift:
        # nothing after this reads the weights)
        comm = {"buckets": dp.measure_buckets()}
        ne = max(3, min(args.steps, 10))

        def timed_eager_ms(on: bool) -> float:
            dp.comm_enabled = on
            for _ in range(2):
                loader.next()
                step_body()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t = time.perf_counter()
            for _ in range(ne):
                loader.next()
                step_body()
            torch.cuda.synchronize()
            ms = torch.tensor([(time.perf_counter() - t) / ne * 1e3], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(ms, op=dist.ReduceOp.MAX)
            return float(ms.item())

        on, off = timed_eager_ms(True), timed_eager_ms(False)
        dp.comm_enabled = True
        comm.update({"eager_ms_comm_on": round(on, 4), "eager_ms_comm_off": round(off, 4),
                     "comm_exposed_ms": round(on - off, 4)})
    phases = None
    if args.phases > 0:                     # outside the timed region: per-phase breakdown of an eager step
        from distributed_tensorflow_ibm_mnist_amd.runtime.timers import PhaseTimer
        timer = PhaseTimer(dev)
        for _ in range(args.phases):
            loader.next()
            dp.train_step(timer)
        phases = timer.summary()
    global_batch = args.batch * world
    ms = el / max(args.steps, 1) * 1e3
    value = global_batch * args.steps / el
    if rank == 0:
        fwd, tot = spec.flops_per_image()
        out = {
            "metric": "images/sec (whole node) MNIST LeNet-5" if args.model == "lenet5"
            else f"images/sec (whole node) MNIST {MODEL_LABEL[args.model]}",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_ms": args.prewarm_ms,
            "prewarm_steps": n_pre,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision if args.impl == "hip" else "bf16",
            "data": f"synthetic 28x28x{args.in_channels} (on-device generated MNIST-like glyphs), random-init weights",
            "config": {
                "model": MODEL_LABEL[args.model],
                "global_batch": global_batch,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "dist_backend": args.dist_backend if world > 1 else None,
                "impl": args.impl,
                "hip_graph": use_graph,
                "optimizer": args.optimizer,
                "input": mode if fused_in else "prep",
                "lenet_bwd": ("fused" if getattr(net, "fused_bwd", False) else "split") if args.model == "lenet5" else None,
                "input_lookahead": getattr(net, "next_input_job", None) is not None,
            },
            "tflops_per_s": round(tot * value / 1e12, 2),
            "final_train_loss": round(stats["cross_entropy"], 5),
            "ms_per_step_eager": round(eager_ms, 4) if eager_ms is not None else (None if use_graph else round(ms, 4)),
            "host_issue_ms_per_step": round((t_enq - t0) / args.steps * 1e3, 4),
            "phase_ms_eager": phases,
            "replicas_in_sync": in_sync,
            "grad_bucket_mb": [round(b.nbytes / 2 ** 20, 3) for b in dp.buckets] if world > 1 else None,
            # per-bucket all-reduce time / bus bandwidth and the exposed communication
            # (eager step with minus without collectives), measured after the timed steps
            "comm": comm,
            "pg": pg,
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),   # None = HIP's default
        }
        print(json.dumps(out), flush=True)
    if pg is not None and pg["shared"] and pg["backend"] == "nccl":
        if rank == 0:
            print(f"[bench] ERROR: ranks {pg['shared']} share one device under nccl; the multi-GPU number "
                  f"is not a {world}-GPU measurement", file=sys.stderr)
        if dist.is_initialized():
            dist.destroy_process_group()
        return 3
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
