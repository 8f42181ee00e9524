#!/usr/bin/env python3
"""Parameter-server capacity on the host, without GPUs: 1 PS + W workers that push the same
gradient back to back (no compute), so the PS's service time per applied update is what is
measured -- the bound of the BASELINE "1 PS + 7 workers" config once every worker owns a
GPU (on a one-GPU box the workers' step graphs time-slice the GPU and hide it,
profiles/r5/ps/).  Transports: shm (CPU PS, native loop on a shared-memory segment),
host (gloo messages, the portable fallback) and ipc (GPU PS: every rank on cuda:0 of a
one-GPU box, peer copies degenerate to device copies -- the PS's own service time, not
xGMI bandwidth).  '' = the CLI default for the model (parallel/ps.default_transport).

    python bench/ps_capacity.py [--model lenet5] [--workers 3,7] [--updates 3000] [--transports shm,host]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, model, transport, updates, q):
    import torch
    import torch.distributed as dist
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import ParameterServer, PSClient
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import default_transport, max_shard_params
    spec = get_model(model, 1)
    init = torch_ref.init_params(spec, seed=0)
    opt = OptConfig(lr0=0.01, momentum=0.9, use_momentum=True, ema_max=0.9999)
    nw = world - 1
    if not transport:
        transport = default_transport(torch.device("cuda"), max_shard_params(param_specs(spec), 1))
    dev = "cuda:0" if transport == "ipc" else "cpu"
    if rank == 0:
        ps = ParameterServer(0, 1, nw, param_specs(spec), init, opt, dev, updates, log=lambda *a: None,
                             transport=transport)
        m0 = updates // 10
        ps.marks = {m0: 0.0, updates: 0.0}
        res = ps.serve()
        el = ps.marks[updates] - ps.marks[m0]
        q.put({"model": model, "transport": ps.tx.name, "workers": nw, "params": ps.fp.total,
               "us_per_update": round(el / (updates - m0) * 1e6, 2),
               "updates_per_s": round((updates - m0) / el, 1),
               "ps_us_per_msg": {k: round(v / max(1, res["applied"]) * 1e6, 2) for k, v in res["phase_s"].items()},
               "per_worker": res["per_worker"]})
    else:
        from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
        net = TorchNet(spec, 2, dev, init, opt)
        net.fp.grads.normal_(0, 1e-3)
        client = PSClient(net, 1, nw, rank - 1, transport=transport)
        client.hello()
        while not client.stop:
            client.push_pull()
        client.done()
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--workers", default="3,7")
    ap.add_argument("--transports", default="shm,host")
    ap.add_argument("--updates", type=int, default=3000)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    for t in args.transports.split(","):
        for w in [int(v) for v in args.workers.split(",")]:
            q = ctx.Queue()
            port = _port()
            procs = [ctx.Process(target=_rank, args=(r, w + 1, port, args.model, t, args.updates, q))
                     for r in range(w + 1)]
            for p in procs:
                p.start()
            out = q.get(timeout=600)
            for p in procs:
                p.join(timeout=120)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
