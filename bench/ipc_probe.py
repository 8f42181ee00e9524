"""Cross-process device-memory hand-off probe (PS ipc data plane).

Two processes on one GPU: rank 0 exports a buffer (torch reductions / hipIpc);
rank 1 maps it.  Each round: rank 1 writes a pattern (copy_ or a kernel), syncs,
signals over gloo; rank 0 checks it with a kernel read, then writes its own
pattern back for rank 1 to check.  Rank 0 reads the buffer before every round so
a stale cached copy would show."""
import os
import sys

import torch
import torch.distributed as dist
from torch.multiprocessing.reductions import reduce_tensor


def main():
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 20)
    mode = sys.argv[2] if len(sys.argv) > 2 else "copy"
    obj = [None]
    if rank == 0:
        buf = torch.zeros(2, n, device=dev)
        torch.cuda.synchronize()
        obj = [reduce_tensor(buf)]
    dist.broadcast_object_list(obj, src=0)
    if rank == 1:
        fn, args = obj[0]
        buf = fn(*args)
    bad = 0
    for it in range(20):
        if rank == 1:
            src = torch.full((n,), float(it + 1), device=dev)
            if mode == "copy":
                buf[0].copy_(src)
            else:
                buf[0].fill_(float(it + 1))
            torch.cuda.current_stream().synchronize()
            dist.send(torch.tensor([it]), 0)
            dist.recv(torch.zeros(1, dtype=torch.int64), 0)
            got = buf[1].clone()
            torch.cuda.synchronize()
            ok = bool((got == -(it + 1)).all())
            bad += not ok
            if not ok:
                print(f"[r1] it {it}: reply stale: {got[:4].tolist()} unique {got.unique()[:8].tolist()}", flush=True)
        else:
            warm = float(buf[0].sum())              # cache the lines before the peer writes
            dist.recv(torch.zeros(1, dtype=torch.int64), 1)
            got = buf[0].clone()
            torch.cuda.synchronize()
            ok = bool((got == it + 1).all())
            bad += not ok
            if not ok:
                print(f"[r0] it {it}: mailbox stale (warm sum {warm}): unique {got.unique()[:8].tolist()}", flush=True)
            buf[1].fill_(-(it + 1))
            torch.cuda.current_stream().synchronize()
            dist.send(torch.tensor([it]), 1)
    print(f"[r{rank}] mode {mode} n {n}: {bad} bad rounds of 20", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
