#!/usr/bin/env python3
"""Do inter-process HIP events work on this runtime?  Producer records an IPC event
after a long device sleep, consumer waits on it in its own stream and times how long
its (trivial) follow-up work takes to complete.  Bounded: every wait has a timeout."""
import json
import sys
import time

import torch
import torch.multiprocessing as mp


def producer(q_out, q_in):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ev = torch.cuda.Event(interprocess=True)
    ev.record()
    q_out.put(ev.ipc_handle())
    q_in.get(timeout=30)                     # consumer opened the event
    torch.cuda._sleep(200_000_000)           # ~0.1-0.2 s of device time
    ev.record()
    q_out.put(time.time())
    torch.cuda.synchronize()
    q_out.put(time.time())


def consumer(q_in, q_out, res):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    h = q_in.get(timeout=30)
    try:
        ev = torch.cuda.Event.from_ipc_handle(dev, h)
    except Exception as e:
        res.put({"ok": False, "error": f"from_ipc_handle: {e}"})
        q_out.put(1)
        return
    q_out.put(1)
    t_rec = q_in.get(timeout=30)
    s = torch.cuda.current_stream()
    s.wait_event(ev)
    x = torch.ones(4, device=dev)
    x += 1
    done = torch.cuda.Event()
    done.record()
    t0 = time.time()
    while not done.query():
        if time.time() - t0 > 20:
            res.put({"ok": False, "error": "consumer stream never released (wait_event hung)"})
            return
        time.sleep(0.001)
    t_done = time.time()
    t_prod = q_in.get(timeout=30)
    res.put({"ok": True, "consumer_done_minus_producer_done_ms": round((t_done - t_prod) * 1e3, 2),
             "waited": t_done - t_rec > 0.05})


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    a, b, res = ctx.Queue(), ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=producer, args=(a, b))
    c = ctx.Process(target=consumer, args=(a, b, res))
    p.start(); c.start()
    try:
        r = res.get(timeout=60)
    except Exception as e:
        r = {"ok": False, "error": f"no result: {e}"}
    for q in (p, c):
        q.join(timeout=10)
        if q.is_alive():
            q.kill()
    print(json.dumps(r))
