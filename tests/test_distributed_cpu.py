"""T5: distributed correctness on the CPU (gloo backend, same code paths as RCCL).

* data parallel: world 2/4 replicas with bucketed, hook-launched all-reduce give
  the same parameters as one process on the concatenated global batch;
* bucket plan: the reference CNN's local3 gradient closes an early bucket;
* parameter-server mode: 1 PS + 2 workers and 2 PS + 1 worker via the real CLI —
  async apply, exact global-step total, PS shutdown, chief-only sharded checkpoint.
"""
import os
import socket
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, steps, B, out_q):
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=0)
    opt = OptConfig(lr0=0.05, use_momentum=True, momentum=0.9, nesterov=True, ema_max=0.9999)
    net = TorchNet(spec, B, "cpu", init, opt)
    dp = DataParallel(net, bucket_cap_mb=0.05)          # several buckets on LeNet's 247 KB
    assert len(dp.buckets) > 1
    g = torch.Generator().manual_seed(123)
    for _ in range(steps):
        x = torch.rand(world * B, 28, 28, 1, generator=g) - 0.5
        y = torch.randint(0, 10, (world * B,), generator=g, dtype=torch.int32)
        net.x0.copy_(x[rank * B:(rank + 1) * B])
        net.labels.copy_(y[rank * B:(rank + 1) * B])
        dp.train_step()
    if rank == 0:
        out_q.put((net.fp.params.clone(), net.fp.ema.clone(), int(net.fp.step.item())))
    dist.barrier()
    dist.destroy_process_group()


def _single(steps, B_global):
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=0)
    opt = OptConfig(lr0=0.05, use_momentum=True, momentum=0.9, nesterov=True, ema_max=0.9999)
    net = TorchNet(spec, B_global, "cpu", init, opt)
    g = torch.Generator().manual_seed(123)
    for _ in range(steps):
        x = torch.rand(B_global, 28, 28, 1, generator=g) - 0.5
        y = torch.randint(0, 10, (B_global,), generator=g, dtype=torch.int32)
        net.x0.copy_(x)
        net.labels.copy_(y)
        net.train_step()
    return net.fp.params.clone(), net.fp.ema.clone()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_matches_single_process_large_batch(world):
    B, steps = 8, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, steps, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    params, ema, step = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_p, ref_e = _single(steps, B * world)
    assert step == steps
    # mean over ranks of per-rank mean gradients == mean over the global batch
    assert torch.allclose(params, ref_p, rtol=1e-5, atol=1e-6), (params - ref_p).abs().max()
    assert torch.allclose(ema, ref_e, rtol=1e-5, atol=1e-6)


def test_bucket_plan_reference_cnn():
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import plan_buckets
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("reference_cnn", 3)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    b = plan_buckets(net, 4 << 20)
    names = [[spec.layers[i].name for i in bk.layers] for bk in b]
    assert names == [["softmax_linear", "local4", "local3"], ["conv2", "conv1"]]
    assert b[0].end == net.fp.total and b[1].start == 0 and b[0].start == b[1].end
    assert b[0].nbytes > 12.8e6                      # the local3 gradient goes out early


def test_bucket_plan_default_cap():
    """The default 0.125 MB cap leaves only a small bucket that cannot overlap backward."""
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import plan_buckets
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    cap = int(0.125 * (1 << 20))
    spec = get_model("lenet5", 1)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    b = plan_buckets(net, cap)
    assert [[spec.layers[i].name for i in bk.layers] for bk in b] == [["softmax_linear", "fc4", "fc3"], ["conv2", "conv1"]]
    assert b[1].nbytes < 16 << 10                    # the tail bucket: conv params only
    spec = get_model("reference_cnn", 3)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    b = plan_buckets(net, cap)
    assert [[spec.layers[i].name for i in bk.layers] for bk in b] == [
        ["softmax_linear", "local4"], ["local3"], ["conv2"], ["conv1"]]


def test_bucket_plan_lockout():
    """A bucket is never closed where the next backward kernel takes every CU (HipNet.bucket_lockout):
    LeNet-5 with the fused head + conv backward becomes ONE end-of-backward bucket, the reference
    CNN keeps its early local3 bucket but folds conv2 into the final one."""
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import plan_buckets
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    cap = int(0.125 * (1 << 20))
    spec = get_model("lenet5", 1)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    idx = {L.name: i for i, L in enumerate(spec.layers)}
    b = plan_buckets(net, cap, lockout={idx["fc3"], idx["conv2"]})
    assert len(b) == 1 and b[0].start == 0 and b[0].end == net.fp.total
    net.bucket_lockout = {idx["fc3"], idx["conv2"]}       # what HipNet reports for this model
    assert len(plan_buckets(net, cap)) == 1
    spec = get_model("reference_cnn", 1)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    idx = {L.name: i for i, L in enumerate(spec.layers)}
    b = plan_buckets(net, cap, lockout={idx["conv2"]})
    assert [[spec.layers[i].name for i in bk.layers] for bk in b] == [
        ["softmax_linear", "local4"], ["local3"], ["conv2", "conv1"]]


def test_dp_reserve_policy():
    """CUs are reserved for collectives only with several ranks AND an early bucket."""
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("reference_cnn", 1)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec), OptConfig())
    assert DataParallel(net, bucket_cap_mb=0.125, world=1).reserve_cus == 0
    assert DataParallel(net, bucket_cap_mb=0.125, world=2).reserve_cus == DataParallel.RESERVE_CUS
    assert DataParallel(net, bucket_cap_mb=64, world=2).reserve_cus == 0       # one bucket: nothing overlaps
    assert DataParallel(net, bucket_cap_mb=0.125, world=2, reserve_cus=3).reserve_cus == 3


def _spawn_main(args, log):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1")
    return subprocess.Popen([sys.executable, os.path.join(ROOT, "main.py")] + args, cwd=ROOT, env=env,
                            stdout=open(log, "w"), stderr=subprocess.STDOUT)


@pytest.mark.parametrize("num_ps,num_workers,backend", [(1, 2, ""), (2, 1, ""), (1, 2, "shm"), (2, 2, "shm")])
def test_ps_mode_cli(tmp_path, num_ps, num_workers, backend):
    """backend shm: CPU parameter servers serving the gradient pushes natively from shared
    memory (parallel/ps.py ShmTransport, csrc/host/ps_shm.h)."""
    base = free_port()
    ps_hosts = ",".join(f"localhost:{base + i}" for i in range(num_ps))
    wk_hosts = ",".join(f"localhost:{base + 100 + i}" for i in range(num_workers))
    d = str(tmp_path / "train")
    common = ["--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=32", "--max_steps=40",
              "--test_interval=20", "--log_step_count_steps=0", "--train_data=synthetic://1500",
              "--test_data=synthetic://300?seed=1", f"--train_dir={d}", f"--ps_hosts={ps_hosts}",
              f"--worker_hosts={wk_hosts}", "--optimizer=momentum"] + ([f"--ps_backend={backend}"] if backend else [])
    procs = []
    for j in range(num_ps):
        procs.append(("ps", j, _spawn_main(common + ["--job_name=ps", f"--task_id={j}"], tmp_path / f"ps{j}.log")))
    for i in range(num_workers):
        procs.append(("w", i, _spawn_main(common + ["--job_name=worker", f"--task_id={i}"],
                                          tmp_path / f"w{i}.log")))
    t0 = time.time()
    for kind, i, p in procs:
        try:
            p.wait(timeout=max(5, 240 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for _, _, q in procs:
                q.kill()
            pytest.fail(f"{kind}{i} hung:\n" + open(tmp_path / f"{'ps' if kind == 'ps' else 'w'}{i}.log").read())
    logs = {f"{k}{i}": open(tmp_path / f"{'ps' if k == 'ps' else 'w'}{i}.log").read() for k, i, _ in procs}
    for (k, i, p) in procs:
        assert p.returncode == 0, logs[f"{k}{i}"][-3000:]
    assert "applied 40 update(s)" in logs["ps0"]                   # exactly max_steps pushes applied
    assert "global_step 40" in logs["ps0"]
    assert f"transport {backend or 'host'}" in logs["ps0"]
    assert "result: global_step=40" in logs["w0"]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.bundle import read_index
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, latest_checkpoint
    prefix = latest_checkpoint(d)
    assert prefix.endswith("model.ckpt-40")
    n, idx = read_index(prefix)
    assert n == num_ps                                              # one data shard per PS
    t = Saver.restore(prefix)
    assert int(t["global_step"]) == 40 and "hidden/weights/Momentum" in t


def test_ps_kill_fails_workers_then_resume(tmp_path):
    """T6: the PS is SIGKILLed mid-run -> every worker exits non-zero (no hang);
    a restarted cluster resumes from the last checkpoint and finishes."""
    d = str(tmp_path / "train")

    def launch(tag, env_extra):
        base = free_port()
        ps_hosts = f"localhost:{base}"
        wk_hosts = ",".join(f"localhost:{base + 100 + i}" for i in range(2))
        common = ["--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=32", "--max_steps=40",
                  "--test_interval=100", "--log_step_count_steps=0", "--train_data=synthetic://1500",
                  "--test_data=synthetic://300?seed=1", f"--train_dir={d}", f"--ps_hosts={ps_hosts}",
                  f"--worker_hosts={wk_hosts}", "--save_checkpoint_steps=5", "--collective_timeout=120"]
        env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1", **env_extra)
        procs = []
        for job, i in [("ps", 0), ("worker", 0), ("worker", 1)]:
            log = tmp_path / f"{tag}_{job}{i}.log"
            procs.append((f"{job}{i}", log, subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "main.py")] + common + [f"--job_name={job}", f"--task_id={i}"],
                cwd=ROOT, env=env, stdout=open(log, "w"), stderr=subprocess.STDOUT)))
        t0 = time.time()
        for name, log, p in procs:
            try:
                p.wait(timeout=max(5, 240 - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                for _, _, q in procs:
                    q.kill()
                pytest.fail(f"{tag} {name} hung:\n" + open(log).read()[-3000:])
        return {name: (p.returncode, open(log).read()) for name, log, p in procs}

    # no supervisor restarts the PS here: the workers wait MNISTX_PS_RECOVERY_TIMEOUT for a
    # new session generation, then give up and exit non-zero
    r1 = launch("kill", {"MNIST_FI_KILL_RANK_AT_STEP": "0:17", "MNISTX_PS_RECOVERY_TIMEOUT": "10"})
    assert r1["ps0"][0] == -9, r1["ps0"][1][-2000:]
    assert "fault injection: SIGKILL" in r1["ps0"][1]
    for w in ("worker0", "worker1"):
        assert r1[w][0] != 0, r1[w][1][-2000:]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    lc = latest_checkpoint(d)
    assert lc is not None and 5 <= int(lc.rsplit("-", 1)[1]) <= 17     # async: saves at the first step >= 5k
    r2 = launch("resume", {})
    for name, (rc, out) in r2.items():
        assert rc == 0, (name, out[-2000:])
    assert "restored shard from" in r2["ps0"][1] and os.path.basename(lc) in r2["ps0"][1]   # the PS owns the state
    res = [l for l in r2["worker0"][1].splitlines() if l.startswith("result:")][-1]
    assert "global_step=40" in res
    # continues from the checkpoint, not from scratch: exactly the missing updates are applied
    assert f"applied {40 - int(lc.rsplit('-', 1)[1])} update(s)" in r2["ps0"][1]


def test_dp_rank_kill_elastic_restart_resumes(tmp_path):
    """T6 (DP): rank 1 is SIGKILLed at step 12 of a 2-rank torchrun job; the elastic
    agent tears the group down and restarts it (--max-restarts 1), the new attempt
    resumes from the chief's last checkpoint (step 10) and finishes at 40.  Only the
    chief writes checkpoints / events."""
    d = str(tmp_path / "train")
    # GLOO_SOCKET_IFNAME=lo: the container hostname may not resolve.  The restarted
    # attempt must not read the dead attempt's store keys (cluster._attempt_store).
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1", MNIST_FI_KILL_RANK_AT_STEP="1:12",
               GLOO_SOCKET_IFNAME="lo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=1",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "main.py"),
           "--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=40",
           "--test_interval=100", "--log_step_count_steps=0", "--train_data=synthetic://1500",
           "--test_data=synthetic://300?seed=1", "--eval_examples=300", f"--train_dir={d}",
           "--save_checkpoint_steps=5", "--collective_timeout=60"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "restored" in out.lower() and "model.ckpt-10" in out, out[-4000:]
    results = [l for l in out.splitlines() if l.startswith("result:")]
    results = [l for l in out.replace("result:", "\nresult:").splitlines() if l.startswith("result:")]
    assert len(results) == 2 and all("global_step=40" in l for l in results), results
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    assert latest_checkpoint(d).endswith("model.ckpt-40")
    ev = [f for f in os.listdir(d) if f.startswith("events.out.tfevents")]
    assert len(ev) <= 2, ev          # one per attempt, chief only


def test_ps_async_arrival_order_slow_worker(tmp_path):
    """Async semantics: with one worker slowed, the PS keeps applying the fast
    workers' pushes in arrival order (no lock-step): the fast workers' applied
    counts exceed the slow one's, and the total is exactly max_steps."""
    base = free_port()
    ps_hosts = f"localhost:{base}"
    wk_hosts = ",".join(f"localhost:{base + 100 + i}" for i in range(3))
    d = str(tmp_path / "train")
    common = ["--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=60",
              "--test_interval=1000", "--log_step_count_steps=0", "--train_data=synthetic://600",
              "--test_data=synthetic://100?seed=1", f"--train_dir={d}", f"--ps_hosts={ps_hosts}",
              f"--worker_hosts={wk_hosts}", "--save_checkpoint_secs=0", "--eval_examples=100"]
    os.environ["MNIST_FI_SLOW_WORKER"] = "2:0.25"
    try:
        procs = [("ps0", _spawn_main(common + ["--job_name=ps", "--task_id=0"], tmp_path / "ps0.log"))]
        for i in range(3):
            procs.append((f"w{i}", _spawn_main(common + ["--job_name=worker", f"--task_id={i}"],
                                               tmp_path / f"w{i}.log")))
    finally:
        del os.environ["MNIST_FI_SLOW_WORKER"]
    t0 = time.time()
    for name, p in procs:
        try:
            p.wait(timeout=max(5, 240 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for _, q in procs:
                q.kill()
            pytest.fail(f"{name} hung:\n" + open(tmp_path / f"{name}.log").read()[-3000:])
    logs = {n: open(tmp_path / f"{n}.log").read() for n, _ in procs}
    for n, p in procs:
        assert p.returncode == 0, logs[n][-3000:]
    import re
    m = re.search(r"applied (\d+) update\(s\), per worker \[(\d+), (\d+), (\d+)\]", logs["ps0"])
    assert m, logs["ps0"][-2000:]
    applied, c0, c1, c2 = map(int, m.groups())
    assert applied == 60 and c0 + c1 + c2 == 60
    assert min(c0, c1) > c2, (c0, c1, c2)            # the slow worker did not hold the others back
    assert "transport host" in logs["ps0"]


@pytest.mark.parametrize("nesterov,ema", [(True, 0.9999), (False, -1.0)])
def test_ps_native_apply_bitwise_torch_update(nesterov, ema):
    """The shm PS's native update (csrc/host/ps_shm.h) is bitwise the reference-semantics
    update (runtime/torchnet.torch_update): momentum / Nesterov, staircase LR decay, weight
    decay and the EMA -- both single-threaded (LeNet) and threaded (reference CNN) shards."""
    from distributed_tensorflow_ibm_mnist_amd import _host
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import FlatParams, OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import torch_update
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs
    cfg = OptConfig(lr0=0.05, decay_rate=0.5, decay_steps=2, momentum=0.9, use_momentum=True, nesterov=nesterov,
                    ema_max=ema)
    opt = [cfg.lr0, cfg.decay_rate, float(cfg.decay_steps), cfg.momentum, float(cfg.nesterov),
           float(cfg.use_momentum), cfg.ema_max]
    for model in ("lenet5", "reference_cnn"):
        spec = get_model(model, 1)
        init = torch_ref.init_params(spec, seed=0)
        a = FlatParams.build(param_specs(spec), init, "cpu", pads={})
        b = FlatParams.build(param_specs(spec), init, "cpu", pads={})
        wd = torch.zeros_like(a.params)
        for e in a.entries:
            if e.wd:
                wd[e.off:e.off + e.n] = e.wd
        g = torch.Generator().manual_seed(1)
        for step in range(4):
            gr = torch.randn(a.total, generator=g) * 0.01
            a.grads.copy_(gr)
            a.step.fill_(step)
            torch_update(a, cfg, 1.0)
            _host.ps_apply_once(b.params.data_ptr(), gr.data_ptr(), b.mom.data_ptr(), b.ema.data_ptr(),
                                wd.data_ptr(), b.total, opt, step)
        assert torch.equal(a.params, b.params) and torch.equal(a.mom, b.mom), model
        if ema >= 0:
            assert torch.equal(a.ema, b.ema), model


def test_ps_push_stamp_helpers():
    """A push slot = the slice padded to an even length + an int64 stamp in its last 8 bytes."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import slot_len, stamp_view
    for n in (1, 2, 7, 61706):
        L = slot_len(n)
        assert L >= n + 2 and L % 2 == 0
        slot = torch.zeros(L)
        stamp_view(slot).fill_(123456789012)
        assert int(stamp_view(slot)) == 123456789012 and slot[:n].abs().sum() == 0   # stamp never overlaps data


@pytest.mark.parametrize("backend", ["", "shm"])
def test_ps_corrupt_push_is_rejected_and_names_worker(tmp_path, backend):
    """Push integrity (host transport, and the shm data plane's native check): worker 1's
    5th push carries a wrong sequence stamp (MNIST_FI_CORRUPT_PUSH=1:5); the PS rejects it
    BEFORE applying it and exits non-zero naming that worker; the workers do not hang."""
    base = free_port()
    ps_hosts = f"localhost:{base}"
    wk_hosts = ",".join(f"localhost:{base + 100 + i}" for i in range(2))
    d = str(tmp_path / "train")
    common = ["--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=40",
              "--test_interval=1000", "--log_step_count_steps=0", "--train_data=synthetic://600",
              "--test_data=synthetic://100?seed=1", f"--train_dir={d}", f"--ps_hosts={ps_hosts}",
              f"--worker_hosts={wk_hosts}", "--save_checkpoint_secs=0", "--eval_examples=100",
              "--collective_timeout=60"] + ([f"--ps_backend={backend}"] if backend else [])
    os.environ["MNIST_FI_CORRUPT_PUSH"] = "1:5"
    try:
        procs = [("ps0", _spawn_main(common + ["--job_name=ps", "--task_id=0"], tmp_path / "ps0.log"))]
        for i in range(2):
            procs.append((f"w{i}", _spawn_main(common + ["--job_name=worker", f"--task_id={i}"],
                                               tmp_path / f"w{i}.log")))
    finally:
        del os.environ["MNIST_FI_CORRUPT_PUSH"]
    t0 = time.time()
    for name, p in procs:
        try:
            p.wait(timeout=max(5, 200 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for _, q in procs:
                q.kill()
            pytest.fail(f"{name} hung:\n" + open(tmp_path / f"{name}.log").read()[-3000:])
    logs = {n: open(tmp_path / f"{n}.log").read() for n, _ in procs}
    assert procs[0][1].returncode != 0, logs["ps0"][-2000:]
    if backend == "shm":
        assert "PushIntegrityError" in logs["ps0"] and "push from worker 1 failed its sequence-stamp check" \
            in logs["ps0"], logs["ps0"][-2000:]
    else:
        assert "PushIntegrityError" in logs["ps0"] and "push from worker 1 carries stamp 1005" in logs["ps0"], \
            logs["ps0"][-2000:]
        assert "announced 5" in logs["ps0"]
    for n, p in procs[1:]:
        assert p.returncode is not None            # no hang: the workers fail once the PS is gone


def test_ps_worker_weight_loss_terms():
    """PS workers run no local optimizer; the weight-decay loss terms still enter
    total_loss (mnist_input.py:112-114,231) via ps.weight_l2_into."""
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import weight_l2_into
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("reference_cnn", 1)
    net = TorchNet(spec, 2, "cpu", torch_ref.init_params(spec, seed=3), OptConfig())
    net.x0.copy_(torch.rand(2, 28, 28, 1) - 0.5)
    net.labels.copy_(torch.tensor([1, 7], dtype=torch.int32))
    net.forward()
    net.loss_and_grad()
    net.backward()
    weight_l2_into(net.fp)
    net.finalize(2, increment=False)
    want = sum(0.004 * 0.5 * float(net.fp.param_view(f"{n}/weights").square().sum()) for n in ("local3", "local4"))
    st = net.read_stats()
    assert want > 0.01
    assert abs((st["total_loss"] - st["cross_entropy"]) - want) < 1e-4 * want
    assert int(net.fp.step.item()) == 0


def _sup_flags(d, backend=""):
    return ["--impl=torch", "--cpu", "--model=mlp", "--in_channels=1", "--batch_size=32", "--max_steps=40",
            "--test_interval=100", "--log_step_count_steps=0", "--train_data=synthetic://1500",
            "--test_data=synthetic://300?seed=1", f"--train_dir={d}", "--save_checkpoint_steps=5",
            "--collective_timeout=60"] + ([f"--ps_backend={backend}"] if backend else [])


def test_ps_supervisor_restarts_after_ps_death(tmp_path):
    """Whole-job recovery (--recover_ps 0): the PS is SIGKILLed at step 17 of attempt 0;
    the supervisor tears the attempt down, starts attempt 1 (fault injection is off on
    restarts), the PS restores its shard from the last checkpoint and the job
    finishes at exactly max_steps."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.supervisor import supervise
    d = str(tmp_path / "train")
    logs = str(tmp_path / "logs")
    msgs = []
    os.environ["MNIST_FI_KILL_RANK_AT_STEP"] = "0:17"
    try:
        rc = supervise(_sup_flags(d), num_ps=1, num_workers=2, max_restarts=2, log_dir=logs, timeout_s=400,
                       log=msgs.append, recover_ps=False)
    finally:
        os.environ.pop("MNIST_FI_KILL_RANK_AT_STEP", None)
    assert rc == 0, msgs
    assert any("attempt 1 finished" in m for m in msgs), msgs
    ps1 = open(os.path.join(logs, "attempt1_ps0.log")).read()
    assert "restored shard from" in ps1
    w0 = open(os.path.join(logs, "attempt1_worker0.log")).read()
    assert "result: global_step=40" in w0, w0[-2000:]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    assert latest_checkpoint(d).endswith("model.ckpt-40")


@pytest.mark.parametrize("num_ps,kill_rank,backend", [(1, 0, ""), (2, 1, ""), (1, 0, "shm"), (2, 1, "shm")])
def test_ps_session_recovery_in_place(tmp_path, num_ps, kill_rank, backend):
    """In-place session recovery (MonitoredTrainingSession's, main.py:140-146): a PS is
    SIGKILLed at step 17; the supervisor relaunches ONLY that PS, which restores its
    shard from the last checkpoint and opens session generation 1; both workers (same
    processes: no attempt 1) recreate their session and rejoin, a surviving PS (2-PS
    case) rejoins on the workers' RESET keeping its state, and the job ends at
    max_steps with a checkpoint of every shard."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.supervisor import supervise
    d = str(tmp_path / "train")
    logs = str(tmp_path / "logs")
    msgs = []
    os.environ["MNIST_FI_KILL_RANK_AT_STEP"] = f"{kill_rank}:17"
    try:
        rc = supervise(_sup_flags(d, backend), num_ps=num_ps, num_workers=2, max_restarts=2, log_dir=logs,
                       timeout_s=400, log=msgs.append)
    finally:
        os.environ.pop("MNIST_FI_KILL_RANK_AT_STEP", None)
    read = lambda n: open(os.path.join(logs, n)).read()
    assert rc == 0, (msgs, read(f"attempt0_ps{kill_rank}_restart1.log")[-2000:])
    assert any(f"ps{kill_rank} exited with -9; restarting it in place" in m for m in msgs), msgs
    assert not any("attempt 1" in m for m in msgs), msgs              # no whole-job restart
    assert not os.path.exists(os.path.join(logs, "attempt1_worker0.log"))
    assert "fault injection: SIGKILL" in read(f"attempt0_ps{kill_rank}.log")
    rs = read(f"attempt0_ps{kill_rank}_restart1.log")
    assert "restored shard from" in rs and "opening session generation 1" in rs, rs[-2000:]
    for w in ("worker0", "worker1"):
        out = read(f"attempt0_{w}.log")
        assert "The current session will be recreated" in out and "joined generation 1" in out, out[-2000:]
    if num_ps == 2:
        survivor = read(f"attempt0_ps{1 - kill_rank}.log")
        assert "rejoining session generation 1" in survivor, survivor[-2000:]
    w0 = read("attempt0_worker0.log")
    res = [l for l in w0.splitlines() if l.startswith("result:")][-1]
    assert "global_step=40" in res, w0[-2000:]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.bundle import read_index
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    lc = latest_checkpoint(d)
    assert lc.endswith("model.ckpt-40")
    assert read_index(lc)[0] == num_ps


def test_ps_supervisor_never_restarts_a_fatal_ps(tmp_path):
    """A PS that rejects a corrupt push (MNIST_FI_CORRUPT_PUSH) exits with EXIT_FATAL;
    the supervisor neither relaunches it in place nor restarts the job."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.supervisor import EXIT_FATAL, supervise
    d = str(tmp_path / "train")
    logs = str(tmp_path / "logs")
    msgs = []
    os.environ["MNIST_FI_CORRUPT_PUSH"] = "1:5"
    try:
        rc = supervise(_sup_flags(d) + ["--ps_backend=host"], num_ps=1, num_workers=2, max_restarts=2,
                       log_dir=logs, timeout_s=300, log=msgs.append)
    finally:
        os.environ.pop("MNIST_FI_CORRUPT_PUSH", None)
    assert rc == EXIT_FATAL, msgs
    assert any("(fatal); not restarting" in m for m in msgs), msgs
    assert not any("restarting it in place" in m or "attempt 1" in m for m in msgs), msgs
    assert "PushIntegrityError" in open(os.path.join(logs, "attempt0_ps0.log")).read()


def test_is_peer_loss_classification():
    """Only lost-peer control-plane errors enter PS recovery; a HIP / CUDA failure that
    happens to mention a timeout is re-raised at once (it is not a lost peer)."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import PushIntegrityError, is_peer_loss
    assert is_peer_loss(RuntimeError("[../third_party/gloo/gloo/transport/tcp/pair.cc:534] Connection closed by peer"))
    assert is_peer_loss(RuntimeError("Gloo: Timed out waiting 60000ms for recv operation to complete"))
    assert not is_peer_loss(RuntimeError("HIP error: hipErrorLaunchTimeOut: the launch timed out"))
    assert not is_peer_loss(RuntimeError("CUDA error: unspecified launch failure (connection to gloo lost?)"))
    assert not is_peer_loss(RuntimeError("socket timeout"))          # no gloo: not ours to recover
    assert not is_peer_loss(PushIntegrityError("gloo connection closed"))
    # a device string inside a gloo transport error is not a compute error
    assert is_peer_loss(RuntimeError("Gloo connection closed by peer while sending tensor on cuda:0"))
    assert not is_peer_loss(RuntimeError("hipErrorIllegalAddress: gloo connection reset"))


def test_default_ps_transport_by_shard_size():
    """GPU ranks: shm (CPU PS) for small shards, ipc (GPU PS) above 1 M parameters per shard;
    the same answer from the model's specs (PS side) and from a worker's FlatParams."""
    import torch
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.parallel.ps import default_transport, max_shard_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import FlatParams
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs
    gpu = torch.device("cuda", 0)
    lenet = param_specs(get_model("lenet5", 1))
    ref = param_specs(get_model("reference_cnn", 3))
    assert max_shard_params(lenet, 1) == 61706
    assert max_shard_params(ref, 1) == 3464714
    assert max_shard_params(ref, 2) == max_shard_params(FlatParams.build(ref, {}, "cpu", pads={}), 2)
    assert default_transport(gpu, max_shard_params(lenet, 1)) == "shm"
    assert default_transport(gpu, max_shard_params(ref, 1)) == "ipc"
    assert default_transport(torch.device("cpu"), max_shard_params(ref, 1)) == "host"


def test_shm_segment_enospc_is_a_clean_error(monkeypatch, tmp_path):
    """The shm segment reserves its pages at creation (posix_fallocate): a /dev/shm too small
    for it is an OSError there -- setup_transport's fallback -- not a SIGBUS at first touch;
    the half-made file is removed."""
    import errno
    from distributed_tensorflow_ibm_mnist_amd.parallel import ps as psm

    def full(fd, off, n):
        raise OSError(errno.ENOSPC, "No space left on device")
    monkeypatch.setattr(psm.os, "posix_fallocate", full)
    path = str(tmp_path / "seg")
    with pytest.raises(OSError):
        psm.ShmSegment(path, psm.ShmLayout(1000, 2), create=True)
    assert not os.path.exists(path)


def test_shm_worker_pins_only_its_own_page_aligned_block(monkeypatch, tmp_path):
    """A GPU worker of the shm data plane registers (hipHostRegister) only its own block, once
    its worker index is known (worker_open), and that block starts on a page boundary."""
    from distributed_tensorflow_ibm_mnist_amd.parallel import ps as psm
    lay = psm.ShmLayout(1000, 3)
    assert lay.HDR % 4096 == 0 and lay.wblock % 4096 == 0
    seg = psm.ShmSegment(str(tmp_path / "seg"), lay, create=True)
    calls = []
    monkeypatch.setattr(psm.ShmSegment, "pin", lambda self, worker=None: calls.append(worker) or True)
    tx = psm.ShmTransport(None, 1, 3)
    tx.segs = {0: seg}
    tx.want_pin = True
    tx.worker_open(2, None)
    assert calls == [2]
    seg.close()
