"""Parameter-server mode on the MI355X (``/root/reference/main.py:56-62,80-82``,
``/root/reference/mnist_input.py:261-264``).

One GPU box rehearses the 1 PS + N workers topology with every process on the
same card: the ``ipc`` data plane (PS-owned device mailboxes, one-sided copies,
gloo control plane) is exactly the code that runs across 8 GPUs, where the
copies cross xGMI instead of staying in one HBM.  HIP workers, fused K9 apply
on the PS, async arrival order, stop at ``max_steps``, clean PS exit, PS-owned
sharded checkpoint; and the PS bench mode's JSON line.
"""
import json
import os
import re
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(tmp_path, transport, num_ps=1, num_workers=2, max_steps=60, model="lenet5", in_channels=1, batch=256):
    base = free_port()
    ps_hosts = ",".join(f"localhost:{base + i}" for i in range(num_ps))
    wk_hosts = ",".join(f"localhost:{base + 100 + i}" for i in range(num_workers))
    d = str(tmp_path / f"train_{transport}_{num_ps}")
    common = [f"--model={model}", f"--in_channels={in_channels}", f"--batch_size={batch}", f"--max_steps={max_steps}",
              "--test_interval=30", "--log_step_count_steps=0", "--train_data=synthetic://8000",
              "--test_data=synthetic://512?seed=1", "--eval_examples=512", f"--train_dir={d}",
              f"--ps_hosts={ps_hosts}", f"--worker_hosts={wk_hosts}", f"--ps_backend={transport}",
              "--optimizer=momentum", "--base_lr=0.02"]
    # every worker starts pushing only once all have said HELLO (the per-worker counts below)
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="2", MNISTX_PS_START_BARRIER="1")
    procs = []
    for job, n in (("ps", num_ps), ("worker", num_workers)):
        for i in range(n):
            log = tmp_path / f"{transport}_{job}{i}.log"
            procs.append((f"{job}{i}", log, subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "main.py")] + common + [f"--job_name={job}", f"--task_id={i}"],
                cwd=ROOT, env=env, stdout=open(log, "w"), stderr=subprocess.STDOUT)))
    t0 = time.time()
    for name, log, p in procs:
        try:
            p.wait(timeout=max(5, 200 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for _, _, q in procs:
                q.kill()
            pytest.fail(f"{name} hung:\n" + open(log).read()[-3000:])
    logs = {name: open(log).read() for name, log, _ in procs}
    for name, _, p in procs:
        assert p.returncode == 0, (name, logs[name][-3000:])
    return d, logs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("transport", ["ipc", "host", "shm"])
def test_ps_mode_hip_workers_one_gpu(tmp_path, dev, transport):
    d, logs = _launch(tmp_path, transport)
    assert f"transport {transport}" in logs["ps0"]
    m = re.search(r"applied (\d+) update\(s\), per worker \[(\d+), (\d+)\]", logs["ps0"])
    assert m, logs["ps0"][-2000:]
    assert int(m.group(1)) == 60 and int(m.group(2)) + int(m.group(3)) == 60
    assert min(int(m.group(2)), int(m.group(3))) > 0            # both workers contributed
    assert "result: global_step=60" in logs["worker0"]
    # training made progress: the chief's held-out evaluation (Logger hook) at the end.  Async:
    # a fast worker can push the first 30+ updates before the chief's first step returns (graph
    # capture), so the chief may see only the final crossing of test_interval
    accs = [float(a) for a in re.findall(r"test accuracy ([0-9.]+)", logs["worker0"])]
    assert len(accs) >= 1 and accs[-1] > 0.3, accs
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, latest_checkpoint
    p = latest_checkpoint(d)
    assert p.endswith("model.ckpt-60")
    t = Saver.restore(p)
    assert int(t["global_step"]) == 60 and "fc3/weights/Momentum" in t


@pytest.mark.timeout(300)
def test_ps_mode_reference_cnn_default_transport(tmp_path, dev):
    """The reference's own model and configuration (3.46 M parameters, 3 input channels,
    batch 128: /root/reference/main.py:80-82, mnist_input.py:13-15,261-264) through the
    DEFAULT data plane, which for a shard this size is the GPU PS of ipc
    (parallel/ps.default_transport): every update applied, both workers contributing."""
    d, logs = _launch(tmp_path, "", max_steps=40, model="reference_cnn", in_channels=3, batch=128)
    assert "transport ipc" in logs["ps0"], logs["ps0"][-2000:]
    m = re.search(r"applied (\d+) update\(s\), per worker \[(\d+), (\d+)\]", logs["ps0"])
    assert m, logs["ps0"][-2000:]
    assert int(m.group(1)) == 40 and min(int(m.group(2)), int(m.group(3))) > 0
    assert "result: global_step=40" in logs["worker0"]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, latest_checkpoint
    t = Saver.restore(latest_checkpoint(d))
    assert int(t["global_step"]) == 40 and t["local3/weights"].shape == (3136, 1024)


@pytest.mark.timeout(300)
def test_ps_mode_two_ps_ipc(tmp_path, dev):
    """k=2 PS shards: both apply exactly max_steps updates (consistent shard counts)."""
    d, logs = _launch(tmp_path, "ipc", num_ps=2, num_workers=2, max_steps=40)
    for j in (0, 1):
        assert re.search(r"applied 40 update\(s\)", logs[f"ps{j}"]), logs[f"ps{j}"][-2000:]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.bundle import read_index
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    n, _ = read_index(latest_checkpoint(d))
    assert n == 2


@pytest.mark.timeout(300)
def test_ps_transports_bitwise_equal_one_worker(dev):
    """With ONE worker the PS run is deterministic: the ipc data plane (device
    mailboxes) and the host-staged one must leave bitwise-identical parameters."""
    sums = {}
    for t in ("ipc", "host"):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
               "--mode", "ps", "--ps_transport", t, "--batch", "256", "--steps", "20", "--warmup", "2"]
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=200,
                           env=dict(os.environ, OMP_NUM_THREADS="2"))
        assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert d["global_step"] == 22
        sums[t] = d["param_checksum"]
    assert sums["ipc"] == sums["host"], sums


@pytest.mark.timeout(300)
@pytest.mark.parametrize("transport", ["ipc", "shm"])
def test_bench_ps_mode_json(dev, transport):
    """transport shm: the PS is a CPU task serving a shared-memory segment natively (it never
    opens the GPU); the workers DMA to / from pinned slots."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
           "--mode", "ps", "--batch", "4096", "--steps", "10", "--warmup", "2", "--ps_transport", transport]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out[-3000:]
    d = json.loads(line[0])
    assert d["config"]["parallelism"] == "ps1+w2" and d["global_step"] == 24
    assert d["value"] > 0 and sum(d["applied_per_worker"]) == 24
    # serve-loop phase split (host us per applied update)
    assert set(d["ps_us_per_msg"]) == {"idle", "apply", "reply"} and d["ps_us_per_msg"]["apply"] > 0
    # data plane per GRAD message, per worker: push / pull us and GB/s
    assert len(d["ps_comm"]) == 2 and d["transport_used"] == transport
    assert d["config"]["ps_device"] == ("cpu" if transport == "shm" else "cuda")
    for c in d["ps_comm"]:
        assert c["msgs"] >= 1 and c["push_us"] > 0 and c["push_GBps"] > 0 and c["pull_us"] > 0
        assert c["bytes_per_push"] >= c["bytes_per_pull"] > 0          # the push carries the 8-byte stamp


@pytest.mark.timeout(300)
def test_ps_ipc_corrupt_push_aborts_naming_worker(dev):
    """Push integrity on the device data plane: worker 0's 4th push carries a wrong
    sequence stamp (MNIST_FI_CORRUPT_PUSH=0:4); the fused K9 kernel skips it and the
    PS aborts with an error naming worker 0 (a stale / torn gradient is never applied
    silently)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
           "--mode", "ps", "--ps_transport", "ipc", "--batch", "256", "--steps", "150", "--warmup", "2"]
    # 150 steps: the workers race for a shared update budget, and one run where worker 0's
    # cold first step took 122 ms left it a single push of 44 (its 4th never came)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2", MNIST_FI_CORRUPT_PUSH="0:4"))
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-3000:]
    assert "PushIntegrityError" in out and "push from worker 0 failed its sequence-stamp check" in out, out[-3000:]


def test_ps_session_recovery_ipc(tmp_path):
    """In-place session recovery on the GPU data plane: HIP workers with the ipc
    transport, the PS SIGKILLed at step 17 and relaunched alone by the supervisor;
    the workers (same processes) re-map the new PS's mailboxes and finish at max_steps."""
    from distributed_tensorflow_ibm_mnist_amd.parallel.supervisor import supervise
    d = str(tmp_path / "train")
    logs = str(tmp_path / "logs")
    flags = ["--model=lenet5", "--in_channels=1", "--batch_size=256", "--max_steps=40", "--test_interval=1000",
             "--log_step_count_steps=0", "--train_data=synthetic://8000", "--test_data=synthetic://512?seed=1",
             "--eval_examples=512", f"--train_dir={d}", "--ps_backend=ipc", "--save_checkpoint_steps=5",
             "--optimizer=momentum", "--base_lr=0.02", "--collective_timeout=60"]
    msgs = []
    os.environ["MNIST_FI_KILL_RANK_AT_STEP"] = "0:17"
    try:
        rc = supervise(flags, num_ps=1, num_workers=2, max_restarts=1, log_dir=logs, timeout_s=180,
                       log=msgs.append)
    finally:
        os.environ.pop("MNIST_FI_KILL_RANK_AT_STEP", None)
    read = lambda n: open(os.path.join(logs, n)).read()
    assert rc == 0, (msgs, read("attempt0_worker0.log")[-2000:])
    assert not any("attempt 1" in m for m in msgs), msgs
    rs = read("attempt0_ps0_restart1.log")
    assert "restored shard from" in rs and "transport ipc" in rs, rs[-2000:]
    for w in ("worker0", "worker1"):
        assert "joined generation 1" in read(f"attempt0_{w}.log")
    res = [l for l in read("attempt0_worker0.log").splitlines() if l.startswith("result:")][-1]
    assert "global_step=40" in res
