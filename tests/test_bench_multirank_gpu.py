"""The driver's multi-GPU bench launch form (``torch.distributed.run --nnodes=1
--nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``), rehearsed on
one MI355X: RCCL refuses two ranks on one device, so the ranks share cuda:0 over
the gloo backend (host-staged all-reduce of the same gradient buckets).  Checks
the contract the 8-GPU scaling run relies on: exactly one JSON line (rank 0),
n_gpus / global_batch / parallelism scaled by the world size, the HIP kernels
running on every rank, and replicas holding identical weights after the timed
steps."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("model,batch", [("lenet5", 4096), ("reference_cnn", 1024)])
def test_bench_torchrun_two_ranks_one_gpu(model, batch):
    port = str(29900 + (os.getpid() % 50) + (0 if model == "lenet5" else 50))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", port,
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--model", model, "--batch", str(batch), "--dist_backend", "gloo", "--phases", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 6 and out["warmup"] == 2
    assert out["config"]["global_batch"] == 2 * batch and out["config"]["per_gpu_batch"] == batch
    assert out["config"]["parallelism"] == "dp2" and out["config"]["impl"] == "hip"
    assert out["replicas_in_sync"] is True
    assert out["grad_bucket_mb"] and out["value"] > 0
    assert out["final_train_loss"] == out["final_train_loss"]     # not NaN
    # communication evidence for the scaling run: every bucket's all-reduce
    # alone and the exposed communication of an eager step
    comm = out["comm"]
    assert len(comm["buckets"]) == len(out["grad_bucket_mb"])
    for b in comm["buckets"]:
        assert b["allreduce_us"] > 0 and b["busbw_GBps"] > 0 and b["algbw_GBps"] > 0 and b["layers"]
    assert comm["eager_ms_comm_on"] > 0 and comm["eager_ms_comm_off"] > 0
    assert "comm_exposed_ms" in comm
    # the process group as the ranks saw it: gloo, 2 ranks, both on the one visible device
    pg = out["pg"]
    assert pg["backend"] == "gloo" and pg["world_size"] == 2 and len(pg["ranks"]) == 2
    assert [r["rank"] for r in pg["ranks"]] == [0, 1] and pg["shared"] == [[0, 1]]
    assert 0 < pg["timed_s_min"] <= pg["timed_s_max"]


def test_bench_one_rank_rccl_comm_probe():
    """The RCCL path on one GPU (--force_collectives 1): the per-bucket all-reduce probe
    and the exposed-communication measurement run on a real RCCL process group."""
    port = str(29800 + (os.getpid() % 50))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "2", "--batch", "4096",
           "--force_collectives", "1", "--phases", "0", "--graph", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "2", "MASTER_PORT": port})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    comm = out["comm"]
    assert comm is not None and len(comm["buckets"]) >= 1
    assert all(b["allreduce_us"] > 0 and b["algbw_GBps"] > 0 for b in comm["buckets"])
    assert comm["eager_ms_comm_on"] > 0 and comm["eager_ms_comm_off"] > 0
    pg = out["pg"]
    assert pg["backend"] == "nccl" and pg["world_size"] == 1 and pg["shared"] == [] and pg["distinct_devices"] == 1
    assert pg["rccl_version"] and (pg["ranks"][0]["pci"] or pg["ranks"][0]["uuid"])
