"""hipGraph capture of the data-parallel step WITH its RCCL bucket all-reduces,
rehearsed on one MI355X with a one-rank RCCL group (8-GPU runs are the driver's):
graph replays must equal eager DP steps bitwise, and bench.py must run the
captured DP step (--force_collectives 1 --graph 1)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph
from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
spec = get_model(sys.argv[3], 1)
init = torch_ref.init_params(spec, seed=4)
B = 256
g = torch.Generator(device=dev).manual_seed(0)
xs = [(torch.rand(B, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16) for _ in range(5)]
ys = [torch.randint(0, 10, (B,), device=dev, generator=g, dtype=torch.int32) for _ in range(5)]
def run(graph):
    net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05, use_momentum=True, momentum=0.9))
    dp = DataParallel(net, bucket_cap_mb=0.01, force_collectives=True)
    assert len(dp.buckets) >= 2, dp.buckets
    sg = None
    for i in range(5):
        net.x0.copy_(xs[i]); net.labels.copy_(ys[i])
        if graph and sg is None:
            sg = StepGraph(dp.train_step, warmup=1)   # the warm-up is step 0
        elif graph:
            sg.replay()
        else:
            dp.train_step()
    torch.cuda.synchronize()
    return net.fp.params.clone(), int(net.fp.step.item())
pe, se = run(False)
pg, sgs = run(True)
assert se == sgs == 5, (se, sgs)
assert torch.equal(pe, pg), (pe - pg).abs().max().item()
dist.destroy_process_group()
print("DP_GRAPH_OK")
"""


@pytest.mark.parametrize("model", ["lenet5", "reference_cnn"])
def test_dp_step_graph_capture_with_rccl(dev, model, tmp_path):
    p = tmp_path / "dp_graph.py"
    p.write_text(SCRIPT)
    port = str(29600 + (os.getpid() % 200) + (0 if model == "lenet5" else 1))
    r = subprocess.run([sys.executable, str(p), ROOT, port, model], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "DP_GRAPH_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_bench_graph_dp_rehearsal(dev):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "512", "--steps", "10",
                        "--warmup", "3", "--graph", "1", "--force_collectives", "1", "--phases", "0"],
                       capture_output=True, text=True, timeout=240,
                       env={**os.environ, "MASTER_PORT": str(29800 + os.getpid() % 100)})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["hip_graph"] is True and out["value"] > 0
    # the driver contract: exactly --steps timed after --warmup (+ the untimed GEMM prewarm)
    assert out["steps"] == 10 and out["warmup"] == 3 and out["prewarm_ms"] == 300.0
