"""Benchmark plumbing on the CPU: steps-to-99%-train-accuracy (BASELINE.json's
second metric) and the handwriting-style synthetic generator it trains on."""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hand_style_deterministic_and_varied():
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic, parse_uri
    a, la = make_synthetic(300, seed=5, style="hand")
    b, lb = make_synthetic(300, seed=5, style="hand")
    assert torch.equal(a, b) and torch.equal(la, lb) and a.shape == (300, 784) and a.dtype == torch.uint8
    # intra-class variability: same-class samples differ far more than in the glyph style
    g, lg = make_synthetic(300, seed=5, style="glyph")
    def spread(x, l):
        x = x.float()
        return torch.stack([x[l == c].std(0).mean() for c in range(10)]).mean().item()
    assert spread(a, la) > spread(g, lg)
    assert parse_uri("synthetic://100?style=hand")[1] == {"style": "hand"}


def test_steps_to_accuracy_cli():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "steps_to_acc.py"), "--cpu", "--impl=torch",
                          "--model=mlp", "--dataset_size=3000", "--probe=500", "--eval_every=25", "--max_steps=2000",
                          "--batch=64", "--lr=0.05", "--target=0.95"],
                         capture_output=True, text=True, timeout=600, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["unit"] == "steps" and r["higher_is_better"] is False
    assert r["value"] is not None and r["value"] % 25 == 0 and r["final_probe_accuracy"] >= 0.95
    assert r["images_seen"] == r["value"] * 64


def test_phase_timer_dp_step():
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.runtime.timers import PhaseTimer
    from distributed_tensorflow_ibm_mnist_amd.runtime.torchnet import TorchNet
    spec = get_model("mlp", 1)
    net = TorchNet(spec, 16, "cpu", torch_ref.init_params(spec), OptConfig())
    dp = DataParallel(net)
    t = PhaseTimer("cpu")
    for _ in range(3):
        dp.train_step(t)
    s = t.summary()
    assert list(s) == ["forward", "loss", "backward", "allreduce_wait", "update"] and t.steps == 3
    assert all(v >= 0 for v in s.values()) and int(net.fp.step.item()) == 3
