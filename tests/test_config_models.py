"""T1/T2: flags (reference names/defaults), parameter manager, model oracle."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flag_parsing_forms():
    from distributed_tensorflow_ibm_mnist_amd.utils.flags import FlagValues, FlagError
    import distributed_tensorflow_ibm_mnist_amd.utils.flags as fl
    F = FlagValues()
    F._define("job_name", "", "", str, "string")
    F._define("task_id", 0, "", int, "int")
    F._define("log_device_placement", False, "", fl._parse_bool, "bool")
    rest = F.parse(["--job_name=ps", "--task_id", "3", "--log_device_placement", "pos"])
    assert (F.job_name, F.task_id, F.log_device_placement, rest) == ("ps", 3, True, ["pos"])
    F.parse(["--nolog_device_placement"])
    assert F.log_device_placement is False
    F.parse(["--log_device_placement=false"])
    with pytest.raises(FlagError):
        F.parse(["--unknown=1"])
    F.task_id = 0                       # main.py:66 assigns FLAGS.task_id
    assert F.task_id == 0


def _flags_of(script):
    code = ("import runpy\n"
            f"g = runpy.run_path({script!r}, run_name='flags_probe')\n"
            "print(g['FLAGS'].flag_dict())")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return eval(out.stdout.strip().splitlines()[-1])


def test_reference_flag_surface():
    m = _flags_of(os.path.join(ROOT, "main.py"))
    for k, v in {"job_name": "", "ps_hosts": "", "worker_hosts": "", "task_id": 0,
                 "train_dir": "/tmp/mnist_train", "log_device_placement": False}.items():
        assert m[k] == v, k                                   # main.py:12-32
    i = _flags_of(os.path.join(ROOT, "inference.py"))
    for k, v in {"input_dir": "", "output_dir": "", "output_file": "", "model": "", "label_file": "",
                 "prob_thresh": 0.5, "validate": False}.items():
        assert i[k] == v, k                                   # inference.py:17-30


def test_parameter_manager(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.utils import parameter_mgr as pm
    p = tmp_path / "p.yaml"
    p.write_text("max_steps: 77\nbatch_size: 32\noptimizer: nesterov\nmomentum: 0.8\n"
                 "train_data: [a.tfrecords, b.tfrecords]\n")
    pm.configure(str(p), base_lr=0.5)
    assert pm.getMaxSteps() == 77 and pm.getTrainBatchSize() == 32 and pm.getBaseLearningRate() == 0.5
    assert pm.getTrainData() == ["a.tfrecords", "b.tfrecords"]
    o = pm.getOptimizer(0.1)
    assert o.name == "momentum" and o.nesterov and o.momentum == 0.8 and o.learning_rate == 0.1
    with pytest.raises(ValueError):
        pm.configure({"bogus": 1})
    pm.configure({})
    assert pm.getTestInterval() == 100 and pm.getOptimizer(1.0).name == "sgd"


def test_reference_cnn_parity():
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    s = get_model("reference_cnn", 3)
    assert s.num_params() == 3464714
    f, t = s.flops_per_image()
    assert abs(f - 30.65e6) / 30.65e6 < 1e-3 and abs(t - 88.2e6) / 88.2e6 < 1e-3
    assert [n for n, _ in s.param_shapes()] == [
        "conv1/weights", "conv1/biases", "conv2/weights", "conv2/biases", "local3/weights", "local3/biases",
        "local4/weights", "local4/biases", "softmax_linear/weights", "softmax_linear/biases"]
    assert s.shapes()[5] == (7, 7, 64) and s.loss_names()[-1] == "cross_entropy"
    assert get_model("lenet5").num_params() == 61706


def test_init_statistics():
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    s = get_model("reference_cnn", 3)
    p = torch_ref.init_params(s, seed=0)
    w = p["local3/weights"]
    assert w.abs().max().item() <= 2 * 0.04 + 1e-6                  # truncated at 2 sigma
    assert abs(w.std().item() - 0.04 * 0.8796) < 0.002               # std of N(0,1) truncated at 2 = 0.8796
    assert torch.all(p["conv2/biases"] == 0.1) and torch.all(p["conv1/biases"] == 0.0)


def test_lrn_tf_semantics():
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import lrn_tf
    x = torch.randn(2, 12, 3, 3)
    y = lrn_tf(x, 4, 1.0, 0.001 / 9, 0.75)
    for c in range(12):
        s = sum(x[:, k] ** 2 for k in range(max(0, c - 4), min(12, c + 5)))
        assert torch.allclose(y[:, c], x[:, c] * (1.0 + 0.001 / 9 * s) ** -0.75, atol=1e-6)


def test_oracle_losses_and_grad_shapes():
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    s = get_model("reference_cnn", 1)
    p = {k: v.requires_grad_(True) for k, v in torch_ref.init_params(s, seed=1).items()}
    x = torch.rand(4, 784) - 0.5
    logits, acts = torch_ref.forward(s, p, x, keep_activations=True)
    L = torch_ref.losses(s, p, logits, torch.tensor([1, 2, 3, 4]))
    assert set(L) == {"conv1/weight_loss", "conv2/weight_loss", "local3/weight_loss", "local4/weight_loss",
                      "softmax_linear/weight_loss", "cross_entropy", "total_loss"}
    assert L["conv1/weight_loss"].item() == 0.0                     # wd=0.0 still adds a zero term (Q6)
    assert abs(L["local3/weight_loss"].item() - 0.004 * 0.5 * (p["local3/weights"] ** 2).sum().item()) < 1e-4
    L["total_loss"].backward()
    assert acts["pool2"].shape == (4, 7, 7, 64)
    assert all(p[k].grad is not None for k in p)


def test_lr_schedule_and_decay_steps():
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import decay_steps_for
    assert decay_steps_for(128) == 136718                            # Q8: int(50000/128*350)
    c = OptConfig(lr0=0.1, decay_rate=0.1, decay_steps=100)
    assert c.lr_at(0) == 0.1 and c.lr_at(99) == 0.1 and abs(c.lr_at(100) - 0.01) < 1e-12
    assert abs(c.lr_at(250) - 0.001) < 1e-12                          # staircase


def test_synthetic_data_deterministic_and_learnable():
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic, parse_uri
    a, la = make_synthetic(500, seed=3)
    b, lb = make_synthetic(500, seed=3)
    assert torch.equal(a, b) and torch.equal(la, lb) and a.dtype == torch.uint8 and a.shape == (500, 784)
    assert parse_uri("synthetic://100?seed=4&noise=0.1") == (100, {"seed": 4, "noise": 0.1})
    # nearest-class-mean is far above chance -> learnable
    x = a.float()
    means = torch.stack([x[la == c].mean(0) for c in range(10)])
    pred = torch.cdist(x, means).argmin(1)
    assert (pred == la).float().mean().item() > 0.5


def test_shipped_configs_load():
    import glob
    from distributed_tensorflow_ibm_mnist_amd.utils import parameter_mgr as pm
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import parse_uri
    files = sorted(glob.glob(os.path.join(ROOT, "configs", "*.yaml")))
    assert len(files) >= 3
    for f in files:
        pm.configure(f)
        assert pm.getMaxSteps() > 0 and pm.getTrainBatchSize() > 0
        for uri in pm.getTrainData() + pm.getTestData():
            parse_uri(uri)
    pm.configure({})
