"""T4 (CPU variant) / T6: the training CLI end to end on the torch path —
hooks, checkpoint layout + resume, event files / monitor tags, NaN guard and
fault injection."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--impl=torch", "--cpu", "--log_step_count_steps=0", "--train_data=synthetic://1500",
          "--test_data=synthetic://300?seed=1", "--eval_examples=300"]


def run_main(args, env=None, timeout=300):
    e = dict(os.environ, OMP_NUM_THREADS="2", PYTHONUNBUFFERED="1")
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "main.py")] + COMMON + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def result_of(out):
    line = [l for l in out.stdout.splitlines() if l.startswith("result:")][-1]
    return dict(kv.split("=") for kv in line.split()[1:])


def test_train_checkpoint_layout_and_resume(tmp_path):
    d = str(tmp_path / "train")
    r = run_main(["--model=mlp", "--in_channels=1", "--batch_size=32", "--max_steps=30", "--test_interval=10",
                  f"--train_dir={d}", "--save_checkpoint_steps=10", "--optimizer=momentum"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert float(result_of(r)["global_step"]) == 30
    files = os.listdir(d)
    for f in ("checkpoint", "graph.pbtxt", "model.ckpt-30.index", "model.ckpt-30.data-00000-of-00001",
              "model.ckpt-30.meta"):
        assert f in files, f
    assert any(f.startswith("events.out.tfevents") for f in files)
    assert any(f.startswith("events.out.tfevents") for f in os.listdir(os.path.join(d, "log")))
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver
    t = Saver.restore(os.path.join(d, "model.ckpt-30"))
    assert int(t["global_step"]) == 30
    for k in ("hidden/weights", "hidden/weights/ExponentialMovingAverage", "hidden/weights/Momentum",
              "cross_entropy/avg", "total_loss/avg", "softmax_linear/weight_loss/avg"):
        assert k in t, k
    assert t["hidden/weights"].shape == (784, 128)
    # EMA shadow lags the weights but stays close (decay min(0.9999, (1+t)/(10+t)))
    assert 0 < np.abs(t["hidden/weights"] - t["hidden/weights/ExponentialMovingAverage"]).max() < 0.5
    # resume continues the global step
    r2 = run_main(["--model=mlp", "--in_channels=1", "--batch_size=32", "--max_steps=45", "--test_interval=10",
                   f"--train_dir={d}", "--optimizer=momentum"])
    assert r2.returncode == 0, r2.stderr[-2000:]
    assert "Restored from" in r2.stdout and "model.ckpt-30" in r2.stdout
    res = result_of(r2)
    assert float(res["global_step"]) == 45 and float(res["steps"]) == 15


def test_monitor_summaries_reference_cnn(tmp_path):
    d = str(tmp_path / "cnn")
    r = run_main(["--model=reference_cnn", "--in_channels=3", "--batch_size=8", "--max_steps=6",
                  "--test_interval=3", f"--train_dir={d}", "--eval_examples=32", "--log_device_placement"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "device placement" in r.stdout and "local3/weights" in r.stdout
    from distributed_tensorflow_ibm_mnist_amd.obs.events import find_event_files, read_events
    tags = set()
    for f in find_event_files(os.path.join(d, "log")):
        for ev in read_events(f):
            tags |= set(ev["values"])
    for t in ("conv1/weight", "conv1/bias", "conv1/activation", "conv1/weight_norm2", "local4/activation",
              "gradient/local3/weights", "gw_ratio/conv2/weights", "train loss", "train accuracy", "test loss",
              "test accuracy"):
        assert t in tags, t


@pytest.mark.parametrize("every", [4, -1])
def test_nan_guard_fault_injection(tmp_path, every):
    """The NaN guard reads the device flag every N steps, asynchronously: a NaN at
    step k is raised by step k + N (every=-1: N = 100 > max_steps, caught by the end
    hook's final check)."""
    r = run_main(["--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=50", "--test_interval=100",
                  f"--train_dir={tmp_path}", f"--nan_check_steps={every}"], env={"MNIST_FI_NAN_AT_STEP": "5"})
    assert r.returncode != 0
    assert "NaN loss during training" in (r.stderr + r.stdout)
    import re
    m = re.search(r"NaN loss detected at global step (\d+)", r.stdout)
    assert m, r.stdout[-2000:]
    assert 5 <= int(m.group(1)) <= (5 + every if every > 0 else 50)
    # the final-checkpoint end hook must not run after a NaN
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    lc = latest_checkpoint(str(tmp_path))
    assert lc is None or lc.endswith("model.ckpt-0")


def test_no_checkpoint_inside_nan_window(tmp_path):
    """A checkpoint due between a NaN step and the asynchronous NaN check (every 40 steps
    here, saves every 2) must not be written: the saver reads the device flag itself."""
    r = run_main(["--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=30", "--test_interval=100",
                  f"--train_dir={tmp_path}", "--nan_check_steps=40", "--save_checkpoint_steps=2"],
                 env={"MNIST_FI_NAN_AT_STEP": "5"})
    assert r.returncode != 0
    assert "NaN loss during training" in (r.stderr + r.stdout)
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, latest_checkpoint
    lc = latest_checkpoint(str(tmp_path))
    assert lc is not None and int(lc.rsplit("-", 1)[1]) <= 5, lc
    assert np.isfinite(Saver.restore(lc)["hidden/weights"]).all()


def test_crash_and_resume_from_last_checkpoint(tmp_path):
    d = str(tmp_path)
    r = run_main(["--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=40", "--test_interval=100",
                  f"--train_dir={d}", "--save_checkpoint_steps=5"], env={"MNIST_FI_EXIT_AT_STEP": "12"})
    assert r.returncode == 17
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    assert latest_checkpoint(d).endswith("model.ckpt-10")
    r2 = run_main(["--model=mlp", "--in_channels=1", "--batch_size=16", "--max_steps=40", "--test_interval=100",
                   f"--train_dir={d}", "--save_checkpoint_steps=5"])
    assert r2.returncode == 0 and "model.ckpt-10" in r2.stdout
    assert float(result_of(r2)["global_step"]) == 40


def test_inference_cli_after_training(tmp_path):
    d = str(tmp_path / "m")
    r = run_main(["--model=lenet5", "--in_channels=1", "--batch_size=32", "--max_steps=60", "--test_interval=100",
                  f"--train_dir={d}", "--base_lr=0.05", "--optimizer=momentum"])
    assert r.returncode == 0, r.stderr[-2000:]
    from distributed_tensorflow_ibm_mnist_amd.data import idx
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    x, y = make_synthetic(40, seed=9)
    idx.write_dataset(y.numpy(), x.numpy(), 40, 28, 28, str(tmp_path / "png"))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "inference.py"), f"--model={d}", "--impl=torch",
                          "--validate", f"--val_data=png://{tmp_path / 'png'}", f"--output_dir={tmp_path}",
                          "--output_file=val.json"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Predictions are Finished in" in out.stdout
    import json
    res = json.load(open(tmp_path / "val.json"))
    assert res["summary"]["count"] == 40 and res["summary"]["accuracy"] > 0.3
    assert os.path.exists(tmp_path / "val.csv")
