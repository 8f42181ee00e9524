"""T4 on the default CLI path: ``main.py`` / ``inference.py`` with ``--impl=hip``.

The reference loop (``/root/reference/main.py:140-156``) and predictor
(``/root/reference/inference.py:67-110``), run end to end on the HIP kernels
with the hipGraph-captured step:

* the defaults (reference CNN, 3-channel input, hipGraph): ``--max_steps=1``
  performs exactly one update, and a resume at ``max_steps - 1`` exactly one more;
* SIGKILL mid-run (``MNIST_FI_KILL_RANK_AT_STEP``), resume from the last
  checkpoint: the final parameters, EMA shadows and momentum slots equal an
  uninterrupted run BITWISE (deterministic kernels + seekable loader);
* the chief's ``train_dir/log`` events carry the reference's DLMAO tags, and the
  conv activations are the pre-pool ReLU outputs (``main.py:97-100``);
* ``inference.py --impl=hip`` on that checkpoint agrees with ``--impl=torch``
  (fp32 CPU oracle) within bf16 tolerance.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

DATA = ["--train_data=synthetic://4000", "--test_data=synthetic://512?seed=1", "--eval_examples=256"]


def run(args, env_extra=None, timeout=180, script="main.py"):
    env = dict(os.environ, PYTHONUNBUFFERED="1", **(env_extra or {}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def result_line(out):
    lines = [l for l in out.splitlines() if l.startswith("result:")]
    assert lines, out[-3000:]
    return dict(kv.split("=", 1) for kv in lines[-1][len("result: "):].split())


def final_state(d):
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, latest_checkpoint
    p = latest_checkpoint(d)
    assert p is not None
    return p, Saver.restore(p)


@pytest.mark.timeout(400)
def test_defaults_one_step_and_resume_one_more(tmp_path, dev):
    d = str(tmp_path / "t")
    common = ["--batch_size=32", "--test_interval=1000", f"--train_dir={d}", "--log_step_count_steps=0"] + DATA
    rc, out = run(common + ["--max_steps=1"])
    assert rc == 0, out[-3000:]
    assert result_line(out)["global_step"] in ("1", "1.0"), out[-2000:]
    p, t = final_state(d)
    assert p.endswith("model.ckpt-1") and int(t["global_step"]) == 1
    rc, out = run(common + ["--max_steps=2"])
    assert rc == 0, out[-3000:]
    assert "Restored from" in out and "model.ckpt-1" in out
    assert result_line(out)["global_step"] in ("2", "2.0")
    p, t = final_state(d)
    assert p.endswith("model.ckpt-2") and int(t["global_step"]) == 2


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model,cin", [("reference_cnn", 3), ("lenet5", 1)])
def test_kill_resume_bitwise_and_events(tmp_path, dev, model, cin):
    common = [f"--model={model}", f"--in_channels={cin}", "--batch_size=64", "--max_steps=30",
              "--test_interval=10", "--save_checkpoint_steps=10", "--log_step_count_steps=0",
              "--optimizer=momentum", "--base_lr=0.05"] + DATA
    da, db = str(tmp_path / "killed"), str(tmp_path / "straight")
    rc, out = run(common + [f"--train_dir={da}"], {"MNIST_FI_KILL_RANK_AT_STEP": "0:15"})
    assert rc == -9, out[-3000:]
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import latest_checkpoint
    assert latest_checkpoint(da).endswith("model.ckpt-10")
    rc, out = run(common + [f"--train_dir={da}"])
    assert rc == 0 and "model.ckpt-10" in out, out[-3000:]
    rc, out2 = run(common + [f"--train_dir={db}"])
    assert rc == 0, out2[-3000:]
    pa, ta = final_state(da)
    pb, tb = final_state(db)
    assert pa.endswith("model.ckpt-30") and pb.endswith("model.ckpt-30")
    keys = [k for k in tb if k.endswith(("/weights", "/biases", "/ExponentialMovingAverage", "/Momentum"))]
    assert len(keys) >= 18
    for k in keys:
        assert np.array_equal(np.asarray(ta[k]), np.asarray(tb[k])), k

    # chief DLMAO summaries (main.py:95-109) in train_dir/log
    from distributed_tensorflow_ibm_mnist_amd.obs.events import find_event_files, read_events
    tags, acts = set(), {}
    for f in find_event_files(os.path.join(db, "log")):
        for ev in read_events(f):
            tags |= set(ev["values"])
            for t, v in ev["values"].items():
                if t.endswith("/activation"):
                    acts[t] = v
    want = {"train loss", "train accuracy", "test loss", "test accuracy", "conv1/weight", "conv1/bias",
            "conv1/activation", "conv1/weight_norm2", "conv2/activation", "gradient/conv1/weights",
            "gw_ratio/conv1/weights"}
    assert want <= tags, want - tags
    # the conv activation is the pre-pool ReLU output of 64 sampled images
    cout1 = 32 if model == "reference_cnn" else 6
    a1 = acts["conv1/activation"]
    assert a1["num"] == 64 * 28 * 28 * cout1 and a1["min"] >= 0.0, a1
    a2 = acts["conv2/activation"]
    oh2, c2 = (14, 64) if model == "reference_cnn" else (10, 16)
    assert a2["num"] == 64 * oh2 * oh2 * c2 and a2["min"] >= 0.0, a2

    # inference on the checkpoint: HIP kernels vs the fp32 PyTorch oracle on the CPU
    res = {}
    for impl in ("hip", "torch"):
        rc, out = run([f"--model={db}", "--validate", "--val_data=synthetic://600?seed=2",
                       f"--output_dir={tmp_path / 'inf'}", f"--output_file={impl}.json", f"--impl={impl}"],
                      script="inference.py")
        assert rc == 0 and "Predictions are Finished" in out, out[-3000:]
        res[impl] = json.load(open(tmp_path / "inf" / f"{impl}.json"))
    rh, rt = res["hip"]["results"], res["torch"]["results"]
    assert len(rh) == len(rt) == 600
    agree = np.mean([a["prediction"] == b["prediction"] for a, b in zip(rh, rt)])
    assert agree >= 0.98, agree
    same = [(a["probability"], b["probability"]) for a, b in zip(rh, rt) if a["prediction"] == b["prediction"]]
    diff = max(abs(x - y) for x, y in same)
    assert diff < 0.05, diff
    assert abs(res["hip"]["summary"]["accuracy"] - res["torch"]["summary"]["accuracy"]) <= 0.02
