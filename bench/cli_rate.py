#!/usr/bin/env python3
"""The training CLI's own step rate (main.py, StepCounterHook ``global_step/sec``) next to
``bench.py``'s ms/step on the same box, for LeNet-5 at the reference batch (128, hipGraph
step) and at the BASELINE batch (65536).

main.py runs as a child process with its defaults (summaries every 100 steps, NaN guard
every --log_step_count_steps steps, checkpoint timer 600 s); the test-summary evaluation is
moved past the last step so no timed window contains it.  The first rate window (graph
capture, clock ramp) is dropped; the JSON line gives the median of the rest and the
bench.py numbers measured right after.

    python bench/cli_rate.py [--steps128 4000] [--steps64k 400]
"""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


MODEL, CIN = "lenet5", 1


def run_cli(batch, steps, every):
    cfg = "reference_cnn_synth.yaml" if MODEL == "reference_cnn" else "lenet5_synth.yaml"
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-u", os.path.join(ROOT, "main.py"), f"--train_dir={d}",
               f"--config={os.path.join(ROOT, 'configs', cfg)}", f"--model={MODEL}", f"--in_channels={CIN}",
               f"--batch_size={batch}", f"--max_steps={steps}", f"--test_interval={steps + 1}",
               f"--log_step_count_steps={every}"]
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if out.returncode != 0:
            sys.stderr.write(out.stdout[-3000:] + out.stderr[-3000:])
            raise SystemExit(f"main.py failed ({out.returncode})")
        rates = [float(m) for m in re.findall(r"global_step/sec: ([0-9.eE+-]+)", out.stdout + out.stderr)]
    if len(rates) < 2:
        raise SystemExit(f"too few rate lines: {rates}")
    med = statistics.median(rates[1:])
    return {"batch": batch, "steps": steps, "log_every": every, "rates": [round(r, 2) for r in rates],
            "global_step_per_sec": round(med, 2), "ms_per_step": round(1e3 / med, 4),
            "images_per_sec": round(med * batch, 0)}


def run_bench(batch):
    steps = "2000" if batch <= 1024 else "50"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--batch", str(batch), "--steps", steps, "--warmup", "10",
           "--model", MODEL, "--in_channels", str(CIN)]
    if batch <= 1024:
        cmd += ["--graph", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-3000:])
        raise SystemExit("bench.py failed")
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps128", type=int, default=4000)
    ap.add_argument("--steps64k", type=int, default=400)
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--in_channels", type=int, default=1)
    ap.add_argument("--big_batch", type=int, default=65536, help="the second batch (0 = only 128)")
    args = ap.parse_args()
    global MODEL, CIN
    MODEL, CIN = args.model, args.in_channels
    res = {}
    runs = [(128, args.steps128, 500)] + ([(args.big_batch, args.steps64k, 50)] if args.big_batch else [])
    for batch, steps, every in runs:
        cli = run_cli(batch, steps, every)
        b = run_bench(batch)
        cli["bench_ms_per_step"] = b["ms_per_step"]
        cli["cli_vs_bench"] = round(b["ms_per_step"] / cli["ms_per_step"], 3)
        res[str(batch)] = cli
        print(json.dumps(cli), flush=True)
    print(json.dumps({"cli_rate": res}), flush=True)


if __name__ == "__main__":
    main()
