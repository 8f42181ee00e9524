"""``train()`` — the reference trainer (``main.py:70-156``) on the MI355X runtime.

Flow (same order as the reference):
  setup_distribute → chief election (task 0) → chief Monitor + FileWriter on
  ``train_dir/log`` → model / loss / optimizer (LR schedule, EMA) → hooks
  [StopAtStep(max_steps), NaN guard, (+chief) Logger] → MonitoredTrainingSession
  → step loop with the reference's progress prints.
A PS task runs the parameter-server loop and returns when every worker is done
(the reference's PS blocked forever in ``server.join()``, Q9).
"""
from __future__ import annotations

import os
import sys
import time
from typing import Dict, Optional

import numpy as np
import torch

from .. import models
from ..data import sources
from ..models import torch_ref
from ..models.spec import Conv, Dense
from ..parallel.cluster import Cluster, setup_distribute, shutdown
from ..runtime.params import OptConfig
from ..utils import parameter_mgr as pm
from .hooks import FaultInjectionHook, LoggerHook, NanTensorHook, StopAtStepHook
from .replica import Replica, state_tensors
from .session import MonitoredTrainingSession

NUM_EPOCHS_PER_DECAY = 350.0      # mnist_input.py:21
MOVING_AVERAGE_DECAY = 0.9999     # mnist_input.py:20


def decay_steps_for(batch_size: int) -> int:
    """mnist_input.py:248-249 — int(NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN / B * 350)."""
    return int(sources.NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN / batch_size * NUM_EPOCHS_PER_DECAY)


def param_specs(spec):
    out = []
    for L in spec.weights():
        shp = (L.kh, L.kw, L.cin, L.cout) if isinstance(L, Conv) else (L.din, L.dout)
        out.append((f"{L.name}/weights", shp, L.wd))
        out.append((f"{L.name}/biases", (shp[-1],), None))
    return out


def load_data(entries, in_channels: int, log=print):
    imgs, labs, c = sources.load_split(entries)
    if c != in_channels and not (c == 1 and in_channels == 3):
        imgs = sources.convert_channels(imgs, c, in_channels)
        c = in_channels
    return torch.from_numpy(np.ascontiguousarray(imgs)), torch.from_numpy(labs), c


def placement_table(replica, cl: Cluster) -> str:
    """``--log_device_placement`` (main.py:31-32,145-146): where every variable,
    gradient bucket and kernel runs."""
    net = replica.net
    dev = str(replica.device)
    lines = [f"device placement (rank {cl.rank}/{cl.world}, mode {cl.mode}, backend {cl.backend or 'none'}"
             + (f", PS data plane {cl.transport}" if cl.mode == "ps" else "") + "):"]
    for e in net.fp.entries:
        lines.append(f"  {e.name:34s} {str(e.shape):22s} fp32 master + EMA{' + Momentum' if net.opt.use_momentum else ''}"
                     f" -> {dev if cl.mode != 'ps' else 'ps shard'}")
    for lay in getattr(net, "layers", []):
        lines.append(f"  kernel {lay.name:18s} {type(lay).__name__:14s} -> {dev}")
    if hasattr(replica, "dp") and replica.dp.world > 1:
        lines.append(replica.dp.describe())
    return "\n".join(lines)


def train(FLAGS, log=print) -> Dict[str, float]:
    pm.configure(FLAGS.config or None, **{k: v for k, v in {
        "max_steps": FLAGS.max_steps, "test_interval": FLAGS.test_interval, "batch_size": FLAGS.batch_size,
        "base_lr": FLAGS.base_lr, "lr_decay": FLAGS.lr_decay, "optimizer": FLAGS.optimizer,
        "momentum": FLAGS.momentum, "train_data": FLAGS.train_data, "test_data": FLAGS.test_data,
        "val_data": FLAGS.val_data}.items() if v not in (None, "", -1)})
    max_steps = pm.getMaxSteps()                  # main.py:38-40
    test_interval = pm.getTestInterval()
    batch_size = pm.getTrainBatchSize()
    impl = FLAGS.impl
    want_gpu = impl == "hip" or (impl == "torch" and torch.cuda.is_available() and not FLAGS.cpu)
    if impl == "hip" and not torch.cuda.is_available():
        raise RuntimeError("--impl=hip needs an MI355X (HIP device); use --impl=torch for the CPU path")
    # the PS data plane's default depends on the largest PS shard (parallel/ps.default_transport)
    n_ps = len([h for h in (FLAGS.ps_hosts or "").split(",") if h.strip()])
    shard_params = 0
    if n_ps and FLAGS.worker_hosts and not FLAGS.ps_backend:
        from ..parallel.ps import max_shard_params
        shard_params = max_shard_params(param_specs(models.get_model(FLAGS.model, FLAGS.in_channels)), n_ps)
    cl = setup_distribute(FLAGS.job_name, FLAGS.ps_hosts, FLAGS.worker_hosts, FLAGS.task_id, want_gpu=want_gpu,
                          timeout_s=FLAGS.collective_timeout, log=log, ps_backend=FLAGS.ps_backend,
                          dp_backend=FLAGS.dp_backend, ps_shard_params=shard_params)
    try:
        return _train(FLAGS, cl, max_steps, test_interval, batch_size, impl, log)
    finally:
        shutdown()


def _train(FLAGS, cl: Cluster, max_steps, test_interval, batch_size, impl, log) -> Dict[str, float]:
    spec = models.get_model(FLAGS.model, FLAGS.in_channels)
    lr0 = pm.getBaseLearningRate()
    opt = OptConfig.from_spec(pm.getOptimizer(lr0), decay_steps_for(batch_size), pm.getLearningRateDecay(),
                              MOVING_AVERAGE_DECAY)
    init = torch_ref.init_params(spec, seed=FLAGS.seed)
    if cl.mode == "ps" and cl.job_name == "ps":
        from ..ckpt.saver import Saver, latest_checkpoint
        from ..parallel.ps import ParameterServer
        prefix = latest_checkpoint(FLAGS.train_dir) if FLAGS.train_dir else None
        restore = Saver.restore(prefix) if prefix else None
        if prefix:
            log(f"[ps {cl.task_id}] restored shard from {prefix}")
        ps = ParameterServer(cl.task_id, cl.num_ps, cl.num_workers, param_specs(spec), init, opt, cl.device,
                             max_steps, restore=restore, log=log, transport=cl.transport, cluster=cl)
        from ..parallel.ps import EXIT_FATAL, PushIntegrityError
        try:
            res = ps.serve()
        except PushIntegrityError as e:
            # an error no restart would fix: a distinct exit code the supervisor never restarts
            log(f"[ps {cl.task_id}] fatal: PushIntegrityError: {e}")
            sys.stdout.flush()
            raise SystemExit(EXIT_FATAL)
        return {"global_step": float(res["global_step"])}

    # Q1: the reference trains on the *test* list (inputs(eval_data=True), main.py:85)
    train_entries = pm.getTestData() if FLAGS.train_on_eval_split else pm.getTrainData()
    x_tr, y_tr, c_tr = load_data(train_entries, spec.in_channels, log)
    x_ev, y_ev, _ = load_data(pm.getTestData(), c_tr if c_tr == spec.in_channels else spec.in_channels, log)
    if x_ev.shape[1] != x_tr.shape[1]:
        x_ev = torch.from_numpy(sources.convert_channels(x_ev.numpy(), x_ev.shape[1] // 784, c_tr))
    dp_group = None
    base = Replica(spec, impl, batch_size, cl.device, init, opt, x_tr, y_tr, c_tr, x_ev, y_ev,
                   seed=FLAGS.seed, shard=not FLAGS.no_shard, use_graph=FLAGS.hip_graph,
                   bucket_mb=FLAGS.bucket_mb, group=dp_group if cl.mode == "dp" else None,
                   fused_input=True if FLAGS.fused_input else getattr(FLAGS, "input_mode", "prep"), precision=getattr(FLAGS, "precision", "bf16"),
                   dp_graph=getattr(FLAGS, "hip_graph_dp", False)) \
        if cl.mode != "ps" else _ps_base(spec, impl, batch_size, cl, init, opt, x_tr, y_tr, c_tr, x_ev, y_ev, FLAGS)
    replica = base
    if cl.mode == "ps":
        from ..parallel.ps import PSWorkerReplica
        replica = PSWorkerReplica(base, cl.num_ps, cl.num_workers, cl.task_id, transport=cl.transport, cluster=cl,
                                  log=log)
    is_chief = cl.is_chief
    if FLAGS.log_device_placement:
        log(placement_table(replica, cl))

    monitor = None
    if is_chief:                                               # main.py:75-78,95-109
        from ..obs.monitor import Monitor
        monitor = Monitor(os.path.join(FLAGS.train_dir, "log"), test_interval, max_steps, replica,
                          eval_examples=FLAGS.eval_examples, log=log)
        monitor.register_reference_summaries()

    # main.py:137-138; the NaN flag is checked asynchronously every N steps
    nan_every = getattr(FLAGS, "nan_check_steps", -1)
    if nan_every is None or nan_every <= 0:
        nan_every = FLAGS.log_step_count_steps if FLAGS.log_step_count_steps > 0 else 100
    hooks = [StopAtStepHook(last_step=max_steps), NanTensorHook(fail_on_nan_loss=True, every_n_steps=nan_every,
                                                                log=log)]
    fi = FaultInjectionHook(cl.rank)
    if fi.active():
        hooks.insert(0, fi)
    if is_chief:
        hooks.append(LoggerHook(test_interval, monitor))                                 # main.py:139
    meta = {"model": spec.name, "in_channels": spec.in_channels, "impl": impl, "mode": cl.mode,
            "precision": getattr(FLAGS, "precision", "bf16"),
            "world": cl.world, "batch_size": batch_size, "flags": {k: v for k, v in FLAGS.flag_dict().items()
                                                                   if isinstance(v, (int, float, str, bool))}}
    t0 = time.time()
    steps = 0
    with MonitoredTrainingSession(replica, is_chief, FLAGS.train_dir if is_chief or cl.mode == "dp" else None,
                                  hooks, save_checkpoint_secs=FLAGS.save_checkpoint_secs,
                                  save_checkpoint_steps=FLAGS.save_checkpoint_steps,
                                  save_summaries_steps=FLAGS.save_summaries_steps,
                                  log_step_count_steps=FLAGS.log_step_count_steps, max_to_keep=FLAGS.max_to_keep,
                                  meta=meta, log=log, restore=cl.mode != "ps") as mon_sess:
        while not mon_sess.should_stop():
            if FLAGS.verbose_steps:                            # main.py:149-150 (Q11: opt-in)
                log("training")
                log(steps)
            mon_sess.run()
            steps += 1
            if steps % 100 == 0:
                log("%d steps executed on worker %d." % (steps, cl.task_id))   # main.py:153
            if getattr(replica, "stop_requested", False):
                break
        replica.synchronize()
    log("%d steps executed on worker %d." % (steps, cl.task_id))                # main.py:154
    if cl.mode == "ps":
        replica.finish()
    if monitor is not None:
        monitor.flush()                                                         # main.py:155-156
        monitor.close()
    dt = time.time() - t0
    st = replica.read_stats()
    res = {"global_step": float(replica.global_step), "steps": float(steps), "seconds": dt,
           "images_per_sec": steps * replica.examples_per_step / max(dt, 1e-9), **st}
    return res


def _ps_base(spec, impl, batch_size, cl, init, opt, x_tr, y_tr, c_tr, x_ev, y_ev, FLAGS):
    """A PS-mode worker: own input stream (reference P3: no sharding), no DP group."""
    return Replica(spec, impl, batch_size, cl.device, init, opt, x_tr, y_tr, c_tr, x_ev, y_ev,
                   seed=FLAGS.seed + 7919 * cl.task_id, shard=False, use_graph=False, bucket_mb=FLAGS.bucket_mb,
                   standalone=True, precision=getattr(FLAGS, "precision", "bf16"))
