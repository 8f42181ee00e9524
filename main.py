#!/usr/bin/env python3
"""Distributed MNIST training — CLI-compatible with the reference ``main.py``.

    python main.py [--train_dir=/tmp/mnist_train] [--config=params.yaml]
    # data parallel (RCCL all-reduce over xGMI), one process per GPU:
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py
    # parameter-server mode (reference semantics), e.g. 1 PS + 2 workers on one node:
    python main.py --job_name=ps     --task_id=0 --ps_hosts=localhost:2222 --worker_hosts=localhost:2223,localhost:2224
    python main.py --job_name=worker --task_id=0 --ps_hosts=localhost:2222 --worker_hosts=localhost:2223,localhost:2224
    python main.py --job_name=worker --task_id=1 --ps_hosts=localhost:2222 --worker_hosts=localhost:2223,localhost:2224

Reference flags (main.py:12-32): job_name, ps_hosts, worker_hosts, task_id,
train_dir, log_device_placement.  Hyper-parameters come from the parameter
manager (``--config`` YAML/JSON or ``MNISTX_PARAMS``), as DLI's
tf_parameter_mgr provided them; the extra flags below override it.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_ibm_mnist_amd.utils import flags  # noqa: E402

FLAGS = flags.FLAGS

# ---- reference flags (main.py:12-32)
flags.DEFINE_string("job_name", "", 'One of "ps", "worker"')
flags.DEFINE_string("ps_hosts", "", "Comma-separated list of hostname:port for the parameter server jobs.")
flags.DEFINE_string("worker_hosts", "", "Comma-separated list of hostname:port for the worker jobs.")
flags.DEFINE_integer("task_id", 0, "Task ID of the worker/replica running the training.")
flags.DEFINE_string("train_dir", "/tmp/mnist_train", "Directory where to write event logs and checkpoint.")
flags.DEFINE_boolean("log_device_placement", False, "Whether to log device placement.")

# ---- parameter manager (tf_parameter_mgr) source + overrides
flags.DEFINE_string("config", "", "YAML/JSON hyper-parameter file (the DLI job config replacement)")
flags.DEFINE_integer("max_steps", -1, "override getMaxSteps()")
flags.DEFINE_integer("test_interval", -1, "override getTestInterval()")
flags.DEFINE_integer("batch_size", -1, "override getTrainBatchSize() (per replica)")
flags.DEFINE_float("base_lr", -1, "override getBaseLearningRate()")
flags.DEFINE_float("lr_decay", -1, "override getLearningRateDecay()")
flags.DEFINE_string("optimizer", "", "override getOptimizer(): sgd | momentum | nesterov")
flags.DEFINE_float("momentum", -1, "momentum for --optimizer=momentum|nesterov")
flags.DEFINE_string("train_data", "", "override getTrainData() (comma list: TFRecords, synthetic://, idx://, png://)")
flags.DEFINE_string("test_data", "", "override getTestData()")
flags.DEFINE_string("val_data", "", "override getValData()")

# ---- framework flags
flags.DEFINE_string("model", "reference_cnn", "reference_cnn | lenet5 | mlp")
flags.DEFINE_integer("in_channels", 3, "model input channels: 3 = DLI RGB records (reference), 1 = grayscale")
flags.DEFINE_string("impl", "hip", "hip = MI355X HIP kernels; torch = plain PyTorch (CPU path / baseline)")
flags.DEFINE_boolean("cpu", False, "force the CPU (torch impl, gloo)")
flags.DEFINE_string("precision", "bf16", "HIP compute precision: bf16 (bf16 operands, fp32 accumulate) | fp32 "
                    "(the reference's tf.float32: fp32 activations and fp32 MFMA)")
flags.DEFINE_integer("seed", 0, "random seed (weights, shuffling)")
flags.DEFINE_boolean("train_on_eval_split", False, "parity with the reference, which trains on getTestData() (Q1)")
flags.DEFINE_boolean("no_shard", False, "every DP rank reads the whole dataset in its own order (reference P3)")
flags.DEFINE_boolean("verbose_steps", False, "print 'training' + step on every step like the reference (Q11)")
flags.DEFINE_boolean("hip_graph", True, "capture the training step in a hipGraph (single GPU)")
flags.DEFINE_boolean("hip_graph_dp", False, "data parallel: also capture the step with its RCCL all-reduces "
                     "(rehearsed with one-rank RCCL and gloo ranks sharing a GPU; a real multi-GPU capture is "
                     "UNVERIFIED -- the eager DP path is the default)")
flags.DEFINE_float("bucket_mb", 0.125, "gradient all-reduce bucket cap (MB); every bucket but the last overlaps backward")
flags.DEFINE_boolean("fused_input", False, "HIP: first fused conv reads the uint8 dataset through the batch index")
flags.DEFINE_string("input_mode", "bf16", "HIP input path: bf16 | u8 (the first fused conv gathers the resident "
                    "training set, normalised once to bf16 / in the kernels from uint8) | prep (a per-step "
                    "gather+normalise kernel); models whose first layer cannot gather fall back to prep")
flags.DEFINE_float("save_checkpoint_secs", 600, "checkpoint every N seconds (TF default 600)")
flags.DEFINE_integer("save_checkpoint_steps", 0, "checkpoint every N steps (0: off)")
flags.DEFINE_integer("save_summaries_steps", 100, "loss/accuracy scalars every N steps")
flags.DEFINE_integer("log_step_count_steps", 100, "global_step/sec every N steps")
flags.DEFINE_integer("max_to_keep", 5, "checkpoints to keep")
flags.DEFINE_integer("nan_check_steps", -1, "NaN guard: read the device NaN flag every N steps, asynchronously "
                     "(a NaN at step k raises by step k + N); -1 = --log_step_count_steps (100 when that is 0)")
flags.DEFINE_integer("eval_examples", 10000, "examples per test-summary evaluation (0: whole split)")
flags.DEFINE_string("ps_backend", "", "PS-mode data plane: '' (GPU: shm for PS shards up to 1 M parameters, e.g. "
                    "LeNet-5, ipc above, e.g. the reference CNN; CPU: host) | shm (CPU parameter server "
                    "serving a shared-memory segment natively; one host) | ipc (xGMI peer copies into a GPU PS) | "
                    "host / gloo (staged through host memory)")
flags.DEFINE_string("dp_backend", "", "DP transport override: '' (RCCL on GPU, gloo on CPU) | gloo (host-staged; "
                    "lets several ranks share one GPU for a rehearsal)")
flags.DEFINE_float("collective_timeout", 600.0, "process-group timeout (s): a hung peer fails the job")


def main(argv=None):
    if FLAGS.ps_hosts and FLAGS.job_name in ("ps", "worker") and "GPU_MAX_HW_QUEUES" not in os.environ:
        # PS mode only (data-parallel workers keep HIP's default queues, so the RCCL stream
        # does not share a queue with compute): PS tasks are often co-located on one GPU,
        # and one hardware queue per process keeps their queues from oversubscribing the
        # GPU's scheduler (0.21-0.25 ms per applied update vs 0.47-0.51 at the default 4,
        # profiles/r3/ps/).  Set before HIP starts; a value the user set is kept.
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MNISTX_PS_HW_QUEUES", "1")
    from distributed_tensorflow_ibm_mnist_amd.train.trainer import train
    res = train(FLAGS)
    if res:
        print("result: " + " ".join(f"{k}={v:.6g}" if isinstance(v, float) else f"{k}={v}" for k, v in res.items()))
    return 0


if __name__ == "__main__":
    flags.run(main)
