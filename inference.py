#!/usr/bin/env python3
"""Batch prediction — CLI-compatible with the reference ``inference.py``.

    python inference.py --model=<ckpt_dir> --input_dir=<images> --output_dir=<dir> \
        --output_file=result.json [--label_file=labels.txt] [--prob_thresh=0.5]
    python inference.py --model=<ckpt_dir> --validate --output_dir=... --output_file=...

Reference flags (inference.py:17-30): input_dir, output_dir, output_file, model,
label_file, prob_thresh, validate.  Behaviour:
* image mode: every ``input_dir/*.{jpg,jpeg,png}``, decoded (1 channel),
  centre crop/pad to 28×28; validate mode: ``getValData()`` records;
* batches of 128 with a smaller final batch; softmax probabilities;
* restores the raw variables of the latest checkpoint (``--use_ema`` restores
  the EMA shadows instead);
* prints ``Predictions are Finished in X s.`` and writes the result file.
The two reference bugs are fixed (Q3): the input is fed with the model's channel
count (gray replicated to 3 for the DLI-layout model) and normalised exactly as in
training (``x/255 - 0.5``); ``--per_image_standardization`` restores the reference's
preprocessing for parity experiments.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from distributed_tensorflow_ibm_mnist_amd.utils import flags  # noqa: E402

FLAGS = flags.FLAGS
flags.DEFINE_string("input_dir", "", "Directory where to put the predicted images.")
flags.DEFINE_string("output_dir", "", "Directory where to put the inference result.")
flags.DEFINE_string("output_file", "", "File name of the inference result.")
flags.DEFINE_string("model", "", "The pre-trained model referring to the checkpoint.")
flags.DEFINE_string("label_file", "", "Labels of the image classes.")
flags.DEFINE_float("prob_thresh", 0.5, "The prediction probability threshold to display.")
flags.DEFINE_boolean("validate", False, "Evaluating this model with validation dataset or not.")
# framework flags
flags.DEFINE_string("config", "", "parameter-manager config (for getValData())")
flags.DEFINE_string("val_data", "", "override getValData()")
flags.DEFINE_string("arch", "", "model architecture (default: from the checkpoint .meta)")
flags.DEFINE_integer("in_channels", 0, "model input channels (default: from the checkpoint .meta)")
flags.DEFINE_boolean("use_ema", False, "restore <var>/ExponentialMovingAverage shadows")
flags.DEFINE_boolean("per_image_standardization", False, "reference preprocessing (parity; Q3)")
flags.DEFINE_string("impl", "auto", "hip | torch | auto")
flags.DEFINE_string("precision", "bf16", "HIP compute precision: bf16 | fp32 (the reference's tf.float32)")
flags.DEFINE_integer("batch_size", 128, "inference batch (inference.py:34)")

BATCH_SIZE = 128
IMAGE_SIZE = 28


def _standardize(x: np.ndarray) -> np.ndarray:
    """tf.image.per_image_standardization."""
    x = x.astype(np.float32)
    n = x[0].size
    m = x.reshape(len(x), -1).mean(1)
    s = np.maximum(x.reshape(len(x), -1).std(1), 1.0 / np.sqrt(n))
    return (x - m[:, None, None, None]) / s[:, None, None, None]


def predict(FLAGS):
    import torch
    from distributed_tensorflow_ibm_mnist_amd import models
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, get_checkpoint_state
    from distributed_tensorflow_ibm_mnist_amd.data import idx as idxmod, sources
    from distributed_tensorflow_ibm_mnist_amd.obs.results import writeClassificationResult
    from distributed_tensorflow_ibm_mnist_amd.utils import parameter_mgr as pm

    pm.configure(FLAGS.config or None, val_data=FLAGS.val_data or None)
    ckpt = get_checkpoint_state(FLAGS.model)                                   # inference.py:89
    if not (ckpt and ckpt.model_checkpoint_path):
        raise SystemExit(f"no checkpoint found in {FLAGS.model!r}")
    prefix = ckpt.model_checkpoint_path
    from distributed_tensorflow_ibm_mnist_amd.ckpt.metagraph import read_meta_json
    meta = read_meta_json(prefix + ".meta") if os.path.exists(prefix + ".meta") else {}
    arch = FLAGS.arch or meta.get("model", "reference_cnn")
    cin = FLAGS.in_channels or int(meta.get("in_channels", 3))
    spec = models.get_model(arch, cin)

    # ---- inputs
    if FLAGS.validate:
        imgs, labels, c = sources.load_split(pm.getValData())                 # inference.py:62-65
        imgs = imgs.reshape(len(imgs), 28, 28, c)
        if c != 1:
            imgs = imgs.mean(-1, keepdims=True).round().astype(np.uint8)
        names = [f"val_{i}" for i in range(len(imgs))]
    else:
        files = idxmod.list_images(FLAGS.input_dir)                            # inference.py:38-47
        imgs = np.stack([idxmod.decode_image(p, 1, IMAGE_SIZE) for p in files]) if files else \
            np.zeros((0, 28, 28, 1), np.uint8)
        labels = np.full(len(imgs), -1, dtype=np.int32)
        names = files
    if FLAGS.per_image_standardization:
        x = _standardize(imgs)
    else:
        x = imgs.astype(np.float32) / 255.0 - 0.5                              # training normalisation
    if cin != 1:
        x = np.repeat(x, cin, axis=-1)

    # ---- model
    tensors = Saver.restore(prefix)                                            # inference.py:86-91
    params = {}
    for L in spec.weights():
        for kind in ("weights", "biases"):
            n = f"{L.name}/{kind}"
            key = f"{n}/ExponentialMovingAverage" if FLAGS.use_ema else n
            params[n] = torch.from_numpy(np.asarray(tensors[key], dtype=np.float32))
    impl = FLAGS.impl
    if impl == "auto":
        impl = "hip" if torch.cuda.is_available() else "torch"
    dev = torch.device("cuda", 0) if impl == "hip" else torch.device("cpu")
    B = FLAGS.batch_size
    from distributed_tensorflow_ibm_mnist_amd.train.replica import build_net
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    net = build_net(impl, spec, B, dev, params, OptConfig(), FLAGS.precision)

    start = time.time()
    probs = []
    for s in range(0, len(x), B):                                              # inference.py:94-101
        nb = min(B, len(x) - s)
        xb = torch.from_numpy(x[s:s + nb]).to(dev)
        net.x0.view(-1)[: xb.numel()].copy_(xb.reshape(-1).to(net.x0.dtype))
        probs.append(net.probs(nb).float().cpu().numpy()[:, : spec.num_classes])
    prediction = np.concatenate(probs) if probs else np.zeros((0, spec.num_classes), np.float32)
    print("Predictions are Finished in %.2f s." % (time.time() - start))       # inference.py:102
    out_path = os.path.join(FLAGS.output_dir, FLAGS.output_file or "inference_result.json")
    if FLAGS.validate:
        res = writeClassificationResult(out_path, names, prediction, ground_truth=labels)
        print("validation accuracy: %.4f over %d images" % (res["summary"].get("accuracy", float("nan")),
                                                            len(names)))
    else:
        writeClassificationResult(out_path, names, prediction, prob_thresh=FLAGS.prob_thresh,
                                  label_file=FLAGS.label_file)
    return prediction


def main(argv=None):
    predict(FLAGS)
    return 0


if __name__ == "__main__":
    flags.run(main)
