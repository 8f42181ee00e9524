"""Dataset resolution: the file lists the parameter manager hands out
(``getTrainData/getTestData/getValData``, ``mnist_input.py:47-50``) → uint8
image matrix + int32 labels (+ channel count), ready for ``DeviceDataset``.

Accepted entries (a list may mix several of the same kind):
* TFRecord paths / globs in the reference schema (``image_raw`` + ``label``);
* ``synthetic://N?seed=S&noise=F`` — generated MNIST-shaped data;
* ``idx://DIR?split=train|test`` — raw MNIST IDX files (optionally .gz);
* ``png://DIR`` — the ``{0..9}/*.png`` tree written by ``convert_mnist.py``.
"""
from __future__ import annotations

import urllib.parse
from typing import List, Sequence, Tuple

import numpy as np

from . import idx as idx_mod
from .synthetic import make_synthetic, parse_uri
from .tfrecord import load_mnist_tfrecords

# reference constants (mnist_input.py:12-23)
IMAGE_SIZE = 28
IMAGE_PIXELS = 2352        # 28*28*3: DLI stores RGB-converted MNIST
IMAGE_LAYERS = 3
NUM_CLASSES = 10
NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN = 50000   # CIFAR value kept for decay_steps parity (Q8)
NUM_EXAMPLES_PER_EPOCH_FOR_EVAL = 10000


def _load_one_kind(entries: Sequence[str]) -> Tuple[np.ndarray, np.ndarray, int]:
    kind = entries[0].split("://", 1)[0] if "://" in entries[0] else "tfrecord"
    if kind == "synthetic":
        imgs, labs = [], []
        for e in entries:
            n, opts = parse_uri(e)
            a, b = make_synthetic(n, **opts)
            imgs.append(a.numpy())
            labs.append(b.numpy())
        return np.concatenate(imgs), np.concatenate(labs), 1
    if kind == "idx":
        imgs, labs = [], []
        for e in entries:
            u = urllib.parse.urlparse(e)
            path = (u.netloc + u.path) or "."
            split = urllib.parse.parse_qs(u.query).get("split", ["train"])[-1]
            lab, pix, n, r, c = idx_mod.read(split, path)
            imgs.append(pix.reshape(n, r * c))
            labs.append(lab.astype(np.int32))
        return np.concatenate(imgs), np.concatenate(labs), 1
    if kind == "png":
        imgs, labs = [], []
        for e in entries:
            u = urllib.parse.urlparse(e)
            a, b = idx_mod.load_png_tree(u.netloc + u.path)
            imgs.append(a)
            labs.append(b)
        return np.concatenate(imgs), np.concatenate(labs), 1
    return load_mnist_tfrecords(entries)


def load_split(entries: Sequence[str]) -> Tuple[np.ndarray, np.ndarray, int]:
    """Returns (images uint8 [N, 784*C], labels int32 [N], channels C)."""
    entries = list(entries)
    if not entries:
        raise ValueError("empty data list")
    kinds = {e.split("://", 1)[0] if "://" in e else "tfrecord" for e in entries}
    if len(kinds) != 1:
        raise ValueError(f"mixed data kinds in one list: {sorted(kinds)}")
    imgs, labels, c = _load_one_kind(entries)
    if labels.min() < 0 or labels.max() >= NUM_CLASSES:
        raise ValueError("labels out of range 0..9")
    return np.ascontiguousarray(imgs), labels.astype(np.int32), c


def convert_channels(imgs: np.ndarray, c_from: int, c_to: int) -> np.ndarray:
    """Host-side channel conversion (e.g. 3-channel DLI records -> grayscale)."""
    if c_from == c_to:
        return imgs
    n = imgs.shape[0]
    x = imgs.reshape(n, -1, c_from)
    if c_from == 1:
        return np.repeat(x, c_to, axis=2).reshape(n, -1)
    if c_to == 1:
        return x.mean(axis=2).round().astype(np.uint8).reshape(n, -1)
    raise ValueError(f"cannot convert {c_from} -> {c_to} channels")
