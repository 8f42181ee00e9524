"""Checkpoint saver / restorer with the reference's directory layout.

Layout written under ``--train_dir``::

    checkpoint                           CheckpointState (text proto)
    model.ckpt-<step>.index              tensor-bundle SSTable
    model.ckpt-<step>.data-0000i-of-0000N
    model.ckpt-<step>.meta               MetaGraphDef (variable graph; model description in any_info)
    graph.pbtxt                          text GraphDef of the variable graph

Variable names follow the reference graph: trainables (``conv1/weights``...),
``global_step``, weight-EMA shadows ``<var>/ExponentialMovingAverage``
(``mnist_input.py:265-267``), optimizer slots ``<var>/Momentum``, and the
zero-debiased loss averages ``<loss>/avg`` (+ ``/biased``, ``/local_step``;
``mnist_input.py:288-290``).  ``max_to_keep`` defaults to TF's 5.

``.meta`` is a serialized ``MetaGraphDef`` of the checkpoint's VARIABLE graph
(``ckpt/metagraph.py``: VariableV2 / initializer / Assign / read nodes and the
``variables`` / ``trainable_variables`` / ``global_step`` collections, no
saver_def), so ``tf.train.import_meta_graph`` + a default ``Saver`` can restore the
bundle by name; the model description (architecture, input channels, precision,
mode, step) rides in ``MetaInfoDef.any_info`` as JSON.  ``graph.pbtxt`` is the
text ``GraphDef`` of the same graph.  There is no compute graph to serialize (the
model is a static kernel plan over a ``ModelSpec``) and no TensorFlow in the image
to import the result with: parity unpinned, structure pinned by decoding it
(``tests/test_formats.py``).  The reference's inference (``inference.py:86-91``)
rebuilds its graph from code and reads only the ``checkpoint`` state file +
``.index``/``.data`` bundle, which are written in TF's tensor-bundle format.
"""
from __future__ import annotations

import dataclasses
import os
import re
import time
from typing import Dict, List, Mapping, Optional

import numpy as np

from .bundle import read_bundle, read_index, write_bundle, data_path
from .metagraph import build_meta_graph, graph_pbtxt, trainable_names


@dataclasses.dataclass
class CheckpointState:
    model_checkpoint_path: str
    all_model_checkpoint_paths: List[str]


def _q(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def write_checkpoint_state(train_dir: str, latest: str, all_paths: List[str]) -> None:
    def rel(p: str) -> str:
        return os.path.basename(p) if os.path.dirname(os.path.abspath(p)) == os.path.abspath(train_dir) else p
    lines = [f"model_checkpoint_path: {_q(rel(latest))}"]
    lines += [f"all_model_checkpoint_paths: {_q(rel(p))}" for p in all_paths]
    tmp = os.path.join(train_dir, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(train_dir, "checkpoint"))


def get_checkpoint_state(ckpt_dir: str) -> Optional[CheckpointState]:
    """``tf.train.get_checkpoint_state`` (inference.py:89)."""
    path = os.path.join(ckpt_dir, "checkpoint")
    if not os.path.exists(path):
        return None
    latest, all_paths = None, []
    for line in open(path):
        m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).replace('\\"', '"').replace("\\\\", "\\")
        if not os.path.isabs(v):
            v = os.path.join(ckpt_dir, v)
        if k == "model_checkpoint_path":
            latest = v
        elif k == "all_model_checkpoint_paths":
            all_paths.append(v)
    if latest is None:
        return None
    return CheckpointState(latest, all_paths or [latest])


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    st = get_checkpoint_state(ckpt_dir)
    if st and os.path.exists(st.model_checkpoint_path + ".index"):
        return st.model_checkpoint_path
    return None


class Saver:
    def __init__(self, max_to_keep: int = 5, basename: str = "model.ckpt"):
        self.max_to_keep = max_to_keep
        self.basename = basename

    def save(self, train_dir: str, step: int, tensors: Mapping[str, np.ndarray], meta: Optional[dict] = None,
             num_shards: int = 1, shard_of: Optional[Mapping[str, int]] = None) -> str:
        os.makedirs(train_dir, exist_ok=True)
        prefix = os.path.join(train_dir, f"{self.basename}-{int(step)}")
        write_bundle(prefix, tensors, num_shards=num_shards, shard_of=shard_of)
        meta = dict(meta or {})
        meta.update({"global_step": int(step), "saved_at": time.time(),
                     "variables": {k: [str(np.asarray(v).dtype), list(np.shape(v))] for k, v in tensors.items()}})
        with open(prefix + ".meta", "wb") as f:
            f.write(build_meta_graph(tensors, trainable_names(tensors), meta))
        st = get_checkpoint_state(train_dir)
        paths = [p for p in (st.all_model_checkpoint_paths if st else []) if p != prefix] + [prefix]
        while self.max_to_keep and len(paths) > self.max_to_keep:
            self._delete(paths.pop(0))
        write_checkpoint_state(train_dir, prefix, paths)
        return prefix

    @staticmethod
    def _delete(prefix: str) -> None:
        try:
            n, _ = read_index(prefix)
        except Exception:
            n = 1
        for p in [prefix + ".index", prefix + ".meta"] + [data_path(prefix, s, n) for s in range(n)]:
            if os.path.exists(p):
                os.remove(p)

    @staticmethod
    def restore(prefix: str, names: Optional[list] = None) -> Dict[str, np.ndarray]:
        return read_bundle(prefix, names)


def write_graph_pbtxt(train_dir: str, tensors: Mapping[str, np.ndarray]) -> None:
    """graph.pbtxt: the text GraphDef of the checkpoint's variable graph (ckpt/metagraph.py)."""
    with open(os.path.join(train_dir, "graph.pbtxt"), "w") as f:
        f.write(graph_pbtxt(tensors))
