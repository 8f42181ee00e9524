"""TFRecord + ``tf.Example`` I/O (replaces TFRecordReader / ParseSingleExample).

Record schema of the reference (``mnist_input.py:29-33``, ``inference.py:52-56``):
``{'image_raw': bytes (uint8 pixels), 'label': int64}``.  DLI's converter wrote
28×28×3 images (2352 bytes, ``mnist_input.py:13-15``); 784-byte grayscale
records are accepted too (the channel count is inferred from the record size).

Framing and CRC-32C are native (``csrc/host/runtime.cpp``); decoding a whole
file set is one multi-threaded C++ call.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Iterable, List, Sequence, Tuple, Union

import numpy as np

from ..ops._ext import host
from ..utils import proto


def encode_example(features: Dict[str, Union[bytes, int, Sequence[int], Sequence[float]]]) -> bytes:
    """Serialize a tf.train.Example (Features map of Bytes/Int64/Float lists)."""
    entries = []
    for name in sorted(features):
        v = features[name]
        if isinstance(v, (bytes, bytearray)):
            feat = proto.f_bytes(1, proto.f_bytes(1, bytes(v)))                 # BytesList
        elif isinstance(v, (int, np.integer)):
            feat = proto.f_bytes(3, proto.f_packed_varints(1, [int(v)]))        # Int64List
        elif len(v) and isinstance(v[0], float):
            feat = proto.f_bytes(2, proto.f_bytes(1, np.asarray(v, dtype="<f4").tobytes()))  # FloatList (packed)
        else:
            feat = proto.f_bytes(3, proto.f_packed_varints(1, [int(x) for x in v]))
        entry = proto.f_bytes(1, name) + proto.f_bytes(2, feat)
        entries.append(proto.f_bytes(1, entry))
    return proto.f_bytes(1, b"".join(entries))


def decode_example(b: bytes) -> Dict[str, Union[bytes, List[int], List[float]]]:
    """Python decoder (tests / tools); bulk decoding uses the C++ path."""
    out: Dict[str, Union[bytes, List[int], List[float]]] = {}
    for f, _, feats in proto.fields(b):
        if f != 1:
            continue
        for f2, _, entry in proto.fields(feats):
            if f2 != 1:
                continue
            d = proto.to_dict(entry)
            name = d[1][0].decode()
            feature = proto.to_dict(d[2][0])
            if 1 in feature:
                vals = proto.to_dict(feature[1][0]).get(1, [])
                out[name] = vals[0] if len(vals) == 1 else list(vals)
            elif 3 in feature:
                ints: List[int] = []
                for ff, wt, v in proto.fields(feature[3][0]):
                    if wt == proto.WT_LEN:
                        i = 0
                        while i < len(v):
                            x, i = proto.read_varint(v, i)
                            ints.append(proto.signed64(x))
                    else:
                        ints.append(proto.signed64(v))
                out[name] = ints
            elif 2 in feature:
                floats: List[float] = []
                for ff, wt, v in proto.fields(feature[2][0]):
                    floats.extend(np.frombuffer(v, dtype="<f4").tolist())
                out[name] = floats
    return out


class TFRecordWriter:
    def __init__(self, path: str, append: bool = False):
        self.path = path
        self._buf: List[bytes] = []
        if not append:
            host().tfrecord_write(path, [], False)

    def write(self, record: bytes) -> None:
        self._buf.append(record)
        if len(self._buf) >= 1024:
            self.flush()

    def flush(self) -> None:
        if self._buf:
            host().tfrecord_write(self.path, self._buf, True)
            self._buf = []

    def close(self) -> None:
        self.flush()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read_records(path: str, verify: bool = True) -> List[bytes]:
    return host().tfrecord_read(path, verify)


def expand(paths: Iterable[str]) -> List[str]:
    out: List[str] = []
    for p in paths:
        hits = sorted(glob.glob(p))
        if not hits and not os.path.exists(p):
            raise ValueError("Failed to find file: " + p)   # mnist_input.py:53-55
        out.extend(hits or [p])
    return out


def load_mnist_tfrecords(paths: Sequence[str], threads: int = 4) -> Tuple[np.ndarray, np.ndarray, int]:
    """Returns (images uint8 [N, HW*C], labels int32 [N], channels)."""
    files = expand(paths)
    blob, labels, per = host().decode_mnist_files(files, "image_raw", "label", True, threads)
    n = len(labels)
    if per % 784 != 0:
        raise ValueError(f"image_raw has {per} bytes; expected a multiple of 784 (28x28xC)")
    imgs = np.frombuffer(blob, dtype=np.uint8).reshape(n, per)
    return imgs, np.asarray(labels, dtype=np.int32), per // 784


def write_mnist_tfrecords(path: str, images: np.ndarray, labels: np.ndarray) -> None:
    """Write records in the reference/DLI schema (image_raw bytes + int64 label)."""
    with TFRecordWriter(path) as w:
        for img, lab in zip(images, labels):
            w.write(encode_example({"image_raw": np.ascontiguousarray(img, dtype=np.uint8).tobytes(),
                                    "label": int(lab)}))
