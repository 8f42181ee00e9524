"""Minimal protobuf wire-format codec.

TensorFlow's .proto files are not available here (no TF install), so the few
messages the framework must read/write byte-compatibly are encoded by hand:
``tf.Example`` (TFRecord datasets, ``mnist_input.py:27-33``), ``Event`` /
``Summary`` / ``HistogramProto`` (event files, ``main.py:78,133``),
``BundleHeaderProto`` / ``BundleEntryProto`` (tensor-bundle checkpoints) and
``CheckpointState`` (the ``checkpoint`` text file).
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Tuple, Union

WT_VARINT, WT_I64, WT_LEN, WT_I32 = 0, 1, 2, 5


def varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def key(field: int, wt: int) -> bytes:
    return varint((field << 3) | wt)


def f_varint(field: int, v: int) -> bytes:
    return key(field, WT_VARINT) + varint(int(v))


def f_bytes(field: int, b: Union[bytes, str]) -> bytes:
    if isinstance(b, str):
        b = b.encode()
    return key(field, WT_LEN) + varint(len(b)) + b


def f_double(field: int, v: float) -> bytes:
    return key(field, WT_I64) + struct.pack("<d", v)


def f_float(field: int, v: float) -> bytes:
    return key(field, WT_I32) + struct.pack("<f", v)


def f_fixed32(field: int, v: int) -> bytes:
    return key(field, WT_I32) + struct.pack("<I", v & 0xFFFFFFFF)


def f_packed_doubles(field: int, vals) -> bytes:
    body = b"".join(struct.pack("<d", float(v)) for v in vals)
    return f_bytes(field, body)


def f_packed_varints(field: int, vals) -> bytes:
    return f_bytes(field, b"".join(varint(int(v)) for v in vals))


def read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = 0
    v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def fields(b: bytes) -> Iterator[Tuple[int, int, Union[int, bytes]]]:
    """Yield (field, wire_type, value) for a serialized message."""
    i = 0
    n = len(b)
    while i < n:
        k, i = read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == WT_VARINT:
            v, i = read_varint(b, i)
        elif wt == WT_I64:
            v = b[i:i + 8]
            i += 8
        elif wt == WT_LEN:
            ln, i = read_varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == WT_I32:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, wt, v


def to_dict(b: bytes) -> Dict[int, List]:
    d: Dict[int, List] = {}
    for f, _, v in fields(b):
        d.setdefault(f, []).append(v)
    return d


def signed64(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v
