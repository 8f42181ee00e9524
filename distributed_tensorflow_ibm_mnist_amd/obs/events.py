"""TensorBoard event files (``events.out.tfevents.*``) without TensorFlow.

Replaces ``tf.summary.FileWriter`` (``main.py:78,133-135,155-156``) and the
summary/step-counter output of ``MonitoredTrainingSession`` [TF1-lib].  Records
are TFRecord-framed (native CRC-32C framing) serialized ``Event`` protos:

    Event{wall_time=1 double, step=2 int64, file_version=3 string, summary=5}
    Summary{value=1 repeated Value{tag=1, simple_value=2 float, histo=5}}
    HistogramProto{min=1, max=2, num=3, sum=4, sum_squares=5,
                   bucket_limit=6 packed double, bucket=7 packed double}

Histograms use TF's default bucket edges (±1e-12·1.1^k up to 1e20, plus ±DBL_MAX).
"""
from __future__ import annotations

import os
import socket
import struct
import sys
import time
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..ops._ext import host
from ..utils import proto


def _default_buckets() -> np.ndarray:
    pos = []
    v = 1e-12
    while v < 1e20:
        pos.append(v)
        v *= 1.1
    pos.append(sys.float_info.max)
    neg = [-x for x in reversed(pos)]
    return np.asarray(neg + [0.0] + pos, dtype=np.float64)


BUCKET_LIMITS = _default_buckets()


def scalar_value(tag: str, value: float) -> bytes:
    return proto.f_bytes(1, tag) + proto.f_float(2, float(value))


def histogram_proto(values: np.ndarray) -> bytes:
    v = np.asarray(values, dtype=np.float64).reshape(-1)
    if v.size == 0:
        v = np.zeros(1)
    idx = np.searchsorted(BUCKET_LIMITS, v, side="left")
    counts = np.bincount(idx, minlength=len(BUCKET_LIMITS)).astype(np.float64)
    nz = np.nonzero(counts)[0]
    lo, hi = (nz[0], nz[-1]) if nz.size else (0, 0)
    # TF emits the contiguous bucket range that holds data
    limits = BUCKET_LIMITS[lo:hi + 1]
    buckets = counts[lo:hi + 1]
    return (proto.f_double(1, float(v.min())) + proto.f_double(2, float(v.max())) +
            proto.f_double(3, float(v.size)) + proto.f_double(4, float(v.sum())) +
            proto.f_double(5, float((v * v).sum())) + proto.f_packed_doubles(6, limits) +
            proto.f_packed_doubles(7, buckets))


def histogram_value(tag: str, values: np.ndarray) -> bytes:
    return proto.f_bytes(1, tag) + proto.f_bytes(5, histogram_proto(values))


def summary(values: Sequence[bytes]) -> bytes:
    return b"".join(proto.f_bytes(1, v) for v in values)


def event(step: int, wall_time: Optional[float] = None, summary_bytes: Optional[bytes] = None,
          file_version: Optional[str] = None) -> bytes:
    out = proto.f_double(1, time.time() if wall_time is None else wall_time)
    if step:
        out += proto.f_varint(2, int(step))
    if file_version is not None:
        out += proto.f_bytes(3, file_version)
    if summary_bytes is not None:
        out += proto.f_bytes(5, summary_bytes)
    return out


class EventFileWriter:
    """``tf.summary.FileWriter`` equivalent (chief-only by convention)."""

    def __init__(self, logdir: str, filename_suffix: str = "", flush_secs: float = 120.0):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
                                         f"{filename_suffix}")
        self._pending: List[bytes] = [event(0, file_version="brain.Event:2")]
        self._last_flush = time.time()
        self.flush_secs = flush_secs
        host().tfrecord_write(self.path, [], False)
        self.flush()

    def add_event(self, ev: bytes) -> None:
        self._pending.append(ev)
        if time.time() - self._last_flush > self.flush_secs or len(self._pending) > 256:
            self.flush()

    def add_summary(self, summary_bytes: bytes, global_step: int) -> None:
        self.add_event(event(global_step, summary_bytes=summary_bytes))

    def add_scalars(self, scalars: Dict[str, float], global_step: int) -> None:
        self.add_summary(summary([scalar_value(k, v) for k, v in scalars.items()]), global_step)

    def add_histograms(self, hists: Dict[str, np.ndarray], global_step: int) -> None:
        self.add_summary(summary([histogram_value(k, v) for k, v in hists.items()]), global_step)

    def flush(self) -> None:
        if self._pending:
            host().tfrecord_write(self.path, self._pending, True)
            self._pending = []
        self._last_flush = time.time()

    def close(self) -> None:
        self.flush()


# ------------------------------------------------------------------ reader (tests / tools)
def read_events(path: str) -> Iterator[dict]:
    for rec in host().tfrecord_read(path, True):
        d = proto.to_dict(rec)
        ev = {"wall_time": struct.unpack("<d", d[1][0])[0] if 1 in d else 0.0,
              "step": proto.signed64(d[2][0]) if 2 in d else 0,
              "file_version": d[3][0].decode() if 3 in d else None, "values": {}}
        if 5 in d:
            for f, _, val in proto.fields(d[5][0]):
                if f != 1:
                    continue
                vd = proto.to_dict(val)
                tag = vd[1][0].decode()
                if 2 in vd:
                    ev["values"][tag] = struct.unpack("<f", vd[2][0])[0]
                elif 5 in vd:
                    h = proto.to_dict(vd[5][0])
                    ev["values"][tag] = {
                        "min": struct.unpack("<d", h[1][0])[0], "max": struct.unpack("<d", h[2][0])[0],
                        "num": struct.unpack("<d", h[3][0])[0], "sum": struct.unpack("<d", h[4][0])[0],
                        "bucket": np.frombuffer(h[7][0], dtype="<f8").tolist() if 7 in h else []}
        yield ev


def find_event_files(logdir: str) -> List[str]:
    return sorted(os.path.join(logdir, f) for f in os.listdir(logdir) if f.startswith("events.out.tfevents"))
