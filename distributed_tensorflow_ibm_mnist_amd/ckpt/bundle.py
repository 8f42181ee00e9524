"""TensorFlow tensor-bundle checkpoint format (``.index`` SSTable + ``.data-*``).

The reference checkpoints through ``MonitoredTrainingSession(checkpoint_dir=...)``
(``main.py:140-146``) and restores with ``Saver().restore`` (``inference.py:
86-91``).  To keep the *same layout*  without TensorFlow, this
module writes the bundle format byte-for-byte:

* ``<prefix>.index``: leveldb-format SSTable (built natively, ``_host.
  sstable_build``) mapping ``""`` → ``BundleHeaderProto`` and each tensor name →
  ``BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c}``;
* ``<prefix>.data-0000i-of-0000N``: raw little-endian tensor bytes; with N>1
  (parameter-server mode) each PS shard owns one data file (P4).

Only uncompressed blocks are produced/accepted (TF readers handle both).
"""
from __future__ import annotations

import os
from typing import Dict, Mapping, Optional, Tuple

import numpy as np

from ..ops._ext import host
from ..utils import proto

# tensorflow/core/framework/types.proto
DTYPES = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
          np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
          np.dtype(np.float16): 19}
DT_BFLOAT16 = 14
NP_OF = {v: k for k, v in DTYPES.items()}


def data_path(prefix: str, shard: int, num_shards: int) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def _header(num_shards: int) -> bytes:
    # BundleHeaderProto{num_shards=1, endianness=LITTLE(0), version=VersionDef{producer=1}}
    return proto.f_varint(1, num_shards) + proto.f_bytes(3, proto.f_varint(1, 1))


def _entry(dtype: int, shape: Tuple[int, ...], shard: int, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(proto.f_bytes(2, proto.f_varint(1, d)) for d in shape)
    out = proto.f_varint(1, dtype) + proto.f_bytes(2, dims)
    if shard:
        out += proto.f_varint(3, shard)
    if offset:
        out += proto.f_varint(4, offset)
    out += proto.f_varint(5, size) + proto.f_fixed32(6, crc)
    return out


def write_bundle(prefix: str, tensors: Mapping[str, np.ndarray], num_shards: int = 1,
                 shard_of: Optional[Mapping[str, int]] = None) -> None:
    """Write ``prefix.index`` + data shard(s).  ``shard_of`` maps name -> shard."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)) or ".", exist_ok=True)
    H = host()
    names = sorted(tensors)
    blobs = [bytearray() for _ in range(num_shards)]
    entries = [(b"", _header(num_shards))]
    for name in names:
        a = np.asarray(tensors[name], order="C")  # (ascontiguousarray would make 0-d scalars 1-d)
        if a.dtype.byteorder == ">":
            a = a.astype(a.dtype.newbyteorder("<"))
        if a.dtype not in DTYPES:
            raise TypeError(f"{name}: unsupported dtype {a.dtype}")
        shard = int(shard_of.get(name, 0)) if shard_of else 0
        raw = a.tobytes()
        off = len(blobs[shard])
        blobs[shard] += raw
        entries.append((name.encode(), _entry(DTYPES[a.dtype], tuple(a.shape), shard, off, len(raw),
                                              H.masked_crc32c(raw))))
    for s in range(num_shards):
        tmp = data_path(prefix, s, num_shards) + ".tempstate"
        with open(tmp, "wb") as f:
            f.write(bytes(blobs[s]))
        os.replace(tmp, data_path(prefix, s, num_shards))
    tmp = prefix + ".index.tempstate"
    with open(tmp, "wb") as f:
        f.write(H.sstable_build(entries))
    os.replace(tmp, prefix + ".index")


def read_index(prefix: str) -> Tuple[int, Dict[str, dict]]:
    with open(prefix + ".index", "rb") as f:
        kv = host().sstable_parse(f.read(), True)
    num_shards = 1
    out: Dict[str, dict] = {}
    for k, v in kv:
        d = proto.to_dict(v)
        if k == b"":
            num_shards = d.get(1, [1])[0]
            continue
        shape = []
        if 2 in d:
            for f, _, dim in proto.fields(d[2][0]):
                if f == 2:
                    shape.append(proto.to_dict(dim).get(1, [0])[0])
        out[k.decode()] = {
            "dtype": d.get(1, [0])[0], "shape": tuple(shape), "shard": d.get(3, [0])[0],
            "offset": d.get(4, [0])[0], "size": d.get(5, [0])[0],
            "crc32c": int.from_bytes(d[6][0], "little") if 6 in d else None,
        }
    return num_shards, out


def read_bundle(prefix: str, names: Optional[list] = None, verify: bool = True) -> Dict[str, np.ndarray]:
    num_shards, index = read_index(prefix)
    data: Dict[int, bytes] = {}
    out: Dict[str, np.ndarray] = {}
    H = host()
    for name, e in index.items():
        if names is not None and name not in names:
            continue
        s = e["shard"]
        if s not in data:
            with open(data_path(prefix, s, num_shards), "rb") as f:
                data[s] = f.read()
        raw = data[s][e["offset"]:e["offset"] + e["size"]]
        if verify and e["crc32c"] is not None and H.masked_crc32c(raw) != e["crc32c"]:
            raise IOError(f"checksum mismatch for {name} in {prefix}")
        if e["dtype"] not in NP_OF:
            raise TypeError(f"{name}: unsupported dtype enum {e['dtype']}")
        out[name] = np.frombuffer(raw, dtype=NP_OF[e["dtype"]]).reshape(e["shape"]).copy()
    return out
