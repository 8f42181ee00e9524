"""TF1 ``MetaGraphDef`` (``model.ckpt-N.meta``) and text ``GraphDef`` (``graph.pbtxt``)
for a checkpoint, written with the in-tree protobuf codec (``utils/proto.py``).

The reference's ``MonitoredTrainingSession`` saver writes both files
(``/root/reference/main.py:140-146``).  This framework has no TF graph -- the model
is a static kernel plan -- so the graph written here is the VARIABLE graph of the
checkpoint: for every saved tensor ``v`` the four nodes ``tf.Variable`` creates
(``v`` VariableV2, ``v/Initializer/zeros`` Const, ``v/Assign``, ``v/read``
Identity), the ``variables`` / ``trainable_variables`` / ``global_step``
collections (``VariableDef`` records) and no ``saver_def`` -- so
``tf.train.import_meta_graph`` builds a default ``Saver`` over the imported
variables and ``saver.restore(sess, prefix)`` reads this framework's tensor
bundle by variable name.  The model description the repo's own tools need
(architecture, input channels, precision...) rides in ``MetaInfoDef.any_info`` as
JSON (``read_meta_json``).

Field numbers follow tensorflow/core/protobuf/meta_graph.proto, saver.proto,
framework/{graph,node_def,attr_value,tensor,tensor_shape,types,variable,
versions}.proto (TF 1.15).  Parity unpinned: no TensorFlow is installed to
import the result; ``tests/test_formats.py`` pins the structure by decoding it.
"""
from __future__ import annotations

import json
import struct
from typing import Dict, Iterable, List, Mapping, Optional

import numpy as np

from ..utils.proto import f_bytes, f_varint, to_dict

DT_FLOAT, DT_INT32, DT_INT64 = 1, 3, 9
_DT = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.int64): DT_INT64, np.dtype(np.int32): DT_INT32}
_DT_NAME = {DT_FLOAT: "DT_FLOAT", DT_INT32: "DT_INT32", DT_INT64: "DT_INT64"}
GRAPH_PRODUCER = 134          # TF 1.15 GRAPH_DEF_VERSION
ANY_TYPE_URL = "type.googleapis.com/mnistx.CheckpointMeta"


def _shape(dims: Iterable[int]) -> bytes:           # TensorShapeProto
    return b"".join(f_bytes(2, f_varint(1, int(d))) for d in dims)


def _attr(key: str, value: bytes) -> bytes:         # map<string, AttrValue> entry
    return f_bytes(5, f_bytes(1, key) + f_bytes(2, value))


def _zeros_tensor(dt: int, dims) -> bytes:          # TensorProto: one value broadcast to the shape
    body = f_varint(1, dt) + f_bytes(2, _shape(dims))
    if dt == DT_FLOAT:
        body += f_bytes(5, struct.pack("<f", 0.0))   # packed float_val
    elif dt == DT_INT64:
        body += f_bytes(10, b"\x00")                 # packed int64_val
    else:
        body += f_bytes(7, b"\x00")                  # packed int_val (TensorProto field 7; 6 is double_val)
    return body


def _node(name: str, op: str, inputs: List[str], attrs: List[bytes]) -> bytes:
    return (f_bytes(1, name) + f_bytes(2, op) + b"".join(f_bytes(3, i) for i in inputs) + b"".join(attrs))


def _var_nodes(name: str, dt: int, dims) -> List[bytes]:
    return [
        _node(name, "VariableV2", [], [_attr("shape", f_bytes(7, _shape(dims))), _attr("dtype", f_varint(6, dt)),
                                       _attr("container", f_bytes(2, b"")), _attr("shared_name", f_bytes(2, b""))]),
        _node(f"{name}/Initializer/zeros", "Const", [],
              [_attr("dtype", f_varint(6, dt)), _attr("value", f_bytes(8, _zeros_tensor(dt, dims)))]),
        _node(f"{name}/Assign", "Assign", [name, f"{name}/Initializer/zeros"],
              [_attr("T", f_varint(6, dt)), _attr("validate_shape", f_varint(5, 1)), _attr("use_locking", f_varint(5, 1))]),
        _node(f"{name}/read", "Identity", [name], [_attr("T", f_varint(6, dt))]),
    ]


def _variable_def(name: str, trainable: bool) -> bytes:
    return (f_bytes(1, f"{name}:0") + f_bytes(2, f"{name}/Assign") + f_bytes(3, f"{name}/read:0")
            + f_bytes(6, f"{name}/Initializer/zeros:0") + f_varint(7, 1 if trainable else 0))


def _dtype_of(v) -> int:
    dt = np.asarray(v).dtype
    if dt not in _DT:
        raise ValueError(f"unsupported checkpoint dtype {dt}")
    return _DT[dt]


def build_meta_graph(tensors: Mapping[str, np.ndarray], trainable: Iterable[str], meta: Optional[dict] = None) -> bytes:
    """Serialized MetaGraphDef of the variable graph of `tensors` (+ `meta` as JSON in any_info)."""
    trainable = set(trainable)
    names = sorted(tensors)
    nodes = b"".join(f_bytes(1, n) for name in names
                     for n in _var_nodes(name, _dtype_of(tensors[name]), np.shape(tensors[name])))
    graph = nodes + f_bytes(4, f_varint(1, GRAPH_PRODUCER))           # GraphDef.node*, versions
    any_info = f_bytes(1, ANY_TYPE_URL) + f_bytes(2, json.dumps(meta or {}, sort_keys=True))
    info = f_bytes(1, "") + f_bytes(3, any_info) + f_bytes(5, "1.15.0")  # MetaInfoDef
    colls = []

    def coll(key: str, defs: List[bytes]) -> bytes:               # CollectionDef.bytes_list
        return f_bytes(4, f_bytes(1, key) + f_bytes(2, f_bytes(2, b"".join(f_bytes(1, d) for d in defs))))
    colls.append(coll("variables", [_variable_def(n, n in trainable) for n in names]))
    tr = [n for n in names if n in trainable]
    if tr:
        colls.append(coll("trainable_variables", [_variable_def(n, True) for n in tr]))
    if "global_step" in tensors:
        colls.append(coll("global_step", [_variable_def("global_step", False)]))
    return f_bytes(1, info) + f_bytes(2, graph) + b"".join(colls)


def graph_pbtxt(tensors: Mapping[str, np.ndarray]) -> str:
    """Text-format GraphDef of the same variable graph (what the saver hook's graph.pbtxt holds)."""
    out = []

    def shape_txt(dims) -> str:
        return " ".join(f"dim {{ size: {int(d)} }}" for d in dims)
    for name in sorted(tensors):
        dt = _DT_NAME[_dtype_of(tensors[name])]
        dims = np.shape(tensors[name])
        zero = "float_val: 0.0" if dt == "DT_FLOAT" else "int64_val: 0" if dt == "DT_INT64" else "int_val: 0"
        out.append(f'node {{\n  name: "{name}"\n  op: "VariableV2"\n'
                   f'  attr {{ key: "container" value {{ s: "" }} }}\n'
                   f'  attr {{ key: "dtype" value {{ type: {dt} }} }}\n'
                   f'  attr {{ key: "shape" value {{ shape {{ {shape_txt(dims)} }} }} }}\n'
                   f'  attr {{ key: "shared_name" value {{ s: "" }} }}\n}}')
        out.append(f'node {{\n  name: "{name}/Initializer/zeros"\n  op: "Const"\n'
                   f'  attr {{ key: "dtype" value {{ type: {dt} }} }}\n'
                   f'  attr {{ key: "value" value {{ tensor {{ dtype: {dt} tensor_shape {{ {shape_txt(dims)} }} '
                   f'{zero} }} }} }}\n}}')
        out.append(f'node {{\n  name: "{name}/Assign"\n  op: "Assign"\n  input: "{name}"\n'
                   f'  input: "{name}/Initializer/zeros"\n  attr {{ key: "T" value {{ type: {dt} }} }}\n'
                   f'  attr {{ key: "use_locking" value {{ b: true }} }}\n'
                   f'  attr {{ key: "validate_shape" value {{ b: true }} }}\n}}')
        out.append(f'node {{\n  name: "{name}/read"\n  op: "Identity"\n  input: "{name}"\n'
                   f'  attr {{ key: "T" value {{ type: {dt} }} }}\n}}')
    out.append(f"versions {{\n  producer: {GRAPH_PRODUCER}\n}}")
    return "\n".join(out) + "\n"


def trainable_names(names: Iterable[str]) -> List[str]:
    """The reference's trainables: every layer's weights and biases (mnist_input.py:136-205);
    EMA shadows, optimizer slots, loss averages and global_step are not."""
    return [n for n in names if n.endswith("/weights") or n.endswith("/biases")]


def read_meta_json(path: str) -> Dict:
    """The JSON model description of a checkpoint's .meta: MetaInfoDef.any_info of a
    MetaGraphDef, or (checkpoints of earlier rounds) the whole file as JSON."""
    raw = open(path, "rb").read()
    if raw[:1] in (b"{", b"["):
        return json.loads(raw.decode())
    info = to_dict(to_dict(raw)[1][0])
    anyv = to_dict(info[3][0])
    if anyv.get(1, [b""])[0].decode() != ANY_TYPE_URL:
        return {}
    return json.loads(anyv[2][0].decode())


__all__ = ["build_meta_graph", "graph_pbtxt", "read_meta_json", "trainable_names"]
