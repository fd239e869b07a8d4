"""ONNX model files without onnx / onnxruntime: a minimal protobuf schema of the ONNX IR (ModelProto,
GraphProto, NodeProto, AttributeProto, TensorProto — field numbers from onnx/onnx.proto3, the public
IR spec) assembled at run time like grpc/schema.py does for backend.proto, then decoded with the
protobuf runtime that ships with grpcio.

Used to read the weights (graph initializers, recursively through If / Loop subgraphs and Constant
nodes) of the gallery's ONNX checkpoints — silero-vad (backend/go/vad/silero/vad.go:15-54 loads
silero_vad.onnx) — into state dicts for this framework's own kernels. No ONNX graph is executed:
the model's math is re-implemented natively (models/vad.py); parity against onnxruntime is unpinned
(no onnxruntime in this image).
"""
from __future__ import annotations

import numpy as np

_PKG = "mxonnx"
# (message, [(field, number, type, label)]) ; type: scalar name or message name
_SCHEMA = {
    "TensorProto": [("dims", 1, "int64", "repeated"), ("data_type", 2, "int32", ""),
                    ("float_data", 4, "float", "repeated"), ("int32_data", 5, "int32", "repeated"),
                    ("string_data", 6, "bytes", "repeated"), ("int64_data", 7, "int64", "repeated"),
                    ("name", 8, "string", ""), ("raw_data", 9, "bytes", ""), ("double_data", 10, "double", "repeated"),
                    ("uint64_data", 11, "uint64", "repeated"), ("doc_string", 12, "string", ""),
                    ("data_location", 14, "int32", "")],
    "AttributeProto": [("name", 1, "string", ""), ("f", 2, "float", ""), ("i", 3, "int64", ""), ("s", 4, "bytes", ""),
                       ("t", 5, "TensorProto", ""), ("g", 6, "GraphProto", ""), ("floats", 7, "float", "repeated"),
                       ("ints", 8, "int64", "repeated"), ("strings", 9, "bytes", "repeated"),
                       ("tensors", 10, "TensorProto", "repeated"), ("graphs", 11, "GraphProto", "repeated"),
                       ("doc_string", 13, "string", ""), ("type", 20, "int32", ""), ("ref_attr_name", 21, "string", "")],
    "NodeProto": [("input", 1, "string", "repeated"), ("output", 2, "string", "repeated"), ("name", 3, "string", ""),
                  ("op_type", 4, "string", ""), ("attribute", 5, "AttributeProto", "repeated"),
                  ("doc_string", 6, "string", ""), ("domain", 7, "string", "")],
    "GraphProto": [("node", 1, "NodeProto", "repeated"), ("name", 2, "string", ""),
                   ("initializer", 5, "TensorProto", "repeated"), ("doc_string", 10, "string", "")],
    "OperatorSetIdProto": [("domain", 1, "string", ""), ("version", 2, "int64", "")],
    "ModelProto": [("ir_version", 1, "int64", ""), ("producer_name", 2, "string", ""),
                   ("producer_version", 3, "string", ""), ("domain", 4, "string", ""), ("model_version", 5, "int64", ""),
                   ("doc_string", 6, "string", ""), ("graph", 7, "GraphProto", ""),
                   ("opset_import", 8, "OperatorSetIdProto", "repeated")],
}
_SCALAR = {"double": 1, "float": 2, "int64": 3, "uint64": 4, "int32": 5, "bool": 8, "string": 9, "bytes": 12}
# TensorProto.DataType -> numpy
DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
          9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}
_CLASSES = None


def _classes():
    global _CLASSES
    if _CLASSES is None:
        from google.protobuf import descriptor_pb2 as d
        from google.protobuf import descriptor_pool, message_factory
        fd = d.FileDescriptorProto(name="mx_onnx_subset.proto", package=_PKG, syntax="proto2")
        for mname, fields in _SCHEMA.items():
            m = fd.message_type.add(name=mname)
            for name, num, typ, label in fields:
                f = m.field.add(name=name, number=num)
                f.label = 3 if label == "repeated" else 1
                if typ in _SCALAR:
                    f.type = _SCALAR[typ]
                    if label == "repeated" and typ not in ("string", "bytes"):
                        f.options.packed = True  # ONNX writes repeated numerics packed
                else:
                    f.type = 11
                    f.type_name = f".{_PKG}.{typ}"
        pool = descriptor_pool.DescriptorPool()
        pool.Add(fd)
        _CLASSES = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{n}")) for n in _SCHEMA}
    return _CLASSES


def tensor_to_numpy(t) -> np.ndarray:
    dt = DTYPES.get(int(t.data_type))
    if dt is None:
        raise ValueError(f"ONNX tensor {t.name!r}: unsupported data type {t.data_type}")
    shape = tuple(int(x) for x in t.dims)
    if t.data_location == 1:
        raise ValueError(f"ONNX tensor {t.name!r} keeps its data in an external file")
    if t.raw_data:
        a = np.frombuffer(t.raw_data, dtype=np.dtype(dt).newbyteorder("<"))
    elif dt == np.float32:
        a = np.asarray(t.float_data, np.float32)
    elif dt == np.float64:
        a = np.asarray(t.double_data, np.float64)
    elif dt in (np.int64,):
        a = np.asarray(t.int64_data, np.int64)
    elif dt in (np.uint64, np.uint32):
        a = np.asarray(t.uint64_data, dt)
    elif dt == np.float16:  # stored as uint16 bit patterns in int32_data
        a = np.asarray(t.int32_data, np.uint16).view(np.float16)
    else:
        a = np.asarray(t.int32_data).astype(dt)
    return a.reshape(shape).copy() if shape else a.reshape(()).copy()


def load_model(path_or_bytes):
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    m = _classes()["ModelProto"]()
    m.ParseFromString(bytes(data))
    return m


def _walk(graph, prefix: str, out: dict, nodes: list):
    for t in graph.initializer:
        out[prefix + t.name] = tensor_to_numpy(t)
    for n in graph.node:
        nodes.append((prefix, n))
        for a in n.attribute:
            if n.op_type == "Constant" and a.name == "value" and a.HasField("t"):
                out[prefix + (n.output[0] if n.output else a.t.name)] = tensor_to_numpy(a.t)
            if a.HasField("g"):
                _walk(a.g, f"{prefix}{n.name or n.op_type}/{a.name}/", out, nodes)
            for i, g in enumerate(a.graphs):
                _walk(g, f"{prefix}{n.name or n.op_type}/{a.name}{i}/", out, nodes)


def initializers(path_or_bytes) -> tuple[dict[str, np.ndarray], list]:
    """-> ({qualified name: array} of every initializer / Constant, [(scope, NodeProto)] of every node).
    Subgraph tensors are qualified "<node>/<attr>/<name>" (If branches: then_branch / else_branch)."""
    m = load_model(path_or_bytes)
    out: dict[str, np.ndarray] = {}
    nodes: list = []
    _walk(m.graph, "", out, nodes)
    return out, nodes


def make_model(tensors: dict[str, np.ndarray], subgraph: dict[str, np.ndarray] | None = None) -> bytes:
    """Serialise a weights-only ONNX model (tests / converters): `tensors` as graph initializers and,
    optionally, `subgraph` inside an If node's then_branch (the silero-vad v5 layout)."""
    C = _classes()
    rev = {v: k for k, v in DTYPES.items()}

    def tp(name, a):
        a = np.ascontiguousarray(a)
        t = C["TensorProto"](name=name, data_type=rev[a.dtype.type], raw_data=a.astype(a.dtype.newbyteorder("<")).tobytes())
        t.dims.extend(a.shape)
        return t

    g = C["GraphProto"](name="main")
    g.initializer.extend(tp(k, v) for k, v in tensors.items())
    if subgraph:
        sub = C["GraphProto"](name="then")
        sub.initializer.extend(tp(k, v) for k, v in subgraph.items())
        node = g.node.add(op_type="If", name="If_0")
        node.attribute.add(name="then_branch", type=5, g=sub)
    m = C["ModelProto"](ir_version=8, producer_name="localai_tfp_amd", graph=g)
    m.opset_import.add(domain="", version=16)
    return m.SerializeToString()
