"""ONNX protobuf schema (onnx/onnx.proto, IR version 8-9) rebuilt as dynamic
descriptors -- the ``onnx`` package is not installed and no protoc is
needed.  Field numbers / wire types follow the public ONNX IR spec, so files
written here load in any ONNX runtime and ONNX files from elsewhere parse
here.  Nested messages are declared flat (``TypeProto_Tensor`` for
``TypeProto.Tensor``); only names differ, the wire format is identical.
"""
from __future__ import annotations

from typing import Dict

from google.protobuf import descriptor_pb2, descriptor_pool

try:  # protobuf >= 4
    from google.protobuf import message_factory as _mf

    def _get_cls(desc):
        return _mf.GetMessageClass(desc)
except Exception:  # pragma: no cover
    from google.protobuf.message_factory import MessageFactory

    _FACT = MessageFactory()

    def _get_cls(desc):
        return _FACT.GetPrototype(desc)

PKG = "onnx"
O, R = "optional", "repeated"

# TensorProto.DataType
FLOAT, UINT8, INT8, UINT16, INT16, INT32, INT64, STRING, BOOL, FLOAT16, DOUBLE, UINT32, UINT64 = \
    1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13
BFLOAT16 = 16

# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_GRAPH, A_FLOATS, A_INTS, A_STRINGS, A_TENSORS, A_GRAPHS = \
    1, 2, 3, 4, 5, 6, 7, 8, 9, 10

MESSAGES = {
    "StringStringEntryProto": [(O, "string", "key", 1), (O, "string", "value", 2)],
    "OperatorSetIdProto": [(O, "string", "domain", 1), (O, "int64", "version", 2)],
    "TensorShapeProto_Dimension": [(O, "int64", "dim_value", 1), (O, "string", "dim_param", 2),
                                   (O, "string", "denotation", 3)],
    "TensorShapeProto": [(R, "TensorShapeProto_Dimension", "dim", 1)],
    "TypeProto_Tensor": [(O, "int32", "elem_type", 1), (O, "TensorShapeProto", "shape", 2)],
    "TypeProto": [(O, "TypeProto_Tensor", "tensor_type", 1), (O, "string", "denotation", 6)],
    "ValueInfoProto": [(O, "string", "name", 1), (O, "TypeProto", "type", 2), (O, "string", "doc_string", 3)],
    "TensorProto_Segment": [(O, "int64", "begin", 1), (O, "int64", "end", 2)],
    "TensorProto": [
        (R, "int64", "dims", 1), (O, "int32", "data_type", 2), (O, "TensorProto_Segment", "segment", 3),
        (R, "float", "float_data", 4, "packed"), (R, "int32", "int32_data", 5, "packed"),
        (R, "bytes", "string_data", 6), (R, "int64", "int64_data", 7, "packed"), (O, "string", "name", 8),
        (O, "bytes", "raw_data", 9), (R, "double", "double_data", 10, "packed"),
        (R, "uint64", "uint64_data", 11, "packed"), (O, "string", "doc_string", 12),
        (R, "StringStringEntryProto", "external_data", 13), (O, "int32", "data_location", 14)],
    "AttributeProto": [
        (O, "string", "name", 1), (O, "float", "f", 2), (O, "int64", "i", 3), (O, "bytes", "s", 4),
        (O, "TensorProto", "t", 5), (O, "GraphProto", "g", 6), (R, "float", "floats", 7),
        (R, "int64", "ints", 8), (R, "bytes", "strings", 9), (R, "TensorProto", "tensors", 10),
        (R, "GraphProto", "graphs", 11), (O, "string", "doc_string", 13), (O, "int32", "type", 20),
        (O, "string", "ref_attr_name", 21)],
    "NodeProto": [
        (R, "string", "input", 1), (R, "string", "output", 2), (O, "string", "name", 3),
        (O, "string", "op_type", 4), (R, "AttributeProto", "attribute", 5), (O, "string", "doc_string", 6),
        (O, "string", "domain", 7)],
    "GraphProto": [
        (R, "NodeProto", "node", 1), (O, "string", "name", 2), (R, "TensorProto", "initializer", 5),
        (O, "string", "doc_string", 10), (R, "ValueInfoProto", "input", 11), (R, "ValueInfoProto", "output", 12),
        (R, "ValueInfoProto", "value_info", 13)],
    "ModelProto": [
        (O, "int64", "ir_version", 1), (O, "string", "producer_name", 2), (O, "string", "producer_version", 3),
        (O, "string", "domain", 4), (O, "int64", "model_version", 5), (O, "string", "doc_string", 6),
        (O, "GraphProto", "graph", 7), (R, "OperatorSetIdProto", "opset_import", 8),
        (R, "StringStringEntryProto", "metadata_props", 14)],
}

_SCALAR = {
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
}


def _build():
    f = descriptor_pb2.FileDescriptorProto()
    f.name = "singa_amd_onnx.proto"
    f.package = PKG
    f.syntax = "proto2"
    for mname, fields in MESSAGES.items():
        m = f.message_type.add()
        m.name = mname
        for spec in fields:
            label, tname, fname, num = spec[:4]
            fd = m.field.add()
            fd.name, fd.number = fname, num
            fd.label = (descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED if label == R
                        else descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
            if tname in _SCALAR:
                fd.type = _SCALAR[tname]
                if len(spec) > 4 and spec[4] == "packed":
                    fd.options.packed = True
            else:
                fd.type = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
                fd.type_name = f".{PKG}.{tname}"
    return f


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(_build())
_CLS: Dict[str, type] = {}


def cls(name: str) -> type:
    if name not in _CLS:
        _CLS[name] = _get_cls(_POOL.FindMessageTypeByName(f"{PKG}.{name}"))
    return _CLS[name]


def new(name: str):
    return cls(name)()


def load_model(path_or_bytes) -> object:
    """Parse an ONNX ModelProto (protobuf wire format; nothing is executed)."""
    m = new("ModelProto")
    if isinstance(path_or_bytes, (bytes, bytearray)):
        m.ParseFromString(bytes(path_or_bytes))
    else:
        with open(path_or_bytes, "rb") as f:
            m.ParseFromString(f.read())
    return m


def save_model(m, path: str) -> None:
    with open(path, "wb") as f:
        f.write(m.SerializeToString())
