"""Configuration schemas (reference C2, src/proto/{model,cluster,topology}.proto)
rebuilt as dynamic protobuf descriptors -- no protoc needed.

Field names, numbers, labels, types and proto2 defaults match the reference
exactly so its text-format ``.conf`` files (examples/mnist/*.conf) parse
unchanged through ``google.protobuf.text_format``.  The schema is declared
here as compact tables and turned into a ``FileDescriptorProto`` at import.

Usage::

    from singa_amd.config import schema
    model = schema.parse_text("ModelProto", open("mlp.conf").read())
    model.updater.base_learning_rate
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, text_format

try:  # protobuf >= 4
    from google.protobuf import message_factory as _mf

    def _get_cls(desc):
        return _mf.GetMessageClass(desc)
except Exception:  # pragma: no cover
    from google.protobuf.message_factory import MessageFactory

    _FACT = MessageFactory()

    def _get_cls(desc):
        return _FACT.GetPrototype(desc)

PKG = "singa"
O, R, Q = "optional", "repeated", "required"

# enum tables: name -> [(value_name, number)]
ENUMS_TOP: Dict[str, List[Tuple[str, int]]] = {
    "Phase": [("kTrain", 0), ("kValidation", 1), ("kTest", 2)],
    "PartitionType": [("kDataPartition", 0), ("kLayerPartition", 1), ("kNone", 2)],
    "ConnectionType": [("kOneToOne", 0), ("kOneToAll", 1)],
}
NESTED_ENUMS: Dict[str, Dict[str, List[Tuple[str, int]]]] = {
    "ModelProto": {"GradCalcAlg": [("kBackPropagation", 1), ("kContrastiveDivergence", 2)]},
    "ParamProto": {"InitMethod": [("kConstant", 0), ("kGaussain", 1), ("kUniform", 2), ("kPretrained", 3),
                                  ("kGaussainSqrtFanIn", 4), ("kUniformSqrtFanIn", 5),
                                  ("kUniformSqrtFanInOut", 6)]},
    "Record": {"Type": [("kSingleLabelImage", 0)]},
    "UpdaterProto": {"Type": [("kAdaGrad", 1), ("kAdaDelta", 2), ("kNesterov", 3), ("kSGD", 4), ("kRMSProp", 5)],
                     "ChangeProto": [("kFixed", 0), ("kInverse_t", 1), ("kInverse", 2), ("kExponential", 3),
                                     ("kLinear", 4), ("kStep", 5)]},
    "LRNProto": {"NormRegion": [("ACROSS_CHANNELS", 0), ("WITHIN_CHANNEL", 1)]},
    "PoolingProto": {"PoolMethod": [("MAX", 0), ("AVE", 1)]},
}

# message tables: name -> [(label, type, field, number, default)]
MESSAGES: Dict[str, List[Tuple]] = {
    "ModelProto": [
        (O, "string", "name", 1, None), (O, "string", "train_folder", 2, "train"),
        (O, "string", "test_folder", 3, "test"), (O, "string", "validation_folder", 4, "validation"),
        (O, "int32", "display_after_steps", 6, 0), (O, "int32", "display_frequency", 7, 0),
        (O, "int32", "validation_after_steps", 10, 0), (O, "int32", "validation_frequency", 11, 0),
        (O, "int32", "test_after_steps", 13, 0), (O, "int32", "test_frequency", 14, 0),
        (O, "bool", "prefetch", 15, True), (O, "int32", "train_steps", 20, None),
        (O, "int32", "validation_steps", 21, None), (O, "int32", "test_steps", 22, None),
        (O, "int32", "step", 29, 0), (O, "UpdaterProto", "updater", 31, None),
        (O, "ModelProto.GradCalcAlg", "alg", 32, "kBackPropagation"), (O, "NetProto", "neuralnet", 40, None),
        (O, "bool", "debug", 41, False),
    ],
    "NetProto": [(R, "LayerProto", "layer", 1, None), (O, "PartitionType", "partition_type", 3, "kNone")],
    "ParamProto": [
        (O, "string", "name", 1, None), (O, "int32", "id", 2, None), (R, "int32", "shape", 3, None),
        (O, "int32", "split_threshold", 4, 5000000), (O, "int32", "partition_dim", 5, -1),
        (O, "ParamProto.InitMethod", "init_method", 7, "kConstant"), (O, "float", "value", 8, 1.0),
        (O, "float", "low", 9, -1.0), (O, "float", "high", 10, 1.0), (O, "float", "mean", 11, 0.0),
        (O, "float", "std", 12, 1.0), (O, "float", "learning_rate_multiplier", 13, 1.0),
        (O, "float", "weight_decay_multiplier", 14, 1.0),
    ],
    "LayerProto": [
        (O, "string", "name", 1, None), (O, "string", "type", 2, None), (R, "string", "srclayers", 3, None),
        (O, "int32", "locationid", 4, 0), (O, "int32", "partitionid", 5, 0),
        (O, "PartitionType", "partition_type", 6, None), (R, "string", "share_ary", 11, None),
        (R, "ParamProto", "param", 12, None), (R, "string", "share_param", 13, None),
        (R, "Phase", "exclude", 20, None),
        (O, "ConvolutionProto", "convolution_param", 21, None), (O, "ConcateProto", "concate_param", 31, None),
        (O, "DataProto", "data_param", 22, None), (O, "DropoutProto", "dropout_param", 23, None),
        (O, "InnerProductProto", "inner_product_param", 24, None), (O, "LRNProto", "lrn_param", 25, None),
        (O, "MnistProto", "mnist_param", 26, None), (O, "PoolingProto", "pooling_param", 27, None),
        (O, "SliceProto", "slice_param", 32, None), (O, "SplitProto", "split_param", 33, None),
        (O, "ReLUProto", "relu_param", 28, None), (O, "RGBImage", "rgbimage_param", 34, None),
        (O, "SoftmaxLossProto", "softmaxloss_param", 29, None), (O, "TanhProto", "tanh_param", 30, None),
    ],
    "RGBImage": [(O, "float", "scale", 1, 1.0), (O, "int32", "cropsize", 2, 0), (O, "bool", "mirror", 3, False)],
    "SplitProto": [(O, "int32", "num_splits", 1, None)],
    "TanhProto": [(O, "float", "outer_scale", 1, 1.0), (O, "float", "inner_scale", 2, 1.0)],
    "SoftmaxLossProto": [(O, "int32", "topk", 1, 1), (O, "float", "scale", 2, 1.0)],
    "ConvolutionProto": [
        (O, "uint32", "num_filters", 1, None), (O, "bool", "bias_term", 2, True), (O, "uint32", "pad", 3, 0),
        (O, "uint32", "stride", 4, 1), (Q, "uint32", "kernel", 5, None),
    ],
    "ConcateProto": [(O, "int32", "concate_dimension", 1, None), (O, "int32", "concate_num", 2, None)],
    "DataProto": [(O, "string", "source", 1, None), (O, "string", "path", 2, None),
                  (O, "uint32", "batchsize", 4, None), (O, "uint32", "random_skip", 5, 0)],
    "MnistProto": [
        (O, "int32", "kernel", 1, 0), (O, "float", "sigma", 2, 0.0), (O, "float", "alpha", 3, 0.0),
        (O, "float", "beta", 4, 0.0), (O, "float", "gamma", 5, 0.0), (O, "int32", "resize", 6, 0),
        (O, "int32", "elastic_freq", 7, 0), (O, "float", "norm_a", 8, 1.0), (O, "float", "norm_b", 9, 0.0),
    ],
    "DropoutProto": [(O, "float", "dropout_ratio", 1, 0.5)],
    "InnerProductProto": [(O, "uint32", "num_output", 1, None), (O, "bool", "bias_term", 2, True)],
    "LRNProto": [(O, "uint32", "local_size", 1, 5), (O, "float", "alpha", 2, 1.0), (O, "float", "beta", 3, 0.75),
                 (O, "LRNProto.NormRegion", "norm_region", 4, "ACROSS_CHANNELS"), (O, "float", "knorm", 5, 1.0)],
    "PoolingProto": [(O, "PoolingProto.PoolMethod", "pool", 1, "MAX"), (Q, "uint32", "kernel", 2, None),
                     (O, "uint32", "pad", 4, 0), (O, "uint32", "stride", 3, 1)],
    "SliceProto": [(O, "int32", "slice_dimension", 1, None), (O, "int32", "slice_num", 2, None)],
    "ReLUProto": [(O, "float", "negative_slope", 1, 0.0)],
    "Record": [(O, "Record.Type", "type", 1, "kSingleLabelImage"), (O, "SingleLabelImageRecord", "image", 2, None)],
    "Datum": [(O, "int32", "channels", 1, None), (O, "int32", "height", 2, None), (O, "int32", "width", 3, None),
              (O, "bytes", "data", 4, None), (O, "int32", "label", 5, None), (R, "float", "float_data", 6, None),
              (O, "bool", "encoded", 7, False)],
    "SingleLabelImageRecord": [(R, "int32", "shape", 1, None), (O, "int32", "label", 2, None),
                               (O, "bytes", "pixel", 3, None), (R, "float", "data", 4, None)],
    "UpdaterProto": [
        (O, "UpdaterProto.Type", "type", 1, "kAdaGrad"), (O, "bool", "hogwild", 2, True),
        (O, "float", "momentum", 4, 0.0), (O, "float", "weight_decay", 5, 0.0), (O, "float", "gamma", 6, 1.0),
        (O, "float", "pow", 7, 0.0), (O, "float", "delta", 8, 0.0000001), (O, "float", "rho", 9, 0.9),
        (O, "float", "base_learning_rate", 12, None), (O, "float", "final_learning_rate", 13, None),
        (O, "int32", "learning_rate_change_frequency", 14, None),
        (O, "UpdaterProto.ChangeProto", "learning_rate_change_method", 16, "kFixed"),
        (O, "int32", "sync_frequency", 17, 1), (O, "int32", "warmup_steps", 25, 10),
        (O, "float", "moving_rate", 26, 0.0), (O, "string", "param_type", 27, "Elastic"),
    ],
    "BlobProto": [(O, "int32", "num", 1, 0), (O, "int32", "channels", 2, 0), (O, "int32", "height", 3, 0),
                  (O, "int32", "width", 4, 0), (R, "float", "data", 5, "packed"), (R, "float", "diff", 6, "packed")],
    # cluster.proto
    "ClusterProto": [
        (O, "int32", "nworkers", 1, None), (O, "int32", "nservers", 2, None), (O, "int32", "start_port", 3, 6723),
        (O, "int32", "nprocs_per_group", 5, 1), (O, "int32", "nthreads_per_procs", 6, 1),
        (O, "int32", "nthreads_per_server", 7, 1), (Q, "string", "workspace", 10, None),
        (O, "string", "vis_subfolder", 11, "vis"), (O, "string", "log_subfolder", 12, "log"),
        (O, "bool", "synchronous", 15, False), (O, "int32", "largest_message", 20, 1048576),
        (O, "float", "bandwidth", 21, 100.0),
    ],
    # topology.proto (pm prototype)
    "Topology": [(Q, "int32", "nservers", 2, None), (Q, "int32", "nworker_groups", 3, None),
                 (R, "int32", "nserver_groups", 4, None), (R, "ServerGroup", "server_group", 5, None),
                 (Q, "int32", "port", 6, None), (Q, "int32", "server_threads", 7, None),
                 (Q, "int32", "worker_threads", 8, None)],
    "ServerGroup": [(Q, "int32", "id", 9, None), (Q, "int32", "sync_interval", 10, None),
                    (R, "int32", "neighbor", 11, None)],
}

_SCALAR = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
}
_LABEL = {O: descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL,
          R: descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED,
          Q: descriptor_pb2.FieldDescriptorProto.LABEL_REQUIRED}


def _is_enum(tname: str) -> bool:
    if tname in ENUMS_TOP:
        return True
    if "." in tname:
        m, e = tname.split(".", 1)
        return e in NESTED_ENUMS.get(m, {})
    return False


def _fmt_default(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    f = descriptor_pb2.FileDescriptorProto()
    f.name = "singa_amd_config.proto"
    f.package = PKG
    f.syntax = "proto2"
    for ename, vals in ENUMS_TOP.items():
        e = f.enum_type.add()
        e.name = ename
        for vn, num in vals:
            v = e.value.add()
            v.name, v.number = vn, num
    for mname, fields in MESSAGES.items():
        m = f.message_type.add()
        m.name = mname
        for ename, vals in NESTED_ENUMS.get(mname, {}).items():
            e = m.enum_type.add()
            e.name = ename
            for vn, num in vals:
                v = e.value.add()
                v.name, v.number = vn, num
        for label, tname, fname, num, default in fields:
            fd = m.field.add()
            fd.name, fd.number, fd.label = fname, num, _LABEL[label]
            if tname in _SCALAR:
                fd.type = _SCALAR[tname]
                if default == "packed":
                    fd.options.packed = True
                elif default is not None:
                    fd.default_value = _fmt_default(default)
            elif _is_enum(tname):
                fd.type = descriptor_pb2.FieldDescriptorProto.TYPE_ENUM
                fd.type_name = f".{PKG}.{tname}"
                if default is not None:
                    fd.default_value = str(default)
            else:
                fd.type = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
                fd.type_name = f".{PKG}.{tname}"
    return f


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_build_file())
_CLASSES: Dict[str, type] = {}


def message_class(name: str) -> type:
    if name not in _CLASSES:
        _CLASSES[name] = _get_cls(_POOL.FindMessageTypeByName(f"{PKG}.{name}"))
    return _CLASSES[name]


def new(name: str):
    return message_class(name)()


def parse_text(name: str, text: str):
    """Parse a text-format message (``#`` comments allowed)."""
    msg = new(name)
    text_format.Parse(text, msg)
    return msg


def read_text_file(name: str, path: str):
    """ReadProtoFromTextFile (reference src/utils/common.cc:56-63)."""
    with open(path, "r") as fh:
        return parse_text(name, fh.read())


def to_text(msg) -> str:
    return text_format.MessageToString(msg)


def enum_name(msg, field: str) -> str:
    fd = msg.DESCRIPTOR.fields_by_name[field]
    return fd.enum_type.values_by_number[getattr(msg, field)].name
