"""sonnx: export -> serialize -> parse -> import round trips (outputs must
match the source model), fine-tuning an imported graph, and hand-built ONNX
graphs through the importer (oracle: PyTorch fp32 of the same op).
The reference has no ONNX support: parity unpinned, round-trip tested."""
import math

import numpy as np
import pytest
import torch

from singa_amd import autograd, device, opt, sonnx, tensor
from singa_amd.sonnx import onnx_proto as P
from singa_amd.tensor import Tensor


def _roundtrip(m, xs, atol=1e-4, **kw):
    device.get_default_device().SetRandSeed(0)
    m.compile(xs, is_train=False)
    autograd.training = False
    ref = m.forward(*xs, **kw)
    mp = sonnx.to_onnx(m, xs, **kw)
    blob = mp.SerializeToString()
    rep = sonnx.prepare(P.load_model(blob))
    out = rep.run(xs)[0]
    np.testing.assert_allclose(out.data.float().numpy(), ref.data.float().numpy(), atol=atol, rtol=1e-4)
    return mp


def _img(n, c, h, w, seed=0):
    return tensor.from_numpy(np.random.RandomState(seed).randn(n, c, h, w).astype(np.float32))


def test_roundtrip_mlp_cnn():
    from singa_amd.models import cnn, mlp

    mp = _roundtrip(mlp.MLP((32, 16), activation="stanh"), [_img(4, 1, 6, 6)])
    assert {n.op_type for n in mp.graph.node} >= {"MatMul", "Add", "Tanh", "Flatten"}
    mp = _roundtrip(cnn.CNN(), [_img(2, 1, 28, 28)])
    assert {"Conv", "MaxPool"} <= {n.op_type for n in mp.graph.node}


def test_roundtrip_resnet18_and_alexnet():
    from singa_amd.models import alexnet, resnet

    m = resnet.resnet18(num_classes=10)
    mp = _roundtrip(m, [_img(2, 3, 32, 32)], atol=2e-3)
    ops = {n.op_type for n in mp.graph.node}
    assert {"Conv", "BatchNormalization", "Relu", "Add", "GlobalAveragePool", "MaxPool"} <= ops
    names = {i.name for i in mp.graph.initializer}
    assert "conv1.W" in names and any(k.endswith("running_mean") for k in names)
    _roundtrip(alexnet.AlexNet(10, small=True), [_img(2, 3, 32, 32)], atol=1e-3)


def test_roundtrip_bert_tiny():
    from singa_amd.models import bert

    ids = tensor.from_numpy(np.random.RandomState(0).randint(0, 1000, (2, 16)).astype(np.int64))
    mp = _roundtrip(bert.bert_tiny(dropout=0.0), [ids], atol=1e-3)
    ops = {n.op_type for n in mp.graph.node}
    assert {"Gather", "LayerNormalization", "Softmax", "MatMul", "Erf", "Transpose", "Reshape"} <= ops


def test_sonnx_model_finetunes(tmp_path):
    from singa_amd.models import cnn

    x = _img(8, 1, 28, 28)
    y = tensor.from_numpy(np.random.RandomState(1).randint(0, 10, 8).astype(np.int32))
    m = cnn.CNN()
    m.compile([x], is_train=False)
    path = str(tmp_path / "cnn.onnx")
    sonnx.export(m, [x], path)
    sm = sonnx.SONNXModel(path)
    assert len(sm.get_params()) == 8
    sm.set_optimizer(opt.SGD(0.01, 0.9))
    sm.compile([x], is_train=True)
    ls = [float(sm(x, y)[1].data) for _ in range(6)]
    assert ls[-1] < ls[0], ls


def _graph(nodes, inputs, outputs, inits=()):
    g = P.new("GraphProto")
    g.node.extend(nodes)
    for n, a in inputs:
        g.input.append(sonnx._value_info(n, a.shape))
    for n in outputs:
        g.output.append(sonnx._value_info(n, ()))
    for n, a in inits:
        g.initializer.append(sonnx.numpy_to_tensorproto(a, n))
    m = P.new("ModelProto")
    m.ir_version = 8
    m.graph.CopyFrom(g)
    o = m.opset_import.add()
    o.version = 17
    return m


def _run1(node, arrays, inits=()):
    autograd.training = False  # ONNX semantics: inference (BatchNormalization uses running stats)
    names = [f"x{i}" for i in range(len(arrays))]
    m = _graph([node], list(zip(names, arrays)), list(node.output), inits)
    return sonnx.prepare(m).run([Tensor(data=torch.from_numpy(a), requires_grad=False) for a in arrays])


R = np.random.RandomState(3)
A = R.randn(2, 3, 4).astype(np.float32)


@pytest.mark.parametrize("op,attrs,fn", [
    ("Relu", {}, lambda a: np.maximum(a, 0)),
    ("Sigmoid", {}, lambda a: 1 / (1 + np.exp(-a))),
    ("Tanh", {}, np.tanh),
    ("Abs", {}, np.abs),
    ("Neg", {}, np.negative),
    ("Exp", {}, np.exp),
    ("Erf", {}, lambda a: torch.erf(torch.from_numpy(a)).numpy()),
    ("LeakyRelu", {"alpha": 0.1}, lambda a: np.where(a > 0, a, 0.1 * a)),
    ("Elu", {"alpha": 0.5}, lambda a: np.where(a > 0, a, 0.5 * (np.exp(a) - 1))),
    ("Softplus", {}, lambda a: np.log1p(np.exp(a))),
    ("Softsign", {}, lambda a: a / (1 + np.abs(a))),
    ("HardSigmoid", {"alpha": 0.2, "beta": 0.5}, lambda a: np.clip(0.2 * a + 0.5, 0, 1)),
    ("Softmax", {"axis": -1}, lambda a: np.exp(a) / np.exp(a).sum(-1, keepdims=True)),
    ("Transpose", {"perm": [2, 0, 1]}, lambda a: a.transpose(2, 0, 1)),
    ("Flatten", {"axis": 1}, lambda a: a.reshape(2, -1)),
    ("ReduceMean", {"axes": [1], "keepdims": 0}, lambda a: a.mean(1)),
])
def test_import_unary_ops(op, attrs, fn):
    out = _run1(sonnx.make_node(op, ["x0"], ["y"], **attrs), [A])[0]
    np.testing.assert_allclose(out.data.numpy(), fn(A), rtol=1e-4, atol=1e-5)


def test_import_shape_ops():
    sh = np.asarray([3, 8], np.int64)
    out = _run1(sonnx.make_node("Reshape", ["x0", "s"], ["y"]), [A], [("s", sh)])[0]
    assert out.shape == (3, 8)
    out = _run1(sonnx.make_node("Slice", ["x0", "st", "en", "ax"], ["y"]), [A],
                [("st", np.asarray([1], np.int64)), ("en", np.asarray([3], np.int64)),
                 ("ax", np.asarray([2], np.int64))])[0]
    np.testing.assert_allclose(out.data.numpy(), A[:, :, 1:3])
    outs = _run1(sonnx.make_node("Split", ["x0", "sp"], ["a", "b"], axis=2), [A],
                 [("sp", np.asarray([1, 3], np.int64))])
    assert outs[0].shape == (2, 3, 1) and outs[1].shape == (2, 3, 3)
    out = _run1(sonnx.make_node("Concat", ["x0", "x1"], ["y"], axis=0), [A, A])[0]
    assert out.shape == (4, 3, 4)
    out = _run1(sonnx.make_node("Gather", ["x0", "i"], ["y"], axis=1), [A], [("i", np.asarray([2, 0], np.int64))])[0]
    np.testing.assert_allclose(out.data.numpy(), A[:, [2, 0]])
    out = _run1(sonnx.make_node("Unsqueeze", ["x0", "ax"], ["y"]), [A], [("ax", np.asarray([0], np.int64))])[0]
    assert out.shape == (1, 2, 3, 4)
    out = _run1(sonnx.make_node("Where", ["c", "x0", "x1"], ["y"]), [A, -A], [("c", A > 0)])[0]
    np.testing.assert_allclose(out.data.numpy(), np.abs(A))


def test_import_conv_gemm_bn():
    x = R.randn(2, 3, 8, 8).astype(np.float32)
    w = R.randn(4, 3, 3, 3).astype(np.float32)
    b = R.randn(4).astype(np.float32)
    out = _run1(sonnx.make_node("Conv", ["x0", "w", "b"], ["y"], kernel_shape=[3, 3], pads=[1, 1, 1, 1],
                                strides=[2, 2]), [x], [("w", w), ("b", b)])[0]
    ref = torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b), 2, 1)
    np.testing.assert_allclose(out.data.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    a2 = R.randn(5, 6).astype(np.float32)
    wt = R.randn(4, 6).astype(np.float32)
    out = _run1(sonnx.make_node("Gemm", ["x0", "w", "c"], ["y"], transB=1, alpha=0.5, beta=2.0), [a2],
                [("w", wt), ("c", b)])[0]
    np.testing.assert_allclose(out.data.numpy(), 0.5 * a2 @ wt.T + 2.0 * b, rtol=1e-4, atol=1e-4)
    sc, bi, mu, var = (R.rand(3).astype(np.float32) + 0.5 for _ in range(4))
    out = _run1(sonnx.make_node("BatchNormalization", ["x0", "s", "b", "m", "v"], ["y"], epsilon=1e-5), [x],
                [("s", sc), ("b", bi), ("m", mu), ("v", var)])[0]
    ref = (x - mu[:, None, None]) / np.sqrt(var[:, None, None] + 1e-5) * sc[:, None, None] + bi[:, None, None]
    np.testing.assert_allclose(out.data.numpy(), ref, rtol=1e-4, atol=1e-4)


def test_tensorproto_roundtrip_dtypes():
    for a in (np.arange(6, dtype=np.int64).reshape(2, 3), R.randn(3).astype(np.float32), np.asarray([True, False])):
        b = sonnx.tensorproto_to_numpy(sonnx.numpy_to_tensorproto(a, "t"))
        np.testing.assert_array_equal(a, b)
    t = P.new("TensorProto")  # float_data (non-raw) encoding written by other exporters
    t.dims.extend([2])
    t.data_type = P.FLOAT
    t.float_data.extend([1.5, -2.0])
    np.testing.assert_array_equal(sonnx.tensorproto_to_numpy(t), [1.5, -2.0])


def test_sonnx_mixed_precision_import():
    """compute_dtype=bf16: GEMM operands cast (fp32 master weights), outputs
    stay close to the fp32 import, and fine-tuning still converges."""
    from singa_amd.models import bert

    ids = tensor.from_numpy(np.random.RandomState(0).randint(0, 1000, (4, 16)).astype(np.int64))
    y = tensor.from_numpy(np.array([0, 1, 1, 0], np.int32))
    device.get_default_device().SetRandSeed(0)
    m = bert.bert_tiny(dropout=0.0)
    m.compile([ids], is_train=False)
    blob = sonnx.to_onnx(m, [ids]).SerializeToString()
    ref = sonnx.prepare(P.load_model(blob)).run([ids])[0].data.float().numpy()
    sm = sonnx.SONNXModel(P.load_model(blob), compute_dtype=torch.bfloat16)
    out = sm.rep.run([ids])[0].data.float().numpy()
    np.testing.assert_allclose(out, ref, atol=5e-2, rtol=5e-2)
    assert all(p.dtype == torch.float32 for p in sm.get_params().values())
    sm.set_optimizer(opt.SGD(0.01))
    sm.compile([ids], is_train=True)
    ls = [float(sm(ids, y)[1].data.float()) for _ in range(8)]
    assert ls[-1] < ls[0], ls


def test_exported_bert_is_batch_independent():
    from singa_amd.models import bert

    rng = np.random.RandomState(0)
    ids2 = tensor.from_numpy(rng.randint(0, 1000, (2, 16)).astype(np.int64))
    ids5 = tensor.from_numpy(rng.randint(0, 1000, (5, 16)).astype(np.int64))
    m = bert.bert_tiny(dropout=0.0)
    m.compile([ids2], is_train=False)
    blob = sonnx.to_onnx(m, [ids2]).SerializeToString()
    out = sonnx.prepare(P.load_model(blob)).run([ids5])[0].data.numpy()
    autograd.training = False
    np.testing.assert_allclose(out, m.forward(ids5).data.numpy(), atol=1e-4)


@pytest.mark.parametrize("fuse_gelu", ["0", "1"])
def test_import_fusion_plan_bert_matches_unfused(monkeypatch, fuse_gelu):
    """Import-time fusion maps the exported Linear / GELU / attention chains
    back onto the fused operators (with SINGA_AMD_FUSE_GELU=1 a Linear
    feeding a GELU becomes one GEMM with the GELU epilogue); fused and
    unfused imports give the same outputs and parameter gradients (fp32,
    CPU)."""
    from singa_amd.models import bert
    monkeypatch.setenv("SINGA_AMD_FUSE_GELU", fuse_gelu)

    ids = tensor.from_numpy(np.random.RandomState(0).randint(0, 1000, (3, 16)).astype(np.int64))
    y = tensor.from_numpy(np.array([0, 1, 1], np.int32))
    device.get_default_device().SetRandSeed(0)
    m = bert.bert_tiny(dropout=0.0)
    m.compile([ids], is_train=False)
    blob = sonnx.to_onnx(m, [ids]).SerializeToString()
    kinds = {}
    res = []
    for fuse in (False, True):
        rep = sonnx.prepare(P.load_model(blob), fuse=fuse)
        for st in rep.fused.values():
            kinds[st.kind] = kinds.get(st.kind, 0) + 1
        autograd.training = True
        out = rep.run([ids])[0]
        loss = autograd.softmax_cross_entropy(out, y)
        grads = {p.name: g.data.clone() for p, g in autograd.backward(loss)}
        autograd.training = False
        res.append((out.data.clone(), grads))
    # bert_tiny: 2 layers x (qkv, proj, fc1, fc2) + pooler + classifier; the
    # residual tails Add -> LayerNormalization: 2 per layer + the embeddings'
    want = {"linear": 8, "linear_gelu": 2} if fuse_gelu == "1" else {"linear": 10, "gelu": 2}
    assert kinds == {**want, "qkv_attention": 2, "add_ln": 5}, kinds
    (o0, g0), (o1, g1) = res
    np.testing.assert_allclose(o1.numpy(), o0.numpy(), atol=1e-5, rtol=1e-5)
    assert set(g0) == set(g1) and len(g0) > 20
    for k in g0:
        np.testing.assert_allclose(g1[k].numpy(), g0[k].numpy(), atol=1e-5, rtol=1e-4, err_msg=k)


def test_import_fusion_respects_other_consumers():
    """A MatMul whose output is also a graph output is not fused with its Add."""
    x = R.randn(4, 6).astype(np.float32)
    w = R.randn(6, 5).astype(np.float32)
    b = R.randn(5).astype(np.float32)
    nodes = [sonnx.make_node("MatMul", ["x0", "w"], ["t"]), sonnx.make_node("Add", ["t", "b"], ["y"])]
    for outs, n_fused in ((["y"], 1), (["y", "t"], 0)):
        m = _graph(nodes, [("x0", x)], outs, [("w", w), ("b", b)])
        rep = sonnx.prepare(m)
        assert len(rep.fused) == n_fused
        autograd.training = False
        got = rep.run([Tensor(data=torch.from_numpy(x), requires_grad=False)])
        np.testing.assert_allclose(got[0].data.numpy(), x @ w + b, rtol=1e-5, atol=1e-5)


def test_import_scalar_params_stay_learnable():
    """An untagged one-element initializer feeding Mul (a learnable
    temperature) is a parameter; the GELU chain's sqrt 2 / 1 / 0.5 are frozen
    only because the fused pattern consumed them; the exporter's tagged
    constants are never parameters."""
    x = R.randn(4, 6).astype(np.float32)
    temp = np.asarray([1.7], np.float32)
    m = _graph([sonnx.make_node("Mul", ["x0", "temp"], ["y"])], [("x0", x)], ["y"], [("temp", temp)])
    rep = sonnx.prepare(m)
    assert "temp" in rep.params() and not rep.is_const("temp")
    autograd.training = True
    out = rep.run([Tensor(data=torch.from_numpy(x), requires_grad=False)])[0]
    grads = {p.name: g.data for p, g in autograd.backward(autograd.reduce_sum(out, keepdims=0))}
    autograd.training = False
    np.testing.assert_allclose(float(grads["temp"].reshape(-1)[0]), x.sum(), rtol=1e-5)
    # untagged GELU constants: frozen by the matched pattern
    sq, one, half = (np.asarray([v], np.float32) for v in (math.sqrt(2.0), 1.0, 0.5))
    nodes = [sonnx.make_node("Div", ["x0", "sq"], ["a"]), sonnx.make_node("Erf", ["a"], ["b"]),
             sonnx.make_node("Add", ["b", "one"], ["c"]), sonnx.make_node("Mul", ["x0", "c"], ["d"]),
             sonnx.make_node("Mul", ["d", "half"], ["y"])]
    rep = sonnx.prepare(_graph(nodes, [("x0", x)], ["y"], [("sq", sq), ("one", one), ("half", half)]))
    assert [st.kind for st in rep.fused.values()] == ["gelu"]
    assert all(rep.is_const(n) for n in ("sq", "one", "half")) and not rep.params()
    # exporter-tagged initializers (bert's GELU / attention constants) are never parameters
    from singa_amd.models import bert
    ids = tensor.from_numpy(np.random.RandomState(0).randint(0, 1000, (2, 16)).astype(np.int64))
    mb = bert.bert_tiny(dropout=0.0)
    mb.compile([ids], is_train=False)
    mp = sonnx.to_onnx(mb, [ids])
    tagged = {t.name for t in mp.graph.initializer if t.doc_string == sonnx.CONST_TAG}
    assert tagged and not (tagged & set(sonnx.prepare(mp, fuse=False).params()))
