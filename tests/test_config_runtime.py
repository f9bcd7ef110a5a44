"""Config-driven path: reference .conf parsing, NeuralNet construction and
partitioning (reference src/test/test_neuralnet.cc expectations), Worker."""
import os

import numpy as np
import pytest
import torch

from singa_amd import autograd
from singa_amd.config import schema
from singa_amd.runtime import NeuralNet, Worker

REF = "/root/reference/examples/mnist"


def conv_test_net(partition=None):
    """The 8-layer conv net of the reference NeuralNet tests."""
    txt = """
    layer { name: "data" type: "kShardData" data_param { batchsize: 8 path: "/nonexistent" } }
    layer { name: "mnist" type: "kMnistImage" srclayers: "data" }
    layer { name: "label" type: "kLabel" srclayers: "data" }
    layer { name: "conv1" type: "kConvolution" srclayers: "mnist" param {} param {}
            convolution_param { num_filters: 8 kernel: 2 } }
    layer { name: "relu1" type: "kReLU" srclayers: "conv1" }
    layer { name: "pool1" type: "kPooling" srclayers: "relu1" pooling_param { kernel: 4 stride: 2 } }
    layer { name: "fc1" type: "kInnerProduct" srclayers: "pool1" param {} param {}
            inner_product_param { num_output: 10 } }
    layer { name: "loss" type: "kSoftmaxLoss" srclayers: "fc1" srclayers: "label" }
    """
    net = schema.parse_text("NetProto", txt)
    for l in net.layer:
        for p in l.param:
            p.init_method = p.kUniform
            p.low, p.high = -0.1, 0.1
    if partition:
        net.partition_type = partition
    return net


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference examples not mounted")
@pytest.mark.parametrize("f,msg", [("mlp.conf", "ModelProto"), ("conv.conf", "ModelProto"),
                                   ("cluster.conf", "ClusterProto"), ("topology.conf", "Topology")])
def test_reference_confs_parse_unchanged(f, msg):
    m = schema.read_text_file(msg, os.path.join(REF, f))
    assert m.IsInitialized()
    if msg == "ModelProto":
        assert len(m.neuralnet.layer) > 0
        assert schema.enum_name(m.updater, "type") == "kSGD"


def test_proto2_defaults():
    up = schema.new("UpdaterProto")
    assert schema.enum_name(up, "type") == "kAdaGrad" and up.param_type == "Elastic" and up.warmup_steps == 10
    assert schema.new("ClusterProto").start_port == 6723


def test_neuralnet_no_partition():
    net = NeuralNet(conv_test_net())
    assert len(net.layers) == 8
    assert net.layers[0].name == "data" and net.layers[-1].name == "loss"
    assert net.shapes["conv1"] == (8, 8, 27, 27)
    assert net.shapes["pool1"] == (8, 8, 12, 12)


def test_neuralnet_data_partition_count():
    net = NeuralNet(conv_test_net("kDataPartition"), group_size=3)
    assert len(net.layers) == 28  # reference test_neuralnet.cc DataPartition
    assert net.layers[0].name == "data"


def _run(net, seed=0):
    torch.manual_seed(seed)
    for l in net.layers:
        if l.is_data:
            l.source.rng = np.random.RandomState(7)
    autograd.training = True
    outs = net.forward(True)
    loss = net.total_loss(outs)
    grads = {}
    for p, g in autograd.backward(loss):
        grads.setdefault(p.name, []).append(g.data.clone())
    autograd.training = False
    return float(loss.data), grads


@pytest.mark.parametrize("ptype,g", [("kDataPartition", 2), ("kDataPartition", 4), ("kLayerPartition", 2)])
def test_partitioned_equals_unpartitioned(ptype, g):
    base = NeuralNet(conv_test_net(), seed=3)
    part = NeuralNet(conv_test_net(ptype), group_size=g, seed=3)
    # copy unpartitioned weights into the partitioned net's original layers
    for l in base.layers:
        if l.params and ptype == "kDataPartition":
            for pl in part.layers:
                if getattr(pl, "origin", None) is not None and pl.origin.name == l.name:
                    for a, b in zip(pl.params, l.params):
                        a.data.copy_(b.data)
    if ptype == "kLayerPartition":
        # partition slices were copied from the (seed-identical) original params at build
        pass
    lb, gb = _run(base)
    lp, gp = _run(part)
    assert abs(lb - lp) < 1e-4, (lb, lp)
    if ptype == "kDataPartition":
        for k, v in gb.items():
            assert torch.allclose(v[0], sum(gp[k]), atol=1e-5), k


def test_hybrid_partition_builds():
    net = conv_test_net("kLayerPartition")
    net.layer[-2].partition_type = "kDataPartition"
    net.layer[-1].partition_type = "kDataPartition"
    nn = NeuralNet(net, group_size=2)
    types = [l.type_name for l in nn.layers]
    assert "kSlice" in types and "kConcate" in types
    loss, _ = _run(nn)
    assert np.isfinite(loss)


def test_worker_trains_lenet_style():
    txt = """
    name: "lenet-test" train_steps: 40 test_steps: 2 test_frequency: 20 display_frequency: 20
    updater { base_learning_rate: 0.05 type: kSGD momentum: 0.9 learning_rate_change_method: kFixed }
    neuralnet {
      layer { name: "data" type: "kShardData" data_param { batchsize: 16 path: "/nonexistent" } }
      layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
      layer { name: "label" type: "kLabel" srclayers: "data" }
      layer { name: "conv1" type: "kConvolution" srclayers: "mnist" convolution_param { num_filters: 8 kernel: 5 }
              param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
      layer { name: "pool1" type: "kPooling" srclayers: "conv1" pooling_param { pool: MAX kernel: 2 stride: 2 } }
      layer { name: "ip1" type: "kInnerProduct" srclayers: "pool1" inner_product_param { num_output: 10 }
              param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
      layer { name: "loss" type: "kSoftmaxLoss" srclayers: "ip1" srclayers: "label" }
    }"""
    m = schema.parse_text("ModelProto", txt)
    logs = []
    w = Worker(m, data_override={"*": {"shape": (28, 28), "nclass": 10}}, log=logs.append)
    # fixed batch so the net can memorise it
    src = w.train_net.layers[0].source
    img, lab = src.next()
    src.next = lambda: (img, lab)
    w.run()
    train_hist = [h for h in w.history if h[0] == "train"]
    assert train_hist[-1][2][0] < train_hist[0][2][0]
    assert any(l.startswith("test:") for l in logs)


_MLP_NET = """
    name: "mlp-threads" train_steps: 6 display_frequency: 0
    updater { base_learning_rate: 0.05 type: kSGD momentum: 0.9 learning_rate_change_method: kFixed hogwild: %s }
    neuralnet {
      layer { name: "data" type: "kShardData" data_param { batchsize: 8 path: "/nonexistent" } }
      layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
      layer { name: "label" type: "kLabel" srclayers: "data" }
      layer { name: "ip1" type: "kInnerProduct" srclayers: "mnist" inner_product_param { num_output: 16 }
              param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
      layer { name: "tanh1" type: "kTanh" srclayers: "ip1" }
      layer { name: "ip2" type: "kInnerProduct" srclayers: "tanh1" inner_product_param { num_output: 10 }
              param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
      layer { name: "loss" type: "kSoftmaxLoss" srclayers: "ip2" srclayers: "label" }
    }"""


def _thread_worker(k, hogwild, fixed_seed=True, dev=None):
    m = schema.parse_text("ModelProto", _MLP_NET % ("true" if hogwild else "false"))
    cp = schema.new("ClusterProto")
    cp.nworkers, cp.nthreads_per_procs, cp.workspace = 1, k, ""
    ov = {"shape": (6, 6), "nclass": 10}
    if fixed_seed:
        ov["seed"] = 3
    return Worker(m, cp, dev=dev, data_override={"*": ov}, log=lambda s: None)


def test_executor_threads_aggregated_equals_single():
    """P3, aggregated mode: k threads on identical data sum k identical
    gradients and apply ONE update with grad_scale 1/k == the 1-thread run."""
    w1 = _thread_worker(1, False)
    w2 = _thread_worker(2, False)
    assert len(w2.replicas) == 2 and w2.replicas[1].params()[0] is not w2.train_net.params()[0]
    assert w2.replicas[1].params()[0].data.data_ptr() == w2.train_net.params()[0].data.data_ptr()
    w1.run()
    w2.run()
    np.testing.assert_allclose(w1.store.w.numpy(), w2.store.w.numpy(), rtol=1e-6, atol=1e-7)


def test_executor_threads_hogwild_trains():
    w = _thread_worker(3, True, fixed_seed=False)
    first = w.train_one_batch(0)
    for s in range(1, 30):
        last = w.train_one_batch(s)
    assert np.isfinite(last).all()
    assert w.updater.step_counter == 30


def _mnist_layer(params: str):
    from singa_amd import device
    from singa_amd.runtime.layers import create_layer
    from singa_amd.tensor import Tensor
    lp = schema.parse_text("LayerProto", 'name: "mnist" type: "kMnistImage" srclayers: "data" '
                                         'mnist_param { %s }' % params)
    layer = create_layer(lp)
    dev = device.get_default_device()
    layer.setup([(4, 28, 28)], dev)
    img = torch.zeros(4, 28, 28)
    img[:, 10:18, 12:16] = 255.0  # a bar ("1")
    x = {"image": Tensor(device=dev, data=img, requires_grad=False),
         "label": Tensor(device=dev, data=torch.tensor([1, 7, 3, 4]), requires_grad=False)}
    return layer, x, img


def test_mnist_layer_no_augmentation_is_exact():
    """All MnistProto deformation fields default to 0: plain x/norm_a - norm_b
    (reference src/worker/layer.cc:438-444), identical in train and test."""
    layer, x, img = _mnist_layer("norm_a: 255 norm_b: 0.5")
    for training in (True, False):
        out = layer.forward([x], training).data
        assert torch.allclose(out, img / 255 - 0.5)


@pytest.mark.parametrize("params", ["gamma: 15", "beta: 15", "kernel: 5 sigma: 2 alpha: 3",
                                    "gamma: 10 beta: 10 kernel: 5 sigma: 2 alpha: 3 elastic_freq: 2"])
def test_mnist_layer_deformations(params):
    """Scaling / rotation-or-shear / elastic distortion (the intent of the
    commented-out code at src/worker/layer.cc:405-436): the training output
    moves pixels but keeps the value range and roughly the ink mass; the
    test-phase output stays undeformed."""
    layer, x, img = _mnist_layer("norm_a: 255 " + params)
    out = layer.forward([x], True).data
    assert out.shape == img.shape
    assert not torch.allclose(out, img / 255)
    assert out.min() >= -1e-5 and out.max() <= 1 + 1e-5
    mass_in, mass_out = (img / 255).sum((1, 2)), out.sum((1, 2))
    assert torch.all((mass_out / mass_in - 1).abs() < 0.45)
    assert torch.allclose(layer.forward([x], False).data, img / 255)


def test_mnist_layer_elastic_freq():
    layer, x, img = _mnist_layer("norm_a: 255 kernel: 5 sigma: 2 alpha: 3 elastic_freq: 2")
    outs = [layer.forward([x], True).data for _ in range(2)]
    assert not torch.allclose(outs[0], img / 255)  # batch 0: distorted
    assert torch.allclose(outs[1], img / 255)      # batch 1: skipped


@pytest.mark.parametrize("method,kw,check", [
    ("kConstant", dict(value=0.5), lambda d: bool(np.all(d == 0.5))),
    ("kUniform", dict(low=-0.2, high=0.3), lambda d: d.min() >= -0.2 and d.max() <= 0.3 and abs(d.mean() - 0.05) < 0.1),
    ("kUniform", dict(low=-1, high=1, value=2), lambda d: d.min() >= -2 and d.max() <= 2 and abs(d.std() - 2 / 3 ** .5) < 0.1),
    ("kUniformSqrtFanIn", dict(low=-1, high=1, value=1),  # U * value / sqrt(fan_in / 3), fan_in = 75
     lambda d: np.abs(d).max() <= 1 / (75 / 3) ** .5 + 1e-6 and abs(d.std() - (1 / 3 ** .5) / (25 ** .5)) < 0.1),
    ("kUniformSqrtFanInOut", dict(low=-1, high=1, value=1),  # U * value / sqrt(s0 + s1)
     lambda d: np.abs(d).max() <= 1 / (50 + 100) ** .5 + 1e-6),
    ("kGaussain", dict(mean=0.3, std=0.5), lambda d: abs(d.mean() - 0.3) < 0.1 and abs(d.std() - 0.5) < 0.1),
    ("kGaussainSqrtFanIn", dict(mean=0.0, std=1.0, value=1),  # N * value / sqrt(s0)
     lambda d: abs(d.mean()) < 0.1 and abs(d.std() - 1 / 50 ** .5) < 0.1),
])
def test_param_init_distributions(method, kw, check):
    """Port of the reference's Param init tests (src/test/model/test_param.cc:
    25-140): every init method over 5000 samples, mean / std within 0.1."""
    from singa_amd import device
    from singa_amd.config import schema
    from singa_amd.runtime.param import make_param

    p = schema.new("ParamProto")
    p.name = "w"
    p.init_method = getattr(p, method)
    for k, v in kw.items():
        setattr(p, k, v)
    t = make_param((50, 100), p, device.get_default_device(), fan_in=75,
                   generator=torch.Generator().manual_seed(1))
    d = t.data.numpy().ravel()
    assert d.size == 5000 and check(d)


def test_rgb_image_layer_crop_mirror_unsigned():
    """kRGBImage (reference RGBImageLayer, src/worker/layer.cc:573-643) with
    its quirks fixed (Appendix A #12): the crop is written also without
    mirroring, the mirror decision is one draw, centre crop at test time,
    random crop + mirror in training, then * scale.  (Unsigned pixel decoding
    is the record decoder's job: shard.cc DecodeRecordToFloat.)"""
    from singa_amd import device, tensor
    from singa_amd.runtime.layers import create_layer

    p = schema.new("LayerProto")
    p.name, p.type = "rgb", "kRGBImage"
    p.rgbimage_param.cropsize = 4
    p.rgbimage_param.mirror = True
    p.rgbimage_param.scale = 0.5
    lay = create_layer(p)
    dev = device.get_default_device()
    lay.setup([(2, 3, 6, 6)], dev)
    img = torch.arange(2 * 3 * 6 * 6, dtype=torch.float32).reshape(2, 3, 6, 6) % 256  # includes values > 127
    src = {"image": tensor.Tensor(data=img)}
    y = lay.forward([src], training=False).data
    assert y.shape == (2, 3, 4, 4)
    assert torch.equal(y, img[..., 1:5, 1:5] * 0.5)  # centre crop
    seen = set()
    for _ in range(40):
        y = lay.forward([src], training=True).data
        assert y.shape == (2, 3, 4, 4) and float(y.min()) >= 0
        found = None
        for h0 in range(3):
            for w0 in range(3):
                c = img[..., h0:h0 + 4, w0:w0 + 4] * 0.5
                if torch.equal(y, c):
                    found = (h0, w0, False)
                elif torch.equal(y, torch.flip(c, dims=[-1])):
                    found = (h0, w0, True)
        assert found is not None
        seen.add(found)
    assert len({s[:2] for s in seen}) > 3 and {s[2] for s in seen} == {False, True}
