"""Config-driven path on the MI355X: the reference LeNet/MLP confs run through
NeuralNet + Worker on a RocmGPU (HIP conv/pool/softmax-xent/optimiser
kernels), and partitioned nets equal unpartitioned ones on the GPU."""
import os

import numpy as np
import pytest
import torch

from singa_amd.config import schema
from singa_amd.runtime import NeuralNet, Worker

pytestmark = pytest.mark.gpu
REF = "/root/reference/examples/mnist"

LENET = """
name: "lenet-gpu" train_steps: 60 test_steps: 2 test_frequency: 30 display_frequency: 20
updater { base_learning_rate: 0.02 type: kSGD momentum: 0.9 weight_decay: 0.0005 learning_rate_change_method: kFixed }
neuralnet {
  layer { name: "data" type: "kShardData" data_param { batchsize: 64 path: "/nonexistent" } }
  layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
  layer { name: "label" type: "kLabel" srclayers: "data" }
  layer { name: "conv1" type: "kConvolution" srclayers: "mnist" convolution_param { num_filters: 20 kernel: 5 }
          param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
  layer { name: "pool1" type: "kPooling" srclayers: "conv1" pooling_param { pool: MAX kernel: 2 stride: 2 } }
  layer { name: "conv2" type: "kConvolution" srclayers: "pool1" convolution_param { num_filters: 50 kernel: 5 }
          param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
  layer { name: "pool2" type: "kPooling" srclayers: "conv2" pooling_param { pool: MAX kernel: 2 stride: 2 } }
  layer { name: "ip1" type: "kInnerProduct" srclayers: "pool2" inner_product_param { num_output: 500 }
          param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
  layer { name: "relu1" type: "kReLU" srclayers: "ip1" }
  layer { name: "ip2" type: "kInnerProduct" srclayers: "relu1" inner_product_param { num_output: 10 }
          param { init_method: kUniformSqrtFanIn low: -1 high: 1 } param { init_method: kConstant value: 0 } }
  layer { name: "loss" type: "kSoftmaxLoss" srclayers: "ip2" srclayers: "label" softmaxloss_param { topk: 1 } }
}"""


def _fixed_batch(w):
    src = w.train_net.layers[0].source
    img, lab = src.next()
    src.next = lambda: (img, lab)


def test_worker_lenet_on_gpu(gpu):
    from singa_amd.device import create_cuda_gpu

    dev = create_cuda_gpu()
    m = schema.parse_text("ModelProto", LENET)
    logs = []
    w = Worker(m, dev=dev, data_override={"*": {"shape": (28, 28), "nclass": 10}}, log=logs.append)
    _fixed_batch(w)
    w.run()
    p = w.train_net.params()[0]
    assert p.data.is_cuda
    hist = [h for h in w.history if h[0] == "train"]
    assert hist[-1][2][0] < 0.5 * hist[0][2][0], hist
    assert any(l.startswith("test:") for l in logs)


def test_lenet_gpu_matches_cpu_first_step(gpu):
    """Same seed on CppCPU and RocmGPU: identical init, losses agree."""
    from singa_amd.device import create_cuda_gpu, get_default_device

    m = schema.parse_text("ModelProto", LENET)
    out = []
    for dev in (get_default_device(), create_cuda_gpu()):
        net = NeuralNet(m.neuralnet, dev=dev, seed=5, data_override={"*": {"shape": (28, 28), "nclass": 10,
                                                                          "seed": 9}})
        outs = net.forward(training=False)
        out.append(float(net.total_loss(outs).data.float().cpu()))
    assert abs(out[0] - out[1]) < 2e-2 * max(1.0, abs(out[0])), out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference examples not mounted")
def test_reference_mlp_conf_steps_on_gpu(gpu):
    from singa_amd.device import create_cuda_gpu

    m = schema.read_text_file("ModelProto", os.path.join(REF, "mlp.conf"))
    m.train_steps = 20
    m.display_frequency = 10
    m.test_steps = 0
    m.validation_steps = 0
    w = Worker(m, dev=create_cuda_gpu(), data_override={"*": {"shape": (28, 28), "nclass": 10, "batch": 100}},
               log=lambda s: None)
    _fixed_batch(w)
    w.run()
    hist = [h for h in w.history if h[0] == "train"]
    assert np.isfinite(hist[-1][2][0]) and hist[-1][2][0] < hist[0][2][0]


@pytest.mark.parametrize("ptype,g", [("kDataPartition", 2), ("kLayerPartition", 2)])
def test_partitioned_equals_unpartitioned_gpu(gpu, ptype, g):
    from singa_amd.device import create_cuda_gpu

    txt = """
    layer { name: "data" type: "kShardData" data_param { batchsize: 8 path: "/nonexistent" } }
    layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
    layer { name: "label" type: "kLabel" srclayers: "data" }
    layer { name: "ip1" type: "kInnerProduct" srclayers: "mnist" param {} param {}
            inner_product_param { num_output: 16 } }
    layer { name: "tanh1" type: "kTanh" srclayers: "ip1" }
    layer { name: "ip2" type: "kInnerProduct" srclayers: "tanh1" param {} param {}
            inner_product_param { num_output: 10 } }
    layer { name: "loss" type: "kSoftmaxLoss" srclayers: "ip2" srclayers: "label" }
    """
    dev = create_cuda_gpu()
    losses = []
    for part in (None, ptype):
        net = schema.parse_text("NetProto", txt)
        for l in net.layer:
            for p in l.param:
                p.init_method = p.kUniform
                p.low, p.high = -0.1, 0.1
        if part:
            net.partition_type = part
        nn = NeuralNet(net, group_size=g if part else 1, dev=dev, seed=3,
                       data_override={"*": {"shape": (12, 12), "seed": 4}})
        outs = nn.forward(training=True)
        losses.append(float(nn.total_loss(outs).data.float().cpu()))
    assert abs(losses[0] - losses[1]) < 1e-3 * max(1.0, abs(losses[0])), losses


def test_executor_threads_on_gpu_streams():
    """P3 on the GPU: 2 executor threads (one HIP stream each) on identical
    data in aggregated mode == the single-thread run."""
    from test_config_runtime import _thread_worker
    from singa_amd import device

    dev = device.create_rocm_gpu()
    outs = []
    for k in (1, 2):
        dev.SetRandSeed(0)
        w = _thread_worker(k, False, dev=dev)
        assert (w.streams is not None) == (k > 1)
        w.run()
        outs.append(w.store.w.detach().cpu().numpy())
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-4, atol=1e-5)
