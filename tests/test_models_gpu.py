"""Model zoo + attention on the MI355X (bf16 MFMA paths)."""
import numpy as np
import pytest
import torch

from singa_amd import autograd, device, opt, tensor
from singa_amd.tensor import Tensor

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H,S,D,masked", [(2, 4, 64, 64, False), (3, 2, 128, 64, True), (1, 12, 512, 64, True)])
def test_attention_native_vs_fp32(gpu, B, H, S, D, masked):
    from singa_amd.ops import functional as F

    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, S, D, device=gpu, generator=g).bfloat16() for _ in range(3))
    mask = None
    if masked:
        mask = torch.zeros(B, 1, 1, S, device=gpu)
        mask[..., S - S // 4:] = -10000.0
    o, p = F.attention_fwd(q, k, v, mask)
    qf, kf, vf = q.float().requires_grad_(), k.float().requires_grad_(), v.float().requires_grad_()
    s = qf @ kf.transpose(-1, -2) / D ** 0.5
    if mask is not None:
        s = s + mask
    ref = torch.softmax(s, -1) @ vf
    assert (o.float() - ref).abs().max().item() < 3e-2
    do = torch.randn_like(ref)
    ref.backward(do)
    dq, dk, dv = F.attention_bwd(q, k, v, p, do.bfloat16())
    for a, b in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        err = (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6)
        assert err < 4e-2, err


def _img(n, c, h, w, dev, k=10):
    rng = np.random.RandomState(0)
    return (tensor.from_numpy(rng.randn(n, c, h, w).astype(np.float32)).to_device(dev),
            tensor.from_numpy(rng.randint(0, k, n).astype(np.int32)).to_device(dev))


@pytest.mark.parametrize("name", ["cnn", "alexnet", "vgg16", "mlp"])
def test_model_trains_gpu(gpu, name):
    from singa_amd.models import alexnet, cnn, mlp, vgg

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(0)
    if name == "cnn":
        m, (x, y), lr = cnn.CNN(), _img(32, 1, 28, 28, dev), 0.01
    elif name == "alexnet":
        m, (x, y), lr = alexnet.AlexNet(100, compute_dtype=torch.bfloat16), _img(8, 3, 224, 224, dev, 100), 0.002
    elif name == "vgg16":
        m, (x, y), lr = vgg.VGG(16, 10, small=True), _img(8, 3, 32, 32, dev), 0.005
    else:
        m, (x, y), lr = mlp.deep_big_simple(), _img(64, 1, 28, 28, dev), 0.01
    m.set_optimizer(opt.SGD(lr, 0.9))
    m.compile([x], is_train=True)
    ls = []
    for _ in range(8):
        _, l = m(x, y)
        ls.append(float(l.data.float().cpu()))
    assert all(np.isfinite(ls)) and ls[-1] < ls[0], ls


def test_bert_tiny_gpu_matches_cpu_loss(gpu):
    from singa_amd.models import bert

    rng = np.random.RandomState(0)
    ids_np = rng.randint(0, 1000, (4, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 4).astype(np.int32)
    losses = []
    init = None
    for dev in (device.get_default_device(), device.create_rocm_gpu()):
        dev.SetRandSeed(3)
        m = bert.bert_tiny(dropout=0.0, compute_dtype=torch.bfloat16)
        ids = tensor.from_numpy(ids_np).to_device(dev)
        y = tensor.from_numpy(y_np).to_device(dev)
        m.set_optimizer(opt.SGD(0.01, 0.9))
        m.compile([ids], is_train=True)
        if init is None:  # CPU and GPU generators differ: start the GPU model from the CPU weights
            init = {k: v.data.clone() for k, v in m.get_states().items()}
        else:
            m.set_states(init)
        ls = []
        for _ in range(6):
            _, l = m(ids, y)
            ls.append(float(l.data.float().cpu()))
        losses.append(ls)
    assert abs(losses[0][0] - losses[1][0]) < 5e-2 * max(1, abs(losses[0][0])), losses
    assert losses[1][-1] < losses[1][0]


def test_sonnx_import_runs_on_gpu(gpu):
    """ResNet-18 exported on the CPU, imported on the MI355X: same logits
    (the GPU conv runs bf16 MFMA internally)."""
    from singa_amd import autograd, sonnx
    from singa_amd.models import resnet
    from singa_amd.sonnx import onnx_proto as P

    cpu = device.get_default_device()
    cpu.SetRandSeed(0)
    x = tensor.from_numpy(np.random.RandomState(0).randn(4, 3, 32, 32).astype(np.float32))
    m = resnet.resnet18(num_classes=10)
    m.compile([x], is_train=False)
    autograd.training = False
    ref = m.forward(x).data.float().numpy()
    blob = sonnx.to_onnx(m, [x]).SerializeToString()
    rep = sonnx.prepare(P.load_model(blob), device.create_rocm_gpu())
    out = rep.run([x.data.numpy()])[0]
    assert out.data.is_cuda
    err = np.abs(out.data.float().cpu().numpy() - ref).max() / (np.abs(ref).max() + 1e-6)
    assert err < 5e-2, err
