"""Per-parameter gradient comparison, GPU (bf16 MFMA) vs CPU fp32, for a
model zoo network started from identical weights (debugging aid)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def build(name, small):
    from singa_amd.models import alexnet, cnn, resnet, vgg

    if name == "alexnet":
        return alexnet.create_model(num_classes=10 if small else 1000, small=small, dropout=0.0,
                                    compute_dtype=torch.bfloat16), (32 if small else 224), (10 if small else 1000)
    if name == "vgg":
        return vgg.create_model(11, num_classes=10, compute_dtype=torch.bfloat16, small=True, dropout=0.0), 32, 10
    if name == "resnet":
        return resnet.create_model(18, num_classes=10, compute_dtype=torch.bfloat16), 32, 10
    return cnn.create_model(), 28, 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--env", default="")
    a = ap.parse_args()
    from singa_amd import device, opt, tensor

    rng = np.random.RandomState(0)
    grads, init = [], None
    for dev in (device.get_default_device(), device.create_rocm_gpu()):
        dev.SetRandSeed(1)
        m, hw, ncls = build(a.model, a.small)
        cin = 1 if a.model == "cnn" else 3
        x_np = np.random.RandomState(0).standard_normal((a.batch, cin, hw, hw)).astype(np.float32)
        y_np = np.random.RandomState(1).randint(0, ncls, a.batch).astype(np.int32)
        x = tensor.from_numpy(x_np).to_device(dev)
        y = tensor.from_numpy(y_np).to_device(dev)
        m.set_optimizer(opt.SGD(0.0))
        m.compile([x], is_train=True)
        if init is None:
            init = {k: v.data.clone() for k, v in m.get_states().items()}
        else:
            m.set_states(init)
        _, l = m(x, y)
        print(dev.lang(), "loss", float(l.data.float().cpu()))
        grads.append({k: p.grad_view.detach().float().cpu().clone() for k, p in m.get_params().items()})
    for k, gc in grads[0].items():
        gg = grads[1][k]
        cos = float((gc * gg).sum() / (gc.norm() * gg.norm() + 1e-30))
        rel = float((gc - gg).norm() / (gc.norm() + 1e-30))
        print(f"{k:24s} {tuple(gc.shape)!s:22s} |g|cpu {gc.norm():.4e} |g|gpu {gg.norm():.4e} cos {cos:.5f} rel {rel:.4f}")


if __name__ == "__main__":
    main()
