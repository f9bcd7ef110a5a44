"""Yardstick only (not part of the framework): the same ResNet-50 v1.5 training
step written in plain PyTorch (MIOpen convs, bf16 autocast, channels_last,
SGD momentum) on the same GPU, so singa_amd's bench number can be read
against the vendor-library path.  Not used by bench.py."""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, inp, planes, stride, down):
        super().__init__()
        self.c1 = nn.Conv2d(inp, planes, 1, bias=False)
        self.b1 = nn.BatchNorm2d(planes)
        self.c2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(planes)
        self.c3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.b3 = nn.BatchNorm2d(planes * 4)
        self.down = nn.Sequential(nn.Conv2d(inp, planes * 4, 1, stride, bias=False),
                                  nn.BatchNorm2d(planes * 4)) if down else None

    def forward(self, x):
        o = torch.relu(self.b1(self.c1(x)))
        o = torch.relu(self.b2(self.c2(o)))
        o = self.b3(self.c3(o))
        return torch.relu(o + (self.down(x) if self.down is not None else x))


class R50(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, inp = [], 64
        for i, (p, n) in enumerate(zip((64, 128, 256, 512), (3, 4, 6, 3))):
            for j in range(n):
                s = (1 if i == 0 else 2) if j == 0 else 1
                layers.append(Bottleneck(inp, p, s, j == 0))
                inp = p * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(x.mean((2, 3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    m = R50().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = nn.functional.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss
    import os
    import sys
    import threading

    def heartbeat():  # MIOpen's first-call kernel search prints nothing for minutes at b1024
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[yardstick] alive {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()
        print(f"warmup step {i} done", file=sys.stderr, flush=True)  # MIOpen's first-call searches are slow
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"yardstick": "pytorch-miopen resnet50 bf16 autocast channels_last", "images_per_s":
                      a.batch * a.steps / el, "ms_per_step": 1e3 * el / a.steps, "batch": a.batch,
                      "torch": torch.__version__, "miopen_find_mode": os.environ.get("MIOPEN_FIND_MODE", "default")}))


if __name__ == "__main__":
    main()
