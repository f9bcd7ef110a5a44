"""Worker checkpoint / resume (reference: ``Worker::Resume`` was a TODO,
src/worker/worker.cc:65-67; ``ModelProto.step`` "last snapshot step" was
never read).

A checkpoint is a zip with ``tensors.safetensors`` (parameters by
``<layer>/<index>`` of the local layers, optimiser slots ``opt/s1`` /
``opt/s2``, and the EASGD centre / RandomSync snapshot) and ``meta.json``
(step, optimiser counters, the model conf text, data-source positions).
Loading executes nothing from the file (safetensors + JSON only).  Resumed
runs continue the step counter, LR schedule and sync cadence, so
``train(k) + resume + train(n-k)`` reproduces ``train(n)``.
"""
from __future__ import annotations

import json
import os
import zipfile

import torch


def _param_table(net):
    out = {}
    for l in net.layers:
        if not net.is_local(l):
            continue
        for i, p in enumerate(l.params):
            out.setdefault(id(p), (f"{l.name}/{i}", p))
    return dict(out.values())


def save_worker(w, path: str) -> None:
    from safetensors.torch import save as st_save

    from ..config import schema

    tens = {}
    for k, p in _param_table(w.train_net).items():
        tens["param/" + k] = p.data.detach().float().contiguous().cpu()
    ost = w.updater.get_states()
    meta_opt = {}
    for k, v in ost.items():
        if isinstance(v, torch.Tensor):
            tens["opt/" + k] = v.contiguous().cpu()
        else:
            meta_opt[k] = v
    sync = getattr(w, "sync", None)
    if sync is not None:
        for attr in ("centre", "snapshot"):
            t = getattr(sync, attr, None)
            if t is not None:
                tens["sync/" + attr] = t.detach().contiguous().cpu()
    draws = {l.name: int(getattr(l, "draws", 0)) for l in w.train_net.layers if l.is_data}
    meta = {"step": int(getattr(w, "step", 0)), "opt": meta_opt, "model": schema.to_text(w.model),
            "nsync": int(getattr(sync, "nsync", 0)) if sync is not None else 0, "data_draws": draws}
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    with zipfile.ZipFile(tmp, "w") as z:
        z.writestr("tensors.safetensors", st_save(tens))
        z.writestr("meta.json", json.dumps(meta))
    os.replace(tmp, path)  # atomic: a crash never leaves a half-written checkpoint


def load_worker(w, path: str) -> dict:
    from safetensors.torch import load as st_load

    with zipfile.ZipFile(path, "r") as z:
        tens = st_load(z.read("tensors.safetensors"))
        meta = json.loads(z.read("meta.json").decode())
    table = _param_table(w.train_net)
    for k, p in table.items():
        key = "param/" + k
        if key not in tens:
            raise KeyError(f"checkpoint {path} has no tensor {key}")
        p.data.copy_(tens[key].reshape(p.data.shape).to(p.data.dtype))
    w.store.sync_low()
    ost = dict(meta.get("opt", {}))
    for k, v in tens.items():
        if k.startswith("opt/"):
            ost[k[4:]] = v
    w.updater.set_states(ost)
    sync = getattr(w, "sync", None)
    if sync is not None:
        for attr in ("centre", "snapshot"):
            if "sync/" + attr in tens:
                setattr(sync, attr, tens["sync/" + attr].to(w.store.w.device))
        sync.nsync = int(meta.get("nsync", 0))
        sync.resumed = True
    for l in w.train_net.layers:  # fast-forward the data sources
        n = int(meta.get("data_draws", {}).get(l.name, 0))
        if l.is_data and n and w.train_net.is_local(l):
            for _ in range(n):
                l.source.next()
            l.draws = n
    w.start_step = int(meta.get("step", 0))
    return meta
