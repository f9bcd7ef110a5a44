"""``singa_amd.model`` -- SINGA's Model API with HIP-graph execution.

``Model.compile(inputs, is_train, use_graph)`` materialises every layer's
parameters with one forward pass and, when an optimiser is set, re-homes them
into a flat :class:`singa_amd.opt.ParamStore`.  With ``use_graph=True`` on a
RocmGPU, the whole ``train_one_batch`` (forward, backward, all-reduce hooks
and the fused optimiser update) is captured ONCE into a HIP graph and then
replayed -- the MI355X replacement for SINGA's buffered-op graph executor: no
Python or launch overhead per op after capture.  Inputs are static device
buffers (as in SINGA graph mode): pass the same Tensor objects every step, or
different ones whose contents are copied into the captured inputs.

Checkpoints (``save_states`` / ``load_states``) are zip files holding a
safetensors blob of every parameter/state tensor, optimiser slots, and a JSON
dict of auxiliary values -- the resume path the reference left as a TODO
(``Worker::Resume``, src/worker/worker.cc:65-67).
"""
from __future__ import annotations

import io
import json
import os
import zipfile
from typing import Dict, Optional

import numpy as np
import torch

from . import autograd
from . import layer
from . import memory as _mem
from . import stream as _stream
from .ops import functional as _F
from .ops import glue as G
from .tensor import Tensor


class Model(layer.Layer):
    def __init__(self):
        super().__init__()
        self.training = True
        self.graph_mode = False
        self.sequential = False
        self.optimizer = None
        self.compute_dtype = torch.float32
        self._graphs: Dict[str, tuple] = {}
        self._warm: Dict[str, int] = {}
        self._pool = None
        self.graph_warmup = 2
        # a capture that raises: False -> re-raise; True -> log, switch this
        # model to eager execution and run the step eagerly (bench.py)
        self.graph_fallback = False
        self.graph_error: Optional[str] = None

    # ---------------------------------------------------------------- config
    def set_optimizer(self, optimizer) -> None:
        self.optimizer = optimizer

    def set_compute_dtype(self, dtype) -> None:
        self.compute_dtype = dtype

    def train(self, mode: bool = True) -> None:
        self.training = mode

    def eval(self) -> None:
        self.train(False)

    def graph(self, mode: bool = True, sequential: bool = False) -> None:
        self.graph_mode = mode
        self.sequential = sequential

    def on_device(self, dev) -> None:
        for p in self.get_states().values():
            p.to_device(dev)

    def compile(self, inputs, is_train: bool = True, use_graph: bool = False, sequential: bool = False):
        """Initialise parameters with one (tape-free) forward pass."""
        prev = autograd.training
        autograd.training = False
        try:
            self.forward(*inputs)
        finally:
            autograd.training = prev
        self.training = is_train
        self.graph(use_graph, sequential)
        if self.optimizer is not None and is_train:
            self._attach_optimizer()

    def _attach_optimizer(self) -> None:
        opt = self.optimizer
        if getattr(opt, "store", None) is not None:
            return
        params = self._flat_params()
        if not params:
            return
        gpu = params[0].data.is_cuda
        mixed = gpu and self.compute_dtype == torch.bfloat16
        opt.attach(params, mixed_bf16=mixed)

    # ------------------------------------------------------------ execution
    def __call__(self, *args, **kwargs):
        if not self._initialized:
            self._initialized = True
        fn = self.train_one_batch if self.training else self.forward
        if self.training and self.optimizer is not None and getattr(self.optimizer, "store", None) is None:
            # first call without compile(): materialise params, then attach
            prev = autograd.training
            autograd.training = False
            self.forward(*args[:self._n_forward_args(args)])
            autograd.training = prev
            self._attach_optimizer()
        use_graph = self.graph_mode and args and isinstance(args[0], Tensor) and args[0].data.is_cuda
        if not use_graph:
            autograd.training = self.training
            arena = self.training and args and isinstance(args[0], Tensor) and args[0].data.is_cuda
            if arena:  # one zeroing launch for every reduction workspace of the step
                _F.ARENA.begin(args[0].data.device)
            try:
                return fn(*args, **kwargs)
            finally:
                if arena:
                    _F.ARENA.end()
        return self._run_graph(fn, args, kwargs)

    def _n_forward_args(self, args) -> int:
        import inspect

        try:
            n = len([p for p in inspect.signature(self.forward).parameters.values()
                     if p.default is inspect.Parameter.empty and p.kind == p.POSITIONAL_OR_KEYWORD])
        except (TypeError, ValueError):
            n = 1
        return max(1, min(n, len(args)))

    def _run_graph(self, fn, args, kwargs):
        key = "train" if self.training else "eval"
        autograd.training = self.training
        opt = self.optimizer
        if key not in self._graphs:
            n = self._warm.get(key, 0)
            if n < self.graph_warmup:
                self._warm[key] = n + 1
                if self.training:
                    _F.ARENA.begin(args[0].data.device)
                try:
                    return fn(*args, **kwargs)
                finally:
                    _F.ARENA.end()
            _stream.device_synchronize(args[0].data.device)
            if opt is not None:
                getattr(opt, "opt", opt).graph_mode = True
                opt.prepare_step()
            sc0 = opt.step_counter if opt is not None else 0
            dev = args[0].device
            keep: list = []
            _F.CAPTURE_KEEP = keep

            def body():
                # first captured kernel: advance the device RNG epoch, so
                # dropout masks differ on every replay (host-side Philox
                # offsets are frozen into the captured launches)
                dev.advance_rng_epoch()
                if self.training:
                    _F.ARENA.begin(args[0].data.device)  # the arena's zeroing kernel is captured too
                try:
                    return fn(*args, **kwargs)
                finally:
                    _F.ARENA.end()

            try:
                if os.environ.get("SINGA_AMD_GRAPH_FAIL_TEST") == "1":  # test hook: a capture that raises
                    raise RuntimeError("SINGA_AMD_GRAPH_FAIL_TEST: capture refused")
                if os.environ.get("SINGA_AMD_NATIVE_GRAPH", "1") != "0":
                    # framework-owned capture (hipStreamBeginCapture on a native
                    # stream); the step's memory is the graph's private native
                    # pool -- one per graph, so the eval graph's static outputs
                    # never share blocks with the train graph's temporaries
                    g = _stream.new_step_graph(args[0].data.device)
                    out = g.capture(body)
                else:
                    g = torch.cuda.CUDAGraph()
                    if self._pool is None:
                        self._pool = {}
                    pool = self._pool.setdefault(key, torch.cuda.graph_pool_handle())
                    gp = _mem.graph_pool(args[0].data.device)
                    keep.append(gp)
                    with torch.cuda.graph(g, pool=pool), gp:
                        out = body()
            except Exception as e:
                _F.CAPTURE_KEEP = None
                if not self.graph_fallback:
                    raise
                return self._eager_after_failed_capture(fn, args, kwargs, e)
            finally:
                _F.CAPTURE_KEEP = None
            if opt is not None:
                opt.step_counter = sc0  # capture does not execute; replay below does
            self._graphs[key] = (g, tuple(args), out, keep)
        g, sargs, out = self._graphs[key][:3]
        for a, s in zip(args, sargs):
            if isinstance(a, Tensor) and a is not s and a.data.data_ptr() != s.data.data_ptr():
                G.copy_(s.data, G.reshape(a.data, s.shape))
        if opt is not None and self.training:
            opt.prepare_step()
        g.replay()
        if opt is not None and self.training:
            if hasattr(opt, "post_replay"):
                opt.post_replay()
            opt.step_counter += 1
        return out

    def _eager_after_failed_capture(self, fn, args, kwargs, err):
        """The capture raised: this model runs eagerly from now on.  The
        optimiser leaves graph mode (its eager ``step()`` writes lr / t again)
        and gets the hyper-parameters of the step about to run."""
        import sys

        self.graph_error = f"{type(err).__name__}: {err}"[:300]
        print(f"singa_amd.Model: HIP-graph capture failed ({self.graph_error}); running eagerly", file=sys.stderr)
        self.reset_graph()
        self.graph(False, self.sequential)
        opt = self.optimizer
        if opt is not None:
            getattr(opt, "opt", opt).graph_mode = False
            opt.prepare_step()
        autograd.training = self.training
        if self.training:
            _F.ARENA.begin(args[0].data.device)
        try:
            return fn(*args, **kwargs)
        finally:
            _F.ARENA.end()

    def reset_graph(self) -> None:
        gs, self._graphs = self._graphs, {}
        for g, _, _, keep in gs.values():
            if hasattr(g, "release"):
                g.release()  # the graph, then its private memory
        pools = [k for ent in gs.values() for k in ent[3] if isinstance(k, _mem.graph_pool)]
        del gs
        for k in pools:
            k.release()
        self._warm.clear()

    def forward(self, *args, **kwargs):
        raise NotImplementedError

    def train_one_batch(self, *args, **kwargs):
        raise NotImplementedError

    # -------------------------------------------------------- checkpointing
    def save_states(self, fpath: str, aux_states: Optional[dict] = None) -> None:
        from safetensors.torch import save as st_save

        states = {k: v.data.detach().float().contiguous().cpu() if v.data.is_floating_point()
                  else v.data.detach().contiguous().cpu() for k, v in self.get_states().items()}
        aux_t, aux_j = {}, {}
        for k, v in (aux_states or {}).items():
            if isinstance(v, Tensor):
                aux_t["aux/" + k] = v.data.detach().contiguous().cpu()
            elif isinstance(v, torch.Tensor):
                aux_t["aux/" + k] = v.detach().contiguous().cpu()
            elif isinstance(v, np.ndarray):
                aux_t["aux/" + k] = torch.from_numpy(np.ascontiguousarray(v))
            else:
                aux_j[k] = v
        opt_meta = {}
        if self.optimizer is not None:
            ost = self.optimizer.get_states()
            for k, v in ost.items():
                if isinstance(v, torch.Tensor):
                    aux_t["opt/" + k] = v.contiguous()
                else:
                    opt_meta[k] = v
        blob = st_save({**states, **aux_t})
        d = os.path.dirname(os.path.abspath(fpath))
        os.makedirs(d, exist_ok=True)
        with zipfile.ZipFile(fpath, "w", compression=zipfile.ZIP_STORED) as z:
            z.writestr("tensors.safetensors", blob)
            z.writestr("meta.json", json.dumps({"aux": aux_j, "opt": opt_meta, "format": "singa_amd-1"}))

    def load_states(self, fpath: str) -> dict:
        from safetensors.torch import load as st_load

        with zipfile.ZipFile(fpath, "r") as z:
            tens = st_load(z.read("tensors.safetensors"))
            meta = json.loads(z.read("meta.json").decode())
        states = {k: v for k, v in tens.items() if not k.startswith(("aux/", "opt/"))}
        self.set_states(states)
        aux = dict(meta.get("aux", {}))
        for k, v in tens.items():
            if k.startswith("aux/"):
                aux[k[4:]] = v
        if self.optimizer is not None:
            ost = dict(meta.get("opt", {}))
            for k, v in tens.items():
                if k.startswith("opt/"):
                    ost[k[4:]] = v
            if ost:
                self.optimizer.set_states(ost)
        return aux
