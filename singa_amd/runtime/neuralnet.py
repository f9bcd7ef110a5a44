"""NeuralNet (reference C23, src/worker/neuralnet.cc): builds the layer DAG
from a ``NetProto``, topologically sorts it (native ``_core.Graph``), infers
shapes, optionally partitions it across a worker group, shares weights
between train/test/validation nets, and exports a node-link JSON graph.

Partitioning (P4 data partition on dim 0, P5 layer partition on dim 1, P6
placement by ``locationid``) follows the reference's graph-rewrite rules
(CreatePartitonedGraph, neuralnet.cc:198-323): partitioned layers become
``name-00..name-(g-1)`` nodes; Slice / Concate / Split nodes are inserted on
mixed edges; fan-out gets a Split; edges that cross locations get a
BridgeSrc -> BridgeDst pair.  Unlike the reference (where the partitioned net
was never executed and the connection layers were stubs), the partitioned
net here runs: data-partition replicas share their parameters (and loss
replicas are scaled by 1/g, the reference ParamManager's grad_scale=1/k
aggregation), layer-partition replicas own their slice of the parameters,
and the result equals the unpartitioned net (tests/test_neuralnet.py).
"""
from __future__ import annotations

import json
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import autograd
from ..config import schema
from ..ops import functional as F
from ..ops import glue as G
from ..tensor import Tensor
from .layers import RefLayer, create_layer


class _Node:
    def __init__(self, name, origin, loc, pid, slice_dim=-1, concate_dim=-1):
        self.name, self.origin, self.loc, self.pid = name, origin, loc, pid
        self.slice_dim, self.concate_dim = slice_dim, concate_dim
        self.srcs: List["_Node"] = []
        self.dsts: List["_Node"] = []


class _PGraph:
    def __init__(self):
        self.nodes: "OrderedDict[str, _Node]" = OrderedDict()

    def add(self, name, *a, **k) -> _Node:
        base, i = name, 1
        while name in self.nodes:
            name = f"{base}#{i}"
            i += 1
        n = _Node(name, *a, **k)
        self.nodes[name] = n
        return n

    @staticmethod
    def edge(a: _Node, b: _Node):
        if b not in a.dsts:
            a.dsts.append(b)
            b.srcs.append(a)

    @staticmethod
    def remove(a: _Node, b: _Node):
        a.dsts.remove(b)
        b.srcs.remove(a)

    def slice_node(self, src, dsts, slice_dim, connect=True):
        n = self.add("slice-" + src.name, "kSlice", src.loc, src.pid, slice_dim=slice_dim)
        self.edge(src, n)
        if connect:
            for d in dsts:
                self.edge(n, d)
        return n

    def concate_node(self, srcs, dst, concate_dim):
        n = self.add("concate-" + dst.name, "kConcate", dst.loc, dst.pid, concate_dim=concate_dim)
        self.edge(n, dst)
        for s in srcs:
            self.edge(s, n)
        return n

    def split_node(self, src, dsts):
        n = self.add("split-" + src.name, "kSplit", src.loc, src.pid)
        self.edge(src, n)
        for d in dsts:
            self.edge(n, d)
        return n

    def bridge(self, src, dst):
        """Replace edge src->dst by src->BridgeSrc->BridgeDst->dst, keeping
        the positions in src.dsts / dst.srcs (concate order = partition id)."""
        a = self.add(f"s-{src.name}-{dst.name}", "kBridgeSrc", src.loc, src.pid)
        b = self.add(f"d-{src.name}-{dst.name}", "kBridgeDst", dst.loc, dst.pid)
        src.dsts[src.dsts.index(dst)] = a
        a.srcs.append(src)
        self.edge(a, b)
        b.dsts.append(dst)
        dst.srcs[dst.srcs.index(src)] = b

    def sort(self) -> List[_Node]:
        from .. import _core

        g = _core.Graph()
        for n in self.nodes.values():
            g.add_node(n.name)
        for n in self.nodes.values():
            for d in n.dsts:
                g.add_edge(n.name, d.name)
        order = g.sort()
        self.nodes = OrderedDict((k, self.nodes[k]) for k in order)
        return list(self.nodes.values())


def _micro_slice(out, i: int, m: int):
    """Micro-batch i of m of a data layer's output (views along dim 0)."""
    if isinstance(out, dict):
        return {k: _micro_slice(v, i, m) for k, v in out.items()}
    B = out.data.shape[0]
    if B % m:
        raise ValueError(f"batch {B} does not split into {m} micro-batches")
    k = B // m
    return Tensor(device=out.device, data=out.data[i * k:(i + 1) * k], requires_grad=False)


class NeuralNet:
    def __init__(self, net_proto, group_size: int = 1, phase: str = "kTrain", dev=None,
                 data_override: Optional[dict] = None, seed: int = 0, devices: Optional[List] = None,
                 comm=None):
        from ..device import get_default_device

        self.dev = dev or get_default_device()
        self.devices = devices  # per-location device list (placement, P6, one process)
        # group communicator: locations are owned by the group's processes
        # (location l -> group rank l % size), bridges become p2p send/recv
        self.comm = comm if comm is not None and comm.world_size > 1 else None
        self.dist = self.comm is not None
        self.before_layer = None  # hook(params) before a layer's forward (per-parameter EASGD waits)
        if self.dist:
            group_size = max(group_size, self.comm.world_size)
        self.group_size = group_size
        self.phase = phase
        default_pt = schema.enum_name(net_proto, "partition_type")
        protos = []
        for lp in net_proto.layer:
            excl = [schema.message_class("LayerProto").DESCRIPTOR.fields_by_name["exclude"].enum_type
                    .values_by_number[e].name for e in lp.exclude]
            if phase in excl:
                continue
            protos.append(lp)
        self.layers: List[RefLayer] = []
        self.name2layer: Dict[str, RefLayer] = {}
        for lp in protos:
            pt = schema.enum_name(lp, "partition_type") if lp.HasField("partition_type") else default_pt
            layer = create_layer(lp, partition_type=pt)
            self.layers.append(layer)
            self.name2layer[layer.name] = layer
        self.gen = torch.Generator().manual_seed(seed)
        data_override = data_override or {}
        for l in self.layers:
            if l.is_data:
                ov = data_override.get(l.name, data_override.get("*", {}))
                l.configure(synthetic_shape=ov.get("shape", (28, 28)), nclass=ov.get("nclass", 10),
                            seed=ov.get("seed", seed), prefetch=ov.get("prefetch", True))
                if "batch" in ov:
                    l.batch = int(ov["batch"])
                    l.source.batch = l.batch
                    if l.source.prefetcher is not None:
                        raise ValueError("batch override is not supported for shard-backed data layers")
        self._construct()
        self.partitioned = group_size > 1 and any(l.partition_type != "kNone" for l in self.layers)
        self.placed = len({l.locationid for l in self.layers}) > 1
        self.partitioned = self.partitioned or self.placed  # placement alone still needs bridges
        if self.partitioned:
            self._partition()
        self._assign_param_ids()

    # ------------------------------------------------------------- construct
    def _construct(self):
        from .. import _core

        g = _core.Graph()
        for l in self.layers:
            g.add_node(l.name)
        for l in self.layers:
            for s in l.srcs:
                if s not in self.name2layer:
                    raise KeyError(f"layer {l.name}: unknown src layer {s}")
                g.add_edge(s, l.name)
        order = g.sort()
        self.layers = [self.name2layer[n] for n in order]
        self.order = order
        self.dsts: Dict[str, List[str]] = {l.name: [] for l in self.layers}
        for l in self.layers:
            for s in l.srcs:
                self.dsts[s].append(l.name)
        shapes: Dict[str, tuple] = {}
        for l in self.layers:
            src_shapes = []
            for s in l.srcs:
                src_shapes.append(shapes[s])
            shapes[l.name] = l.setup(src_shapes, self._dev_of(l.locationid), self.gen)
        self.shapes = shapes

    def _dev_of(self, loc: int):
        if self.devices:
            return self.devices[loc % len(self.devices)]
        return self.dev

    # ------------------------------------------------------------- partition
    def _partition(self):
        g = self.group_size
        pg = _PGraph()
        l2n: Dict[str, List[_Node]] = {}
        for l in self.layers:
            if l.partition_type in ("kDataPartition", "kLayerPartition"):
                l2n[l.name] = [pg.add(f"{l.name}-{i:02d}", l.name, i, i) for i in range(g)]
            else:
                l2n[l.name] = [pg.add(l.name, l.name, l.locationid, 0)]
        for l in self.layers:
            nodes = l2n[l.name]
            tt = l.partition_type
            for si, sname in enumerate(l.srcs):
                src = self.name2layer[sname]
                snodes = l2n[sname]
                st = src.partition_type
                conn = l.connection_type(si)
                part = ("kDataPartition", "kLayerPartition")
                if st == "kNone":
                    if tt == "kDataPartition" or (tt == "kLayerPartition" and conn == "kOneToOne"):
                        pg.slice_node(snodes[0], nodes, l.partition_dimension())
                    elif tt == "kNone":
                        pg.edge(snodes[0], nodes[0])
                    else:
                        pg.split_node(snodes[0], nodes)
                elif (tt == "kNone" and st in part) or (tt == "kLayerPartition" and conn == "kOneToAll"
                                                        and st in part):
                    for n in nodes:
                        pg.concate_node(snodes, n, src.partition_dimension())
                elif (st == "kLayerPartition" and tt == "kDataPartition") or (
                        st == "kDataPartition" and tt == "kLayerPartition"):
                    slices = [pg.slice_node(sn, nodes, l.partition_dimension(), connect=False) for sn in snodes]
                    for n in nodes:
                        pg.concate_node(slices, n, src.partition_dimension())
                else:  # same partitioning, one-to-one
                    for a, b in zip(snodes, nodes):
                        pg.edge(a, b)
        order = pg.sort()
        for i, n in enumerate(order):
            if i > 0 and len(n.dsts) > 1 and n.origin not in ("kSlice", "kSplit"):
                sp = pg.add("split-" + n.name, "kSplit", n.loc, n.pid)
                for d in n.dsts:  # keep each consumer's input position
                    d.srcs[d.srcs.index(n)] = sp
                sp.dsts, n.dsts = list(n.dsts), [sp]
                sp.srcs.append(n)
        for n in list(pg.sort()):
            for d in list(n.dsts):
                if n.loc != d.loc:
                    pg.bridge(n, d)
        order = pg.sort()
        self.graph_nodes = order
        self._instantiate_partitioned(order)

    def _instantiate_partitioned(self, order: List[_Node]):
        from .layers import create_layer as mk

        g = self.group_size
        orig = self.name2layer
        new_layers: List[RefLayer] = []
        by_name: Dict[str, RefLayer] = {}
        shapes: Dict[str, tuple] = {}
        self.slice_route: Dict[str, Dict[str, int]] = {}
        for n in order:
            if n.origin in ("kSlice", "kConcate", "kSplit", "kBridgeSrc", "kBridgeDst"):
                lp = schema.new("LayerProto")
                lp.name, lp.type, lp.locationid, lp.partitionid = n.name, n.origin, n.loc, n.pid
                if n.origin == "kSlice":
                    lp.slice_param.slice_dimension = n.slice_dim
                    lp.slice_param.slice_num = len(n.dsts)
                elif n.origin == "kConcate":
                    lp.concate_param.concate_dimension = n.concate_dim
                    lp.concate_param.concate_num = len(n.srcs)
                elif n.origin == "kSplit":
                    lp.split_param.num_splits = len(n.dsts)
                layer = mk(lp)
            else:
                base = orig[n.origin]
                if base.partition_type == "kNone":
                    layer = base
                else:
                    lp = schema.new("LayerProto")
                    lp.CopyFrom(base.proto)
                    lp.name, lp.locationid, lp.partitionid = n.name, n.loc, n.pid
                    layer = mk(lp, partition_type=base.partition_type)
                    pdim = base.partition_dimension()
                    full = base.shape[pdim]
                    share = full // g + (full % g if n.pid == g - 1 else 0)
                    if base.partition_type == "kLayerPartition" and pdim == 1:
                        layer.nf_override = share
                        layer.part_offset = (full // g) * n.pid
                    if base.partition_type == "kDataPartition":
                        layer.params = base.params  # replicas share the parameters
                        if base.is_loss:
                            layer.loss_scale = 1.0 / g
                    layer.origin = base
            layer.srcs = [s.name for s in n.srcs]
            layer.graph_dsts = [d.name for d in n.dsts]
            new_layers.append(layer)
            by_name[n.name] = layer
        # shapes / params for the new layers
        for layer in new_layers:
            src_shapes = []
            for s in layer.srcs:
                sl = by_name[s]
                if sl.type_name == "kSlice":
                    src_shapes.append(sl.shapes[sl.graph_dsts.index(layer.name)])
                else:
                    src_shapes.append(shapes[s])
            if layer.partition_type == "kLayerPartition" and getattr(layer, "origin", None) is not None \
                    and not layer.params:
                base = layer.origin
                shapes[layer.name] = layer.setup(src_shapes, self._dev_of(layer.locationid), self.gen)
                # take this partition's slice of the unpartitioned params
                off = getattr(layer, "part_offset", None)
                if not base.params or off is None:
                    continue
                w = base.params[0].data
                if base.type_name == "kConvolution":
                    G.copy_(layer.params[0].data, w[off:off + layer.nf])
                else:
                    G.copy_(layer.params[0].data, w[:, off:off + layer.hdim])
                if len(base.params) > 1:
                    nb = layer.params[1].shape[0]
                    G.copy_(layer.params[1].data, base.params[1].data[off:off + nb])
            else:
                shapes[layer.name] = layer.setup(src_shapes, self._dev_of(layer.locationid), self.gen)
        self.layers = new_layers
        self.name2layer = by_name
        self.shapes = shapes
        self.order = [l.name for l in new_layers]

    def _assign_param_ids(self):
        seen, pid = set(), 0
        for l in self.layers:
            for p in l.params:
                if id(p) not in seen:
                    seen.add(id(p))
                    if p.param_meta is None:
                        p.param_meta = {}
                    p.param_meta["id"] = pid
                    pid += 1
        self.num_params = pid

    # -------------------------------------------------------------- execute
    def _rank_of(self, loc: int) -> int:
        return loc % self.comm.world_size

    def is_local(self, l: RefLayer) -> bool:
        return not self.dist or self._rank_of(l.locationid) == self.comm.rank

    def params(self) -> List[Tensor]:
        """Parameters of the layers this process executes."""
        out, seen = [], set()
        for l in self.layers:
            if not self.is_local(l):
                continue
            for p in l.params:
                if id(p) not in seen:
                    seen.add(id(p))
                    out.append(p)
        return out

    def loss_layers(self) -> List[RefLayer]:
        return [l for l in self.layers if l.is_loss and self.is_local(l)]

    def forward(self, training: bool = True, micro: Optional[tuple] = None) -> Dict[str, object]:
        """Run every (local) layer in the global topological order; returns
        name -> output.  Cross-process bridges send/receive (see
        :mod:`singa_amd.parallel.bridge`); cross-device inputs are moved.
        ``micro`` = (i, m): micro-batch i of m (pipelined execution,
        :mod:`singa_amd.parallel.pipeline`): data layers draw their batch at
        i == 0 and every pass consumes its 1/m slice of it."""
        from ..parallel import bridge as B

        autograd.training = training
        outs: Dict[str, object] = {}
        self._extra_roots = []
        self._mb_batch = getattr(self, "_mb_batch", {})
        if getattr(self, "_pending", None) is None and self.dist:
            # the config-driven data layers always yield full batches: fixed
            # message shapes, so receives may post from the cached headers
            self._pending = B.P2PChannel(self.comm, static_shapes=True)
        for l in self.layers:
            if not self.is_local(l):
                continue
            ldev = self._dev_of(l.locationid)
            if self.dist and l.type_name == "kBridgeDst":
                src = self.name2layer[l.srcs[0]]
                if not self.is_local(src):
                    y = B.BridgeRecv(self.comm, self._rank_of(src.locationid), self._pending)(ldev)
                    if y.requires_grad:
                        self._extra_roots.append((y, G.zeros_like(y.data)))
                    outs[l.name] = y
                    continue
            xs = []
            for s in l.srcs:
                o = outs[s]
                if isinstance(o, list):  # slice: pick this consumer's part
                    src = self.name2layer[s]
                    dsts = getattr(src, "graph_dsts", None) or self.dsts.get(s, [])
                    o = o[dsts.index(l.name)]
                if isinstance(o, Tensor) and o.data.device != ldev.torch_device:
                    o = B.to_device(o, ldev)
                xs.append(o)
            if micro is not None and l.is_data:
                i, m = micro
                if i == 0 or l.name not in self._mb_batch:
                    self._mb_batch[l.name] = l.forward(xs, training)
                outs[l.name] = _micro_slice(self._mb_batch[l.name], i, m)
                continue
            if self.dist and l.type_name == "kBridgeSrc":
                dst = self.name2layer[l.graph_dsts[0]]
                if not self.is_local(dst):
                    r = B.bridge_send(xs[0], self.comm, self._rank_of(dst.locationid), self._pending)
                    if r is not None:
                        self._extra_roots.append((r, None))
                    outs[l.name] = xs[0]
                    continue
            if self.before_layer is not None and l.params:
                self.before_layer(l.params)  # (per-parameter EASGD: join this layer's exchange)
            outs[l.name] = l.forward(xs, training)
        self.outputs = outs
        return outs

    def backward_roots(self, outs) -> tuple:
        """(roots, seeds) for :func:`autograd.backward`: the local loss plus,
        in a distributed group, every bridge endpoint."""
        roots, seeds = [], []
        loss = self.total_loss(outs)
        if loss is not None:
            roots.append(loss)
            seeds.append(None)
        for t, d in getattr(self, "_extra_roots", []):
            roots.append(t)
            seeds.append(d)
        return roots, seeds

    def finish_step(self) -> None:
        """Complete outstanding bridge sends."""
        from ..parallel import bridge as B

        B.wait_all(getattr(self, "_pending", []))

    def replica_keys(self) -> List[tuple]:
        """(base layer, param index, numel) of every data-partition-replicated
        parameter, in the same order on every process of the group."""
        keys = []
        for l in self.layers:
            base = getattr(l, "origin", None)
            if base is None or base.partition_type != "kDataPartition" or not base.params:
                continue
            if any(k[0] is base for k in keys):
                continue
            for i, p in enumerate(base.params):
                keys.append((base, i, p.data.numel()))
        return keys

    def sync_replica_grads(self) -> None:
        """Sum the gradients of data-partition replicas held by different
        processes of the group (the reference ParamManager aggregated
        shared-param gradients in-process, param_manager.cc:169-187)."""
        if not self.dist:
            return
        keys = getattr(self, "_rkeys", None)
        if keys is None:
            keys = self._rkeys = self.replica_keys()
        if not keys:
            return
        held = {id(p) for p in self.params()}
        total = sum(k[2] for k in keys)
        buf = G.zeros((total,), torch.float32, self.dev.torch_device)
        o = 0
        spans = []
        for base, i, n in keys:
            p = base.params[i]
            if id(p) in held and p.grad_view is not None:
                G.copy_(buf[o:o + n], G.reshape(p.grad_view, (-1,)))
                spans.append((p, o, n))
            o += n
        self.comm.all_reduce(buf)
        for p, o, n in spans:
            G.copy_(p.grad_view, buf[o:o + n].reshape(p.grad_view.shape))

    def total_loss(self, outs) -> Optional[Tensor]:
        losses = [outs[l.name] for l in self.loss_layers()]
        if not losses:
            return None
        tot = losses[0]
        for t in losses[1:]:
            tot = autograd.add(tot, t)
        return tot

    def metrics(self, reduce: bool = True) -> np.ndarray:
        """[loss, precision] summed over loss layers (reference metric blob);
        summed over the processes of a distributed group (``reduce``)."""
        m = np.zeros(2, np.float64)
        for l in self.loss_layers():
            if hasattr(l, "metric"):
                m += np.array([float(l.metric[0]), float(l.metric[1])]) * (l.loss_scale if l.loss_scale else 1)
        if self.dist and reduce:
            t = torch.tensor(m, dtype=torch.float32, device=self.dev.torch_device)
            self.comm.all_reduce(t)
            m = t.cpu().double().numpy()
        return m

    def share_weights(self, other: "NeuralNet") -> None:
        """Share parameter storage with ``other`` (test/validation nets)."""
        src = {}
        for l in other.layers:  # exact layer (incl. partition replicas) first, then its origin
            src.setdefault(l.name, l.params)
            src.setdefault(getattr(l, "origin", l).name, l.params)
        for l in self.layers:
            key = l.name if l.name in src else getattr(l, "origin", l).name
            if key in src and len(src[key]) == len(l.params):
                for a, b in zip(l.params, src[key]):
                    a.data = b.data
                    a.low = b.low
                l.params = src[key]

    def share_weights_private_grads(self, other: "NeuralNet", store, gbuf: torch.Tensor) -> None:
        """Executor-thread replica (P3): share ``other``'s weight storage but
        accumulate gradients into ``gbuf`` (same flat layout as ``store.g``),
        so concurrent backward passes never write the same gradient memory."""
        off = {id(p): (o, p) for p, o in zip(store.params, store.offsets)}
        src = {l.name: l.params for l in other.layers}
        for l in self.layers:
            if l.name not in src or len(src[l.name]) != len(l.params):
                continue
            mine = []
            for b in src[l.name]:
                t = Tensor(device=b.device, data=b.data, requires_grad=True, stores_grad=True, name=b.name)
                t.low, t.param_meta = b.low, b.param_meta
                o, _ = off[id(b)]
                t.grad_view = store._view(gbuf, o, b.data.shape)
                mine.append(t)
            l.params = mine

    def to_json(self) -> str:
        """Node-link JSON (colour by locationid), script/graph.py compatible."""
        from .. import _core

        g = _core.Graph()
        for l in self.layers:
            g.add_node(l.name)
        for l in self.layers:
            for s in l.srcs:
                g.add_edge(s, l.name)
        return g.to_json([l.locationid for l in self.layers])

    def debug_info(self) -> str:
        """norm1 (mean |x|) of every layer output and parameter (reference
        NeuralNet::DebugInfo; Blob::asum_data is a mean, Appendix A #14)."""
        lines = []

        def norm1(t):
            return float(G.reduce(F.unary("abs", G.to(t, torch.float32)), None, "mean", out_dtype=torch.float32))
        for l in self.layers:
            o = getattr(self, "outputs", {}).get(l.name)
            if isinstance(o, Tensor):
                lines.append(f"layer {l.name} data norm1 {norm1(o.data):.6f}")
            for p in l.params:
                g = p.grad_view
                gs = f" grad norm1 {norm1(g):.6f}" if g is not None else ""
                lines.append(f"param {p.name} data norm1 {norm1(p.data):.6f}{gs}")
        return "\n".join(lines)

    def __repr__(self):
        return "NeuralNet(" + ", ".join(f"{l.name}:{self.shapes.get(l.name)}" for l in self.layers) + ")"
