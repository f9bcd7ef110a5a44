"""Cluster topology (reference C16, include/utils/cluster.h:20-121).

The reference assigns roles by a global ``procsID`` read from a hostfile:
workers ``[0, nworkers)``, servers ``[nworkers, nworkers+nservers)``; worker
groups are ``procsid / nprocs_per_group``; each process runs
``nthreads_per_procs`` executor threads; ports derive from ``start_port``.

On an MI355X node the process is a GPU rank (``torch.distributed``), so:

* ``procsID`` = global rank, hostfile/ports = the env:// rendezvous;
* a worker *group* = ``nprocs_per_group`` consecutive ranks that jointly run
  one (partitioned) net -- P4/P5/P6 across GPUs, bridges over RCCL p2p;
* groups exchange parameters with EASGD / RandomSync (or, with
  ``synchronous: true`` -- declared but never read by the reference, P10 --
  gradient all-reduce every step);
* servers are dissolved into collectives; ``nservers > 1`` selects the
  key-sharded EASGD centre (reduce-scatter/all-gather, the PS key sharding
  P7) instead of a replicated one;
* ``bandwidth`` feeds RandomSync's sample-ratio model; ``workspace`` /
  ``vis_subfolder`` / ``log_subfolder`` are created like the reference.

Sub-communicators: ``group_comm`` (the ranks of my group, for bridges and
replica-gradient all-reduce) and ``peer_comm`` (the ranks holding the same
partition in every group, for inter-group sync).
"""
from __future__ import annotations

import os
from typing import Optional

from ..parallel.communicator import Communicator, init_distributed


class Cluster:
    _instance: Optional["Cluster"] = None

    def __init__(self, proto=None, comm: Optional[Communicator] = None, procs_id: Optional[int] = None,
                 make_folders: bool = True):
        from ..config import schema

        self.proto = proto if proto is not None else schema.new("ClusterProto")
        self.comm = comm or init_distributed()
        p = self.proto
        self.world = self.comm.world_size
        self.global_procsid = self.comm.rank if procs_id is None else int(procs_id)
        nw = p.nworkers if p.HasField("nworkers") and p.nworkers > 0 else self.world
        self._nworkers = min(nw, self.world) if self.world > 1 else nw
        self._nprocs_per_group = max(1, p.nprocs_per_group)
        if self.world > 1 and self.world % self._nprocs_per_group:
            raise ValueError(f"world size {self.world} is not a multiple of nprocs_per_group "
                             f"{self._nprocs_per_group}")
        self.group_comm: Optional[Communicator] = None
        self.peer_comm: Optional[Communicator] = None
        if self.world > 1:
            self._build_subcomms()
        if make_folders and p.HasField("workspace") and p.workspace:
            for sub in (p.vis_subfolder, p.log_subfolder):
                os.makedirs(os.path.join(p.workspace, sub), exist_ok=True)

    # ------------------------------------------------------------ singleton
    @classmethod
    def get(cls, proto=None, comm=None, procs_id=None) -> "Cluster":
        if cls._instance is None:
            cls._instance = cls(proto, comm, procs_id)
        return cls._instance

    @classmethod
    def reset(cls):
        cls._instance = None

    # -------------------------------------------------------------- roles
    def nworkers(self) -> int:
        return self._nworkers

    def nservers(self) -> int:
        return self.proto.nservers

    def am_i_worker(self) -> bool:
        return 0 <= self.global_procsid < self._nworkers

    def am_i_server(self) -> bool:
        """Servers are dissolved into collectives: no process takes the role."""
        return False

    def nprocs_per_group(self) -> int:
        return self._nprocs_per_group

    def nthreads_per_procs(self) -> int:
        return max(1, self.proto.nthreads_per_procs)

    def nthreads_per_server(self) -> int:
        return max(1, self.proto.nthreads_per_server)

    def groupid(self) -> int:
        return self.global_procsid // self._nprocs_per_group

    def ngroups(self) -> int:
        return max(1, self._nworkers // self._nprocs_per_group)

    def group_procsid(self) -> int:
        return self.global_procsid % self._nprocs_per_group

    def nthreads_per_group(self) -> int:
        return self.nthreads_per_procs() * self._nprocs_per_group

    def group_threadid(self, local_threadid: int = 0) -> int:
        return self.group_procsid() * self.nthreads_per_procs() + local_threadid

    def synchronous(self) -> bool:
        return bool(self.proto.synchronous)

    def bandwidth(self) -> float:
        return float(self.proto.bandwidth)

    def workspace(self) -> str:
        return self.proto.workspace

    def visualization_folder(self) -> str:
        return os.path.join(self.proto.workspace, self.proto.vis_subfolder)

    def log_folder(self) -> str:
        return os.path.join(self.proto.workspace, self.proto.log_subfolder)

    def sharded_centre(self) -> bool:
        return self.proto.nservers > 1

    # ------------------------------------------------------ communicators
    def group_ranks(self, gid: Optional[int] = None):
        g = self.groupid() if gid is None else gid
        return list(range(g * self._nprocs_per_group, (g + 1) * self._nprocs_per_group))

    def peer_ranks(self, gpid: Optional[int] = None):
        q = self.group_procsid() if gpid is None else gpid
        return [g * self._nprocs_per_group + q for g in range(self.world // self._nprocs_per_group)]

    def _build_subcomms(self):
        # every rank must create every group in the same order (torch.distributed rule)
        ng = self.world // self._nprocs_per_group
        for g in range(ng):
            c = self.comm.split(self.group_ranks(g))
            if c is not None:
                self.group_comm = c
        for q in range(self._nprocs_per_group):
            c = self.comm.split(self.peer_ranks(q))
            if c is not None:
                self.peer_comm = c

    def __repr__(self):
        return (f"Cluster(procsid={self.global_procsid}, nworkers={self._nworkers}, group={self.groupid()}/"
                f"{self.ngroups()}, group_procsid={self.group_procsid()}/{self._nprocs_per_group})")
