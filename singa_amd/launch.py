"""Local multi-process launcher (reference C29, examples/mnist/run.sh: ssh
fan-out of one ``singa`` process per hostfile line).  One process per GPU:

    python -m singa_amd.launch --nproc 8 -- --model_conf m.conf --cluster_conf c.conf

* ``--nproc`` defaults to ``ClusterProto.nworkers`` of ``--cluster_conf`` (or
  the number of visible GPUs, or 1);
* ranks get ``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
  MASTER_PORT`` (env:// rendezvous replaces the hostfile + PING/PONG);
* failure detection: the launcher polls its children; when one exits
  non-zero it terminates the others (the reference left peers blocked in
  ``Router::Bind`` forever) and, with ``--max_restarts``,
  relaunches the whole job resuming from ``--checkpoint`` if it exists
  (checkpoint-based elastic recovery);
* ``--nservers N`` also starts N native parameter-server processes (the
  reference's server role, csrc/runtime/ps.cc) and switches the workers'
  inter-group exchange to them (``SINGA_AMD_PS=native``);
* the launcher itself never touches the GPU.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _default_nproc(args_after: List[str]) -> int:
    if "--cluster_conf" in args_after:
        path = args_after[args_after.index("--cluster_conf") + 1]
        try:
            from .config import schema

            c = schema.read_text_file("ClusterProto", path)
            if c.nworkers > 0:
                return c.nworkers
        except Exception:
            pass
    try:
        import torch

        n = torch.cuda.device_count()  # does not initialise the GPU on this image
        if n > 0:
            return n
    except Exception:
        pass
    return 1


def run_job(nproc: int, child_args: List[str], module: str = "singa_amd", poll_s: float = 0.2,
            timeout_s: float = 0.0, env_extra=None, nservers: int = 0, cmd: Optional[List[str]] = None) -> int:
    """Start ``nproc`` ranks (plus ``nservers`` PS processes) and wait.  Each
    child runs ``cmd + child_args`` (default ``python -m <module>``) with the
    rank environment; children share this process's stdout/stderr.  Returns
    0 when every child exits 0, otherwise the first failing child's code
    (124 on ``timeout_s``) after terminating the rest."""
    port = _free_port()
    procs = []
    prog = list(cmd) if cmd else [sys.executable, "-m", module]
    # native parameter-server processes (reference roles procsID >= nworkers):
    # they do not join the workers' process group
    for i in range(nservers):
        env = dict(os.environ)
        env.update(SINGA_AMD_ROLE="server", SINGA_AMD_SERVER_ID=str(i), SINGA_AMD_PS="native",
                   SINGA_AMD_NWORKERS=str(nproc))
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
            env.pop(k, None)
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(prog + child_args, env=env, start_new_session=True))
    for r in range(nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(nproc))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if nservers:
            env["SINGA_AMD_PS"] = "native"
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(prog + child_args, env=env, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                i, rc = bad[0]
                print(f"[launch] rank {i} exited with {rc}; stopping the job", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s and time.time() - t0 > timeout_s:
                print(f"[launch] job timed out after {timeout_s}s", file=sys.stderr)
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        i = argv.index("--")
        mine, child = argv[:i], argv[i + 1:]
    else:
        mine, child = [], argv
    ap = argparse.ArgumentParser(prog="singa_amd.launch")
    ap.add_argument("--nproc", type=int, default=0)
    ap.add_argument("--module", default="singa_amd")
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=0.0)
    ap.add_argument("--nservers", type=int, default=0,
                    help="also start N native parameter-server processes (SINGA_AMD_PS=native)")
    a = ap.parse_args(mine)
    n = a.nproc or _default_nproc(child)
    ckpt = child[child.index("--checkpoint") + 1] if "--checkpoint" in child else ""
    rc = run_job(n, child, a.module, timeout_s=a.timeout, nservers=a.nservers)
    attempt = 0
    while rc != 0 and attempt < a.max_restarts:
        attempt += 1
        args = list(child)
        probe = ckpt.replace("{rank}", "0")
        if ckpt and os.path.exists(probe) and "--resume" not in args:
            args += ["--resume", ckpt]
        print(f"[launch] restart {attempt}/{a.max_restarts}" + (f" resuming from {ckpt}" if "--resume" in args
                                                                 else ""), file=sys.stderr)
        rc = run_job(n, args, a.module, timeout_s=a.timeout, nservers=a.nservers)
    return rc


if __name__ == "__main__":
    sys.exit(main())
