"""bench.py self-launch (``python bench.py --gpus N`` with no WORLD_SIZE):
the parent spawns N ranks with the rendezvous environment, rank 0's JSON
line reaches the parent's stdout, a failing rank stops its peers and the
job exits non-zero.  Stub workers stand in for the GPU bench (CPU only)."""
import json
import os
import subprocess
import sys
import textwrap
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent("""
    import json, os, sys, time
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
    assert os.environ["LOCAL_RANK"] == str(r)
    mode = sys.argv[1]
    if mode == "ok":
        if r == 0:
            print(json.dumps({"n_gpus": w, "args": sys.argv[1:]}), flush=True)
        sys.exit(0)
    if mode == "fail":
        if r == 1:
            sys.exit(3)
        time.sleep(60)  # the launcher must kill this rank
    if mode == "hang":
        time.sleep(60)
""")


def _run(tmp_path, mode, n=2, timeout=0.0):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    code = (f"import sys; sys.path.insert(0, {REPO!r}); import bench; "
            f"sys.exit(bench.self_launch({n}, [{mode!r}], {timeout}, script={str(stub)!r}))")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    return p, time.time() - t0


def test_self_launch_relays_rank0_json(tmp_path):
    p, _ = _run(tmp_path, "ok", n=4)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["args"] == ["ok"]


def test_self_launch_failure_stops_peers(tmp_path):
    p, dt = _run(tmp_path, "fail", n=3)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert dt < 30  # rank 0's 60 s sleep was cut short
    assert "rank 1 exited with 3" in p.stderr


def test_self_launch_timeout(tmp_path):
    p, dt = _run(tmp_path, "hang", n=2, timeout=2.0)
    assert p.returncode == 124 and dt < 30


def test_bench_parent_does_not_import_torch(tmp_path):
    """The self-launching parent must not initialise the GPU: it does not even
    import torch before spawning (checked with a stub that reports the
    parent's modules through a file)."""
    out = tmp_path / "mods.txt"
    code = (f"import sys; sys.path.insert(0, {REPO!r}); import bench\n"
            f"orig = bench.self_launch\n"
            f"def spy(n, argv, t=0.0, script=None):\n"
            f"    open({str(out)!r}, 'w').write('torch' if 'torch' in sys.modules else 'clean')\n"
            f"    return 0\n"
            f"bench.self_launch = spy\n"
            f"sys.argv = ['bench.py', '--gpus', '2']\n"
            f"sys.exit(bench.main())")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    assert out.read_text() == "clean"


def _bench():
    import importlib
    import sys as _sys
    _sys.path.insert(0, REPO)
    return importlib.import_module("bench")


def test_bench_model_switch_builds_each_config():
    """--model resnet50 / alexnet / bert: the BASELINE configs' models, inputs
    of their shapes and the record fields (built on the CppCPU device, tiny
    batch; the GPU run is the same code)."""
    import numpy as np

    from singa_amd import device

    bench = _bench()
    cpu = device.get_default_device()
    args = bench._parser().parse_args(["--model", "alexnet", "--batch", "2"])
    m, (x, y), o, info = bench._build(args, cpu, 0)
    assert x.shape == (2, 3, 224, 224) and info["unit"] == "images/s" and "AlexNet" in info["metric"]
    assert type(o).__name__ == "SGD" and o.weight_decay == 5e-4
    args = bench._parser().parse_args(["--model", "bert", "--batch", "2", "--seq", "16"])
    m, (ids, y), o, info = bench._build(args, cpu, 0)
    assert ids.shape == (2, 16) and info["unit"] == "sequences/s" and info["seq_len"] == 16
    assert type(o).__name__ == "Adam"
    args = bench._parser().parse_args(["--batch", "2", "--image", "32"])
    m, (x, y), o, info = bench._build(args, cpu, 0)
    assert info["metric"] == "images/sec (whole node) ResNet-50 bf16 training" and x.shape == (2, 3, 32, 32)
    assert bench._parser().parse_args([]).model == "resnet50"
    assert np.asarray(y.data).shape == (2,)


class _StubComm:
    """all_reduce(max/min) as if a peer held `peer` (a host numpy vector)."""

    def __init__(self, peer):
        self.peer = peer

    def all_reduce(self, t, op="sum"):
        import numpy as np
        v = t.numpy()
        v[:] = np.maximum(v, self.peer) if op == "max" else np.minimum(v, self.peer)


class _StubOpt:
    def __init__(self, w, buckets):
        import torch

        class S:
            pass
        self.store = S()
        self.store.w = torch.from_numpy(w)
        self.buckets = buckets


def test_replica_guard_detects_drift():
    """bench.py's cross-rank guard: identical replicas pass bit-exactly; one
    bucket of one rank off by a single lr*g-sized step fails it."""
    import numpy as np

    from singa_amd import device

    bench = _bench()
    cpu = device.get_default_device()
    rng = np.random.RandomState(0)
    w = (rng.randn(10000) * 0.05).astype(np.float32)
    opt_ = _StubOpt(w, [(0, 4000, []), (4000, 10000, [])])
    same = bench.replica_checksums(opt_)
    r = bench.replica_guard(_StubComm(same.copy()), opt_, cpu)
    assert r["ok"] and r["bitwise_equal"] and r["buckets"] == 2
    w2 = w.copy()
    w2[4000:4100] -= np.float32(1e-2) * rng.randn(100).astype(np.float32) * 0.05  # a lost bucket update
    other = bench.replica_checksums(_StubOpt(w2, opt_.buckets))
    r = bench.replica_guard(_StubComm(other), opt_, cpu)
    assert not r["ok"] and r["max_rel_spread"] > 1e-6
