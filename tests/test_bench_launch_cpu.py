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
