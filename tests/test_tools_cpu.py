"""Loader tool (MNIST idx -> shard, Split/SplitN), the ``singa`` CLI, the
local launcher (incl. failure detection + checkpoint-based restart), and
Worker checkpoint/resume."""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_idx(tmp, n=50, h=6, w=6, seed=0):
    rng = np.random.RandomState(seed)
    imgs = rng.randint(0, 256, size=(n, h, w)).astype(np.uint8)
    labs = rng.randint(0, 10, size=n).astype(np.uint8)
    ip, lp = os.path.join(tmp, "img-idx3"), os.path.join(tmp, "lab-idx1")
    with open(ip, "wb") as f:
        f.write(struct.pack(">IIII", 2051, n, h, w) + imgs.tobytes())
    with open(lp, "wb") as f:
        f.write(struct.pack(">II", 2049, n) + labs.tobytes())
    return ip, lp, imgs, labs


def test_loader_mnist_roundtrip_and_split(tmp_path):
    from singa_amd import _core, loader
    from singa_amd.runtime.layers import DataSource

    ip, lp, imgs, labs = _write_idx(str(tmp_path))
    folder = str(tmp_path / "train")
    assert loader.main(["--datasource", "mnist", "--imagefile", ip, "--labelfile", lp,
                        "--shard_folder", folder]) == 0
    sh = _core.Shard(folder, _core.kRead)
    assert sh.count() == 50
    # re-running in append mode inserts nothing new (idempotent, crash-safe)
    assert loader.load_mnist(ip, lp, folder) in (0, 50)
    src = DataSource(folder, 10, prefetch=True)
    x, y = src.next()
    assert x.shape == (10, 6, 6)
    np.testing.assert_array_equal(x, imgs[:10].astype(np.float32))  # pixels decoded unsigned
    np.testing.assert_array_equal(y, labs[:10])
    counts = loader.split_n(3, folder, str(tmp_path / "part"))
    assert counts == [18, 16, 16]
    assert loader.split(20, folder, str(tmp_path / "tv")) == [20, 30]
    with pytest.raises(Exception):
        loader.split(60, folder, str(tmp_path / "bad"))


def test_loader_bad_magic(tmp_path):
    from singa_amd import loader

    ip, lp, _, _ = _write_idx(str(tmp_path))
    with pytest.raises(Exception):
        loader.load_mnist(lp, ip, str(tmp_path / "x"))


def test_imagenet_folder_loader(tmp_path):
    PIL = pytest.importorskip("PIL")
    from PIL import Image

    from singa_amd import _core, loader

    d = tmp_path / "in"
    (d / "img").mkdir(parents=True)
    rng = np.random.RandomState(1)
    with open(d / "rid.txt", "w") as f:
        for i in range(4):
            a = rng.randint(0, 256, size=(10, 12, 3)).astype(np.uint8)
            Image.fromarray(a).save(d / "img" / f"im{i}.png")
            f.write(f"im{i}.png {i}\n")
    mean = np.full((3, 8, 8), 10.0, np.float32)
    loader.write_mean(str(tmp_path / "mean.bin"), mean)
    np.testing.assert_allclose(loader.read_mean(str(tmp_path / "mean.bin")), mean)
    n = loader.load_imagenet(str(d), str(tmp_path / "mean.bin"), 8, 8)
    assert n == 4
    sh = _core.Shard(str(d), _core.kRead)
    k, v = sh.next()
    rec = _core.decode_record(v)
    assert list(rec["shape"]) == [3, 8, 8] and rec["label"] == 0


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.setdefault("OMP_NUM_THREADS", "1")
    if env:
        e.update(env)
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=timeout)


TINY = """
name: "tiny" train_steps: %d display_frequency: 1
updater { type: kSGD base_learning_rate: 0.05 momentum: 0.9 warmup_steps: 1 sync_frequency: 2 moving_rate: 0.5 }
neuralnet {
  layer { name: "data" type: "kShardData" data_param { path: "/nonexistent" batchsize: 8 } }
  layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
  layer { name: "label" type: "kLabel" srclayers: "data" }
  layer { name: "fc1" type: "kInnerProduct" srclayers: "mnist" inner_product_param { num_output: 16 }
          param { init_method: kUniform low: -0.1 high: 0.1 } param { init_method: kConstant value: 0 } }
  layer { name: "tanh1" type: "kTanh" srclayers: "fc1" }
  layer { name: "fc2" type: "kInnerProduct" srclayers: "tanh1" inner_product_param { num_output: 10 }
          param { init_method: kUniform low: -0.1 high: 0.1 } param { init_method: kConstant value: 0 } }
  layer { name: "loss" type: "kSoftmaxLoss" srclayers: "fc2" srclayers: "label" }
}
"""


def test_cli_single_process(tmp_path):
    conf = tmp_path / "m.conf"
    conf.write_text(TINY % 6)
    mj = tmp_path / "metrics.jsonl"
    r = _run(["-m", "singa_amd", "--model_conf", str(conf), "--device", "cpu", "--synthetic", "--data_shape",
              "6,6", "--metrics_json", str(mj), "--checkpoint", str(tmp_path / "ck.zip"),
              "--trace", str(tmp_path / "trace.json")])
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(l) for l in mj.read_text().splitlines()]
    assert len(rows) == 6 and all(np.isfinite(x["loss"]) for x in rows)
    assert os.path.exists(tmp_path / "ck.zip")
    tr = json.loads((tmp_path / "trace.json").read_text())
    assert any(e["name"] == "fc1" for e in tr["traceEvents"])


def test_worker_resume_reproduces(tmp_path):
    from singa_amd.config import schema
    from singa_amd.parallel import communicator
    from singa_amd.runtime import Worker
    from singa_amd.runtime.checkpoint import load_worker, save_worker

    communicator.reset()
    ov = {"*": {"shape": (6, 6), "nclass": 10, "seed": 2}}

    def make(n):
        return Worker(schema.parse_text("ModelProto", TINY % n), log=lambda s: None, seed=0, data_override=ov)

    full = make(8)
    full.run()
    ref = [float(h[2][0]) for h in full.history]
    a = make(4)
    a.run()
    save_worker(a, str(tmp_path / "c.zip"))
    b = make(8)
    load_worker(b, str(tmp_path / "c.zip"))
    b.run()
    got = [float(h[2][0]) for h in a.history] + [float(h[2][0]) for h in b.history]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.timeout(600)
def test_launcher_two_ranks_and_restart(tmp_path):
    """2 ranks (EASGD groups) through the launcher; rank 1 is killed at step 5
    by fault injection; the launcher tears the job down and restarts it from
    the periodic checkpoint."""
    conf = tmp_path / "m.conf"
    conf.write_text(TINY % 10)
    cl = tmp_path / "c.conf"
    cl.write_text(f'nworkers: 2\nworkspace: "{tmp_path}/ws"\n')
    ck = str(tmp_path / "ck-{rank}.zip")
    mj = tmp_path / "m.jsonl"
    r = _run(["-m", "singa_amd.launch", "--nproc", "2", "--max_restarts", "1", "--timeout", "240", "--",
              "--model_conf", str(conf), "--cluster_conf", str(cl), "--device", "cpu", "--synthetic",
              "--data_shape", "6,6", "--checkpoint", ck, "--checkpoint_frequency", "2", "--metrics_json", str(mj)],
             env={"SINGA_AMD_FAULT_STEP": "5", "SINGA_AMD_FAULT_RANK": "1"}, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "exited with 17" in r.stderr and "resuming from" in r.stderr
    assert os.path.exists(tmp_path / "ws" / "vis")
    steps = [json.loads(l)["step"] for l in mj.read_text().splitlines()]
    # the checkpoint taken after step 5 (the one the fault hits) resumes at step 6
    assert steps == [6, 7, 8, 9]


def test_draw_graph_dot_from_conf_and_json(tmp_path):
    """C31 visualisation: the partitioned LeNet conf rendered as Graphviz DOT
    (via the node-link JSON of NeuralNet.to_json), no networkx needed."""
    r = _run(["tools/draw_graph.py", "--model_conf", "examples/mnist/conv.conf", "--group_size", "2"], timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    dot = r.stdout
    assert dot.startswith("digraph") and '"conv1" -> "pool1"' in dot
    js = tmp_path / "g.json"
    js.write_text(json.dumps({"directed": 1, "nodes": [{"id": "a", "color": 0, "shape": "box"},
                                                       {"id": "b", "color": 1, "shape": "ellipse"}],
                              "links": [{"source": 0, "target": 1, "color": 1}]}))
    r = _run(["tools/draw_graph.py", "--json", str(js)], timeout=60)
    assert r.returncode == 0 and '"a" -> "b"' in r.stdout
