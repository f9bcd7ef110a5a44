"""Sanitizer builds of the native host runtime: EVERY _core C++
source (shard, graph, loader, the threaded parameter server, the updaters,
the mmap LMDB reader -- all of csrc/runtime/*.cc but the pybind11 glue) plus
tests/native/runtime_selftest.cc are compiled with ThreadSanitizer and with
AddressSanitizer+UBSan and run; the self-test stresses the PS with several
client threads on shared keys.  Any sanitizer report fails the test.
(GPU-side ASan needs xnack+, which the MI355X pool does not offer, so
sanitizers cover host code only.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "singa_amd", "csrc", "runtime")
SRCS = sorted(os.path.join(RT, f) for f in os.listdir(RT) if f.endswith(".cc") and f != "core_bindings.cc") + [
    os.path.join(ROOT, "tests", "native", "runtime_selftest.cc")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.mark.parametrize("flags,marker", [
    (["-fsanitize=thread"], "ThreadSanitizer"),
    (["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
     "AddressSanitizer"),
])
def test_runtime_under_sanitizer(tmp_path, flags, marker):
    exe = tmp_path / "selftest"
    cmd = ["g++", "-std=c++17", "-g", "-O1", *flags, *SRCS, "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import numpy as np
    from lmdb_writer import datum, write_lmdb
    rng = np.random.RandomState(0)
    items = [(b"%06d" % i, datum(3, 6, 6, rng.randint(0, 256, 108).astype(np.uint8).tobytes(), i % 5))
             for i in range(120)]
    items.append((b"zz", datum(3, 40, 40, rng.randint(0, 256, 4800).astype(np.uint8).tobytes(), 1)))  # overflow page
    write_lmdb(str(tmp_path / "lmdb"), items, leaf_limit=8)
    r = subprocess.run([str(exe), str(tmp_path / "data"), str(tmp_path / "lmdb")], capture_output=True, text=True,
                       env=env, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "runtime selftest ok" in out, out[-4000:]
    assert marker not in out and "runtime error" not in out, out[-4000:]
