"""Sanitizer builds of the native host runtime: the _core C++
sources plus tests/native/runtime_selftest.cc are compiled with
ThreadSanitizer and with AddressSanitizer+UBSan and run; any sanitizer
report fails the test.  (GPU-side ASan needs xnack+, which the MI355X pool
does not offer, so sanitizers cover host code only.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "singa_amd", "csrc", "runtime")
SRCS = [os.path.join(RT, f) for f in ("shard.cc", "graph.cc", "loader.cc")] + [
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
    r = subprocess.run([str(exe), str(tmp_path / "data")], capture_output=True, text=True, env=env, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "runtime selftest ok" in out, out[-4000:]
    assert marker not in out and "runtime error" not in out, out[-4000:]
