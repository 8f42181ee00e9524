"""§5.2 race detection / sanitizers: the host C++ runtime (csrc/host/runtime_core.h)
under AddressSanitizer + UndefinedBehaviorSanitizer (round trips and mutation
fuzzing of the TFRecord / tf.Example / SSTable parsers) and ThreadSanitizer (the
multi-threaded TFRecord decoder).  GPU sanitizers are not available on the
MI355X pool, so device code is covered by the numerics tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "runtime_selftest.cpp")
INC = os.path.join(ROOT, "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_runtime_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-msse4.2", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", f"-I{INC}", SRC, "-o", exe, "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "cannot find" in b.stderr and "tsan" in b.stderr:
        pytest.skip("ThreadSanitizer runtime not installed")
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, SELFTEST_TMP=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "ALL OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
