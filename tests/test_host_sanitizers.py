"""Host runtime under sanitizers (SURVEY §5 "Race detection / sanitizers").

tools/host_selftest.cpp drives the multi-threaded synthetic generator, the
multi-threaded wire packer + unpacker, special-row pre-lowering and the CPU
featurizer.  It is compiled twice with g++ -- AddressSanitizer + UBSan
(memory errors, undefined behaviour) and ThreadSanitizer (data races in the
threaded generator / packer / featurizer) -- and must run clean.  Device
code is never sanitizer-built on this pool (no GPU ASan / XNACK).
"""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build(tmp_path, name, flags):
    srcs = [s for s in sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
            if not s.endswith("bindings_host.cpp")]
    exe = str(tmp_path / name)
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", *flags, f"-I{CSRC}",
           os.path.join(ROOT, "tools", "host_selftest.cpp"), *srcs, "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _run(exe, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, "12000", "4"], capture_output=True, text=True, timeout=240, env=env)
    return r


def test_host_runtime_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "selftest_asan", ["-fsanitize=address,undefined",
                                             "-fno-sanitize-recover=undefined",
                                             "-static-libasan"])
    r = _run(exe, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                   "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
    assert "host selftest ok" in r.stdout


def test_host_runtime_tsan(tmp_path):
    exe = _build(tmp_path, "selftest_tsan", ["-fsanitize=thread", "-static-libtsan"])
    r = _run(exe, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        pytest.skip("ThreadSanitizer cannot map its shadow memory on this kernel")
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
    assert "host selftest ok" in r.stdout
