"""Host sanitizers on the native text core and the kernel-launch validation layer.

GPU AddressSanitizer / xnack+ runs are not available on the MI355X pool, so
the sanitizers run on the host C++: csrc/text/text_selftest.cpp is compiled
with ASan+UBSan (out-of-bounds, use-after-free, undefined casts/overflow) and,
separately, with TSan (data races in the thread-parallel batch encode and
featuriser), then executed.  Sanitizer options are compiled into the binary
(__*_default_options), so the child runs in the unchanged environment.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "csrc", "text", "text_selftest.cpp")


def _build_and_run(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags, SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in (r.stderr or ""):
        pytest.skip(f"sanitizer runtime not installed: {r.stderr.strip()[:200]}")
    assert r.returncode == 0, r.stderr
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, f"{name} failed:\n{p.stdout}\n{p.stderr[-4000:]}"
    assert "text core self-test: ok" in p.stdout
    assert "runtime error" not in p.stderr and "WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-4000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_text_core_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], "selftest_asan")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_text_core_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "selftest_tsan")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_binding_validation_layer_asan_ubsan(tmp_path):
    """csrc/binding.cpp's launch-validation layer, built host-only (FD_HOST_VALIDATION) with
    ASan + UBSan against CPU ATen: every launcher is a stub that checks the extents the real
    kernel would touch against the registered buffers; valid calls must pass with no
    violation, invalid ones must be rejected BEFORE any launch (csrc/host_check/)."""
    import torch
    tdir = os.path.dirname(torch.__file__)
    exe = str(tmp_path / "binding_host_check")
    src = os.path.join(REPO, "csrc", "host_check", "binding_host_check.cpp")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-I" + os.path.join(tdir, "include"), "-I" + os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           src, "-L" + os.path.join(tdir, "lib"), "-ltorch_cpu", "-lc10", "-Wl,-rpath," + os.path.join(tdir, "lib"),
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "cannot find" in (r.stderr or ""):
        pytest.skip(f"sanitizer runtime not installed: {r.stderr.strip()[:200]}")
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, f"{p.stdout[-4000:]}\n{p.stderr[-4000:]}"
    assert "binding host check: ok" in p.stdout
    assert "runtime error" not in p.stderr, p.stderr[-4000:]
