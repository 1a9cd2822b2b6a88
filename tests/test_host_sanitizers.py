"""Host sanitizers on the native text core (race detection / sanitizers).

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
