"""Runs the C++ mirror tests (tests/cpp/bloom_tests.cpp): the reference's bloom
tests restated against storage-engine_amd/cpp/lsm_bloom.hpp over the C ABI,
in a process that loads only the system ROCm runtime (no torch) — the way a
C/Rust caller links the library."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "storage-engine_amd", "build", "bloom_tests")


def _bin():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "storage-engine_amd"), "build/bloom_tests"], check=True)
    return BIN


def test_cpp_mirror_host():
    r = subprocess.run([_bin()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu():
    r = subprocess.run([_bin(), "--gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout
