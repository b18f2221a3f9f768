"""The workspace growth policy (storage-engine_amd/csrc/growbuf.hpp, behind
DevBuf::ensure) under memory pressure, with a budgeted mock allocator: a growth
whose old and new buffers do not fit together must free the retired buffers,
then the live one, and succeed.  Host-only, g++."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_growbuf_policy(tmp_path):
    exe = str(tmp_path / "growbuf_test")
    src = os.path.join(ROOT, "tests", "cpp", "growbuf_test.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-fsanitize=address,undefined", "-o", exe, src],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all passed" in r.stdout
