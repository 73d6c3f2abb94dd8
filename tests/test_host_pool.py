"""The library's persistent host pool (verkle-kzg_amd/csrc/host/pool.hpp) used by the verkle
walks, the batched IPA rounds and the multiproof transcript records: coverage over ragged
ranges, nested loops, exception propagation, reuse (tests/cpp/pool_check.cpp)."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_pool(tmp_path):
    exe = tmp_path / "pool_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-pthread", os.path.join(HERE, "cpp", "pool_check.cpp"),
                           "-o", str(exe)])
    d = json.loads(subprocess.check_output([str(exe)], text=True, timeout=120))
    assert d["threads"] >= 1
    assert d["fails"] == 0, d
