"""Radix-2^29 point arithmetic of the accumulate / commit / reduction kernels (csrc/ec29.hpp)
against the 32-bit-limb formulas of csrc/ec.hpp, on the host: mixed-add chains with random
signs, full adds, doublings and the exceptional cases (q = acc, q = -acc, zero operands) for
BLS12-381 G1, BN254 G1 and Bandersnatch, compared as affine points (tests/cpp/ec29_check.cpp)."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_ec29_matches_ec(tmp_path):
    exe = tmp_path / "ec29_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(HERE, "cpp", "ec29_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True, timeout=120)
    res = {d["curve"]: d for d in map(json.loads, out.splitlines())}
    assert set(res) == {"bls12_381", "bn254", "bandersnatch"}
    for curve, d in res.items():
        assert d["checks"] > 200, curve
        assert d["mismatches"] == 0, d

