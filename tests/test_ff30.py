"""Signed radix-2^30 Montgomery arithmetic (csrc/ff30.hpp, the 13-limb BLS12-381 Fq prototype)
checked on the host against Python integers: congruences mod p, the magnitude bounds the header
states, the limb states (exact / near), canonicalisation and the 32-bit Montgomery round trip
including max-limb stress operands (a column overflow shows as a wrong residue); and its mixed
add (ec30.hpp) word for word against the radix-2^29 one (ec29.hpp) on chains of random inputs."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
L = 13
RP = 1 << (30 * L)
R32 = 1 << 384
H = 1 << 29


def val(limbs):
    return sum(v << (30 * j) for j, v in enumerate(limbs))


@pytest.fixture(scope="module")
def lines(tmp_path_factory):
    exe = tmp_path_factory.mktemp("ff30") / "ff30_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(HERE, "cpp", "ff30_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True)
    return [json.loads(ln) for ln in out.splitlines()]


def exact(limbs):
    return all(-H <= v < H for v in limbs[:-1])


def near(limbs):
    return all(-H - 2 <= v < H + 2 for v in limbs[:-1])


def test_ff30_field_ops(lines):
    seen = set()
    for d in lines:
        op = d["op"]
        seen.add(op)
        if op == "mul":
            a, b, r = val(d["a"]), val(d["b"]), val(d["r"])
            assert (r * RP - a * b) % P == 0
            assert abs(r) < abs(a * b) // RP + P // 2 + (P >> 29)
            assert exact(d["r"])
        elif op == "mul2":
            s = val(d["a"]) * val(d["b"]) + val(d["c"]) * val(d["d"])
            r = val(d["r"])
            assert (r * RP - s) % P == 0
            assert abs(r) < abs(s) // RP + P // 2 + (P >> 29)
            assert exact(d["r"])
        elif op == "add" and "r" in d:
            assert val(d["r"]) == val(d["a"]) + val(d["b"]) and near(d["r"])
        elif op == "sub":
            assert val(d["r"]) == val(d["a"]) - val(d["b"]) and near(d["r"])
        elif op == "canon":
            r = sum(v << (30 * j) for j, v in enumerate(d["r"]))
            assert 0 <= r < P and (r - val(d["a"])) % P == 0
        elif op == "mont":
            a = sum(w << (32 * k) for k, w in enumerate(d["a"]))
            back = sum(w << (32 * k) for k, w in enumerate(d["back"]))
            assert back == a
            assert (val(d["r"]) - a * RP * pow(R32, -1, P)) % P == 0
    assert {"mul", "mul2", "add", "sub", "canon", "mont"} <= seen


def test_ff30_madd_matches_radix29(lines):
    res = [d for d in lines if d["op"] == "madd"][0]
    assert res["checked"] == 2560 and res["bad"] == 0
    chains = [d for d in lines if d["op"] == "madd_chain"]
    assert [c["inf"] for c in chains[38:]] == [1, 1]


def test_ff30_add_dbl_and_tables_match_radix29(lines):
    """general adds (with equal / opposite operands), doublings, and pack_aff -> load -> store"""
    res = [d for d in lines if d["op"] == "add" and "checked" in d][0]
    assert res["checked"] == 24 * 36 and res["bad"] == 0 and res["table_bad"] == 0
