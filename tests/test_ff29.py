"""Radix-2^29 Montgomery arithmetic of the accumulate / commit loops (csrc/ff29.hpp), checked on
the host against Python integers: congruences mod p, the output bounds the kernels' bound
analysis relies on (ec29.hpp header), limb normalisation, the packed form and the conversions
to and from the 32-bit-limb Montgomery form. Includes max-limb stress operands (column
accumulator overflow would show as a wrong residue)."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = {
    "bls12_381_fq": (0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab, 14, 12),
    "bn254_fq": (21888242871839275222246405745257275088696311157297823662689037894645226208583, 9, 8),
    "bls12_381_fr": (0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001, 9, 8),
}
M29 = (1 << 29) - 1


def val(limbs):
    return sum(v << (29 * j) for j, v in enumerate(limbs))


@pytest.fixture(scope="module")
def lines(tmp_path_factory):
    exe = tmp_path_factory.mktemp("ff29") / "ff29_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(HERE, "cpp", "ff29_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True)
    return [json.loads(ln) for ln in out.splitlines()]


def test_ff29_ops(lines):
    seen = set()
    for d in lines:
        p, L, N = FIELDS[d["f"]]
        Rp = 1 << (29 * L)
        R = 1 << (32 * N)
        r = val(d["r"])
        op = d["op"]
        seen.add((d["f"], op))
        if op == "mul":
            a, b = val(d["a"]), val(d["b"])
            assert (r * Rp - a * b) % p == 0
            assert r < a * b // Rp + p
            assert all(v <= M29 for v in d["r"][:-1])
        elif op == "mul2":
            s = val(d["a"]) * val(d["b"]) + val(d["c"]) * val(d["d"])
            assert (r * Rp - s) % p == 0
            assert r < s // Rp + p
            assert all(v <= M29 for v in d["r"][:-1])
        elif op == "add":
            assert r == val(d["a"]) + val(d["b"])
            assert all(v <= M29 + 7 for v in d["r"][:-1])
        elif op in ("sub4", "sub16"):
            k = int(op[3:])
            a, b = val(d["a"]), val(d["b"])
            assert r == a - b + k * p
            assert all(v <= M29 + 7 for v in d["r"][:-1])
        elif op == "canon":
            assert r < p and (r - val(d["a"])) % p == 0
        elif op == "unpack":
            assert r == val(d["a"])
        elif op == "mont":
            v = val(d["a"])
            assert (r - v * Rp * pow(R, -1, p)) % p == 0
            back = sum(w << (32 * k) for k, w in enumerate(d["back"]))
            assert back == v
    assert len(seen) == 3 * 8


def test_ff29_zero_test(lines):
    """is_zero_mo29 (product outputs below 2p) agrees with the residue"""
    for d in lines:
        if d["op"] == "mont":
            p = FIELDS[d["f"]][0]
            # "a" of a mont record is canon(r) of the same iteration's product
            assert d["zero_mo"] == (1 if val(d["a"]) % p == 0 else 0)


@pytest.mark.parametrize("lz,ch", [(3, 16), (4, 16), (4, 32), (6, 24)])
def test_mp_chunk_lazy_reduction_bn254_fr(lz, ch):
    """k_mp_chunk's arithmetic (csrc/scheme.hip, shapes LZ x CH of VKZG_MP_SHAPE) restated with
    Python integers: evaluations f (canonical) times r^i R' (radix-2^29 Montgomery, R' = 2^261)
    added into 17 64-bit columns for up to LZ queries, one Montgomery reduction per LZ, the block
    results added with one conditional subtraction each -- == sum f_i r^i mod r for chunks of
    1..CH queries, near-r inputs and all-max-limb canonical inputs included; every column stays
    below 2^64 at every step."""
    import random
    p = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    L, M = 9, (1 << 29) - 1
    Rp = 1 << (29 * L)
    inv = (-pow(p, -1, 1 << 29)) % (1 << 29)
    limbs = lambda x: [(x >> (29 * j)) & M for j in range(L - 1)] + [x >> (29 * (L - 1))]  # noqa: E731
    val = lambda v: sum(a << (29 * j) for j, a in enumerate(v))  # noqa: E731
    pl = limbs(p)
    # the largest limbs a canonical value can have: 8 limbs of 2^29 - 1 under p's top limb - 1
    vmax = val([M] * (L - 1) + [pl[-1] - 1])
    assert vmax < p

    def carry_csub(x):
        v = val(x)
        assert v < 2 * p
        return limbs(v - p if v >= p else v)

    rng = random.Random(3 + lz)
    for trial in range(300):
        cnt = rng.randint(1, ch)
        stress = trial % 4 == 0
        fs = [vmax if stress else rng.randrange(p) if trial % 3 else p - 1 - rng.randrange(5) for _ in range(cnt)]
        rs = [rng.randrange(p) for _ in range(cnt)]
        rm = [vmax if stress else r * Rp % p for r in rs]  # the radix-29 words the kernel reads
        total = [0] * L
        for h in range(0, cnt, lz):
            t = [0] * (2 * L)
            for j in range(h, min(h + lz, cnt)):
                a, b = limbs(fs[j]), limbs(rm[j])
                for y in range(L):
                    for x in range(L):
                        t[x + y] += a[x] * b[y]
            assert max(t) < 1 << 64
            for i in range(L):
                m = ((t[i] & 0xFFFFFFFF) * inv) & M
                for j in range(L):
                    t[i + j] += m * pl[j]
                assert max(t) < 1 << 64
                t[i + 1] += t[i] >> 29
            r = [0] * L
            for j in range(L, 2 * L - 1):
                t[j + 1] += t[j] >> 29
                r[j - L] = t[j] & M
            r[L - 1] = t[2 * L - 1]
            total = carry_csub([u + w for u, w in zip(total, r)])
        total = carry_csub(total)
        want = sum(f * (r if not stress else vmax * pow(Rp, -1, p)) for f, r in zip(fs, rs)) % p
        assert val(total) == want
