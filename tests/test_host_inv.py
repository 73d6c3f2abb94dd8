"""Host field inversion (csrc/ff.hpp fe_inv_host: Bernstein-Yang divsteps on signed 62-bit
limbs, the last serial step of every MSM call and of each IPA round's normalisation) against
Fermat's a^(p-2) on BN254 Fq / Fr, BLS12-381 Fq / Fr and Bandersnatch Fr: random values, the
edges 1, 2, 3, p - 1, p - 2, single bits and runs of ones (tests/cpp/inv_check.cpp)."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_divstep_inverse_matches_fermat(tmp_path):
    exe = tmp_path / "inv_check"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(HERE, "cpp", "inv_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True, timeout=120)
    res = {d["field"]: d for d in map(json.loads, out.splitlines())}
    assert set(res) == {"bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr", "bandersnatch_fr"}
    for name, d in res.items():
        assert d["checks"] > 2000, name
        assert d["mismatches"] == 0, d
