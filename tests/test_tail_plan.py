"""The bit-stage geometry msm_tail_plan picks for each MSM path's tail (csrc/msm_tail.hpp, on the
host; tests/cpp/tail_plan_check.cpp): the row-derived total (urow) only where the U items are the
segment sums themselves (Lseg = 1), the marginal form only within one round of waves, and the
wave count per set (per_w) covering exactly what k_msm_bitsum / PartLoc index."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_tail_plan_geometries(tmp_path):
    exe = tmp_path / "tail_plan_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                           os.path.join(HERE, "cpp", "tail_plan_check.cpp"), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True, timeout=60)
    p = {d["name"]: d for d in map(json.loads, out.splitlines())}
    # 8-way slice: U from the rows, two waves per column sum, 2 items per lane
    s = p["slice8"]
    assert (s["urow"], s["h"], s["pL"], s["K"], s["nb2"]) == (1, 7, 2, 2, 0)
    assert s["per_w"] == 128 * 2 + 256
    # one-GPU radix MSM: marginal form with its five U sums (never urow: U_r are bucket columns)
    r = p["radix1"]
    assert (r["urow"], r["h"], r["K"]) == (0, 7, 4)
    assert r["per_w"] == 128 + 256 + 5 * r["nb2"] and r["nb2"] == (1 << 15) // (64 * 4)
    # a 2^12-bucket shared set: urow on the tie (no U waves), one wave per column
    t = p["shared12"]
    assert (t["urow"], t["h"], t["pL"], t["nb2"]) == (1, 6, 1, 0) and t["per_w"] == 64 + 64
    # two radix sets (the one-call KZG): packed marginal waves, 2 column / 4 row sums per wave, 8 items
    # per lane everywhere, one round; one partial slot per sum
    k = p["kzg2"]
    assert (k["urow"], k["h"], k["K"], k["gL"], k["gH"]) == (0, 7, 8, 2, 4)
    assert k["per_w"] == 128 // 2 + 256 // 4 + 5 * k["nb2"] and 2 * k["per_w"] <= 1024
    assert k["slots"] == 128 + 256 + 5 * k["nb2"]
    # eight per-window sets (GLV variable base): packed marginal waves within one round
    v = p["perwin8"]
    assert v["h"] == 6 and v["urow"] == 0 and v["gL"] * v["gH"] > 1 and 8 * v["per_w"] <= 1024
    assert v["slots"] == 64 + 128 + 4 * v["nb2"]
    # sixteen sets (BN254 2^20): packed too (4 column / 8 row sums per wave), still one round
    b = p["perwin16"]
    assert b["h"] == 6 and (b["gL"], b["gH"]) == (4, 8) and 16 * b["per_w"] <= 1024
    assert b["slots"] == 64 + 128 + b["nb2"]
    for d in p.values():
        assert d["pL"] >= 1 and d["K"] >= 1
        if d["gL"] == 1 and d["gH"] == 1:
            assert d["slots"] == d["per_w"]
