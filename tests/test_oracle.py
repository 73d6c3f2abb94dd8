"""CPU tests of the oracle (test infrastructure): curve KATs, C restatement vs Python restatement,
the committed golden fixtures, and the reference's own round-trip / tamper tests restated
(ipa/mod.rs:382-421, kzg/mod.rs:278-297, multiproof.rs:261-357)."""
import json
import os
import random

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def P(h):
    return None if h is None else (int(h[0], 16), int(h[1], 16))


def test_curve_kats():
    from pyoracle.curves import CURVES
    for C in CURVES.values():
        assert C.is_on_curve(C.g)
        assert C.mul(C.g, C.r - 1) == C.neg(C.g)      # r*G = O
        assert C.add(C.g, C.neg(C.g)) == C.identity()
    # BN254 generator is (1, 2) (ark-bn254 G1)
    assert CURVES["bn254"].g == (1, 2)


def test_domain_generator():
    """omega_n = 5^((r-1)/n) has exact order n (precompute.rs:26)."""
    from pyoracle.protocol import group_gen
    from pyoracle.curves import BN254
    w = group_gen(256)
    assert pow(w, 256, BN254.r) == 1 and pow(w, 128, BN254.r) != 1


def test_golden_msm_python_and_c(oracle_c):
    from pyoracle.curves import CURVES
    for case in load("msm.json")["cases"]:
        C = CURVES[case["curve"]]
        pts = [P(b) for b in case["bases"]]
        if C.kind == "te":
            pts = [(0, 1) if p is None else p for p in pts]
        sc = [int(s, 16) for s in case["scalars"]]
        want = P(case["expected"])
        if case["n"] <= 7:
            assert C.msm(pts, sc) == want
        got = oracle_c.msm(C.name, pts, sc)
        if C.kind == "te" and got == (0, 1) and want is None:
            got = None
        assert got == want, (case["curve"], case["n"])


def test_c_oracle_threads_match(oracle_c):
    from pyoracle.curves import BLS12_381, random_points
    rng = random.Random(5)
    pts = random_points(BLS12_381, 33, rng)
    sc = [rng.randrange(BLS12_381.r) for _ in pts]
    assert oracle_c.msm("bls12_381", pts, sc, 1) == oracle_c.msm("bls12_381", pts, sc, 5)


def test_golden_transcript():
    from pyoracle import arkser
    from pyoracle.curves import BN254
    g = load("transcript.json")
    for h in g["hash_to_field"]:
        assert hex(arkser.hash_to_field(bytes.fromhex(h["msg"]), h["dst"].encode(), BN254.r)) == h["out"]
    for c in g["compressed"]:
        p = P(c["point"])
        assert arkser.ser_point_compressed(p).hex() == c["bytes"]
        assert hex(arkser.to_data_item(p)) == c["to_data_item"]
    # compressed flag semantics: bit7 set iff y is the larger root
    g1 = BN254.g
    assert arkser.ser_point_compressed(g1)[31] & 0x80 == 0
    assert arkser.ser_point_compressed(BN254.neg(g1))[31] & 0x80 == 0x80


def test_ipa_crs_prefix():
    from pyoracle import protocol
    from pyoracle.curves import BN254
    g = load("ipa_crs_bn254.json")
    pts = protocol.ipa_gen_points(8, max_=512)
    assert [P(h) for h in g["points"][:8]] == pts
    assert all(BN254.is_on_curve(p) for p in pts)
    with pytest.raises(ValueError):       # Appendix B.1: default max 256 < N+1 = 257
        protocol.ipa_gen_points(257)


def test_reference_ipa_tests_restated():
    """ipa/mod.rs:382-421 at N = 32: commit proof round trip + tamper; eval proofs in/out of domain."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    crs = [P(h) for h in load("ipa_crs_bn254.json")["points"][:33]]
    ipa = protocol.IPA(32, points=crs)
    data = protocol.LagrangeBasis.from_vec(list(range(32)))
    com = ipa.commit(data)
    cp = ipa.prove_commitment(com, data)
    assert ipa.verify_commitment_proof(com, cp)
    assert not ipa.verify_commitment_proof(BN254.add(com, BN254.g), cp)
    idx = 13
    pr = ipa.prove(com, idx, data)
    assert ipa.verify(com, idx, pr)
    out = ipa.prove(com, 64, data)
    assert ipa.verify(com, 64, out)
    assert not ipa.verify(com, idx, out)


def test_reference_kzg_test_restated():
    """kzg/mod.rs:278-297: CRS 16, data 8: every index verifies, 8..16 give y = 0, index 17 verifies."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    rng = random.Random(9)
    kz = protocol.KZG(16)
    d = protocol.LagrangeBasis([rng.randrange(BN254.r) for _ in range(8)], 16)
    c = kz.commit(d)
    for i in range(16):
        pr = kz.prove(c, i, d)
        assert kz.verify(c, i, pr)
        if i >= 8:
            assert pr["y"] == 0
    assert kz.verify(c, 17, kz.prove(c, 17, d))


def test_golden_ipa_256_proof_verifies():
    from pyoracle import protocol
    crs = [P(h) for h in load("ipa_crs_bn254.json")["points"]]
    g = load("ipa_256.json")
    ipa = protocol.IPA(256, points=crs)
    com = P(g["commitment"])
    for key in ("proof_in_domain", "proof_out_domain"):
        pr = g[key]
        proof = {"l": [P(x) for x in pr["l"]], "r": [P(x) for x in pr["r"]], "tip": int(pr["tip"], 16),
                 "y": int(pr["y"], 16)}
        assert ipa.verify(com, pr["point"], proof)
    cp = g["commitment_proof"]
    proof = {"l": [P(x) for x in cp["l"]], "r": [P(x) for x in cp["r"]], "tip": int(cp["tip"], 16)}
    assert ipa.verify_commitment_proof(com, proof)          # ipa/mod.rs:237-265


def test_golden_multiproof_verifies_and_tamper():
    from pyoracle import protocol
    from pyoracle.curves import BN254
    crs = [P(h) for h in load("ipa_crs_bn254.json")["points"][:33]]
    g = load("multiproof_32.json")
    for name, vc in (("ipa", protocol.IPA(32, points=crs)), ("kzg", protocol.KZG(32))):
        ent = g[name]
        vq = [(P(q["commit"]), q["z"], int(q["y"], 16)) for q in ent["queries"]]
        if name == "ipa":
            pr = ent["proof"]
            proof = {"l": [P(x) for x in pr["l"]], "r": [P(x) for x in pr["r"]], "tip": int(pr["tip"], 16),
                     "y": int(pr["y"], 16)}
        else:
            proof = {"proof": P(ent["proof"]["proof"]), "y": int(ent["proof"]["y"], 16)}
        mp = {"proof": proof, "d": P(ent["d"])}
        assert protocol.verify_multiproof(vc, vq, mp)
        bad = dict(mp, d=BN254.add(mp["d"], BN254.g))
        assert not protocol.verify_multiproof(vc, vq, bad)
        vq2 = list(vq)
        vq2[0] = (vq[0][0], vq[0][1], (vq[0][2] + 1) % BN254.r)
        assert not protocol.verify_multiproof(vc, vq2, mp)


def _mp_golden_arrays(oracle_c, ent, queries_data, N):
    import numpy as np
    coms = [P(c) for c in ent]
    cxy, cinf = oracle_c.points_to_array("bn254", coms)
    data = oracle_c.ints_to_limbs([v for d in queries_data for v in d], 4)
    return data, cxy, cinf


@pytest.mark.parametrize("name", ["ipa", "kzg"])
def test_mpcheck_matches_python_multiproof_goldens(oracle_c, name):
    """oracle/pyoracle/mpcheck.py (the N = 256 / Q = 2^16 checker of the GPU multiproof: field
    phases and commits in C, transcript and inner proof in Python) == the pure-Python
    protocol.prove_multiproof fixtures: multiproof_32.json (N = 32) and multiproof_256.json (the
    reference's width, 20 queries on one z) -- D, the inner proof, and y of every query."""
    import numpy as np
    from pyoracle import mpcheck, protocol
    from pyoracle.curves import BN254
    crs = [P(h) for h in load("ipa_crs_bn254.json")["points"]]
    g32 = load("multiproof_32.json")[name]
    g256 = load("multiproof_256.json")
    cases = [(32, [[int(x, 16) for x in q["data"]] for q in g32["queries"]], [q["commit"] for q in g32["queries"]],
              [q["z"] for q in g32["queries"]], g32),
             (256, [[(int(r0, 16) + i) % BN254.r for i in range(256)] for r0 in g256["r0"]], g256[name]["commits"],
              g256["z"], g256[name])]
    for N, datas, commits, z, ent in cases:
        vc = protocol.IPA(N, points=crs[:N + 1]) if name == "ipa" else protocol.KZG(N)
        data, cxy, cinf = _mp_golden_arrays(oracle_c, commits, datas, N)
        got = mpcheck.multiproof(vc, N, data, cxy, cinf, np.array(z, dtype=np.uint64), nthreads=2)
        assert got["d"] == P(ent["d"])
        if name == "ipa":
            pr = got["proof"]
            assert pr["l"] == [P(x) for x in ent["proof"]["l"]] and pr["r"] == [P(x) for x in ent["proof"]["r"]]
            assert pr["tip"] == int(ent["proof"]["tip"], 16) and pr["y"] == int(ent["proof"]["y"], 16)
        else:
            assert got["proof"]["proof"] == P(ent["proof"]["proof"]) and got["proof"]["y"] == int(ent["proof"]["y"], 16)


def test_multiproof_256_golden_verifies():
    """multiproof_256.json verifies through the oracle verifier (multiproof.rs:178-215) and a
    tampered y is rejected; its z rows hold 20 queries on z = 5 and on z = 200."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    crs = [P(h) for h in load("ipa_crs_bn254.json")["points"]]
    g = load("multiproof_256.json")
    assert g["z"].count(5) >= 20 and g["z"].count(200) >= 20
    ys = [(int(r0, 16) + z) % BN254.r for r0, z in zip(g["r0"], g["z"])]
    ent = g["ipa"]
    vq = [(P(c), z, y) for c, z, y in zip(ent["commits"], g["z"], ys)]
    pr = ent["proof"]
    proof = {"l": [P(x) for x in pr["l"]], "r": [P(x) for x in pr["r"]], "tip": int(pr["tip"], 16),
             "y": int(pr["y"], 16)}
    vc = protocol.IPA(256, points=crs)
    mp = {"proof": proof, "d": P(ent["d"])}
    assert protocol.verify_multiproof(vc, vq, mp)
    vq[7] = (vq[7][0], vq[7][1], (vq[7][2] + 1) % BN254.r)
    assert not protocol.verify_multiproof(vc, vq, mp)


@pytest.mark.parametrize("curve", ["bn254", "bls12_381", "bandersnatch"])
def test_pippenger_baseline_matches_naive(oracle_c, curve):
    """the all-core CPU Pippenger baseline (bench cpu_baseline leg) == the naive restatement of
    utils.rs:16-19 on golden cases (identities, zero / r-1 scalars) and random sizes."""
    import numpy as np
    from pyoracle.curves import CURVES, random_points
    C = CURVES[curve]
    cases = [c for c in load("msm.json")["cases"] if c["curve"] == curve]
    rng = random.Random(9)
    for n in (64, 200, 1500):
        pts = random_points(C, n, rng)
        sc = [rng.randrange(C.r) for _ in pts]
        sc[0], sc[1], sc[2] = 0, C.r - 1, 1
        cases.append({"bases": pts, "scalars": sc})
    for case in cases:
        pts = [P(b) if isinstance(b, list) or b is None else b for b in case["bases"]]
        if C.kind == "te":
            pts = [(0, 1) if p is None else p for p in pts]
        sc = [int(s, 16) if isinstance(s, str) else s for s in case["scalars"]]
        arr, inf = oracle_c.points_to_array(curve, pts)
        lim = oracle_c.ints_to_limbs(sc, 4)
        want = oracle_c.msm_arrays(curve, arr, inf, lim, 2)
        for T in (1, 3):
            got = oracle_c.pip_msm_arrays(curve, arr, inf, lim, T)
            assert got[1] == want[1] and np.array_equal(got[0], want[0]), (curve, len(pts), T)


def test_pippenger_batch_baseline(oracle_c):
    import numpy as np
    from pyoracle.curves import BANDERSNATCH, random_points
    rng = random.Random(4)
    pts = random_points(BANDERSNATCH, 256, rng)
    arr, inf = oracle_c.points_to_array("bandersnatch", pts)
    sc = oracle_c.ints_to_limbs([rng.randrange(BANDERSNATCH.r) for _ in range(256 * 5)], 4)
    xy, oinf = oracle_c.pip_msm_batch_arrays("bandersnatch", arr, inf, sc, 256, 3)
    for j in range(5):
        w = oracle_c.msm_arrays("bandersnatch", arr, inf, sc[j * 256:(j + 1) * 256], 2)
        assert np.array_equal(xy[j], w[0]) and oinf[j] == w[1]


def test_multiproof_field_phases_c_vs_python(oracle_c):
    """the C restatement of prove_multiproof's field phases (CPU baseline of configs[4]) == the
    Python restatement's g and h (multiproof.rs:117-165) for arbitrary challenges r, t."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    r_mod = BN254.r
    rng = random.Random(12)
    N, Q = 32, 23
    pre = protocol.PrecomputedLagrange(N)
    datas = [[rng.randrange(r_mod) for _ in range(N)] for _ in range(Q)]
    z = [rng.randrange(N) for _ in range(Q)]
    z[3] = z[7] = z[11]                                     # repeated points are grouped
    rr, t = rng.randrange(r_mod), rng.randrange(N, r_mod)
    rp = protocol.powers_of(rr, Q, r_mod)
    groups = {}
    for i in range(Q):
        groups.setdefault(z[i], []).append([v * rp[i] % r_mod for v in datas[i]])
    g, h = [0] * N, [0] * N
    invs = protocol.invert_domain_at(t, N, r_mod)
    for zz, lst in groups.items():
        total = [sum(col) % r_mod for col in zip(*lst)]
        q = protocol.LagrangeBasis(total, N).divide_by_vanishing(pre, zz)
        g = [(a + b) % r_mod for a, b in zip(g, q)]
        for ev in lst:
            h = [(a + b * invs[zz]) % r_mod for a, b in zip(h, ev)]
    data = oracle_c.ints_to_limbs([v for d in datas for v in d], 4)
    import numpy as np
    for T in (1, 4):
        cg, ch = oracle_c.mp_field_phases(N, data, np.array(z, dtype=np.uint64), rr, t, pre.omega, T)
        assert [oracle_c.limbs_to_int(x) for x in cg] == g
        assert [oracle_c.limbs_to_int(x) for x in ch] == h


def _pt_fft(C, pts, n, omega, inverse=False):
    """ark-poly fft over points, O(n^2), straight from the definition (no scalar shortcut)"""
    r = C.r
    a = (list(pts) + [None] * n)[:n]
    w = pow(omega, -1, r) if inverse else omega
    out = []
    for i in range(n):
        acc = None
        for j in range(n):
            acc = C.add(acc, C.mul(a[j], pow(w, i * j, r))) if a[j] is not None else acc
        out.append(C.mul(acc, pow(n, -1, r)) if (inverse and acc is not None) else acc)
    return out


def test_prove_all_points_oracle_scalar_shortcut():
    """the oracle's kzg_prove_all_points works on the SRS scalars (L_j = c_j G); recompute one small
    case from the points themselves (G1 FFTs by definition) and compare (kzg/mod.rs:200-235)."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    C, r = BN254, BN254.r
    kz = protocol.KZG(8)
    m = 4
    w4 = protocol.group_gen(4)
    coeffs = [5, 7]                                    # degree 1 -> domain D::new(2) = 2
    evals = [sum(c * pow(w4, i * k, r) for k, c in enumerate(coeffs)) % r for i in range(m)]
    data = protocol.LagrangeBasis(evals, 4)
    got = protocol.kzg_prove_all_points(kz, data)
    assert len(got) == 2
    g1 = _pt_fft(C, kz.lagrange, 8, kz.pre.omega, inverse=True)
    d, D = 1, 2
    chat = [coeffs[d]] + [0] * (d + 1) + coeffs[:d]
    shat = list(reversed(g1[:d])) + [None] * (D - d)
    y = protocol.ark_fft(chat, D, r, protocol.group_gen(D))
    v = _pt_fft(C, shat, D, protocol.group_gen(D))
    u = [C.mul(p, k) if p is not None else None for p, k in zip(v, y)]
    h = _pt_fft(C, u, D, protocol.group_gen(D), inverse=True)
    assert [p for p, _ in got] == h
    assert [yv for _, yv in got] == evals[:2]
    with pytest.raises(protocol.ReferencePanic):
        protocol.kzg_prove_all_points(kz, protocol.LagrangeBasis([0, 0, 0, 0], 4))
