"""GPU parity of the protocol layer (include/vc_scheme.h) against the oracle's golden fixtures:
IPA (ipa/mod.rs), KZG (kzg/mod.rs), multiproof (multiproof.rs), to_data_item (lib.rs:56-67).
Proof bytes are compared exactly; verification results are compared with the reference's own
round-trip / tamper tests (ipa/mod.rs:404-421, kzg/mod.rs:278-297, multiproof.rs:261-357)."""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def P(h):
    return None if h is None else (int(h[0], 16), int(h[1], 16))


def H(x):
    return int(x, 16)


@pytest.fixture(scope="module")
def eng():
    import vkzg
    e = vkzg.Engine("bn254")
    yield e
    e.close()


@pytest.fixture(scope="module")
def crs():
    return [P(h) for h in load("ipa_crs_bn254.json")["points"]]


def test_to_data_item_golden(eng):
    from vkzg import scheme
    comp = load("transcript.json")["compressed"]
    got = scheme.to_data_item(eng, [P(c["point"]) for c in comp])
    assert [hex(g) for g in got] == [c["to_data_item"] for c in comp]


def test_ipa_256_commit_and_proofs_golden(eng, crs):
    from vkzg import scheme
    g = load("ipa_256.json")
    ipa = scheme.IPA(eng, 256, crs)
    data = scheme.LagrangeBasis([H(x) for x in g["data"]])
    com = ipa.commit(data)
    assert com == P(g["commitment"])
    for key in ("proof_in_domain", "proof_out_domain"):
        want = g[key]
        pr = ipa.prove(com, want["point"], data)
        assert pr.y == H(want["y"]) and pr.tip == H(want["tip"])
        assert pr.l == [P(x) for x in want["l"]] and pr.r == [P(x) for x in want["r"]]
        assert ipa.verify(com, want["point"], pr)
    # proof at an out-of-domain point must not verify at an in-domain index (ipa/mod.rs:420)
    out = ipa.prove(com, 1000, data)
    assert not ipa.verify(com, 77, out)


def test_ipa_batched_proofs_match_single(eng, crs):
    """vc_ipa_prove over a batch == the proofs one at a time (no cross-talk between proofs)."""
    from vkzg import scheme
    ipa = scheme.IPA(eng, 32, crs[:33])
    rng = random.Random(5)
    datas = [scheme.LagrangeBasis([rng.randrange(scheme.R_BN254) for _ in range(32)]) for _ in range(5)]
    coms = ipa.commit_batch(datas)
    pts = [3, 40, 31, 0, 12345]
    batch = ipa.prove_batch_points(coms, pts, datas)
    for i in range(5):
        single = ipa.prove_point(coms[i], pts[i], datas[i])
        assert batch[i].as_dict() == single.as_dict()
        assert ipa.verify_point(coms[i], pts[i], batch[i])


def test_reference_ipa_eval_test(eng, crs):
    """ipa/mod.rs:404-421 at N = 32 with data 0..31."""
    from pyoracle import protocol
    from vkzg import scheme
    ipa = scheme.IPA(eng, 32, crs[:33])
    data = scheme.LagrangeBasis(list(range(32)))
    com = ipa.commit(data)
    oracle = protocol.IPA(32, points=crs[:33])
    assert com == oracle.commit(protocol.LagrangeBasis.from_vec(list(range(32))))
    pr = ipa.prove(com, 13, data)
    assert ipa.verify(com, 13, pr)
    assert oracle.verify(com, 13, pr.as_dict())          # the oracle accepts the engine's proof
    po = ipa.prove(com, 64, data)
    assert ipa.verify(com, 64, po) and not ipa.verify(com, 13, po)
    bad = scheme.IPAProof(po.l, po.r, (po.tip + 1) % scheme.R_BN254, po.y)
    assert not ipa.verify(com, 64, bad)


def test_ipa_commitment_proof_golden(eng, crs):
    """prove_commitment (ipa/mod.rs:199-234) at N = 256 == the oracle's proof bytes."""
    from vkzg import scheme
    g = load("ipa_256.json")
    ipa = scheme.IPA(eng, 256, crs)
    data = scheme.LagrangeBasis([H(x) for x in g["data"]])
    com = P(g["commitment"])
    want = g["commitment_proof"]
    pr = ipa.prove_commitment(com, data)
    assert pr.tip == H(want["tip"]) and pr.y == 0
    assert pr.l == [P(x) for x in want["l"]] and pr.r == [P(x) for x in want["r"]]
    assert ipa.verify_commitment_proof(com, pr)


def test_reference_commit_evaluations(eng, crs):
    """ipa/mod.rs:382-402 (test_commit_evaluations) at N = 32: the commitment proof of 0..31
    verifies, and fails against C + G; plus a tampered tip / swapped L, R; the oracle accepts
    the engine's proof."""
    from pyoracle import protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    ipa = scheme.IPA(eng, 32, crs[:33])
    data = scheme.LagrangeBasis(list(range(32)))
    com = ipa.commit(data)
    pr = ipa.prove_commitment(com, data)
    assert ipa.verify_commitment_proof(com, pr)
    assert not ipa.verify_commitment_proof(BN254.add(com, BN254.g), pr)
    bad = scheme.IPAProof(pr.l, pr.r, (pr.tip + 1) % scheme.R_BN254, 0)
    assert not ipa.verify_commitment_proof(com, bad)
    assert not ipa.verify_commitment_proof(com, scheme.IPAProof(pr.r, pr.l, pr.tip, 0))
    oracle = protocol.IPA(32, points=crs[:33])
    assert oracle.verify_commitment_proof(com, {"l": pr.l, "r": pr.r, "tip": pr.tip})


def test_ipa_commitment_proof_batch_and_edges(eng, crs):
    """batched commitment proofs == single ones; short data (max + 1 = 8 of N = 32, the
    reference proves over g[0..max+1]); one value (0 rounds: C == tip * g0); the reference's
    assert on a non-power-of-two length -> error."""
    from pyoracle import protocol
    from vkzg import scheme
    ipa = scheme.IPA(eng, 32, crs[:33])
    oracle = protocol.IPA(32, points=crs[:33])
    rng = random.Random(9)
    datas = [scheme.LagrangeBasis([rng.randrange(scheme.R_BN254) for _ in range(8)]) for _ in range(4)]
    coms = [oracle.commit(protocol.LagrangeBasis.from_vec(d.evals)) for d in datas]
    batch = ipa.prove_commitment_batch(coms, datas)
    for i in range(4):
        single = ipa.prove_commitment(coms[i], datas[i])
        assert batch[i].as_dict() == single.as_dict()
        want = oracle.prove_commitment(coms[i], protocol.LagrangeBasis.from_vec(datas[i].evals))
        assert (batch[i].l, batch[i].r, batch[i].tip) == (want["l"], want["r"], want["tip"])
        assert ipa.verify_commitment_proof(coms[i], batch[i])
    one = scheme.LagrangeBasis([12345])
    c1 = oracle.commit(protocol.LagrangeBasis.from_vec([12345]))
    p1 = ipa.prove_commitment(c1, one)
    assert p1.l == [] and p1.tip == 12345 and ipa.verify_commitment_proof(c1, p1)
    with pytest.raises(Exception):
        ipa.prove_commitment(coms[0], scheme.LagrangeBasis(list(range(6))))


def test_kzg_256_golden(eng):
    from pyoracle.curves import BN254
    from vkzg import scheme, VCError
    g = load("kzg_256.json")
    kz = scheme.KZG(eng, 256, secret=100)
    assert kz.size == 256
    L = kz.lagrange_points()
    cs = [H(c) for c in g["lagrange_scalars"]]
    for j in (0, 1, 77, 255):
        assert L[j] == BN254.mul(BN254.g, cs[j])
    data = scheme.LagrangeBasis([H(x) for x in g["evals"]], 256)
    com = kz.commit(data)
    assert com == P(g["commitment"])
    for op in g["openings"]:
        if "error" in op:
            with pytest.raises(VCError):
                kz.prove(com, op["point"], data)
            continue
        q, y = kz.quotient(op["point"], data)
        assert hex(y) == op["y"]
        assert [hex(v) for v in q[:4]] == op["q_head"] and hex(sum(q) % scheme.R_BN254) == op["q_sum"]
        pr = kz.prove(com, op["point"], data)
        assert pr["proof"] == P(op["proof"]) and hex(pr["y"]) == op["y"]


@pytest.mark.parametrize("curve", ["bn254", "bls12_381"])
def test_kzg_prove_on_fixed_base_tables(curve):
    """A KZG table with fixed-base window tables (vc_fixed_base_precompute) proves a <= 1024-term
    opening on the batched commit's latency path instead of Pippenger: the proof and y equal the
    Pippenger ones (and, on BN254, the golden openings), in and out of the domain, sizes 32 / 256."""
    import ctypes
    import numpy as np
    import vkzg
    from vkzg import scheme
    from vkzg._lib import check, lib
    e = vkzg.Engine(curve)
    try:
        if curve == "bn254":
            g = load("kzg_256.json")
            kz = scheme.KZG(e, 256, secret=100)
            data = scheme.LagrangeBasis([H(x) for x in g["evals"]], 256)
            com = kz.commit(data)
            ops = [op for op in g["openings"] if "error" not in op]
            e.fixed_base_precompute(kz.table, 8)
            for op in ops:
                pr = kz.prove(com, op["point"], data)
                assert pr["proof"] == P(op["proof"]) and hex(pr["y"]) == op["y"], op["point"]
        rng = random.Random(11)
        nl = 8 if curve == "bn254" else 12
        from vkzg import dist
        r = scheme.R_BN254 if curve == "bn254" else dist.BASE_P["bandersnatch"]  # Bandersnatch's base = BLS12-381 r
        for size in (32, 256):
            tid = e.random_bases(size, seed=size)
            ev = vkzg.ints_to_limbs([rng.randrange(r) for _ in range(size - 3)])

            def prove(point):
                pxy = np.zeros(nl, dtype=np.uint64)
                pinf = np.zeros(1, dtype=np.uint8)
                y = np.zeros(4, dtype=np.uint64)
                pt = np.array([(point >> (64 * j)) & (2**64 - 1) for j in range(4)], dtype=np.uint64)
                check(lib().vc_kzg_prove(e.h, tid, size, scheme._p(ev), size - 3, scheme._p(pt), scheme._p(pxy),
                                         scheme._p(pinf), scheme._p(y)), "kzg_prove")
                return pxy.tolist(), int(pinf[0]), y.tolist()

            points = (0, 5, size - 1, size + 7, rng.randrange(r))
            want = [prove(z) for z in points]       # Pippenger
            e.fixed_base_precompute(tid, 8)
            got = [prove(z) for z in points]        # fixed-base latency path
            assert got == want, (curve, size)
    finally:
        e.close()


def test_scratch_pool_reuse_and_stream_switch():
    """Per-call scratch comes from the context's stream-ordered pool (ctx.hpp DevBuf(ctx)):
    repeated KZG opens of different sizes, interleaved IPA proofs, and a switch to another
    stream (vc_ctx_set_stream drains the old one) must reproduce the golden openings exactly."""
    import torch
    import vkzg
    from vkzg import scheme
    g = load("kzg_256.json")
    e = vkzg.Engine("bn254")
    try:
        kz = scheme.KZG(e, 256, secret=100)
        small = scheme.KZG(e, 16)
        data = scheme.LagrangeBasis([H(x) for x in g["evals"]], 256)
        com = kz.commit(data)
        ops = [op for op in g["openings"] if "error" not in op]
        want = [(P(op["proof"]), H(op["y"])) for op in ops]
        rng = random.Random(5)
        d16 = scheme.LagrangeBasis([rng.randrange(scheme.R_BN254) for _ in range(8)], 16)
        c16 = small.commit(d16)
        first16 = small.prove(c16, 3, d16)
        for rep in range(3):
            if rep == 2:  # another stream: pooled blocks freed on the old one must not race
                side = torch.cuda.Stream()
                e.set_stream(side.cuda_stream)
            for op, (pw, yw) in zip(ops, want):
                pr = kz.prove(com, op["point"], data)
                assert pr["proof"] == pw and pr["y"] == yw, (rep, op["point"])
                assert small.prove(c16, 3, d16) == first16
        e.set_stream(None)
    finally:
        e.close()


def test_reference_kzg_test_restated(eng):
    """kzg/mod.rs:278-297: CRS 16, data 8; every index proves (trapdoor check), y = 0 on 8..16, 17 out."""
    from pyoracle import protocol
    from vkzg import scheme
    rng = random.Random(9)
    kz = scheme.KZG(eng, 16)
    ok = protocol.KZG(16)
    data = scheme.LagrangeBasis([rng.randrange(scheme.R_BN254) for _ in range(8)], 16)
    com = kz.commit(data)
    for i in list(range(16)) + [17]:
        pr = kz.prove(com, i, data)
        assert ok.verify(com, i, pr)
        if 8 <= i < 16:
            assert pr["y"] == 0


@pytest.mark.parametrize("name", ["ipa", "kzg"])
def test_multiproof_golden(eng, crs, name):
    from pyoracle import protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    g = load("multiproof_32.json")[name]
    vc = scheme.IPA(eng, 32, crs[:33]) if name == "ipa" else scheme.KZG(eng, 32)
    queries = []
    for q in g["queries"]:
        d = scheme.LagrangeBasis([H(x) for x in q["data"]])
        c = vc.commit(d)
        assert c == P(q["commit"])
        queries.append((d, c, q["z"], H(q["y"])))
    mp = scheme.prove_multiproof(vc, queries)
    assert mp["d"] == P(g["d"])
    vq = [(q[1], q[2], q[3]) for q in queries]
    if name == "ipa":
        want = g["proof"]
        pr = mp["proof"]
        assert pr.l == [P(x) for x in want["l"]] and pr.tip == H(want["tip"]) and pr.y == H(want["y"])
        assert scheme.verify_multiproof(vc, vq, mp)
        bad = dict(mp, d=BN254.add(mp["d"], BN254.g))
        assert not scheme.verify_multiproof(vc, vq, bad)
        vq2 = list(vq)
        vq2[0] = (vq[0][0], vq[0][1], (vq[0][2] + 1) % scheme.R_BN254)
        assert not scheme.verify_multiproof(vc, vq2, mp)
    else:
        assert mp["proof"]["proof"] == P(g["proof"]["proof"]) and mp["proof"]["y"] == H(g["proof"]["y"])
        claim = scheme.verify_multiproof(vc, vq, mp)
        ok = protocol.KZG(32)
        assert ok.verify_point(claim["commitment"], claim["t"], mp["proof"])


@pytest.mark.parametrize("G", [1, 3])
def test_multiproof_sharded_phases_golden(eng, crs, G):
    """the three-phase prover (vc_multiproof_begin / accumulate / finish) with the query set cut
    into G shards accumulated separately (as G ranks would) == the golden multiproof."""
    import numpy as np
    import torch
    from vkzg import dist as vdist
    from vkzg import scheme
    g = load("multiproof_32.json")["ipa"]
    vc = scheme.IPA(eng, 32, crs[:33])
    queries = []
    for q in g["queries"]:
        d = scheme.LagrangeBasis([H(x) for x in q["data"]])
        queries.append((d, vc.commit(d), q["z"], H(q["y"])))
    Q, data, cxy, cinf, z, y = scheme._queries(queries, 32)
    d_data = torch.from_numpy(data.view(np.int64).copy()).cuda()
    if G == 1:
        mp = vdist.multiproof_prove_sharded(vc, cxy, cinf, z, y, d_data.data_ptr(), 0, 1)
    else:
        tr, r, rows = scheme.multiproof_begin(32, cxy, cinf, z, y)
        parts = torch.zeros((G, rows, 32, 4), dtype=torch.int64, device="cuda")
        for k in range(G):
            lo, hi = vdist.shard_range(Q, k, G)
            scheme.multiproof_accumulate(eng, 32, z, lo, hi - lo, d_data[lo * 32:].data_ptr(), r,
                                         parts[k].data_ptr())
        mp = scheme.multiproof_finish_ipa(vc, z, parts.data_ptr(), G, tr)
    assert mp["d"] == P(g["d"])
    want = g["proof"]
    pr = mp["proof"]
    assert pr.l == [P(x) for x in want["l"]] and pr.r == [P(x) for x in want["r"]]
    assert pr.tip == H(want["tip"]) and pr.y == H(want["y"])


def test_ipa_point_on_domain_element_is_domain_error(eng, crs):
    """compute_barycentric_coefficients divides by (point - w^i) (precompute.rs:85): at a domain
    element w^i that is not below N as an integer the reference panics; the engine returns
    VC_E_DOMAIN for both prove and verify instead of all-zero weights (which would let verify
    accept y = 0 for any commitment)."""
    import vkzg
    from vkzg import scheme
    N = 32
    ipa = scheme.IPA(eng, N, crs[:N + 1])
    r = scheme.R_BN254
    omega = pow(5, (r - 1) // N, r)
    data = scheme.LagrangeBasis(list(range(N)))
    com = ipa.commit(data)
    for i in (1, 3, 31):
        pt = pow(omega, i, r)
        assert pt >= N
        with pytest.raises(vkzg.VCError) as ex:
            ipa.prove_point(com, pt, data)
        assert ex.value.status == -8
        good = ipa.prove_point(com, 1000, data)
        with pytest.raises(vkzg.VCError) as ex:
            ipa.verify_point(com, pt, scheme.IPAProof(good.l, good.r, good.tip, 0))
        assert ex.value.status == -8
    # omega^0 = 1 < N is the one-hot branch (precompute.rs:75-79), not an error
    pr = ipa.prove_point(com, 1, data)
    assert pr.y == 1 and ipa.verify_point(com, 1, pr)


@pytest.mark.parametrize("G", [1, 3])
def test_kzg_multiproof_sharded_golden(eng, G):
    """the three-phase prover with the KZG finish (vc_multiproof_finish scheme 1) over G query
    shards == the golden KZG multiproof (multiproof.rs:99-176 over KZG, :310-357)."""
    import numpy as np
    import torch
    from vkzg import dist as vdist
    from vkzg import scheme
    g = load("multiproof_32.json")["kzg"]
    vc = scheme.KZG(eng, 32)
    queries = []
    for q in g["queries"]:
        d = scheme.LagrangeBasis([H(x) for x in q["data"]])
        queries.append((d, vc.commit(d), q["z"], H(q["y"])))
    Q, data, cxy, cinf, z, y = scheme._queries(queries, 32)
    d_data = torch.from_numpy(data.view(np.int64).copy()).cuda()
    if G == 1:
        mp = vdist.multiproof_prove_sharded(vc, cxy, cinf, z, y, d_data.data_ptr(), 0, 1)
    else:
        tr, r, rows = scheme.multiproof_begin(32, cxy, cinf, z, y)
        parts = torch.zeros((G, rows, 32, 4), dtype=torch.int64, device="cuda")
        for k in range(G):
            lo, hi = vdist.shard_range(Q, k, G)
            scheme.multiproof_accumulate(eng, 32, z, lo, hi - lo, d_data[lo * 32:].data_ptr(), r,
                                         parts[k].data_ptr())
        torch.cuda.synchronize()
        mp = scheme.multiproof_finish(vc, z, parts.data_ptr(), G, tr)
    assert mp["d"] == P(g["d"])
    assert mp["proof"]["proof"] == P(g["proof"]["proof"]) and mp["proof"]["y"] == H(g["proof"]["y"])


def test_multiproof_phases_reject_out_of_domain_z(eng):
    """The sharded multiproof's accumulate / finish entry points take z from the caller again:
    a query point outside the domain is VC_E_DOMAIN (the reference panics indexing the Lagrange
    evaluations), an absurd domain size VC_E_INVALID -- validated before any allocation sized
    by the values (multiproof.rs:119-144)."""
    import ctypes
    import numpy as np
    import torch
    import vkzg
    from vkzg import scheme
    from vkzg._lib import lib
    N, Q = 256, 4
    z = np.array([1, 5, 300, 7], dtype=np.uint64)  # 300 >= N
    r = np.array([3, 0, 0, 0], dtype=np.uint64)
    d_data = torch.zeros((Q, N, 4), dtype=torch.int64, device="cuda")
    d_S = torch.zeros((Q, N, 4), dtype=torch.int64, device="cuda")
    with pytest.raises(vkzg.VCError) as ex:
        scheme.multiproof_accumulate(eng, N, z, 0, Q, d_data.data_ptr(), r, d_S.data_ptr())
    assert ex.value.status == -8
    zbig = np.array([1, 5, 1 << 62, 7], dtype=np.uint64)
    with pytest.raises(vkzg.VCError) as ex:
        scheme.multiproof_accumulate(eng, N, zbig, 0, Q, d_data.data_ptr(), r, d_S.data_ptr())
    assert ex.value.status == -8
    st = lib().vc_multiproof_accumulate(eng.h, 1 << 40, Q, z.ctypes.data_as(ctypes.c_void_p), 0, Q,
                                        ctypes.c_void_p(d_data.data_ptr()), r.ctypes.data_as(ctypes.c_void_p),
                                        ctypes.c_void_p(d_S.data_ptr()))
    assert st == -1


def test_ipa_verify_proof_points_on_host_straus(eng, crs):
    """IPA verify's C / L_k / R_k MSM (17 points at N = 32 + ...) runs as Straus on the host pool
    (scheme.hip host_msm): swapped L / R and an identity L_k are rejected, an off-curve L_k is
    VC_E_NOT_ON_CURVE exactly as the GPU upload reports it, and the verdicts match the oracle."""
    import vkzg
    from pyoracle import protocol
    from vkzg import scheme
    ipa = scheme.IPA(eng, 32, crs[:33])
    oracle = protocol.IPA(32, points=crs[:33])
    data = scheme.LagrangeBasis([(7 * i + 3) % 101 for i in range(32)])
    com = ipa.commit(data)
    pr = ipa.prove(com, 77, data)
    assert ipa.verify(com, 77, pr) and oracle.verify(com, 77, pr.as_dict())
    swapped = scheme.IPAProof(pr.r, pr.l, pr.tip, pr.y)
    assert not ipa.verify(com, 77, swapped)
    assert not oracle.verify(com, 77, swapped.as_dict())
    ident = scheme.IPAProof([None] + list(pr.l[1:]), pr.r, pr.tip, pr.y)
    assert not ipa.verify(com, 77, ident)
    assert not oracle.verify(com, 77, ident.as_dict())
    off = scheme.IPAProof([(1, 1)] + list(pr.l[1:]), pr.r, pr.tip, pr.y)
    with pytest.raises(vkzg.VCError) as ex:
        ipa.verify(com, 77, off)
    assert ex.value.status == -6
