"""GPU: one process, several members (include/vc_group.h). Members may repeat a device, so these
run G = 2 and 3 members on the one card of the test box: every group call == the one-context
call and the oracle / golden fixtures (utils.rs:16-19, ipa/mod.rs:130-135, kzg/mod.rs:136-154,
multiproof.rs:99-176, verkle-tree node.rs:205-277)."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def P(h):
    return None if h is None else (int(h[0], 16), int(h[1], 16))


def _group(curve, G):
    from vkzg.group import Group
    return Group(curve, [0] * G)


@pytest.mark.parametrize("curve,n", [("bls12_381", 20000), ("bn254", 4099), ("bandersnatch", 3001)])
@pytest.mark.parametrize("G", [2, 3])
def test_group_msm_both_splits(oracle_c, curve, n, G):
    """vc_group_msm (host scalars) with the point split and the window split == the oracle's
    naive MSM; a sub-range (offset) too."""
    import vkzg
    from vkzg import group as vgroup
    g = _group(curve, G)
    try:
        tid = g.random_bases(n, seed=71)
        e = vkzg.Engine(curve)
        try:
            xy, inf = e.download_bases(e.random_bases(n, seed=71))
        finally:
            e.close()
        sc = vkzg.random_scalars(curve, n, np.random.default_rng(72))
        sc[5] = 0
        want = oracle_c.msm_arrays(curve, xy, inf, sc, 8)
        want_off = oracle_c.msm_arrays(curve, xy[100:], inf[100:], sc[:n - 100], 8)
        for split in (vgroup.SPLIT_POINTS, vgroup.SPLIT_WINDOWS, vgroup.SPLIT_AUTO):
            g.set_msm_split(split)
            got = g.msm(tid, sc)
            assert got[1] == want[1] and np.array_equal(got[0], want[0]), split
            got = g.msm(tid, sc[:n - 100], offset=100)
            assert got[1] == want_off[1] and np.array_equal(got[0], want_off[0]), split
        tiny = g.msm(tid, sc[:1])                      # fewer points than members
        w1 = oracle_c.msm_arrays(curve, xy[:1], inf[:1], sc[:1], 1)
        assert tiny[1] == w1[1] and np.array_equal(tiny[0], w1[0])
    finally:
        g.close()


@pytest.mark.parametrize("G", [2, 3])
def test_group_msm_batch(oracle_c, G):
    """vc_group_msm_batch: contiguous batch slices per member == one context == the oracle."""
    import vkzg
    g = _group("bandersnatch", G)
    e = vkzg.Engine("bandersnatch")
    try:
        tid = g.random_bases(256, seed=9)
        etid = e.random_bases(256, seed=9)
        xy, inf = e.download_bases(etid)
        sc = vkzg.random_scalars("bandersnatch", 256 * 37, np.random.default_rng(3))
        gxy, ginf = g.msm_batch(tid, sc, 256)
        exy, einf = e.msm_batch(etid, sc, 256)
        assert np.array_equal(gxy, exy) and np.array_equal(ginf, einf)
        for j in (0, 17, 36):
            w = oracle_c.msm_arrays("bandersnatch", xy, inf, sc[j * 256:(j + 1) * 256], 4)
            assert np.array_equal(gxy[j], w[0])
    finally:
        e.close()
        g.close()


@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("split", ["ranges", "windows"])
def test_group_kzg_prove_golden(G, split):
    """vc_group_kzg_prove == the golden KZG d = 256 openings (in the domain, at its boundary, outside,
    and the reference's error case), with the default index-range shards (each member its slice of
    the quotient and of the SRS points, one exchange of G field partials) and the window split."""
    import vkzg
    from vkzg import group as vgroup
    from vkzg import scheme
    gd = load("kzg_256.json")
    g = _group("bn254", G)
    try:
        if split == "windows":
            g.set_msm_split(vgroup.SPLIT_WINDOWS)
        tid, size = g.kzg_setup(256)
        ev = vkzg.ints_to_limbs([int(x, 16) for x in gd["evals"]])
        for op in gd["openings"]:
            if "error" in op:
                with pytest.raises(vkzg.VCError):
                    g.kzg_prove(tid, size, ev, op["point"])
                continue
            xy, inf, y = g.kzg_prove(tid, size, ev, op["point"])
            assert scheme._pt(xy, inf) == P(op["proof"]) and hex(y) == op["y"]
    finally:
        g.close()


def _golden_mp(name):
    from vkzg import scheme
    gd = load("multiproof_256.json")
    N, Q = 256, gd["Q"]
    data = scheme.ints_to_limbs([(int(r0, 16) + i) % scheme.R_BN254 for r0 in gd["r0"] for i in range(N)])
    cxy, cinf = scheme._pt_arrays([P(c) for c in gd[name]["commits"]])
    z = np.array(gd["z"], dtype=np.uint64)
    y = np.ascontiguousarray(data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)])
    return gd[name], data, cxy, cinf, z, y


def _check_mp(name, mp, want):
    assert mp["d"] == P(want["d"])
    if name == "ipa":
        pr = mp["proof"]
        assert pr.l == [P(x) for x in want["proof"]["l"]] and pr.r == [P(x) for x in want["proof"]["r"]]
        assert pr.tip == int(want["proof"]["tip"], 16) and pr.y == int(want["proof"]["y"], 16)
    else:
        assert mp["proof"]["proof"] == P(want["proof"]["proof"]) and mp["proof"]["y"] == int(want["proof"]["y"], 16)


@pytest.mark.parametrize("name", ["ipa", "kzg"])
@pytest.mark.parametrize("G", [2, 3])
def test_group_multiproof_golden(name, G):
    """vc_group_multiproof_prove (transcript once, per-point sums of query slices on the members,
    finish on member 0) and vc_group_multiproof_prove_many (P = 4 proofs over the members) ==
    multiproof_256.json (N = 256)."""
    g = _group("bn254", G)
    try:
        if name == "ipa":
            tid = g.upload_points([P(h) for h in load("ipa_crs_bn254.json")["points"]])
        else:
            tid, _ = g.kzg_setup(256)
        want, data, cxy, cinf, z, y = _golden_mp(name)
        sid = 0 if name == "ipa" else 1
        _check_mp(name, g.multiproof_prove(sid, tid, 256, data, cxy, cinf, z, y), want)
        Pn = 4
        tile = lambda a: np.ascontiguousarray(np.broadcast_to(a, (Pn,) + a.shape))  # noqa: E731
        many = g.multiproof_prove_many(sid, tid, 256, tile(data), tile(cxy), tile(cinf), tile(z), tile(y))
        assert len(many) == Pn
        for mp in many:
            _check_mp(name, mp, want)
    finally:
        g.close()


def test_group_verkle_commitment():
    """vc_group_verkle_commitment (one tree, each level's commits in member slices) == the
    one-context commitment, fresh and after an incremental update."""
    import vkzg
    from vkzg import scheme
    from vkzg.verkle import VerkleTree
    rng = random.Random(17)
    N = 4
    keys1 = [tuple(rng.randrange(12) for _ in range(N)) for _ in range(600)]
    keys2 = [tuple(rng.randrange(12) for _ in range(N)) for _ in range(80)]
    vals = {k: bytes(rng.randrange(256) for _ in range(32)) for k in keys1 + keys2}

    def build(keys, t):
        for k in keys:
            try:
                t.insert_single(k, vals[k])
            except Exception:
                pass

    def commitments(commit):
        t = VerkleTree(N)
        build(keys1, t)
        a = commit(t)
        build(keys2, t)
        b = commit(t)
        assert t.stats()["dirty"] == 0
        return a, b

    e = vkzg.Engine("bn254")
    try:
        kz = scheme.KZG(e, 256)
        want = commitments(lambda t: t.commitment(e, kz.table))
    finally:
        e.close()
    for G in (2, 3):
        g = _group("bn254", G)
        try:
            tid, _ = g.kzg_setup(256)
            assert commitments(lambda t: g.verkle_commitment(t, tid)) == want
        finally:
            g.close()


def test_group_errors():
    """unknown table -> VC_E_TABLE; a bad argument -> VC_E_INVALID; the group stays usable."""
    import vkzg
    g = _group("bn254", 2)
    try:
        with pytest.raises(vkzg.VCError) as ex:
            g.msm(7, np.zeros((4, 4), dtype=np.uint64))
        assert ex.value.status == -4
        tid = g.random_bases(64, seed=1)
        with pytest.raises(vkzg.VCError) as ex:
            g.msm(tid, np.zeros((65, 4), dtype=np.uint64))
        assert ex.value.status == -5
        xy, inf = g.msm(tid, np.zeros((64, 4), dtype=np.uint64))
        assert inf == 1
    finally:
        g.close()


def test_group_multiproof_fewer_queries_than_members():
    """Q < G: the empty slices contribute zero sums (cleared on member 0's stream before the
    finish reads them); the proof equals the one-member group's (vc_multiproof_prove)."""
    want_g, data, cxy, cinf, z, y = _golden_mp("ipa")
    Q = 2
    data, cxy, cinf = data[:Q * 256], cxy[:Q], cinf[:Q]
    z, y = z[:Q], y[:Q]
    out = []
    for G in (1, 3):
        g = _group("bn254", G)
        try:
            tid = g.upload_points([P(h) for h in load("ipa_crs_bn254.json")["points"]])
            out.append(g.multiproof_prove(0, tid, 256, data, cxy, cinf, z, y))
        finally:
            g.close()
    a, b = out
    assert a["d"] == b["d"]
    assert a["proof"].l == b["proof"].l and a["proof"].r == b["proof"].r
    assert a["proof"].tip == b["proof"].tip and a["proof"].y == b["proof"].y


def test_group_peer_path():
    """members on one device copy within it (VC_GROUP_PEER_SAME); distinct devices report direct
    peer access or staged copies -- never an error."""
    import torch
    g = _group("bn254", 2)
    try:
        assert g.peer_path(0, 1) == 0 and g.peer_path(1, 0) == 0 and g.peer_path(0, 0) == 0
    finally:
        g.close()
    if torch.cuda.device_count() > 1:
        from vkzg.group import Group
        g = Group("bn254", [0, 1])
        try:
            assert g.peer_path(0, 1) in (1, 2) and g.peer_path(1, 0) in (1, 2)
        finally:
            g.close()


def test_group_msm_2e20_chunked_point_split():
    """configs[1] through vc_group_msm's point split on G = 2 members: each member's 2^19-point
    share copies its host scalars in chunks under its own MSM (vc_msm_partial, the chunked
    point-range path on the radix copies); the sum == (sum k_i s_i) G over P_i = s_i G; and
    vc_msm_partial == vc_msm_device_partial on one member."""
    import torch
    import vkzg
    from pyoracle.curves import BLS12_381 as C
    n = 1 << 20
    g = _group("bls12_381", 2)
    try:
        tid = g.random_bases(n, seed=2024)
        s = vkzg.random_base_scalars("bls12_381", 2024, n)
        k = vkzg.random_scalars("bls12_381", n, np.random.default_rng(1234))
        want = C.mul(C.g, vkzg.dot_mod(k, s, C.r))
        from vkzg import group as vgroup
        g.set_msm_split(vgroup.SPLIT_POINTS)
        got = g.msm(tid, k)
        assert vkzg.arrays_to_points("bls12_381", np.asarray(got[0])[None, :],
                                     np.array([got[1]], dtype=np.uint8))[0] == want
        eng = vkzg.Engine.__new__(vkzg.Engine)  # member 0's context, not owned
        eng.h, eng.curve, eng.cid, eng.nl = g.member(0), "bls12_381", vkzg.engine.CURVE_IDS["bls12_381"], 6
        mt = g.member_table(tid, 0)
        half = n // 2
        a = eng.msm_partial(mt, k[half:], offset=half)
        d_k = torch.from_numpy(k[half:].view(np.int64).copy()).cuda()
        b = eng.msm_device_partial(mt, d_k.data_ptr(), half, offset=half)
        from vkzg.engine import partials_sum
        pa, pb = partials_sum("bls12_381", [a]), partials_sum("bls12_381", [b])
        assert pa[1] == pb[1] and np.array_equal(pa[0], pb[0])
        eng.h = None
    finally:
        g.close()


@pytest.mark.parametrize("where", ["in_domain", "beyond_max", "outside"])
@pytest.mark.parametrize("G", [2, 3])
def test_group_kzg_prove_ranges_2e20_trapdoor(where, G):
    """configs[3]'s open at d = 2^20 on BLS12-381 through index-range shards (each member its 1/G
    of the quotient and a point range of the SRS on its radix copies), with max < size so the last
    member's slice lies partly beyond max: the same proof and y as the one-context vc_kzg_prove on
    member 0's context, and pi (s - z) = C - y G (s = 100, kzg/mod.rs:115-154) with C from the
    group MSM. beyond_max opens in the domain at m >= max (y = 0)."""
    import ctypes
    import vkzg
    from pyoracle.curves import BLS12_381 as C
    from vkzg._lib import check, lib
    n = 1 << 20
    g = _group("bls12_381", G)
    try:
        tid, size = g.kzg_setup(n)
        mx = n - 12345
        rng = np.random.default_rng(31 + G)
        ev = vkzg.random_scalars("bls12_381", mx, rng)
        if where == "in_domain":
            point_int = n // 3
            zval = pow(pow(7, (C.r - 1) // n, C.r), point_int, C.r)
        elif where == "beyond_max":
            point_int = n - 100
            zval = pow(pow(7, (C.r - 1) // n, C.r), point_int, C.r)
        else:
            point_int = n + 987654321
            zval = point_int
        xy, inf, y = g.kzg_prove(tid, size, ev, point_int)
        if where == "in_domain":
            assert y == vkzg.limbs_to_int(ev[point_int])
        if where == "beyond_max":
            assert y == 0
        # the one-context open on member 0's context and table
        h0, t0 = g.member(0), g.member_table(tid, 0)
        pt = vkzg.ints_to_limbs([point_int])[0].copy()
        pxy = np.zeros(12, dtype=np.uint64)
        pinf = np.zeros(1, dtype=np.uint8)
        y1 = np.zeros(4, dtype=np.uint64)
        Pp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        check(lib().vc_kzg_prove(h0, t0, size, Pp(ev), mx, Pp(pt), Pp(pxy), Pp(pinf), Pp(y1)), "vc_kzg_prove")
        assert np.array_equal(xy, pxy) and inf == pinf[0] and y == vkzg.limbs_to_int(y1)
        full = np.zeros((n, 4), dtype=np.uint64)
        full[:mx] = ev
        com = _pt_bls(*g.msm(tid, full))
        proof = _pt_bls(xy, inf)
        assert C.mul(proof, (100 - zval) % C.r) == C.add(com, C.neg(C.mul(C.g, y)))
    finally:
        g.close()


def _pt_bls(xy, inf):
    import vkzg
    return vkzg.arrays_to_points("bls12_381", np.asarray(xy)[None, :], np.array([inf], dtype=np.uint8))[0]
