"""GPU: the verkle commitment at the bench's key length N = 32 (bench.py's verkle line) == the
oracle's recursive gen_commitment (reference verkle-tree/src/node.rs:205-277, lib.rs:112-129).

At N = 32 the extension rows are 32 wide and the stem item `bytes_to_item(stem)`
(node.rs:248-250 -> vector-commit/src/lagrange_basis.rs:175-176) really reduces mod r: the stems
of tests/verkle32_keys.py cover every quotient estimate of verkle.cpp's item_of_bytes (k r - 1,
k r, k r + 1 for k = 1..5, 2^256 - 1, stems below k r with k r's top limb) and random stems >= r;
leaf units < 16 and >= 16 fill c1 and c2 (node.rs:226-239). Each tree is committed fresh, then
after two update rounds (~1 % of the keys rewritten plus a few new keys: dirty nodes only, delta
rows on the device path; one rewrite lands below a level-skipping split and adds a second extension
for its stem, as the reference does -- tests/verkle32_keys.py quirk_keys), on the device path (default, every sparse level on the sort-based path,
every level dense), the host path, a 2-member vc_group and 2 SPMD ranks (node slices per level),
over KZG(256) (the bench's scheme) and IPA(256)."""
import json
import os
import random

import pytest

from verkle32_keys import key_set, quirk_keys, value

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
N = 32


def _rounds(seed=11):
    """[(key, value)] per round: the full tree, then two update rounds of ~1 % rewrites + new keys"""
    rng = random.Random(seed)
    keys = key_set(seed)
    first, again = quirk_keys()
    rounds = [[(k, value(rng)) for k in keys + first]]
    extra = key_set(seed + 1, n_random=12)
    for r in range(2):
        upd = [(k, value(rng)) for k in rng.sample(keys, max(3, len(keys) // 100))]
        upd += [(k, value(rng)) for k in extra[r * 6:(r + 1) * 6]]
        if r == 0:  # the update that adds a second extension for one stem (the reference's quirk)
            upd.append((again, value(rng)))
        rounds.append(upd)
    return rounds


def _commit_fns(scheme_name):
    from pyoracle import cref, protocol
    from pyoracle.curves import BN254
    if scheme_name == "kzg":
        cj = protocol.kzg_lagrange_scalars(256)

        def commit(vals):  # L_j = c_j G  ->  sum v_j L_j = (sum c_j v_j) G
            return BN254.mul(BN254.g, sum(c * v for c, v in zip(cj, vals)) % BN254.r)
        return commit
    pts = _ipa_points()

    def commit(vals):
        return cref.msm("bn254", pts[:len(vals)], list(vals), 16)
    return commit


def _ipa_points():
    with open(os.path.join(HERE, "golden", "ipa_crs_bn254.json")) as f:
        return [(int(h[0], 16), int(h[1], 16)) for h in json.load(f)["points"]][:257]


_ORACLE = {}


def _apply(tree, batch, skip_exc):
    for k, v in batch:
        try:
            tree.insert_single(k, v)
        except skip_exc:
            pass


def oracle_roots(scheme_name):
    """the oracle's root after each round (computed once per scheme)"""
    if scheme_name not in _ORACLE:
        from pyoracle import verkle as ov
        commit = _commit_fns(scheme_name)
        o, roots = ov.VerkleTree(N), []
        for batch in _rounds():
            _apply(o, batch, ov.VerklePanic)
            roots.append(o.commitment(commit))
        _ORACLE[scheme_name] = roots
    return _ORACLE[scheme_name]


def _engine_roots(commit):
    """the same rounds through vkzg.verkle.VerkleTree; commit(tree) -> root"""
    from vkzg._lib import VCError
    from vkzg.verkle import VerkleTree
    t, roots = VerkleTree(N), []
    for i, batch in enumerate(_rounds()):
        _apply(t, batch, VCError)
        if i:
            assert t.stats()["dirty"] > 0
        roots.append(commit(t))
        assert t.stats()["dirty"] == 0
    return roots


@pytest.fixture(scope="module")
def eng():
    import vkzg
    e = vkzg.Engine("bn254")
    yield e
    e.close()


@pytest.mark.parametrize("mode", ["dev", "dev-sort", "dev-dense", "dev-selfinv", "host"])
@pytest.mark.parametrize("scheme_name", ["kzg", "ipa"])
def test_verkle32_matches_oracle(eng, oracle_c, scheme_name, mode, monkeypatch):
    """one context: dev = the default device path; dev-sort = every sparse level on the sort-based
    path (VKZG_SPARSE_SMALL_MAX=0); dev-dense = every level as dense rows (VKZG_VERKLE_DENSE=1);
    dev-selfinv = the normalisations' early-queued finish blocks time out at once (1 us) and invert
    their products themselves (VKZG_NORM_EARLY_US=1: the path a stalled host thread takes);
    host = host-built rows (VKZG_VERKLE_DEV=0, the group / SPMD paths' code)"""
    from vkzg import scheme
    if mode == "dev-sort":
        monkeypatch.setenv("VKZG_SPARSE_SMALL_MAX", "0")
    elif mode == "dev-dense":
        monkeypatch.setenv("VKZG_VERKLE_DENSE", "1")
    elif mode == "dev-selfinv":
        monkeypatch.setenv("VKZG_NORM_EARLY_US", "1")
    elif mode == "host":
        monkeypatch.setenv("VKZG_VERKLE_DEV", "0")
    table = scheme.KZG(eng, 256).table if scheme_name == "kzg" else scheme.IPA(eng, 256, _ipa_points()).table
    want = oracle_roots(scheme_name)
    got = _engine_roots(lambda t: t.commitment(eng, table))
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"round {i}"


def test_verkle32_group_matches_oracle(oracle_c):
    """vc_group_verkle_commitment, G = 2 members (each level's rows in member slices)"""
    from vkzg.group import Group
    want = oracle_roots("kzg")
    g = Group("bn254", [0, 0])
    try:
        tid, _ = g.kzg_setup(256)
        got = _engine_roots(lambda t: g.verkle_commitment(t, tid))
    finally:
        g.close()
    assert got == want


def test_verkle32_spmd_matches_oracle(oracle_c):
    """vc_verkle_commitment_sharded, world 2 (two rank threads on the card, host-callback
    exchange: node slices per level, one all-gather per level)"""
    from test_gpu_comm import run_ranks
    from vkzg import scheme
    want = oracle_roots("kzg")

    def body(k, comm, e):
        kz = scheme.KZG(e, 256)
        return _engine_roots(lambda t: comm.verkle_commitment(t, e, kz.table))

    for got in run_ranks(2, "bn254", body):
        assert got == want
