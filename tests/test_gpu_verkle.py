"""GPU: level-batched verkle-tree commitments (vc_verkle_commitment) == the oracle's recursive
gen_commitment (reference node.rs:205-277) over KZG (Lagrange SRS, setup(256), secret 100:
the reference's test_commitment, lib.rs:313-325) and IPA (the golden IPA CRS) -- for fresh
trees, after incremental inserts (only dirty nodes recomputed), and for key lengths 3..5."""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _key(rng, N, arity=255):
    return tuple(rng.randrange(arity) for _ in range(N))


def _val(rng):
    return bytes(rng.randrange(256) for _ in range(32))


@pytest.fixture(scope="module")
def eng():
    import vkzg
    e = vkzg.Engine("bn254")
    yield e
    e.close()


def _schemes(eng):
    from pyoracle import cref, protocol
    from pyoracle.curves import BN254
    from vkzg import scheme
    kzg = scheme.KZG(eng, 256)
    cj = protocol.kzg_lagrange_scalars(256)

    def kzg_commit(vals):  # L_j = c_j G  ->  sum v_j L_j = (sum c_j v_j) G
        s = sum(c * v for c, v in zip(cj, vals)) % BN254.r
        return BN254.mul(BN254.g, s)

    with open(os.path.join(HERE, "golden", "ipa_crs_bn254.json")) as f:
        pts = [(int(h[0], 16), int(h[1], 16)) for h in json.load(f)["points"]]
    ipa = scheme.IPA(eng, 256, pts[:257])

    def ipa_commit(vals):
        return cref.msm("bn254", pts[:len(vals)], list(vals), 16)

    return {"kzg": (kzg.table, kzg_commit), "ipa": (ipa.table, ipa_commit)}


@pytest.mark.parametrize("path", ["dev", "host"])
@pytest.mark.parametrize("dense", ["auto", "0", "1"])
@pytest.mark.parametrize("scheme_name", ["kzg", "ipa"])
@pytest.mark.parametrize("N,arity,n", [(3, 255, 120), (3, 6, 60), (4, 4, 50), (5, 3, 40)])
def test_verkle_commitment_matches_oracle(eng, oracle_c, scheme_name, N, arity, n, dense, path, monkeypatch):
    """path: dev = the device-resident levels (vc_verkle_commitment's default: items stay in a
    device mirror between levels), host = the host-built rows (VKZG_VERKLE_DEV=0, the sharded /
    group paths' code). dense: the level commits' path (VKZG_VERKLE_DENSE, read per call) -- auto
    (dense rows for small levels, sparse otherwise), 0 = every level sparse, 1 = every level dense
    (internal levels on the dev path)."""
    from pyoracle import verkle as ov
    from vkzg.verkle import VerkleTree
    if dense != "auto":
        monkeypatch.setenv("VKZG_VERKLE_DENSE", dense)
    if path == "host":
        monkeypatch.setenv("VKZG_VERKLE_DEV", "0")
    table, commit = _schemes(eng)[scheme_name]
    rng = random.Random(7 * N + arity)
    t, o = VerkleTree(N), ov.VerkleTree(N)

    def insert_some(m):
        for _ in range(m):
            k, v = _key(rng, N, arity), _val(rng)
            try:
                o.insert_single(k, v)
            except ov.VerklePanic:
                continue
            t.insert_single(k, v)

    assert t.commitment(eng, table) == o.commitment(commit)       # empty tree: 256 zeros
    insert_some(n)
    assert t.commitment(eng, table) == o.commitment(commit)
    insert_some(max(1, n // 5))                                      # incremental update
    assert t.stats()["dirty"] > 0
    assert t.commitment(eng, table) == o.commitment(commit)
    assert t.stats()["dirty"] == 0


@pytest.mark.parametrize("small", ["auto", "0"])
@pytest.mark.parametrize("delta", ["1", "0"])
@pytest.mark.parametrize("N,arity", [(3, 6), (4, 4), (3, 255)])
def test_verkle_delta_rounds_match_oracle(eng, oracle_c, N, arity, delta, small, monkeypatch):
    """Several update rounds on the device path: an updated internal node's row is its old
    commitment plus the changed slots' item differences (delta rows, the insert-time slot log:
    path slots, new extensions in empty slots, splits replacing an extension by an internal node,
    several changes to one slot inside a round); VKZG_VERKLE_DELTA=0 recommits full rows. small:
    the sparse commits' latency path (a wave per 64 pairs, the default for levels of <= 2^18
    pairs) or, "0", the sort-based path for every level. Every round's commitment == the
    oracle's recursive gen_commitment."""
    from pyoracle import verkle as ov
    from vkzg.verkle import VerkleTree
    monkeypatch.setenv("VKZG_VERKLE_DELTA", delta)
    if small != "auto":
        monkeypatch.setenv("VKZG_SPARSE_SMALL_MAX", small)
    table, commit = _schemes(eng)["kzg"]
    rng = random.Random(1000 * N + arity)
    t, o = VerkleTree(N), ov.VerkleTree(N)
    inserted = []
    for rnd, m in enumerate([60, 3, 1, 12, 25, 7]):
        for _ in range(m):
            if inserted and rng.random() < 0.4:
                k = rng.choice(inserted)   # rewrite an existing key (its path's slots only)
            else:
                k = _key(rng, N, arity)
            v = _val(rng)
            try:
                o.insert_single(k, v)
            except ov.VerklePanic:
                continue
            t.insert_single(k, v)
            inserted.append(k)
        assert t.commitment(eng, table) == o.commitment(commit), rnd
        assert t.stats()["dirty"] == 0


@pytest.mark.parametrize("small", ["auto", "0", "1000000000"])
def test_verkle_update_equals_fresh_tree(eng, small, monkeypatch):
    """A 40,000-key tree (32-unit keys) committed, 1 % of the keys rewritten, committed again
    (only the dirty nodes: levels of a few hundred rows with ~150 children each, whose rows are
    built on part of the host pool; delta rows) == a fresh tree with the same insertion history
    committed in full. small: the levels' path by size (auto), the sort-based path everywhere (0) or the
    latency path everywhere (10^9 pairs: the 80,000-row extension levels too)."""
    import numpy as np
    if small != "auto":
        monkeypatch.setenv("VKZG_SPARSE_SMALL_MAX", small)
    from vkzg import scheme
    from vkzg.verkle import VerkleTree
    kzg = scheme.KZG(eng, 256)
    rng = np.random.default_rng(5)
    nk = 40_000
    keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    t = VerkleTree(32)
    for i in range(nk):
        t.insert_single(keys[i].tobytes(), vals[i].tobytes())
    t.commitment(eng, kzg.table)
    history = []
    for i in rng.choice(nk, size=nk // 100, replace=False):
        history.append((keys[i].tobytes(), rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()))
        t.insert_single(*history[-1])
    assert t.stats()["dirty"] > 0
    got = t.commitment(eng, kzg.table)
    # the same insertion history replayed into a fresh tree (not the final contents inserted once:
    # the reference's level-skipping splits, node.rs:176-185, make the trie depend on the order --
    # re-inserting a key below such a split can add a second extension for it, so a fresh tree of
    # the final contents may legitimately have another shape and root)
    f = VerkleTree(32)
    for i in range(nk):
        f.insert_single(keys[i].tobytes(), vals[i].tobytes())
    for k, v in history:
        f.insert_single(k, v)
    assert got == f.commitment(eng, kzg.table)


def test_verkle_paths_and_contexts_interleave(oracle_c):
    """One tree committed alternately on the device path of two contexts and on the host path
    (the mirror moves between devices' contexts, is dropped by a host-path commitment and rebuilt
    from the host arrays): every commitment == the oracle's."""
    import vkzg
    from pyoracle import verkle as ov
    from vkzg.verkle import VerkleTree
    e1, e2 = vkzg.Engine("bn254"), vkzg.Engine("bn254")
    try:
        s1, s2 = _schemes(e1)["kzg"], _schemes(e2)["kzg"]
        rng = random.Random(99)
        N = 4
        t, o = VerkleTree(N), ov.VerkleTree(N)
        for step, (eng_, (table, commit), env) in enumerate([(e1, s1, None), (e2, s2, None), (e1, s1, "0"),
                                                             (e1, s1, None), (e2, s2, "0"), (e2, s2, None)]):
            for _ in range(30):
                k, v = _key(rng, N, 8), _val(rng)
                try:
                    o.insert_single(k, v)
                except ov.VerklePanic:
                    continue
                t.insert_single(k, v)
            if env is None:
                os.environ.pop("VKZG_VERKLE_DEV", None)
            else:
                os.environ["VKZG_VERKLE_DEV"] = env
            try:
                assert t.commitment(eng_, table) == o.commitment(commit), step
                assert t.commitment(eng_, table) == o.commitment(commit), step  # nothing dirty
            finally:
                os.environ.pop("VKZG_VERKLE_DEV", None)
    finally:
        e1.close()
        e2.close()


def test_verkle_mirror_moves_between_devices(oracle_c):
    """one tree committed alternately on contexts of devices 0 and 1: the mirror moves with the
    context (mirror_pull reads the old device's mirror and leaves the caller's device current,
    so the new mirror and scratch are allocated on the new context's device). Needs 2 GPUs."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    import vkzg
    from pyoracle import verkle as ov
    from vkzg.verkle import VerkleTree
    e0, e1 = vkzg.Engine("bn254", 0), vkzg.Engine("bn254", 1)
    try:
        s0, s1 = _schemes(e0)["kzg"], _schemes(e1)["kzg"]
        rng = random.Random(5)
        N = 4
        t, o = VerkleTree(N), ov.VerkleTree(N)
        for step, (eng_, (table, commit)) in enumerate([(e0, s0), (e1, s1), (e0, s0), (e1, s1)]):
            for _ in range(40):
                k, v = _key(rng, N, 8), _val(rng)
                try:
                    o.insert_single(k, v)
                except ov.VerklePanic:
                    continue
                t.insert_single(k, v)
            assert t.commitment(eng_, table) == o.commitment(commit), step
    finally:
        e0.close()
        e1.close()


@pytest.mark.parametrize("pieces", ["2", "3", "4"])
def test_verkle_ext_rows_in_pieces(eng, pieces, monkeypatch):
    """The extension rows built and uploaded in pieces (VKZG_VERKLE_EXT_PIECES, an A/B knob: the
    default is one piece) == the one-buffer path (pieces = 1), fresh and after a 1 % update; a
    20,000-key tree of 32-unit keys (uneven pieces at 3)."""
    import numpy as np
    from vkzg import scheme
    from vkzg.verkle import VerkleTree
    kzg = scheme.KZG(eng, 256)
    rng = np.random.default_rng(12)
    nk = 20_000
    keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    upd = [(keys[i].tobytes(), rng.integers(0, 256, size=32, dtype=np.uint8).tobytes())
           for i in rng.choice(nk, size=nk // 100, replace=False)]

    def roots(p):
        monkeypatch.setenv("VKZG_VERKLE_EXT_PIECES", p)
        t = VerkleTree(32)
        for i in range(nk):
            t.insert_single(keys[i].tobytes(), vals[i].tobytes())
        a = t.commitment(eng, kzg.table)
        for k, v in upd:
            t.insert_single(k, v)
        return a, t.commitment(eng, kzg.table)

    assert roots(pieces) == roots("1")


@pytest.mark.parametrize("mode", ["late", "selfinv", "unfused", "nolead"])
def test_verkle_norm_finish_modes(eng, mode, monkeypatch):
    """The verkle levels' normalisation (commit.hip normalize_rows_items): by default the finish
    kernel is queued behind the prep before the host has inverted the block products, its blocks
    waiting on the host's go word. == the finish launched after the inversion (late,
    VKZG_NORM_EARLY=0) and == blocks that stop waiting after 1 us and invert on their own
    (selfinv, VKZG_NORM_EARLY_US=1); fresh and after a 1 % update of a 20,000-key tree (the c1 / c2
    level's 40,000 rows take the device-scan form, the smaller levels the per-block form). unfused:
    the sort-based sparse commits' count / scan / expand / row offsets as separate launches
    (VKZG_SPARSE_FUSED=0) instead of the two fused kernels. nolead: the extension width-4 rows on the
    SRS's own 16-bit fixed-base table instead of the 20-bit table of bases 0..3 (VKZG_VERKLE_LEAD_C=0)."""
    import numpy as np
    from vkzg import scheme
    from vkzg.verkle import VerkleTree
    kzg = scheme.KZG(eng, 256)
    rng = np.random.default_rng(13)
    nk = 20_000
    keys = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    vals = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
    upd = [(keys[i].tobytes(), rng.integers(0, 256, size=32, dtype=np.uint8).tobytes())
           for i in rng.choice(nk, size=nk // 100, replace=False)]

    def roots():
        t = VerkleTree(32)
        for i in range(nk):
            t.insert_single(keys[i].tobytes(), vals[i].tobytes())
        a = t.commitment(eng, kzg.table)
        for k, v in upd:
            t.insert_single(k, v)
        return a, t.commitment(eng, kzg.table)

    want = roots()
    if mode == "late":
        monkeypatch.setenv("VKZG_NORM_EARLY", "0")
    elif mode == "unfused":
        monkeypatch.setenv("VKZG_SPARSE_FUSED", "0")
    elif mode == "nolead":
        monkeypatch.setenv("VKZG_VERKLE_LEAD_C", "0")
    else:
        monkeypatch.setenv("VKZG_NORM_EARLY_US", "1")
    assert roots() == want
