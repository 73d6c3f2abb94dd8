"""configs[4] at the reference's own shape, checked against the oracle: prove_multiproof
(vector-commit/src/multiproof.rs:99-176) at width N = 256 (benches/ipa.rs:18) with Q = 4096 and
Q = 2^16 queries (:19, 111-131). Every row z holds many queries, which is the multi-chunk path of
the engine's per-point sums (MP_CHUNK = 16 queries per chunk, csrc/scheme.hip) and its large-Q
row grouping.

The checker is oracle/pyoracle/mpcheck.py: r and t from the oracle's TranscriptHasher, g and h
from the C field phases (oracle/c/ref_multiproof.c), D and E by the naive C commit, the inner
proof by protocol.low_level_ipa / KZG.prove_point. Proof bytes are compared exactly."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NT = 16  # the GPU box's CPU share per GPU


def _golden():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "multiproof_256.json")) as f:
        return json.load(f)


def _P(h):
    return None if h is None else (int(h[0], 16), int(h[1], 16))


@pytest.fixture(scope="module")
def eng():
    import vkzg
    e = vkzg.Engine("bn254")
    yield e
    e.close()


@pytest.fixture(scope="module")
def crs():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ipa_crs_bn254.json")) as f:
        return [_P(h) for h in json.load(f)["points"]]


def _inputs(Q, N=256, seed=404):
    """uniform evaluations < r; z hits every row, rows 3 and 250 carry 3 * MP_CHUNK + 5 queries
    more than the rest, and the rest is uniform."""
    import vkzg
    rng = np.random.default_rng(seed)
    data = vkzg.random_scalars("bn254", Q * N, rng)
    data[:N] = vkzg.ints_to_limbs([vkzg.SCALAR_R["bn254"] - 1 - i for i in range(N)])   # top of the field
    z = np.concatenate([np.arange(N), np.full(53, 3), np.full(53, 250), rng.integers(0, N, size=Q - N - 106)])
    z = rng.permutation(z).astype(np.uint64)
    return data, z


def _commit_device(eng, table, N, data):
    import torch
    Q = data.shape[0] // N
    d_all = torch.from_numpy(data.view(np.int64).copy()).cuda()
    cxy_d = torch.zeros((Q, 8), dtype=torch.int64, device="cuda")
    cinf_d = torch.zeros(Q, dtype=torch.uint8, device="cuda")
    eng.msm_batch_device(table, N, d_all.data_ptr(), Q, cxy_d.data_ptr(), cinf_d.data_ptr())
    torch.cuda.synchronize()
    return d_all, cxy_d.cpu().numpy().view(np.uint64).copy(), cinf_d.cpu().numpy().copy()


def _check_sample_commits(bases, data, cxy, cinf, N, idx):
    """a few of the engine's query commitments against the oracle's naive commit (utils.rs:16-19)"""
    from pyoracle import cref
    bxy, binf = cref.points_to_array("bn254", bases[:N])
    for k in idx:
        want = cref.msm_arrays("bn254", bxy, binf, data[k * N:(k + 1) * N], 1)
        assert want[1] == cinf[k] and (want[1] or np.array_equal(want[0], cxy[k])), k


def _gpu_multiproof(eng, scheme_id, table, N, data, cxy, cinf, z):
    from vkzg import scheme
    from vkzg._lib import check, lib
    P = scheme._p
    Q = z.shape[0]
    y = np.ascontiguousarray(data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)])
    dxy = np.zeros(8, dtype=np.uint64)
    dinf = np.zeros(1, dtype=np.uint8)
    if scheme_id == 0:
        b, arrs = scheme.IPAProof._alloc(8)
        check(lib().vc_multiproof_prove(eng.h, 0, table, N, Q, P(data), P(cxy), P(cinf), P(z), P(y), P(dxy), P(dinf),
                                        ctypes.byref(b), None, None, None), "vc_multiproof_prove")
        return {"d": scheme._pt(dxy, dinf[0]), "proof": scheme.IPAProof._from(b, arrs)}, y
    kxy = np.zeros(8, dtype=np.uint64)
    kinf = np.zeros(1, dtype=np.uint8)
    ky = np.zeros(4, dtype=np.uint64)
    check(lib().vc_multiproof_prove(eng.h, 1, table, N, Q, P(data), P(cxy), P(cinf), P(z), P(y), P(dxy), P(dinf),
                                    None, P(kxy), P(kinf), P(ky)), "vc_multiproof_prove")
    return {"d": scheme._pt(dxy, dinf[0]), "proof": {"proof": scheme._pt(kxy, kinf[0]), "y": scheme.limbs_to_int(ky)}}, y


def _same_ipa(got, want):
    pr = got["proof"]
    return (got["d"] == want["d"] and pr.l == want["proof"]["l"] and pr.r == want["proof"]["r"]
            and pr.tip == want["proof"]["tip"] and pr.y == want["proof"]["y"])


@pytest.mark.parametrize("name", ["ipa", "kzg"])
def test_multiproof_256_golden(eng, crs, name):
    """multiproof_256.json (pure-Python oracle, Q = 64, 20 queries on z = 5 and on z = 200): the
    engine's query commitments, D and the inner proof, through vc_multiproof_prove."""
    from vkzg import scheme
    g = _golden()
    N = 256
    vc = scheme.IPA(eng, N, crs) if name == "ipa" else scheme.KZG(eng, N)
    queries = []
    for r0, z, cw in zip(g["r0"], g["z"], g[name]["commits"]):
        d = scheme.LagrangeBasis([(int(r0, 16) + i) % scheme.R_BN254 for i in range(N)])
        queries.append((d, _P(cw), z, d[z]))
    if name == "ipa":
        assert vc.commit_batch([q[0] for q in queries]) == [q[1] for q in queries]
    else:
        assert [vc.commit(q[0]) for q in queries[:4]] == [q[1] for q in queries[:4]]
    mp = scheme.prove_multiproof(vc, queries)
    want = g[name]
    assert mp["d"] == _P(want["d"])
    if name == "ipa":
        pr = mp["proof"]
        assert pr.l == [_P(x) for x in want["proof"]["l"]] and pr.r == [_P(x) for x in want["proof"]["r"]]
        assert pr.tip == int(want["proof"]["tip"], 16) and pr.y == int(want["proof"]["y"], 16)
        assert scheme.verify_multiproof(vc, [(q[1], q[2], q[3]) for q in queries], mp)
    else:
        assert mp["proof"]["proof"] == _P(want["proof"]["proof"]) and mp["proof"]["y"] == int(want["proof"]["y"], 16)


@pytest.mark.parametrize("Q", [4096, 1 << 16])
def test_multiproof_n256_ipa_vs_oracle(eng, crs, Q):
    """IPA multiproof at N = 256: the engine's proof == mpcheck's, and the engine's transcript
    challenge r (vc_multiproof_begin) == the oracle's; at Q = 2^16 also the proof-parallel form
    (vc_multiproof_prove_many, P = 2) and 8 query shards accumulated separately."""
    import torch
    from pyoracle import mpcheck, protocol
    from vkzg import dist as vdist
    from vkzg import scheme
    N = 256
    ipa = scheme.IPA(eng, N, crs)
    data, z = _inputs(Q)
    d_all, cxy, cinf = _commit_device(eng, ipa.table, N, data)
    _check_sample_commits(crs, data, cxy, cinf, N, [0, 1, Q // 2, Q - 1])
    got, y = _gpu_multiproof(eng, 0, ipa.table, N, data, cxy, cinf, z)
    want = mpcheck.multiproof(protocol.IPA(N, points=crs), N, data, cxy, cinf, z, nthreads=NT)
    tr, r, rows = scheme.multiproof_begin(N, cxy, cinf, z, y)
    from vkzg._lib import lib
    lib().vc_transcript_free(tr)
    assert scheme.limbs_to_int(r) == want["r"]
    assert got["d"] == want["d"], "D = commit(g) differs: the per-point sums or the quotients"
    assert _same_ipa(got, want)
    if Q == 1 << 16:
        d_two = torch.cat([d_all, d_all])
        many = scheme.prove_multiproof_many(ipa, *(np.ascontiguousarray(np.broadcast_to(a, (2,) + a.shape))
                                                   for a in (cxy, cinf, z, y)), d_two.data_ptr())
        del d_two
        assert all(_same_ipa(m, want) for m in many)
        G = 8
        tr, r, rows = scheme.multiproof_begin(N, cxy, cinf, z, y)
        parts = torch.zeros((G, rows, N, 4), dtype=torch.int64, device="cuda")
        for k in range(G):
            lo, hi = vdist.shard_range(Q, k, G)
            scheme.multiproof_accumulate(eng, N, z, lo, hi - lo, d_all[lo * N:].data_ptr(), r, parts[k].data_ptr())
        torch.cuda.synchronize()
        assert _same_ipa(scheme.multiproof_finish_ipa(ipa, z, parts.data_ptr(), G, tr), want)


def test_multiproof_n256_kzg_vs_oracle(eng):
    """the KZG finish of the same aggregation at N = 256, Q = 4096 == mpcheck over protocol.KZG(256)."""
    from pyoracle import mpcheck, protocol
    from vkzg import scheme
    N, Q = 256, 4096
    kz = scheme.KZG(eng, N)
    okz = protocol.KZG(N)
    assert kz.lagrange_points() == okz.lagrange
    data, z = _inputs(Q, seed=405)
    _d_all, cxy, cinf = _commit_device(eng, kz.table, N, data)
    _check_sample_commits(okz.lagrange, data, cxy, cinf, N, [0, Q - 1])
    got, _y = _gpu_multiproof(eng, 1, kz.table, N, data, cxy, cinf, z)
    want = mpcheck.multiproof(okz, N, data, cxy, cinf, z, nthreads=NT)
    assert got["d"] == want["d"]
    assert got["proof"]["proof"] == want["proof"]["proof"] and got["proof"]["y"] == want["proof"]["y"]


def test_multiproof_begin_accumulate_equals_phases(eng, crs):
    """vc_multiproof_begin_accumulate (the transcript on a helper thread while the shard is planned)
    gives the r and the per-point sums S of vc_multiproof_begin + vc_multiproof_accumulate, for
    the whole query set and for a shard; the transcripts then finish to the same proof."""
    import torch
    from vkzg import scheme
    N, Q = 256, 4096
    data, z = _inputs(Q, N, seed=9)
    ipa = scheme.IPA(eng, N, crs)
    d_all, cxy, cinf = _commit_device(eng, ipa.table, N, data)
    y = np.ascontiguousarray(data.reshape(Q, N, 4)[np.arange(Q), z.astype(np.int64)])
    rows = scheme.multiproof_rows(N, z)
    assert rows == N
    for lo, hi in ((0, Q), (1000, 2500)):
        tr_a, r_a, rows_a = scheme.multiproof_begin(N, cxy, cinf, z, y)
        S_a = torch.zeros((rows, N, 4), dtype=torch.int64, device="cuda")
        d_slice = d_all[lo * N:hi * N]
        scheme.multiproof_accumulate(eng, N, z, lo, hi - lo, d_slice.data_ptr(), r_a, S_a.data_ptr())
        S_b = torch.zeros((rows, N, 4), dtype=torch.int64, device="cuda")
        tr_b, r_b = scheme.multiproof_begin_accumulate(eng, N, cxy, cinf, z, y, lo, hi - lo, d_slice.data_ptr(),
                                                       S_b.data_ptr())
        torch.cuda.synchronize()
        assert rows_a == rows and np.array_equal(r_a, r_b)
        assert torch.equal(S_a, S_b)
        pa = scheme.multiproof_finish(ipa, z, S_a.data_ptr(), 1, tr_a)
        pb = scheme.multiproof_finish(ipa, z, S_b.data_ptr(), 1, tr_b)
        assert pa["d"] == pb["d"] and pa["proof"].l == pb["proof"].l and pa["proof"].tip == pb["proof"].tip
