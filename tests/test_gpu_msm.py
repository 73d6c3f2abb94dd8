"""GPU parity: the HIP Pippenger MSM (vc_msm) against the C restatement of the reference
MSM (oracle/c/ref_curve.c = utils::inner_product, utils.rs:16-19), bit-exact on canonical
affine coordinates, for BN254 G1 (the reference's curve), BLS12-381 G1 and Bandersnatch."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CURVES = ["bn254", "bls12_381", "bandersnatch"]


@pytest.fixture(scope="module")
def engines():
    import vkzg
    es = {c: vkzg.Engine(c) for c in CURVES}
    yield es
    for e in es.values():
        e.close()


def _oracle(cref, curve, xy, inf, sc, threads=16):
    out, oinf = cref.msm_arrays(curve, xy, inf, sc, threads)
    return out, oinf


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 2, 7, 64, 255, 1000, 4099, 20000])
def test_msm_random(engines, oracle_c, curve, n):
    """bit-exact against the C oracle; n = 20000 (GLV: 40000 terms, shared windows of c = 13, one
    set of 2^12 buckets) runs the tail's bit stage in its marginal form (msm_tail_plan, J = 12)"""
    import vkzg
    e = engines[curve]
    rng = np.random.default_rng(1000 + n)
    tid = e.random_bases(n, seed=n)
    xy, inf = e.download_bases(tid)
    assert oracle_c.on_curve(curve, xy)
    sc = vkzg.random_scalars(curve, n, rng)
    got, ginf = e.msm(tid, sc)
    want, winf = _oracle(oracle_c, curve, xy, inf, sc)
    assert ginf == winf
    assert np.array_equal(got, want)


@pytest.mark.parametrize("curve", CURVES)
def test_msm_edge_cases(engines, oracle_c, curve):
    """zero scalars, r-1, repeated bases (P+P doubling path), P + (-P), identity bases, all-equal scalars."""
    import vkzg
    from pyoracle.curves import CURVES as OC
    e = engines[curve]
    C = OC[curve]
    rng = random.Random(7)
    n = 300
    tid = e.random_bases(n, seed=99)
    xy, inf = e.download_bases(tid)
    pts = vkzg.arrays_to_points(curve, xy, inf)
    pts[5] = pts[4]                       # repeated base
    pts[6] = C.neg(pts[4])                # negation
    if curve != "bandersnatch":
        pts[7] = None                     # identity base
    else:
        pts[7] = (0, 1)
    sc = [rng.randrange(C.r) for _ in range(n)]
    sc[0] = 0
    sc[1] = C.r - 1
    sc[2] = 1
    sc[4] = sc[5] = sc[6] = 12345         # P + P - P
    tid2 = e.upload_points(pts)
    xy2, inf2 = vkzg.points_to_arrays(curve, pts)
    got = e.msm(tid2, vkzg.ints_to_limbs(sc))
    want = _oracle(oracle_c, curve, xy2, inf2, vkzg.ints_to_limbs(sc))
    assert got[1] == want[1] and np.array_equal(got[0], want[0])
    # all scalars equal: every term lands in the same buckets (load-balance path)
    same = [sc[10]] * n
    got = e.msm(tid2, vkzg.ints_to_limbs(same))
    want = _oracle(oracle_c, curve, xy2, inf2, vkzg.ints_to_limbs(same))
    assert got[1] == want[1] and np.array_equal(got[0], want[0])
    # all zero -> identity
    got = e.msm(tid2, vkzg.ints_to_limbs([0] * n))
    assert got[1] == 1


@pytest.mark.parametrize("curve", CURVES)
def test_msm_montgomery_scalars(engines, oracle_c, curve):
    import vkzg
    e = engines[curve]
    r = vkzg.SCALAR_R[curve]
    rng = random.Random(3)
    n = 200
    tid = e.random_bases(n, seed=5)
    xy, inf = e.download_bases(tid)
    sc = [rng.randrange(r) for _ in range(n)]
    mont = [(s << 256) % r for s in sc]
    got = e.msm(tid, vkzg.ints_to_limbs(mont), mont=True)
    want = _oracle(oracle_c, curve, xy, inf, vkzg.ints_to_limbs(sc))
    assert np.array_equal(got[0], want[0])


def _glv_edge_scalars(r, n, rng):
    from pyoracle import pippenger
    lam = pippenger.GLV_LAMBDA
    half = lam >> 1
    edge = [0, 1, lam - 1, lam, lam + 1, half, half + 1, lam + half + 1, lam * (half + 1),
            lam * (half + 1) + half + 1, lam * lam, lam * lam + half, r - 1, r - 2, r - lam]
    return (edge + [rng.randrange(r) for _ in range(n)])[:n]


def test_msm_glv_edges(engines, oracle_c):
    """BLS12-381 at n >= 4096 takes the GLV split (k = k1 + lambda k2 over P and phi(P)): the
    balancing edges of the split, repeated / negated / identity bases, Montgomery scalars and
    all-equal scalars, bit-exact against the naive oracle."""
    import vkzg
    from pyoracle import pippenger
    from pyoracle.curves import BLS12_381 as C
    e = engines["bls12_381"]
    n = 4500
    assert pippenger.glv_active("bls12_381", n)
    rng = random.Random(17)
    tid = e.random_bases(n, seed=31)
    xy, inf = e.download_bases(tid)
    pts = vkzg.arrays_to_points("bls12_381", xy, inf)
    pts[20] = pts[21]
    pts[22] = C.neg(pts[21])
    pts[23] = None
    sc = _glv_edge_scalars(C.r, n, rng)
    sc[21] = sc[22] = sc[20]
    tid2 = e.upload_points(pts)
    xy2, inf2 = vkzg.points_to_arrays("bls12_381", pts)
    want = _oracle(oracle_c, "bls12_381", xy2, inf2, vkzg.ints_to_limbs(sc))
    got = e.msm(tid2, vkzg.ints_to_limbs(sc))
    assert got[1] == want[1] and np.array_equal(got[0], want[0])
    mont = [(s << 256) % C.r for s in sc]
    got = e.msm(tid2, vkzg.ints_to_limbs(mont), mont=True)
    assert got[1] == want[1] and np.array_equal(got[0], want[0])
    for v in (pippenger.GLV_LAMBDA, C.r - 1, (pippenger.GLV_LAMBDA >> 1) + 1):
        same = [v] * n
        got = e.msm(tid2, vkzg.ints_to_limbs(same))
        want = _oracle(oracle_c, "bls12_381", xy2, inf2, vkzg.ints_to_limbs(same))
        assert got[1] == want[1] and np.array_equal(got[0], want[0])


def test_msm_glv_rejects_non_subgroup_table(engines, oracle_c):
    """A BLS12-381 table with one curve point outside the prime-order subgroup: phi is not
    [lambda] there, so the engine must see it (k_glv_check) and run the plain MSM -- the result
    is still the reference's sum of k_i P_i."""
    import vkzg
    from pyoracle.curves import BLS12_381 as C
    e = engines["bls12_381"]
    n = 4096
    tid = e.random_bases(n, seed=41)
    xy, inf = e.download_bases(tid)
    pts = vkzg.arrays_to_points("bls12_381", xy, inf)
    rng = random.Random(43)
    p = C.p
    while True:
        x = rng.randrange(p)
        a = (x ** 3 + 4) % p
        y = pow(a, (p + 1) // 4, p)
        if y * y % p == a:
            break
    pts[1000] = (x, y)
    sc = [rng.randrange(C.r) for _ in range(n)]
    tid2 = e.upload_points(pts)
    xy2, inf2 = vkzg.points_to_arrays("bls12_381", pts)
    want = _oracle(oracle_c, "bls12_381", xy2, inf2, vkzg.ints_to_limbs(sc))
    got = e.msm(tid2, vkzg.ints_to_limbs(sc))
    assert got[1] == want[1] and np.array_equal(got[0], want[0])


@pytest.mark.parametrize("curve", CURVES)
def test_msm_offset_and_partials(engines, oracle_c, curve):
    """offset slices + partial accumulators summed = whole MSM (the multi-GPU shard path)."""
    import torch
    import vkzg
    e = engines[curve]
    n = 5000
    rng = np.random.default_rng(11)
    tid = e.random_bases(n, seed=12)
    sc = vkzg.random_scalars(curve, n, rng)
    whole = e.msm(tid, sc)
    dsc = torch.from_numpy(sc.view(np.int64)).cuda()
    parts = []
    for k in range(4):
        lo, hi = k * n // 4, (k + 1) * n // 4
        parts.append(e.msm_device_partial(tid, dsc[lo:].data_ptr(), hi - lo, offset=lo))
    summed = e.partials_sum(np.stack(parts))
    assert np.array_equal(summed[0], whole[0]) and summed[1] == whole[1]


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n,parts", [(7, 2), (300, 3), (5000, 4), (70000, 2)])
def test_msm_window_parts(engines, oracle_c, curve, n, parts):
    """window-sliced partials (the default multi-GPU split): each part equals the oracle's
    window-part MSM, and the parts add up to the whole MSM."""
    import torch
    import vkzg
    from pyoracle import pippenger
    from pyoracle.curves import CURVES as OC
    e = engines[curve]
    rng = np.random.default_rng(21 + n)
    tid = e.random_bases(n, seed=22)
    xy, inf = e.download_bases(tid)
    sc = vkzg.random_scalars(curve, n, rng)
    whole = e.msm(tid, sc)
    dsc = torch.from_numpy(sc.view(np.int64)).cuda()
    accs = [e.msm_device_window_part(tid, dsc.data_ptr(), n, k, parts) for k in range(parts)]
    summed = e.partials_sum(np.stack(accs))
    assert np.array_equal(summed[0], whole[0]) and summed[1] == whole[1]
    if n <= 5000:
        ints = [vkzg.limbs_to_int(row) for row in sc]
        k = parts - 1
        want = _oracle(oracle_c, curve, xy, inf,
                       vkzg.ints_to_limbs(pippenger.part_scalars(curve, ints, k, parts, OC[curve].r)))
        got = e.partials_sum(accs[k][None, :])
        assert got[1] == want[1] and np.array_equal(got[0], want[0])


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("width,batch,c", [(256, 700, 8), (64, 3000, 12), (255, 520, 16), (5, 30000, 20)])
def test_batch_commit_persistent(engines, oracle_c, curve, width, batch, c):
    """large batches take the chunk-major path (width cut into chunks, one piece per (chunk,
    commit), piece combine); sampled commits vs the oracle, for four table window sizes up to
    the 20-bit windows of the bench's config-3 table"""
    import vkzg
    e = engines[curve]
    rng = np.random.default_rng(31 + c)
    tid = e.random_bases(width, seed=width + c)
    xy, inf = e.download_bases(tid)
    e.fixed_base_precompute(tid, c)
    sc = vkzg.random_scalars(curve, width * batch, rng)
    sc[3 * width:4 * width] = 0      # an all-zero commit in the middle
    got_xy, got_inf = e.msm_batch(tid, sc, width)
    for j in sorted({0, 1, 3, batch // 2, batch - 2, batch - 1} | set(rng.integers(0, batch, 10).tolist())):
        want = _oracle(oracle_c, curve, xy, inf, sc[j * width:(j + 1) * width])
        assert got_inf[j] == want[1], j
        if not want[1]:
            assert np.array_equal(got_xy[j], want[0]), j


@pytest.mark.parametrize("curve", CURVES)
def test_batch_commit(engines, oracle_c, curve):
    """vc_msm_batch (fixed-base tables) vs per-commit oracle MSM; width 256 and ragged width."""
    import vkzg
    e = engines[curve]
    rng = np.random.default_rng(21)
    for width, batch in ((256, 6), (37, 5)):
        tid = e.random_bases(width, seed=width)
        xy, inf = e.download_bases(tid)
        e.fixed_base_precompute(tid, 8)
        sc = vkzg.random_scalars(curve, width * batch, rng)
        sc[:width] = 0          # commit 0: all-zero data -> identity
        sc[width, :] = 0        # commit 1 has a zero scalar
        got_xy, got_inf = e.msm_batch(tid, sc, width)
        for j in range(batch):
            want = _oracle(oracle_c, curve, xy, inf, sc[j * width:(j + 1) * width])
            assert got_inf[j] == want[1], j
            if not want[1]:
                assert np.array_equal(got_xy[j], want[0]), j


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("c,windows", [(8, 30), (12, 20), (5, 43)])
def test_batch_commit_mixed_windows(engines, oracle_c, curve, c, windows):
    """fixed-base tables with windows of c and c + 1 bits (vc_fixed_base_precompute_windows): the
    latency path (small batch), the chunk-major path (large batch) and the sparse CSR commits read
    the same mixed schedule; sampled commits vs the oracle, and the reported geometry"""
    import vkzg
    e = engines[curve]
    bits = {"bn254": 254, "bls12_381": 255, "bandersnatch": 253}[curve]
    rng = np.random.default_rng(77 + c)
    width = 40
    tid = e.random_bases(width, seed=c + windows)
    xy, inf = e.download_bases(tid)
    e.fixed_base_precompute(tid, c, windows)
    assert e.fixed_base_geometry(tid) == (c, windows, bits + 1 - c * windows)
    for batch in (4, 900):
        sc = vkzg.random_scalars(curve, width * batch, rng)
        sc[width:2 * width] = 0
        got_xy, got_inf = e.msm_batch(tid, sc, width)
        for j in sorted({0, 1, batch - 1} | set(rng.integers(0, batch, 4).tolist())):
            want = _oracle(oracle_c, curve, xy, inf, sc[j * width:(j + 1) * width])
            assert got_inf[j] == want[1], (batch, j)
            if not want[1]:
                assert np.array_equal(got_xy[j], want[0]), (batch, j)
    # sparse rows (3 non-zeros each) read the same schedule
    from pyoracle.curves import CURVES as OC
    pts = vkzg.arrays_to_points(curve, xy, inf)
    rows = 50
    cols = [int(v) for v in rng.integers(0, width, size=3 * rows)]
    vals = [int.from_bytes(rng.bytes(32), "little") % OC[curve].r for _ in range(3 * rows)]
    ptr = list(range(0, 3 * rows + 1, 3))
    got_xy, got_inf = e.msm_batch_sparse(tid, ptr, cols, vkzg.ints_to_limbs(vals))
    for g in (0, 7, rows - 1):
        want = oracle_c.msm(curve, [pts[k] for k in cols[3 * g:3 * g + 3]], vals[3 * g:3 * g + 3], 4)
        if curve == "bandersnatch" and want == (0, 1):
            want = None
        got = None if got_inf[g] else vkzg.arrays_to_points(curve, got_xy[g:g + 1], got_inf[g:g + 1])[0]
        assert got == want, g
    # a schedule that needs windows wider than c + 1
    with pytest.raises(vkzg.VCError):
        e.fixed_base_precompute(tid, 8, 10)


def test_batch_commit_edwards_identity(engines, oracle_c):
    """Bandersnatch commits that sum to the identity through P + (-P) (Edwards identity (0 : Z : Z)
    with Z != 1): the device normalisation (large batches, k_norm_prep / k_norm_finish) must divide
    by Z like the host path of small batches and report the identity, (0, 1) with inf = 1."""
    import vkzg
    from pyoracle.curves import CURVES as OC
    C = OC["bandersnatch"]
    e = engines["bandersnatch"]
    xy, _ = e.download_bases(e.random_bases(2, seed=3))
    xy = np.array(xy, dtype=np.uint64)
    x0 = vkzg.limbs_to_int(xy[0][:4])
    xy[1][:4] = vkzg.ints_to_limbs([(C.p - x0) % C.p])[0]   # -P = (-x, y)
    xy[1][4:] = xy[0][4:]
    inf = np.zeros(2, dtype=np.uint8)
    tid = e.upload_bases(xy, inf)
    e.fixed_base_precompute(tid, 8)
    rng = np.random.default_rng(8)
    ident_xy = np.array([0, 0, 0, 0, 1, 0, 0, 0], dtype=np.uint64)
    for batch in (3, 100):                               # host latency path, device normalisation
        sc = vkzg.random_scalars("bandersnatch", 2 * batch, rng)
        for j in range(0, batch, 2):
            sc[2 * j + 1] = sc[2 * j]                    # a P + a (-P) = O
        got_xy, got_inf = e.msm_batch(tid, sc, 2)
        for j in range(batch):
            if j % 2 == 0:
                assert got_inf[j] == 1 and np.array_equal(np.asarray(got_xy[j], dtype=np.uint64), ident_xy), (batch, j)
            else:
                want = _oracle(oracle_c, "bandersnatch", xy, inf, sc[2 * j:2 * j + 2])
                assert got_inf[j] == want[1] and np.array_equal(got_xy[j], want[0]), (batch, j)


@pytest.mark.parametrize("curve", CURVES)
def test_batch_commit_sparse(engines, oracle_c, curve):
    """vc_msm_batch_sparse (CSR rows) vs the oracle: empty rows, single non-zeros, long rows
    straddling accumulate threads, repeated columns, a zero scalar, Montgomery input"""
    import vkzg
    from pyoracle.curves import CURVES as OC
    e = engines[curve]
    C = OC[curve]
    rng = np.random.default_rng(5)
    width = 256
    tid = e.random_bases(width, seed=17)
    xy, inf = e.download_bases(tid)
    pts = vkzg.arrays_to_points(curve, xy, inf)
    lens = [0, 1, 2, 5, 0, 256, 300, 3, 1, 0, 40] + list(rng.integers(0, 12, 60))
    ptr = [0]
    cols, vals = [], []
    for L in lens:
        for _ in range(int(L)):
            cols.append(int(rng.integers(0, width)))
            vals.append(int.from_bytes(rng.bytes(32), "little") % C.r)
        ptr.append(len(cols))
    vals[3] = 0
    got_xy, got_inf = e.msm_batch_sparse(tid, ptr, cols, vkzg.ints_to_limbs(vals))
    for g in range(len(lens)):
        lo, hi = ptr[g], ptr[g + 1]
        want = oracle_c.msm(curve, [pts[c] for c in cols[lo:hi]], vals[lo:hi], 4) if hi > lo else None
        if curve == "bandersnatch" and want == (0, 1):
            want = None
        got = None if got_inf[g] else vkzg.arrays_to_points(curve, got_xy[g:g + 1], got_inf[g:g + 1])[0]
        assert got == want, g
    # Montgomery scalars give the same rows
    R = 1 << (256 if curve != "bls12_381" else 256)
    mont = [v * R % C.r for v in vals]
    m_xy, m_inf = e.msm_batch_sparse(tid, ptr, cols, vkzg.ints_to_limbs(mont), mont=True)
    assert np.array_equal(m_xy, got_xy) and np.array_equal(m_inf, got_inf)


@pytest.mark.parametrize("nnz_mod", [0, 1, 255])
def test_batch_commit_sparse_fused_equals_launches(engines, oracle_c, nnz_mod, monkeypatch):
    """The sparse commit's fused count + scan and expand + row offsets (msm.hip
    k_sparse_count_scan / k_sparse_expand_rows: one block per 256 non-zeros, the last block scans
    the block totals) == the separate launches (VKZG_SPARSE_FUSED=0: count, hipcub scan, expand,
    row offsets), bit for bit, on ~40,000 BN254 rows of 0-4 non-zeros whose count is 256 k + nnz_mod
    (the element j = nnz on a block boundary or not), with a sample of rows against the oracle."""
    import vkzg
    from pyoracle.curves import CURVES as OC
    e = engines["bn254"]
    C = OC["bn254"]
    rng = np.random.default_rng(40 + nnz_mod)
    width = 256
    tid = e.random_bases(width, seed=23)
    xy, inf = e.download_bases(tid)
    pts = vkzg.arrays_to_points("bn254", xy, inf)
    lens = list(rng.integers(0, 5, 40_000))
    target = (sum(lens) // 256) * 256 + nnz_mod
    while sum(lens) < target:
        lens.append(1)
    while sum(lens) > target:
        k = int(np.nonzero(lens)[0][-1])
        lens[k] -= 1
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    nnz = int(ptr[-1])
    assert nnz % 256 == nnz_mod
    cols = rng.integers(0, width, nnz).astype(np.uint32)
    vals = [int.from_bytes(rng.bytes(32), "little") % C.r for _ in range(nnz)]
    sc = vkzg.ints_to_limbs(vals)
    monkeypatch.setenv("VKZG_SPARSE_FUSED", "0")
    w_xy, w_inf = e.msm_batch_sparse(tid, ptr, cols, sc)
    monkeypatch.setenv("VKZG_SPARSE_FUSED", "1")
    g_xy, g_inf = e.msm_batch_sparse(tid, ptr, cols, sc)
    assert np.array_equal(g_xy, w_xy) and np.array_equal(g_inf, w_inf)
    for g in list(rng.choice(len(lens), 12, replace=False)) + [len(lens) - 1]:
        lo, hi = int(ptr[g]), int(ptr[g + 1])
        want = oracle_c.msm("bn254", [pts[c] for c in cols[lo:hi]], vals[lo:hi], 4) if hi > lo else None
        got = None if g_inf[g] else vkzg.arrays_to_points("bn254", g_xy[g:g + 1], g_inf[g:g + 1])[0]
        assert got == want, g


@pytest.mark.parametrize("curve", CURVES)
def test_msm_small_on_precomputed_table(engines, oracle_c, curve):
    """vc_msm of <= 1024 host scalars from the start of a table with precomputed fixed-base
    windows takes the fixed-base latency path (capi.cpp vc_msm): == the oracle and == the
    Pippenger pipeline (vc_msm_device) on the same table, for 1, 37 and 256 scalars, a point
    range (offset > 0: Pippenger) and Montgomery-form scalars."""
    import torch
    import vkzg
    e = engines[curve]
    rng = np.random.default_rng(77)
    tid = e.random_bases(300, seed=300)
    xy, inf = e.download_bases(tid)
    e.fixed_base_precompute(tid, 8)
    r = vkzg.SCALAR_R[curve]
    for n in (1, 37, 256):
        sc = vkzg.random_scalars(curve, n, rng)
        want = _oracle(oracle_c, curve, xy, inf, sc)
        got = e.msm(tid, sc)
        assert got[1] == want[1] and (want[1] or np.array_equal(got[0], want[0])), n
        d = torch.from_numpy(sc.view(np.int64).copy()).cuda()
        dev = e.msm_device(tid, d.data_ptr(), n)
        assert dev[1] == got[1] and np.array_equal(dev[0], got[0]), n
        mont = vkzg.ints_to_limbs([(vkzg.limbs_to_int(x) << 256) % r for x in sc])
        gm = e.msm(tid, mont, mont=True)
        assert gm[1] == got[1] and np.array_equal(gm[0], got[0]), n
    sc = vkzg.random_scalars(curve, 40, rng)
    want = _oracle(oracle_c, curve, xy[5:45], inf[5:45], sc)
    got = e.msm(tid, sc, offset=5)
    assert got[1] == want[1] and (want[1] or np.array_equal(got[0], want[0]))
