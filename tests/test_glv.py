"""CPU checks of the GLV split the engine applies to BLS12-381 MSMs (verkle-kzg_amd/csrc/msm.hip:
k_glv_split, k_glv_phi, k_glv_check), through its oracle restatement (oracle/pyoracle/pippenger.py):
the halves recombine to k mod r, stay below 2^127 at every edge of the balancing, the window
slices of the split add up to the whole scalar, and the curve constants do what msm.hip assumes
(phi = [lambda] on the subgroup; the subgroup test rejects points outside it)."""
import random

BETA = 0x1a0111ea397fe699ec02408663d4de85aa0d857d89759ad4897d29650fb85f9b409427eb4f49fffd8bfd00000000aaac
Z2 = 0xd201000000010000 ** 2


def _edge_scalars(r, lam):
    half = lam >> 1
    out = [0, 1, 2, lam - 1, lam, lam + 1, half, half + 1, half + 2, lam + half, lam + half + 1,
           lam * half, lam * (half + 1), lam * (half + 1) + half + 1, lam * lam, lam * lam + half,
           r - 1, r - 2, r - half, r - lam, r, r + 5, (1 << 256) - 1, (1 << 255)]
    rng = random.Random(3)
    out += [rng.randrange(1 << 256) for _ in range(300)]
    return out


def test_glv_split_recombines_and_is_short():
    from pyoracle import pippenger
    from pyoracle.curves import BLS12_381 as C
    lam, r = pippenger.GLV_LAMBDA, C.r
    assert lam * lam + lam + 1 == r
    for k in _edge_scalars(r, lam):
        k1, k2 = pippenger.glv_split(k, r)
        assert (k1 + lam * k2 - k) % r == 0
        assert abs(k1) <= (lam >> 1) + 1 and abs(k2) <= (lam >> 1) + 1
        assert abs(k1) < 1 << 127 and abs(k2) < 1 << 127


def test_glv_window_parts_sum_to_scalar():
    from pyoracle import pippenger
    from pyoracle.curves import BLS12_381 as C
    n = 5000                                            # GLV active
    c, W, _, _ = pippenger.window_slice("bls12_381", n, 0, 1)
    assert (c, W) == (10, 13)
    sc = _edge_scalars(C.r, pippenger.GLV_LAMBDA)
    sc = (sc * (n // len(sc) + 1))[:n]
    for parts in (1, 3, 8):
        tot = [0] * n
        for k in range(parts):
            for i, v in enumerate(pippenger.part_scalars("bls12_381", sc, k, parts, C.r)):
                tot[i] += v
        assert all((t - s) % C.r == 0 for t, s in zip(tot, sc))
    assert pippenger.window_slice("bls12_381", 1 << 20, 0, 1)[:2] == (16, 8)
    # below GLV_MIN_N: 256 digit bits; the size rule's c = 9 leaves a 4-bit top window, so 8 x 32
    assert pippenger.window_slice("bls12_381", 4095, 0, 1)[:2] == (8, 32)


def _mulraw(C, P, k):
    R, Q = None, P
    while k:
        if k & 1:
            R = C.add(R, Q)
        Q = C.add(Q, Q)
        k >>= 1
    return R


def test_glv_curve_constants():
    """phi(P) = (beta x, y) = [lambda] P on the subgroup; the check phi^2(P) + [z^2] P == 0
    (k_glv_check) holds on the subgroup and fails on curve points outside it."""
    from pyoracle import pippenger
    from pyoracle.curves import BLS12_381 as C
    p = C.p
    rng = random.Random(5)
    for _ in range(3):
        P = C.mul(C.g, rng.randrange(1, C.r))
        assert (BETA * P[0] % p, P[1]) == C.mul(P, pippenger.GLV_LAMBDA)
        assert C.add((BETA * BETA * P[0] % p, P[1]), _mulraw(C, P, Z2)) is None
    outside = 0
    while outside < 3:
        x = rng.randrange(p)
        a = (x ** 3 + 4) % p
        y = pow(a, (p + 1) // 4, p)
        if y * y % p != a:
            continue
        P = (x, y)
        assert _mulraw(C, P, C.r) is not None           # not in the r-torsion
        assert C.add((BETA * BETA * x % p, y), _mulraw(C, P, Z2)) is not None
        outside += 1


def test_radix_digits_recombine_and_bound():
    """k_glv_radix / radix_digits (msm.hip): the GLV halves in radix B = 5 * 2^16, 7 signed digits
    |d_w| <= B/2 (bucket |d| - 1 < 5 * 2^15), the top digit never negative and never carrying."""
    from pyoracle import pippenger
    from pyoracle.curves import BLS12_381 as C
    B = pippenger.RADIX_MUL << pippenger.RADIX_C0
    assert B ** 7 // 2 > 1 << 127 and B ** 6 // 2 < 1 << 127
    rng = random.Random(7)
    ks = [0, 1, B // 2, B // 2 + 1, B - 1, B, (1 << 127) - 1, (1 << 126), B ** 6, B ** 6 - 1]
    ks += [rng.randrange(1 << 127) for _ in range(2000)]
    for k in ks:
        d = pippenger.radix_digits(k)
        assert sum(x * B ** w for w, x in enumerate(d)) == k
        assert all(-B // 2 < x <= B // 2 for x in d)
        assert d[-1] >= 0
    # through the GLV split of edge scalars: both halves fit the radix
    for k in _edge_scalars(C.r, pippenger.GLV_LAMBDA):
        k1, k2 = pippenger.glv_split(k, C.r)
        for h in (k1, k2):
            d = pippenger.radix_digits(abs(h))
            assert sum(x * B ** w for w, x in enumerate(d)) == abs(h)


def test_radix_bucket_reduction_identity():
    """the reduction of the 5 * 2^15 radix buckets (segments of Lseg = 5, bit sums over 2^15
    segments, host fold A + 5 sum 2^j T_j) equals sum (b + 1) B_b -- checked over integers at a
    reduced size with the same shape (segments of 5, power-of-two segment count)."""
    from pyoracle import pippenger
    rng = random.Random(11)
    for S in (1, 2, 8, 64):
        for lseg in (1, 4, 5):
            b = [rng.randrange(1 << 64) for _ in range(S * lseg)]
            assert pippenger.radix_bucket_sum(b, lseg) == sum((i + 1) * x for i, x in enumerate(b))
            assert pippenger.radix_bucket_sum_residue(b, lseg) == sum((i + 1) * x for i, x in enumerate(b))


def test_bit_sums_marginal_form():
    """the marginal form of the bit stage (column sums over the low h bits of the segment index,
    row sums over the high J - h bits) gives exactly the bit sums T_j of the bit form, which the
    host fold consumes unchanged -- checked over integers for every split h of J = 2..8."""
    from pyoracle import pippenger
    rng = random.Random(12)
    for J in range(2, 9):
        R = [rng.randrange(1 << 64) for _ in range(1 << J)]
        want = [sum(R[s] for s in range(1 << J) if (s >> j) & 1) for j in range(J)]
        for h in range(1, J):
            assert pippenger.bit_sums_marginal(R, h) == want



def test_bit_sums_marginal_row_total():
    """the row-derived total of the marginal form (TailPlan::urow, Lseg = 1): column sums split
    into pL partial waves give the same T_j, and X (even-hi row sums) + T_h is the total U --
    checked over integers for every split h of J = 2..8 and pL = 1, 2, 4 (where pL divides Hn)."""
    from pyoracle import pippenger
    rng = random.Random(13)
    for J in range(2, 9):
        R = [rng.randrange(1 << 64) for _ in range(1 << J)]
        want = [sum(R[s] for s in range(1 << J) if (s >> j) & 1) for j in range(J)]
        for h in range(1, J):
            for pL in (1, 2, 4):
                if (1 << (J - h)) % pL:
                    continue
                T, U = pippenger.bit_sums_marginal_urow(R, h, pL)
                assert T == want and U == sum(R)


def test_window_choice_top_window_full():
    """vc_msm_windows (host only) for per-window MSMs: the top window is short by at most 2 bits --
    a short top window piles its digits into a few buckets (BN254 at the old c = 11: 2 of 1,024,
    every call then redid its fix-up) -- and the oracle's window_slice follows the same rule."""
    from pyoracle import pippenger
    from vkzg import dist
    for curve in ("bn254", "bls12_381", "bandersnatch"):
        total = pippenger.SCALAR_BITS[curve] + 1
        for lg in range(1, 22):
            for n in (1 << lg, (1 << lg) + (1 << lg) // 2):
                c, W, terms = dist.window_count(curve, n, with_terms=True)
                if terms != 1:
                    continue
                assert (c, W) == pippenger.window_slice(curve, n, 0, 1)[:2]
                assert c - (total - c * (W - 1)) <= 2, (curve, n, c, W)
