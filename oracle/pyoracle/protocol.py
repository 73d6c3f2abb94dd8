"""ORACLE (test infrastructure only) -- the reference's vector-commitment protocol restated in Python.

Each function cites the reference (paths relative to /root/reference) it follows. Quirks of
SURVEY.md Appendix B are reproduced as-is. Group results are canonical affine tuples.

Pinned by: algebraic KATs (curves.py), the reference's own round-trip/tamper tests restated
in tests/ (ipa/mod.rs:382-421, kzg/mod.rs:278-297, multiproof.rs:261-357), and trapdoor
checks for KZG (s = 100 is public, kzg_point_generator.rs:23) in place of pairings.
Transcript / CRS byte conventions are "parity unpinned vs arkworks" (see arkser.py).
"""
import hashlib

from . import arkser
from .curves import BN254, BLS12_381

# multiplicative generators of the scalar fields (arkworks #[generator]); 2-adicity
FR_GEN = {"bn254": (5, 28), "bls12_381": (7, 32)}


# ---------------------------------------------------------------- utils.rs
def inner_product_f(a, b, r):
    """utils.rs:16-19 with T = F: zip-truncating field dot product."""
    return sum(x * y for x, y in zip(a, b)) % r


def vec_add_and_distribute_f(a, b, x, r):
    """utils.rs:31-38: res_i = a_i + x*b_i (scalars)."""
    assert len(a) == len(b)
    return [(ai + x * bi) % r for ai, bi in zip(a, b)]


def vec_add_and_distribute_g(curve, a, b, x):
    """utils.rs:31-38 on points: res_i = a_i + b_i * x."""
    assert len(a) == len(b)
    return [curve.add(ai, curve.mul(bi, x)) for ai, bi in zip(a, b)]


def split(a):
    """utils.rs:40-42."""
    return a[: len(a) // 2], a[len(a) // 2:]


def powers_of(a, n, r):
    """utils.rs:44-55."""
    res, cur = [], 1
    for _ in range(n):
        res.append(cur)
        cur = cur * a % r
    return res


def invert_domain_at(t, n, r):
    """utils.rs:57-62: 1/(t - i) for INTEGER i in 0..n."""
    return [pow((t - i) % r, -1, r) for i in range(n)]


def to_usize(x):
    """utils.rs:72-74: low 64-bit limb of the canonical integer."""
    return int(x) & ((1 << 64) - 1)


# ---------------------------------------------------------------- domain / precompute.rs
def domain_size(n):
    s = 1
    while s < n:
        s <<= 1
    return s


def group_gen(size, curve=BN254):
    g, adic = FR_GEN[curve.name]
    assert size & (size - 1) == 0 and size <= (1 << adic)
    return pow(g, (curve.r - 1) // size, curve.r)


class PrecomputedLagrange:
    """precompute.rs:12-90."""

    def __init__(self, size, curve=BN254):
        self.curve = curve
        r = curve.r
        self.size = size
        self.dsize = domain_size(size)
        self.omega = group_gen(self.dsize, curve)
        # compute_vanishing_evaluations(size, group_gen) precompute.rs:47-58
        self.vanishing = [size * pow(pow(self.omega, i, r), -1, r) % r for i in range(size)]
        self.vanishing_inv = [pow(v, -1, r) for v in self.vanishing]

    def element(self, i):
        return pow(self.omega, i, self.curve.r)

    def compute_barycentric_coefficients(self, point):
        """precompute.rs:72-90; `point < size` compares canonical integers."""
        r = self.curve.r
        point %= r
        res = [0] * self.size
        if point < self.size:
            res[to_usize(point)] = 1
            return res
        t = (pow(point, self.size, r) - 1) * pow(self.size, -1, r) % r
        for i in range(self.size):
            pw = pow(self.omega, i, r)
            res[i] = t * pw % r * pow((point - pw) % r, -1, r) % r
        return res


# ---------------------------------------------------------------- lagrange_basis.rs
class LagrangeBasis:
    """lagrange_basis.rs:15-178. `evals` may be shorter than the domain (max = len)."""

    def __init__(self, evals, dsize, curve=BN254):
        self.curve = curve
        self.evals = [int(e) % curve.r for e in evals]
        self.max_ = len(evals)
        self.dsize = dsize
        self.omega = group_gen(dsize, curve)

    @classmethod
    def from_vec(cls, data, curve=BN254):
        return cls(data, domain_size(len(data)), curve)

    def max(self):
        return self.max_ - 1

    def __getitem__(self, i):
        return self.evals[i]

    def index_to_point(self, i):
        return pow(self.omega, i, self.curve.r)

    def evaluate(self, pre, point):
        """:63-72 three paths."""
        point %= self.curve.r
        if point <= self.max():
            return self.evals[to_usize(point)]
        elif point <= self.dsize:
            return 0
        return self.evaluate_outside_domain(pre, point)

    def evaluate_outside_domain(self, pre, point):
        return inner_product_f(self.evals, pre.compute_barycentric_coefficients(point), self.curve.r)

    def _eval_at(self, i):
        return 0 if i >= self.max_ else self.evals[i]

    def divide_by_vanishing(self, pre, index):
        """:91-119 in-domain quotient at w^index (two field divisions per i)."""
        r = self.curve.r
        n = self.dsize
        q = [0] * n
        index_f = self.index_to_point(index)
        ev = 0 if index >= self.max_ else self.evals[index]
        index_van = pre.vanishing[index]
        for i in range(n):
            if i == index:
                continue
            i_f = self.index_to_point(i)
            sub = (self._eval_at(i) - ev) % r
            q[i] = sub * pow((i_f - index_f) % r, -1, r) % r
            q[index] = (q[index] + sub * index_van % r * pre.vanishing_inv[i] % r
                        * pow((index_f - i_f) % r, -1, r)) % r
        return q

    def divide_by_vanishing_outside_domain(self, pre, point):
        """:121-142 (`divive_by_vanishing_outside_domain`)."""
        r = self.curve.r
        n = self.dsize
        ev = self.evaluate(pre, point)
        invs = [pow((self.index_to_point(i) - point) % r, -1, r) for i in range(n)]
        return [(self._eval_at(i) - ev) * invs[i] % r for i in range(n)]


# ---------------------------------------------------------------- IPA CRS (ipa_point_generator.rs)
def ipa_gen_points(num, seed=b"eth_verkle_oct_2021", max_=256, curve=BN254):
    """IPAPointGenerator::gen (:51-67) with EthereumHashToCurve (:96-108)."""
    if num > max_:
        raise ValueError("OutOfBounds")
    res, i = [], 0
    while len(res) < num:
        b = hashlib.sha256(seed + i.to_bytes(8, "little")).digest()
        P = arkser.from_random_bytes(b, curve)
        if P != "reject":
            res.append(P)
        i += 1
    return res


# ---------------------------------------------------------------- IPA (ipa/mod.rs)
class IPA:
    """IPA<N, G, H, D> over `curve`; key = (g[0..N], q, precompute)."""

    def __init__(self, N, curve=BN254, gen_max=512, points=None):
        self.N = N
        self.curve = curve
        pts = points if points is not None else ipa_gen_points(N + 1, max_=gen_max, curve=curve)
        self.g = pts[:N]          # new_from_vec (:40-51)
        self.q = pts[N]
        self.pre = PrecomputedLagrange(N, curve)

    def commit(self, data):
        """:130-135."""
        return self.curve.msm(self.g, data.evals)

    def prove_point(self, commitment, point, data, transcript=None):
        """:137-154."""
        b = self.pre.compute_barycentric_coefficients(point)
        return low_level_ipa(self.curve, self.g, self.q, data.evals, b, commitment, point, transcript)

    def prove(self, commitment, index, data):
        return self.prove_point(commitment, index, data, None)

    def verify_point(self, commitment, point, proof, transcript=None):
        """:165-181."""
        b = self.pre.compute_barycentric_coefficients(point)
        return low_level_verify_ipa(self.curve, self.g, self.q, b, commitment, point, proof, transcript)

    def verify(self, commitment, index, proof):
        return self.verify_point(commitment, index, proof, None)

    def prove_commitment(self, commitment, data):
        """:199-234."""
        C, r = self.curve, self.curve.r
        mx = data.max()
        a = data.evals[0:mx + 1]
        gens = self.g[0:mx + 1]
        L, R = [], []
        tr = arkser.TranscriptHasher("ipa", C)
        tr.append_point(commitment, "C")
        tr.digest("x", True)
        while len(a) > 1:
            al, ar = split(a)
            gl, gr = split(gens)
            yl = C.msm(gr, al)
            yr = C.msm(gl, ar)
            L.append(yl)
            R.append(yr)
            tr.append_point(yl, "L")
            tr.append_point(yr, "R")
            x = tr.digest("x", True)
            a = vec_add_and_distribute_f(al, ar, x, r)
            gens = vec_add_and_distribute_g(C, gr, gl, x)
        return {"l": L, "r": R, "tip": a[0]}

    def verify_commitment_proof(self, commitment, proof):
        """:237-265."""
        C, r = self.curve, self.curve.r
        gens = self.g[0:2 ** len(proof["l"])]
        c = commitment
        coeffs = [1]
        tr = arkser.TranscriptHasher("ipa", C)
        tr.append_point(commitment, "C")
        tr.digest("x", True)
        for i in range(len(proof["l"])):
            tr.append_point(proof["l"][i], "L")
            tr.append_point(proof["r"][i], "R")
            x = tr.digest("x", True)
            c = C.add(C.add(proof["l"][i], C.mul(c, x)), C.mul(proof["r"][i], x * x % r))
            coeffs = [v for y in coeffs for v in (y * x % r, y)]
        combined = C.msm(gens, coeffs)
        return c == C.mul(combined, proof["tip"])


def low_level_ipa(C, gens, q, a, b, commitment, input_point, transcript=None):
    """ipa/mod.rs:268-319."""
    r = C.r
    ev = inner_product_f(a, b, r)
    gens = gens[0:len(a)]
    data = list(a)
    other = list(b)
    tr = transcript if transcript is not None else arkser.TranscriptHasher("ipa", C)
    tr.append_point(commitment, "C")
    tr.append_fr(input_point, "input point")
    tr.append_fr(ev, "output point")
    L, R = [], []
    w = tr.digest("w", True)
    qp = C.mul(q, w)
    while len(data) > 1:
        dl, dr = split(data)
        gl, gr = split(gens)
        bl, br = split(other)
        yl = C.add(C.msm(gr, dl), C.mul(qp, inner_product_f(dl, br, r)))
        yr = C.add(C.msm(gl, dr), C.mul(qp, inner_product_f(dr, bl, r)))
        L.append(yl)
        R.append(yr)
        tr.append_point(yl, "L")
        tr.append_point(yr, "R")
        x = tr.digest("x", True)
        data = vec_add_and_distribute_f(dl, dr, x, r)
        gens = vec_add_and_distribute_g(C, gr, gl, x)
        other = vec_add_and_distribute_f(br, bl, x, r)
    return {"l": L, "r": R, "tip": data[0], "y": ev}


def low_level_verify_ipa(C, gens, q, b, commitment, input_point, proof, transcript=None):
    """ipa/mod.rs:321-360."""
    r = C.r
    c = commitment
    tr = transcript if transcript is not None else arkser.TranscriptHasher("ipa", C)
    tr.append_point(commitment, "C")
    tr.append_fr(input_point, "input point")
    tr.append_fr(proof["y"], "output point")
    w = tr.digest("w", True)
    coeffs = [1]
    qp = C.mul(q, w)
    c = C.add(c, C.mul(qp, proof["y"]))
    for i in range(len(proof["l"])):
        tr.append_point(proof["l"][i], "L")
        tr.append_point(proof["r"][i], "R")
        x = tr.digest("x", True)
        c = C.add(C.add(proof["l"][i], C.mul(c, x)), C.mul(proof["r"][i], x * x % r))
        coeffs = [v for y in coeffs for v in (y * x % r, y)]
    combined_point = C.msm(gens, coeffs)
    combined_b = inner_product_f(b, coeffs, r)
    rhs = C.add(C.mul(combined_point, proof["tip"]), C.mul(qp, proof["tip"] * combined_b % r))
    return c == rhs


# ---------------------------------------------------------------- KZG (kzg/mod.rs)
def kzg_lagrange_scalars(max_items, secret=100, curve=BN254):
    """KZG::setup (:115-124) = gen (s^i G, kzg_point_generator.rs:32-43) then zero-padded G1 iFFT:
    L_j = c_j G with c_j = n^{-1} sum_{i<m} s^i w^{-ij}  (SURVEY Appendix A.7)."""
    r = curve.r
    n = domain_size(max_items)
    w = group_gen(n, curve)
    winv = pow(w, -1, r)
    ninv = pow(n, -1, r)
    spow = powers_of(secret, max_items, r)
    out = []
    for j in range(n):
        wj = pow(winv, j, r)
        acc, cur = 0, 1
        for i in range(max_items):
            acc += spow[i] * cur
            cur = cur * wj % r
        out.append(acc % r * ninv % r)
    return out


class KZG:
    """KZG<E, H, D>; verification by the trapdoor identity pi*(s - p) == C - y*G (s public)."""

    def __init__(self, max_items, curve=BN254, secret=100):
        self.curve = curve
        self.secret = secret
        cs = kzg_lagrange_scalars(max_items, secret, curve)
        self.lagrange_scalars = cs
        self.lagrange = [curve.mul(curve.g, c) for c in cs]
        self.size = len(self.lagrange)
        self.pre = PrecomputedLagrange(self.size, curve)

    def max_size(self):
        return self.size

    def commit(self, data):
        """:126-134."""
        return self.curve.msm(self.lagrange, data.evals)

    def quotient(self, point, data):
        """the q of prove_point (:136-154), returned with the evaluation y."""
        point %= self.curve.r
        y = data.evaluate(self.pre, point)
        if point <= self.max_size():
            if to_usize(point) >= self.size:
                raise IndexError("vanishing_at out of bounds (reference panics, Appendix B.4)")
            q = data.divide_by_vanishing(self.pre, to_usize(point))
        else:
            q = data.divide_by_vanishing_outside_domain(self.pre, point)
        return q, y

    def prove_point(self, commitment, point, data, transcript=None):
        q, y = self.quotient(point, data)
        return {"proof": self.curve.msm(self.lagrange, q), "y": y}

    def prove(self, commitment, index, data):
        return self.prove_point(commitment, index, data)

    def eval_point(self, point):
        """verify_point's p (:172-179): w^point in domain (strict <) else point."""
        point %= self.curve.r
        if point < self.max_size():
            return pow(self.pre.omega, to_usize(point), self.curve.r)
        return point

    def verify_point(self, commitment, point, proof, transcript=None):
        """:165-189 pairing check e(pi, [s-p]_2) == e(C - yG, H) <=> pi*(s-p) == C - y*G."""
        C = self.curve
        p = self.eval_point(point)
        lhs = C.mul(proof["proof"], (self.secret - p) % C.r)
        rhs = C.add(commitment, C.neg(C.mul(C.g, proof["y"])))
        return lhs == rhs

    def verify(self, commitment, index, proof):
        return self.verify_point(commitment, index, proof)


def ark_fft(vals, n, r, omega, inverse=False):
    """ark-poly Radix2EvaluationDomain fft / ifft of size n (fft_in_place first resizes the input
    to n: truncates or zero-pads). O(n^2): small n only."""
    a = (list(vals) + [0] * n)[:n]
    w = pow(omega, -1, r) if inverse else omega
    out = [sum(a[j] * pow(w, i * j, r) for j in range(n)) % r for i in range(n)]
    if inverse:
        ninv = pow(n, -1, r)
        out = [x * ninv % r for x in out]
    return out


class ReferencePanic(Exception):
    """where the reference panics (index out of bounds)"""


def kzg_prove_all_points(kzg, data):
    """KZG::prove_all_points (kzg/mod.rs:200-235) restated. Every point involved is a known multiple
    of G (the SRS points are c_j G, kzg_lagrange_scalars), and the FFTs over G1 are linear, so the
    computation runs on those scalars and each output is (scalar) G -- the same group elements.
    Returns [(h_hat_i, data[i])]."""
    C = kzg.curve
    r = C.r
    evals = list(data.evals)
    m = domain_size(len(evals))                        # LagrangeBasis::from_vec's domain
    coeffs = ark_fft(evals, m, r, group_gen(m, C), inverse=True)   # interpolate (:204)
    while coeffs and coeffs[-1] == 0:                  # DensePolynomial trims trailing zeros
        coeffs.pop()
    if not coeffs:
        raise ReferencePanic("coeffs[degree] of the zero polynomial")
    d = len(coeffs) - 1                                # poly.degree()
    D = domain_size(2 * d)                             # D::new(degree * 2)
    chat = [coeffs[d]] + [0] * (d + 1) + coeffs[:d]
    g1 = ark_fft(kzg.lagrange_scalars, kzg.size, r, kzg.pre.omega, inverse=True)
    if d > len(g1):
        raise ReferencePanic("g1[0..degree] out of bounds")
    shat = list(reversed(g1[:d])) + [0] * (D - d)
    y = ark_fft(chat, D, r, group_gen(D, C))
    v = ark_fft(shat, D, r, group_gen(D, C))
    u = [a * b % r for a, b in zip(v, y)]
    h = ark_fft(u, D, r, group_gen(D, C), inverse=True)
    if D > len(evals):
        raise ReferencePanic("data[i] out of bounds")
    return [(C.mul(C.g, hi), evals[i]) for i, hi in enumerate(h)]


# ---------------------------------------------------------------- multiproof.rs
def prove_multiproof(vc, queries):
    """multiproof.rs:99-176. queries: list of (data: LagrangeBasis, commit, z:int, y:int)."""
    C = vc.curve
    r = C.r
    n = vc.max_size() if isinstance(vc, KZG) else vc.N
    tr = arkser.TranscriptHasher("multiproof", C)
    for data, com, z, y in queries:
        tr.append_point(com, "C")
        tr.append_usize(z, "z")
        tr.append_fr(y, "y")
    rr = tr.digest("r", True)
    rp = powers_of(rr, len(queries), r)
    scaled = [(q[2], [e * rp[i] % r for e in q[0].evals]) for i, q in enumerate(queries)]
    groups = {}
    for z, ev in scaled:
        groups.setdefault(z, []).append(ev)
    g = [0] * n
    for z, lst in groups.items():
        total = [0] * n
        for ev in lst:
            for k in range(len(ev)):
                total[k] = (total[k] + ev[k]) % r
        lb = LagrangeBasis(total, domain_size(n), C)
        quo = lb.divide_by_vanishing(vc.pre, z)
        for k in range(n):
            g[k] = (g[k] + quo[k]) % r
    gb = LagrangeBasis(g, domain_size(n), C)
    d = vc.commit(gb)
    tr.append_point(d, "D")
    t = tr.digest("t", True)
    invs = invert_domain_at(t, n, r)
    h = [0] * n
    for z, lst in groups.items():
        for ev in lst:
            for k in range(len(ev)):
                h[k] = (h[k] + ev[k] * invs[z]) % r
    e = vc.commit(LagrangeBasis(h, domain_size(n), C))
    tr.append_point(e, "E")
    hmg = LagrangeBasis([(a - b) % r for a, b in zip(h, g)], domain_size(n), C)
    mcom = C.add(e, C.neg(d))
    proof = vc.prove_point(mcom, t, hmg, tr)
    return {"proof": proof, "d": d}


def verify_multiproof(vc, vqueries, mp):
    """multiproof.rs:178-215. vqueries: list of (commit, z, y)."""
    C = vc.curve
    r = C.r
    n = vc.max_size() if isinstance(vc, KZG) else vc.N
    tr = arkser.TranscriptHasher("multiproof", C)
    for com, z, y in vqueries:
        tr.append_point(com, "C")
        tr.append_usize(z, "z")
        tr.append_fr(y, "y")
    rr = tr.digest("r", True)
    tr.append_point(mp["d"], "D")
    t = tr.digest("t", True)
    invs = invert_domain_at(t, n, r)
    coeffs = {}
    order = []
    rpow = 1
    for com, z, y in vqueries:
        ec = rpow * invs[z] % r
        if com not in coeffs:
            coeffs[com] = 0
            order.append(com)
        coeffs[com] = (coeffs[com] + ec) % r
        rpow = rpow * rr % r
    e = C.msm(order, [coeffs[c] for c in order])
    tr.append_point(e, "E")
    return vc.verify_point(C.add(e, C.neg(mp["d"])), t, mp["proof"], tr)
