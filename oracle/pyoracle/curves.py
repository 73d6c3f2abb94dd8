"""ORACLE (test infrastructure only) -- prime fields and curve groups in pure Python big ints.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
It is never the measured or shipped path.

Restates the arkworks 0.4 group law the reference calls through
`utils::inner_product` (vector-commit/src/utils.rs:16-19): `Projective * Fr` is a
double-and-add over the bits of the canonical scalar (arkworks `mul_bigint`,
MSB first, leading zeros skipped) and `Sum` is a sequential fold from zero.
Group elements are unique, so results are compared as canonical affine
coordinates.

Curves:
  * BN254 G1 (short Weierstrass y^2 = x^3 + 3) -- the only curve the reference
    instantiates (vector-commit/Cargo.toml:15, ipa/mod.rs:367).
  * BLS12-381 G1 (y^2 = x^3 + 4) -- north_star curve for KZG (configs 2, 4).
  * Bandersnatch (twisted Edwards a=-5 over BLS12-381 Fr) -- north_star curve
    for IPA/verkle commits (config 3).
Parity for BLS12-381 / Bandersnatch is pinned only by the curve KATs below
(generator on curve, r*G = O); the reference never runs them.
"""

# ---------------------------------------------------------------- constants
BN254_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
BN254_R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

BLS_P = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 16)
BLS_R = int("73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001", 16)
BLS_GX = int("17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb", 16)
BLS_GY = int("08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1", 16)

# Bandersnatch (ark-ed-on-bls12-381-bandersnatch 0.4): base field = BLS12-381 Fr
BAND_Q = BLS_R
BAND_A = BAND_Q - 5
BAND_D = 45022363124591815672509500913686876175488063829319466900776701791074614335719
BAND_R = 13108968793781547619861935127046491459309155893440570251786403306729687672801
BAND_GX = 18886178867200960497001835917649091219057080094937609519140440539760939937304
BAND_GY = 19188667384257783945677642223292697773471335439753913231509108946878080696678


def inv(x, p):
    return pow(x, -1, p)


def sqrt_mod(a, p):
    """Tonelli-Shanks; returns one root or None."""
    a %= p
    if a == 0:
        return 0
    if pow(a, (p - 1) // 2, p) != 1:
        return None
    if p % 4 == 3:
        return pow(a, (p + 1) // 4, p)
    q, s = p - 1, 0
    while q % 2 == 0:
        q //= 2
        s += 1
    z = 2
    while pow(z, (p - 1) // 2, p) != p - 1:
        z += 1
    m, c, t, r = s, pow(z, q, p), pow(a, q, p), pow(a, (q + 1) // 2, p)
    while t != 1:
        i, tt = 0, t
        while tt != 1:
            tt = tt * tt % p
            i += 1
        b = pow(c, 1 << (m - i - 1), p)
        m, c, t, r = i, b * b % p, t * b * b % p, r * b % p
    return r


# ---------------------------------------------------------------- SW a=0
class SWCurve:
    """y^2 = x^3 + b over F_p, a = 0. Affine points are (x, y) tuples, identity None."""

    kind = "sw"

    def __init__(self, name, p, r, b, gx, gy, fbytes):
        self.name, self.p, self.r, self.b = name, p, r, b
        self.g = (gx, gy)
        self.fbytes = fbytes  # bytes per base-field element in the ABI layout

    def identity(self):
        return None

    def is_on_curve(self, P):
        if P is None:
            return True
        x, y = P
        return (y * y - x * x * x - self.b) % self.p == 0

    def neg(self, P):
        if P is None:
            return None
        return (P[0], (-P[1]) % self.p)

    # Jacobian internals (X, Y, Z), identity Z == 0
    def _to_jac(self, P):
        return (0, 1, 0) if P is None else (P[0], P[1], 1)

    def _to_aff(self, J):
        X, Y, Z = J
        if Z == 0:
            return None
        p = self.p
        zi = inv(Z, p)
        zi2 = zi * zi % p
        return (X * zi2 % p, Y * zi2 * zi % p)

    def _jdbl(self, J):
        X, Y, Z = J
        p = self.p
        if Z == 0 or Y == 0:
            return (0, 1, 0)
        A = X * X % p
        B = Y * Y % p
        C = B * B % p
        D = 2 * ((X + B) ** 2 - A - C) % p
        E = 3 * A % p
        F = E * E % p
        X3 = (F - 2 * D) % p
        Y3 = (E * (D - X3) - 8 * C) % p
        Z3 = 2 * Y * Z % p
        return (X3, Y3, Z3)

    def _jadd(self, J1, J2):
        X1, Y1, Z1 = J1
        X2, Y2, Z2 = J2
        p = self.p
        if Z1 == 0:
            return J2
        if Z2 == 0:
            return J1
        Z1Z1 = Z1 * Z1 % p
        Z2Z2 = Z2 * Z2 % p
        U1 = X1 * Z2Z2 % p
        U2 = X2 * Z1Z1 % p
        S1 = Y1 * Z2 * Z2Z2 % p
        S2 = Y2 * Z1 * Z1Z1 % p
        if U1 == U2:
            if S1 == S2:
                return self._jdbl(J1)
            return (0, 1, 0)
        H = (U2 - U1) % p
        I = (2 * H) ** 2 % p
        Jv = H * I % p
        rr = 2 * (S2 - S1) % p
        V = U1 * I % p
        X3 = (rr * rr - Jv - 2 * V) % p
        Y3 = (rr * (V - X3) - 2 * S1 * Jv) % p
        Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % p
        return (X3, Y3, Z3)

    def add(self, P, Q):
        return self._to_aff(self._jadd(self._to_jac(P), self._to_jac(Q)))

    def double(self, P):
        return self._to_aff(self._jdbl(self._to_jac(P)))

    def mul(self, P, k):
        """arkworks mul_bigint: MSB-first double-and-add over canonical bits of k."""
        k %= self.r
        acc = (0, 1, 0)
        Pj = self._to_jac(P)
        for bit in bin(k)[2:] if k else "":
            acc = self._jdbl(acc)
            if bit == "1":
                acc = self._jadd(acc, Pj)
        return self._to_aff(acc)

    def msm(self, points, scalars):
        """utils::inner_product (utils.rs:16-19): zip (truncating) -> map(P*s) -> sum."""
        acc = (0, 1, 0)
        for P, s in zip(points, scalars):
            acc = self._jadd(acc, self._to_jac(self.mul(P, s)))
        return self._to_aff(acc)

    def msm_fast(self, points, scalars, c=8):
        """Same mathematical value as msm(); bucket method, for big fixture generation only."""
        nb = (self.r.bit_length() + c - 1) // c
        total = (0, 1, 0)
        jpts = [self._to_jac(P) for P in points]
        for w in reversed(range(nb)):
            for _ in range(c):
                total = self._jdbl(total)
            buckets = [(0, 1, 0)] * (1 << c)
            for P, s in zip(jpts, scalars):
                d = ((s % self.r) >> (w * c)) & ((1 << c) - 1)
                if d:
                    buckets[d] = self._jadd(buckets[d], P)
            run = (0, 1, 0)
            acc = (0, 1, 0)
            for d in range((1 << c) - 1, 0, -1):
                run = self._jadd(run, buckets[d])
                acc = self._jadd(acc, run)
            total = self._jadd(total, acc)
        return self._to_aff(total)


# ---------------------------------------------------------------- twisted Edwards
class TECurve:
    """a*x^2 + y^2 = 1 + d*x^2*y^2 over F_q. Affine points (x, y); identity (0, 1)."""

    kind = "te"

    def __init__(self, name, p, r, a, d, gx, gy, fbytes):
        self.name, self.p, self.r, self.a, self.d = name, p, r, a, d
        self.g = (gx, gy)
        self.fbytes = fbytes

    def identity(self):
        return (0, 1)

    def is_on_curve(self, P):
        x, y = P
        p = self.p
        return (self.a * x * x + y * y - 1 - self.d * x * x * y * y) % p == 0

    def neg(self, P):
        return ((-P[0]) % self.p, P[1])

    def add(self, P, Q):
        p = self.p
        x1, y1 = P
        x2, y2 = Q
        t = self.d * x1 * x2 * y1 * y2 % p
        x3 = (x1 * y2 + y1 * x2) * inv((1 + t) % p, p) % p
        y3 = (y1 * y2 - self.a * x1 * x2) * inv((1 - t) % p, p) % p
        return (x3, y3)

    def double(self, P):
        return self.add(P, P)

    # extended coords (X, Y, T, Z)
    def _ext(self, P):
        return (P[0], P[1], P[0] * P[1] % self.p, 1)

    def _eadd(self, A, B):
        p = self.p
        X1, Y1, T1, Z1 = A
        X2, Y2, T2, Z2 = B
        a_ = X1 * X2 % p
        b_ = Y1 * Y2 % p
        c_ = self.d * T1 % p * T2 % p
        d_ = Z1 * Z2 % p
        e_ = ((X1 + Y1) * (X2 + Y2) - a_ - b_) % p
        f_ = (d_ - c_) % p
        g_ = (d_ + c_) % p
        h_ = (b_ - self.a * a_) % p
        return (e_ * f_ % p, g_ * h_ % p, e_ * h_ % p, f_ * g_ % p)

    def _aff(self, E):
        X, Y, T, Z = E
        zi = inv(Z, self.p)
        return (X * zi % self.p, Y * zi % self.p)

    def mul(self, P, k):
        k %= self.r
        acc = (0, 1, 0, 1)
        Pe = self._ext(P)
        for bit in bin(k)[2:] if k else "":
            acc = self._eadd(acc, acc)
            if bit == "1":
                acc = self._eadd(acc, Pe)
        return self._aff(acc)

    def msm(self, points, scalars):
        acc = (0, 1, 0, 1)
        for P, s in zip(points, scalars):
            acc = self._eadd(acc, self._ext(self.mul(P, s)))
        return self._aff(acc)

    def msm_fast(self, points, scalars, c=8):
        nb = (self.r.bit_length() + c - 1) // c
        total = (0, 1, 0, 1)
        epts = [self._ext(P) for P in points]
        for w in reversed(range(nb)):
            for _ in range(c):
                total = self._eadd(total, total)
            buckets = [(0, 1, 0, 1)] * (1 << c)
            for P, s in zip(epts, scalars):
                d = ((s % self.r) >> (w * c)) & ((1 << c) - 1)
                if d:
                    buckets[d] = self._eadd(buckets[d], P)
            run = (0, 1, 0, 1)
            acc = (0, 1, 0, 1)
            for d in range((1 << c) - 1, 0, -1):
                run = self._eadd(run, buckets[d])
                acc = self._eadd(acc, run)
            total = self._eadd(total, acc)
        return self._aff(total)


BN254 = SWCurve("bn254", BN254_P, BN254_R, 3, 1, 2, 32)
BLS12_381 = SWCurve("bls12_381", BLS_P, BLS_R, 4, BLS_GX, BLS_GY, 48)
BANDERSNATCH = TECurve("bandersnatch", BAND_Q, BAND_R, BAND_A, BAND_D, BAND_GX, BAND_GY, 32)

CURVES = {c.name: c for c in (BN254, BLS12_381, BANDERSNATCH)}


def random_points(curve, n, rng):
    """n random subgroup points k_i * G (k_i from rng), via one running sum to keep it cheap."""
    step = curve.mul(curve.g, rng.randrange(1, curve.r))
    pts = []
    P = curve.mul(curve.g, rng.randrange(1, curve.r))
    for _ in range(n):
        pts.append(P)
        P = curve.add(P, step)
    return pts
