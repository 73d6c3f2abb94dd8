// Elliptic-curve group law for the MSM engine (host + gfx950 device).
//
//  * SWCurve<Fq>: short Weierstrass y^2 = x^3 + b (a = 0): BN254 G1, BLS12-381 G1.
//    Accumulators are XYZZ (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): mixed add 8M+2S,
//    add 12M+2S, dbl 6M+3S; no inversion, exceptional cases (P == +-Q) handled.
//    Bases are affine (x, y) in Montgomery form; the identity base is skipped by the
//    digit pass (flag), never stored.
//  * TECurve<Fq>: twisted Edwards a*x^2 + y^2 = 1 + d*x^2*y^2 with a = -5 (Bandersnatch).
//    Accumulators are extended (X, Y, T, Z); bases are (x, y, d*x*y) so the unified
//    mixed add is 8M. The formulas are complete: no exceptional branches.
#pragma once
#include "ff.hpp"

namespace vk {

template <class F, bool IL>
VK_HD fe<F> fsqr(const fe<F>& a) {
    return fmul<F, IL>(a, a);
}

template <class F>
struct SWAff {
    fe<F> x, y;
};
template <class F>
struct SWAcc {
    fe<F> x, y, zz, zzz;
};
template <class F>
struct TEAff {
    fe<F> x, y, kt;  // kt = d*x*y
};
template <class F>
struct TEAcc {
    fe<F> X, Y, T, Z;
};

// ================================================================ short Weierstrass, a = 0
// IL = inline field multiplies (latency-bound kernels); same point types either way.
template <class Fq_, int B_, bool IL = false>
struct SWCurve {
    using F = Fq_;
    static constexpr bool is_te = false;
    static constexpr int COEFF_B = B_;
    using Aff = SWAff<F>;
    using Acc = SWAcc<F>;
    using Inl = SWCurve<Fq_, B_, true>;
    static constexpr int AFF_WORDS = 2 * F::N;
    static constexpr int ACC_WORDS = 4 * F::N;

    VK_HD static Acc zero() {
        Acc r;
        r.x = fe_one<F>();
        r.y = fe_one<F>();
        r.zz = fe_zero<F>();
        r.zzz = fe_zero<F>();
        return r;
    }
    VK_HD static bool is_zero(const Acc& a) { return fe_is_zero<F>(a.zz); }
    VK_HD static Acc from_aff(const Aff& p, bool neg) {
        Acc r;
        r.x = p.x;
        r.y = neg ? fe_neg<F>(p.y) : p.y;
        r.zz = fe_one<F>();
        r.zzz = fe_one<F>();
        return r;
    }
    // dbl-2008-s-1
    VK_HD static Acc dbl(const Acc& p) {
        if (is_zero(p)) return p;
        fe<F> U = fe_dbl<F>(p.y);
        fe<F> V = fsqr<F, IL>(U);
        fe<F> W = fmul<F, IL>(U, V);
        fe<F> S = fmul<F, IL>(p.x, V);
        fe<F> X2 = fsqr<F, IL>(p.x);
        fe<F> M = fe_add<F>(fe_dbl<F>(X2), X2);
        Acc r;
        r.x = fe_sub<F>(fsqr<F, IL>(M), fe_dbl<F>(S));
        r.y = fe_sub<F>(fmul<F, IL>(M, fe_sub<F>(S, r.x)), fmul<F, IL>(W, p.y));
        r.zz = fmul<F, IL>(V, p.zz);
        r.zzz = fmul<F, IL>(W, p.zzz);
        return r;
    }
    // doubling of an affine point (used in the madd exceptional case)
    VK_HD static Acc dbl_aff(const fe<F>& x, const fe<F>& y) {
        fe<F> U = fe_dbl<F>(y);
        fe<F> V = fsqr<F, IL>(U);
        fe<F> W = fmul<F, IL>(U, V);
        fe<F> S = fmul<F, IL>(x, V);
        fe<F> X2 = fsqr<F, IL>(x);
        fe<F> M = fe_add<F>(fe_dbl<F>(X2), X2);
        Acc r;
        r.x = fe_sub<F>(fsqr<F, IL>(M), fe_dbl<F>(S));
        r.y = fe_sub<F>(fmul<F, IL>(M, fe_sub<F>(S, r.x)), fmul<F, IL>(W, y));
        r.zz = V;
        r.zzz = W;
        return r;
    }
    // madd-2008-s: acc + (x2, +-y2)
    VK_HD static Acc madd(const Acc& p, const Aff& q, bool neg) {
        fe<F> y2 = neg ? fe_neg<F>(q.y) : q.y;
        if (is_zero(p)) {
            Acc r;
            r.x = q.x;
            r.y = y2;
            r.zz = fe_one<F>();
            r.zzz = fe_one<F>();
            return r;
        }
        fe<F> U2 = fmul<F, IL>(q.x, p.zz);
        fe<F> S2 = fmul<F, IL>(y2, p.zzz);
        fe<F> P = fe_sub<F>(U2, p.x);
        fe<F> R = fe_sub<F>(S2, p.y);
        if (fe_is_zero<F>(P)) {
            if (fe_is_zero<F>(R)) return dbl_aff(q.x, y2);
            return zero();
        }
        fe<F> PP = fsqr<F, IL>(P);
        fe<F> PPP = fmul<F, IL>(P, PP);
        fe<F> Q = fmul<F, IL>(p.x, PP);
        Acc r;
        r.x = fe_sub<F>(fe_sub<F>(fsqr<F, IL>(R), PPP), fe_dbl<F>(Q));
        r.y = fe_sub<F>(fmul<F, IL>(R, fe_sub<F>(Q, r.x)), fmul<F, IL>(p.y, PPP));
        r.zz = fmul<F, IL>(p.zz, PP);
        r.zzz = fmul<F, IL>(p.zzz, PPP);
        return r;
    }
    // add-2008-s
    VK_HD static Acc add(const Acc& p, const Acc& q) {
        if (is_zero(p)) return q;
        if (is_zero(q)) return p;
        fe<F> U1 = fmul<F, IL>(p.x, q.zz);
        fe<F> U2 = fmul<F, IL>(q.x, p.zz);
        fe<F> S1 = fmul<F, IL>(p.y, q.zzz);
        fe<F> S2 = fmul<F, IL>(q.y, p.zzz);
        fe<F> P = fe_sub<F>(U2, U1);
        fe<F> R = fe_sub<F>(S2, S1);
        if (fe_is_zero<F>(P)) {
            if (fe_is_zero<F>(R)) return dbl(p);
            return zero();
        }
        fe<F> PP = fsqr<F, IL>(P);
        fe<F> PPP = fmul<F, IL>(P, PP);
        fe<F> Q = fmul<F, IL>(U1, PP);
        Acc r;
        r.x = fe_sub<F>(fe_sub<F>(fsqr<F, IL>(R), PPP), fe_dbl<F>(Q));
        r.y = fe_sub<F>(fmul<F, IL>(R, fe_sub<F>(Q, r.x)), fmul<F, IL>(S1, PPP));
        r.zz = fmul<F, IL>(fmul<F, IL>(p.zz, q.zz), PP);
        r.zzz = fmul<F, IL>(fmul<F, IL>(p.zzz, q.zzz), PPP);
        return r;
    }
    VK_HD static Acc neg(const Acc& p) {
        Acc r = p;
        r.y = fe_neg<F>(p.y);
        return r;
    }
    // affine normalisation (host/slow path): returns false for the identity
    // BIN: binary extended-Euclid inversion (host callers: ~10x faster than the Fermat chain
    // there); the Fermat chain stays the device default (no data-dependent branches)
    template <bool BIN = false>
    VK_HD static bool to_aff(const Acc& p, fe<F>& x, fe<F>& y) {
        if (is_zero(p)) return false;
        fe<F> izzz = BIN ? fe_inv_bin<F>(p.zzz) : fe_inv<F>(p.zzz);
        fe<F> t = fmul<F, IL>(izzz, p.zz);   // 1/ZZ^(1/2)... ZZ*1/ZZZ = 1/Z
        fe<F> izz = fsqr<F, IL>(t);          // 1/ZZ
        x = fmul<F, IL>(p.x, izz);
        y = fmul<F, IL>(p.y, izzz);
        return true;
    }
};

// ================================================================ twisted Edwards, a = -5
template <class Fq_, class DParam, bool IL = false>
struct TECurve {
    using F = Fq_;
    static constexpr bool is_te = true;
    using Aff = TEAff<F>;
    using Acc = TEAcc<F>;
    using Inl = TECurve<Fq_, DParam, true>;
    static constexpr int AFF_WORDS = 3 * F::N;
    static constexpr int ACC_WORDS = 4 * F::N;

    VK_HD static fe<F> d() {
        fe<F> r;
#pragma unroll
        for (int i = 0; i < F::N; i++) r.v[i] = DParam::d(i);
        return r;
    }
    VK_HD static Acc zero() {
        Acc r;
        r.X = fe_zero<F>();
        r.Y = fe_one<F>();
        r.T = fe_zero<F>();
        r.Z = fe_one<F>();
        return r;
    }
    VK_HD static bool is_zero(const Acc& a) {
        // X == 0 and Y == Z
        return fe_is_zero<F>(a.X) && fe_eq<F>(a.Y, a.Z);
    }
    VK_HD static Acc from_aff(const Aff& p, bool neg) {
        Acc r;
        r.X = neg ? fe_neg<F>(p.x) : p.x;
        r.Y = p.y;
        r.T = fmul<F, IL>(r.X, r.Y);
        r.Z = fe_one<F>();
        return r;
    }
    // unified mixed add (add-2008-hwcd with Z2 = 1, kt = d*T2 precomputed): 8M
    VK_HD static Acc madd(const Acc& p, const Aff& q, bool neg) {
        fe<F> x2 = neg ? fe_neg<F>(q.x) : q.x;
        fe<F> kt = neg ? fe_neg<F>(q.kt) : q.kt;
        fe<F> A = fmul<F, IL>(p.X, x2);
        fe<F> B = fmul<F, IL>(p.Y, q.y);
        fe<F> C = fmul<F, IL>(p.T, kt);
        fe<F> E = fe_sub<F>(fe_sub<F>(fmul<F, IL>(fe_add<F>(p.X, p.Y), fe_add<F>(x2, q.y)), A), B);
        fe<F> Fv = fe_sub<F>(p.Z, C);
        fe<F> G = fe_add<F>(p.Z, C);
        fe<F> H = fe_add<F>(B, fe_mul_small<F, 5>(A));  // B - a*A, a = -5
        Acc r;
        r.X = fmul<F, IL>(E, Fv);
        r.Y = fmul<F, IL>(G, H);
        r.T = fmul<F, IL>(E, H);
        r.Z = fmul<F, IL>(Fv, G);
        return r;
    }
    // unified add (add-2008-hwcd): 9M + 1 const mul
    VK_HD static Acc add(const Acc& p, const Acc& q) {
        fe<F> A = fmul<F, IL>(p.X, q.X);
        fe<F> B = fmul<F, IL>(p.Y, q.Y);
        fe<F> C = fmul<F, IL>(fmul<F, IL>(p.T, q.T), d());
        fe<F> D = fmul<F, IL>(p.Z, q.Z);
        fe<F> E = fe_sub<F>(fe_sub<F>(fmul<F, IL>(fe_add<F>(p.X, p.Y), fe_add<F>(q.X, q.Y)), A), B);
        fe<F> Fv = fe_sub<F>(D, C);
        fe<F> G = fe_add<F>(D, C);
        fe<F> H = fe_add<F>(B, fe_mul_small<F, 5>(A));
        Acc r;
        r.X = fmul<F, IL>(E, Fv);
        r.Y = fmul<F, IL>(G, H);
        r.T = fmul<F, IL>(E, H);
        r.Z = fmul<F, IL>(Fv, G);
        return r;
    }
    // dbl-2008-hwcd: 4M + 4S
    VK_HD static Acc dbl(const Acc& p) {
        fe<F> A = fsqr<F, IL>(p.X);
        fe<F> B = fsqr<F, IL>(p.Y);
        fe<F> C = fe_dbl<F>(fsqr<F, IL>(p.Z));
        fe<F> D = fe_neg<F>(fe_mul_small<F, 5>(A));  // a*A
        fe<F> xy = fe_add<F>(p.X, p.Y);
        fe<F> E = fe_sub<F>(fe_sub<F>(fsqr<F, IL>(xy), A), B);
        fe<F> G = fe_add<F>(D, B);
        fe<F> Fv = fe_sub<F>(G, C);
        fe<F> H = fe_sub<F>(D, B);
        Acc r;
        r.X = fmul<F, IL>(E, Fv);
        r.Y = fmul<F, IL>(G, H);
        r.T = fmul<F, IL>(E, H);
        r.Z = fmul<F, IL>(Fv, G);
        return r;
    }
    VK_HD static Acc neg(const Acc& p) {
        Acc r = p;
        r.X = fe_neg<F>(p.X);
        r.T = fe_neg<F>(p.T);
        return r;
    }
    template <bool BIN = false>
    VK_HD static bool to_aff(const Acc& p, fe<F>& x, fe<F>& y) {
        fe<F> iz = BIN ? fe_inv_bin<F>(p.Z) : fe_inv<F>(p.Z);
        x = fmul<F, IL>(p.X, iz);
        y = fmul<F, IL>(p.Y, iz);
        return !(fe_is_zero<F>(x) && fe_eq<F>(y, fe_one<F>()));
    }
};

// Bandersnatch d (Montgomery form over BLS12-381 Fr)
struct BandD {
    VK_HD static constexpr uint32_t d(int i) {
        constexpr uint32_t v[] = {0x47a2c730u, 0xa8dced1bu, 0xad3cccc7u, 0x381c065au,
                                  0x188351f8u, 0x53ff52e1u, 0x990fe940u, 0x362e8d63u};
        return v[i];
    }
};

using BN254G1 = SWCurve<BN254Fq, 3>;
using BLS381G1 = SWCurve<BLS381Fq, 4>;
using Bandersnatch = TECurve<BLS381Fr, BandD>;

// to_data_item (reference lib.rs:56-67) of a canonical affine BN254 G1 point: its compressed
// encoding (x, the top bit set when y > p - y) read as a little-endian integer mod r -- canonical
// Fr words; the identity maps to 0
VK_HD fe<BN254Fr> to_data_item_canon(const fe<BN254Fq>& x, const fe<BN254Fq>& y, bool inf) {
    fe<BN254Fr> r = fe_zero<BN254Fr>();
    if (inf) return r;
    const fe<BN254Fq> ny = fe_sub<BN254Fq>(fe_zero<BN254Fq>(), y);
    bool neg = false;  // y > p - y (canonical)
    for (int k = 7; k >= 0; k--) {
        if (y.v[k] != ny.v[k]) {
            neg = y.v[k] > ny.v[k];
            break;
        }
    }
    for (int k = 0; k < 8; k++) r.v[k] = x.v[k];
    if (neg) r.v[7] |= 0x80000000u;
    for (int it = 0; it < 6; it++) r = fe_reduce_once<BN254Fr>(r);  // < 2^256 < 6r
    return r;
}


}  // namespace vk
