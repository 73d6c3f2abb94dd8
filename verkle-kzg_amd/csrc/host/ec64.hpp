// Host-side XYZZ point arithmetic on 64-bit limbs, for the serial folds the host runs after an
// MSM (the Horner pass over bit positions in msm.hip's slice_finish, ~128 doublings + ~112 adds
// per 2^20 BLS12-381 MSM). Same Montgomery representation as ec.hpp -- x R with
// R = 2^(32 N) = 2^(64 NL), canonical -- so an ec.hpp accumulator converts by a plain copy of its
// words. The 32-bit-limb device formulas compiled for the host cost 0.9 us per doubling and
// 1.4 us per add at BLS12-381, i.e. ~0.27 ms of host time per MSM; the CIOS multiply here works
// on 64 x 64 -> 128-bit products.
// Group law and exceptional cases are those of SWCurve (ec.hpp: dbl-2008-s-1, add-2008-s).
#pragma once
#include <stdint.h>
#include <string.h>

#include "../ec.hpp"

namespace vk {
namespace h64 {

typedef unsigned __int128 u128;

template <class F>
struct Fld {
    static constexpr int NL = F::N / 2;
    static constexpr uint64_t limb(int i) { return (uint64_t)F::p(2 * i) | ((uint64_t)F::p(2 * i + 1) << 32); }
    static constexpr uint64_t neg_inv() {  // -p^-1 mod 2^64: p0 p0 = 1 mod 8, Newton doubles the bits
        uint64_t x = limb(0);
        for (int k = 0; k < 5; k++) x *= 2 - limb(0) * x;
        return 0 - x;
    }
    static constexpr uint64_t inv = neg_inv();
    struct Arr {
        uint64_t v[NL];
    };
    static constexpr Arr mk() {
        Arr a{};
        for (int i = 0; i < NL; i++) a.v[i] = limb(i);
        return a;
    }
    static constexpr Arr P = mk();
};
template <class F>
struct FldRef {
    const uint64_t* p = Fld<F>::P.v;
    uint64_t inv = Fld<F>::inv;
};
template <class F>
inline FldRef<F> fld() {
    return FldRef<F>();
}

template <class F>
struct E {
    uint64_t v[F::N / 2];
};

template <class F>
inline bool geq_p(const uint64_t* t) {
    const FldRef<F> f = fld<F>();
#pragma GCC unroll 8
    for (int i = Fld<F>::NL - 1; i >= 0; i--) {
        if (t[i] != f.p[i]) return t[i] > f.p[i];
    }
    return true;
}
template <class F>
inline void sub_p(uint64_t* t) {
    const FldRef<F> f = fld<F>();
    uint64_t br = 0;
    for (int i = 0; i < Fld<F>::NL; i++) {
        const u128 d = (u128)t[i] - f.p[i] - br;
        t[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
    }
}

// Montgomery product a b / R (CIOS); a, b < p < 2^(64 NL - 2) -> canonical result
template <class F>
inline E<F> mul(const E<F>& a, const E<F>& b) {
    constexpr int NL = Fld<F>::NL;
    const FldRef<F> f = fld<F>();
    uint64_t t[NL + 2] = {0};
#pragma GCC unroll 8
    for (int i = 0; i < NL; i++) {
        u128 c = 0;
#pragma GCC unroll 8
        for (int j = 0; j < NL; j++) {
            c += (u128)a.v[j] * b.v[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[NL];
        t[NL] = (uint64_t)c;
        t[NL + 1] = (uint64_t)(c >> 64);
        const uint64_t m = t[0] * f.inv;
        c = ((u128)m * f.p[0] + t[0]) >> 64;
#pragma GCC unroll 8
        for (int j = 1; j < NL; j++) {
            c += (u128)m * f.p[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[NL];
        t[NL - 1] = (uint64_t)c;
        t[NL] = t[NL + 1] + (uint64_t)(c >> 64);
    }
    E<F> r;
    memcpy(r.v, t, sizeof r.v);
    if (t[NL] || geq_p<F>(r.v)) sub_p<F>(r.v);
    return r;
}
template <class F>
inline E<F> add(const E<F>& a, const E<F>& b) {
    E<F> r;
    uint64_t c = 0;
    for (int i = 0; i < Fld<F>::NL; i++) {
        const u128 s = (u128)a.v[i] + b.v[i] + c;
        r.v[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    if (c || geq_p<F>(r.v)) sub_p<F>(r.v);
    return r;
}
template <class F>
inline E<F> sub(const E<F>& a, const E<F>& b) {
    const FldRef<F> f = fld<F>();
    E<F> r;
    uint64_t br = 0;
    for (int i = 0; i < Fld<F>::NL; i++) {
        const u128 d = (u128)a.v[i] - b.v[i] - br;
        r.v[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
    }
    if (br) {  // add p back
        uint64_t c = 0;
        for (int i = 0; i < Fld<F>::NL; i++) {
            const u128 s = (u128)r.v[i] + f.p[i] + c;
            r.v[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
    return r;
}
template <class F>
inline bool is_zero(const E<F>& a) {
    uint64_t o = 0;
    for (int i = 0; i < Fld<F>::NL; i++) o |= a.v[i];
    return o == 0;
}

template <class F>
struct Acc {
    E<F> x, y, zz, zzz;
};

template <class C>
inline Acc<typename C::F> from(const typename C::Acc& a) {
    static_assert(sizeof(Acc<typename C::F>) == sizeof(typename C::Acc), "layout");
    Acc<typename C::F> r;
    memcpy(&r, &a, sizeof r);
    return r;
}
template <class C>
inline typename C::Acc to(const Acc<typename C::F>& a) {
    typename C::Acc r;
    memcpy(&r, &a, sizeof r);
    return r;
}

template <class F>
inline Acc<F> zero() {
    Acc<F> r;
    memset(&r, 0, sizeof r);
    const E<F> one = [] {
        E<F> o;
        for (int i = 0; i < Fld<F>::NL; i++) o.v[i] = (uint64_t)F::one(2 * i) | ((uint64_t)F::one(2 * i + 1) << 32);
        return o;
    }();
    r.x = one;
    r.y = one;
    return r;
}
template <class F>
inline bool is_inf(const Acc<F>& a) {
    return is_zero<F>(a.zz);
}

// dbl-2008-s-1
template <class F>
inline Acc<F> dbl(const Acc<F>& p) {
    if (is_inf<F>(p)) return p;
    const E<F> U = add<F>(p.y, p.y);
    const E<F> V = mul<F>(U, U);
    const E<F> W = mul<F>(U, V);
    const E<F> S = mul<F>(p.x, V);
    const E<F> X2 = mul<F>(p.x, p.x);
    const E<F> M = add<F>(add<F>(X2, X2), X2);
    Acc<F> r;
    r.x = sub<F>(mul<F>(M, M), add<F>(S, S));
    r.y = sub<F>(mul<F>(M, sub<F>(S, r.x)), mul<F>(W, p.y));
    r.zz = mul<F>(V, p.zz);
    r.zzz = mul<F>(W, p.zzz);
    return r;
}

// add-2008-s
template <class F>
inline Acc<F> add_pt(const Acc<F>& p, const Acc<F>& q) {
    if (is_inf<F>(p)) return q;
    if (is_inf<F>(q)) return p;
    const E<F> U1 = mul<F>(p.x, q.zz);
    const E<F> U2 = mul<F>(q.x, p.zz);
    const E<F> S1 = mul<F>(p.y, q.zzz);
    const E<F> S2 = mul<F>(q.y, p.zzz);
    const E<F> P = sub<F>(U2, U1);
    const E<F> R = sub<F>(S2, S1);
    if (is_zero<F>(P)) {
        if (is_zero<F>(R)) return dbl<F>(p);
        return zero<F>();
    }
    const E<F> PP = mul<F>(P, P);
    const E<F> PPP = mul<F>(P, PP);
    const E<F> Q = mul<F>(U1, PP);
    Acc<F> r;
    r.x = sub<F>(sub<F>(mul<F>(R, R), PPP), add<F>(Q, Q));
    r.y = sub<F>(mul<F>(R, sub<F>(Q, r.x)), mul<F>(S1, PPP));
    r.zz = mul<F>(mul<F>(p.zz, q.zz), PP);
    r.zzz = mul<F>(mul<F>(p.zzz, q.zzz), PPP);
    return r;
}

}  // namespace h64
}  // namespace vk
