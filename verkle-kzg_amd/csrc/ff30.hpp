// Signed radix-2^30 Montgomery arithmetic (BLS12-381 Fq in 13 limbs instead of ff29.hpp's 14):
// the prototype of DESIGN.md §8's "13 x 30-bit limbs". Constants: ff30_consts.hpp
// (tools/gen_ff30.py); host checks: tests/cpp/ff30_check.cpp + tests/test_ff30.py; GPU A/B
// against the radix-2^29 mixed add: tools/s30probe.hip.
//
// Why signed: unsigned 30-bit limbs make products < 2^60 and a CIOS column of 2 L = 26 of them
// overflows 64 bits. Centred limbs (in [-2^29, 2^29), the top limb takes the rest) keep every
// product at |.| <= 2^58 (v_mad_i64_i32, same issue cost as the unsigned mad), so a column of
// 26 products plus the row carry stays below 2^62.8. 13 x 13 = 169 products per half of a
// multiply against 196: -14 % of the mads.
//
// Values are signed integers congruent to x R' (R' = 2^390): no K p constants in subtractions,
// a - b is limb-wise. Bounds (rho = p / R' = 2^-9.3): a product of |a| < c_a p, |b| < c_b p is
// below (c_a c_b rho + 1/2 (1 + 2^-30)) p in magnitude -- below p for c_a c_b < 300, so a product
// output is congruent to 0 mod p iff all its limbs are 0 (is_zero_mo30).
// Limb states: "exact" (mul outputs: limbs j < L-1 in [-2^29, 2^29)), "near" (norm30 outputs:
// [-2^29 - 2, 2^29 + 2)). Every multiply operand must be exact or near (a raw sum of two would
// make a column of 13 x 2^59 + 13 x 2^58 > 2^63).
#pragma once
#include <stdint.h>

#include "ff.hpp"
#include "ff30_consts.hpp"

namespace vk {

constexpr uint32_t M30 = (1u << 30) - 1;

template <class P>
struct f30 {
    int32_t v[P::L];
};

VK_HD int32_t sext30(uint32_t x) { return (int32_t)(x << 2) >> 2; }

// x as a value of the current basic block (an empty asm the optimiser cannot see through): the
// selector fuses (int64) a * (int64) b into v_mad_i64_i32 only when it sees both sign
// extensions, and an operand extended in an earlier block (a multiply the compiler sank past a
// branch) becomes a 64 x 64-bit product (v_mad_u64_u32 + 2 v_mul_lo_u32 + v_add3). Used at the
// few call sites that need it (ec30.hpp): on every operand it costs registers (216 -> 248 VGPRs
// in tools/s30probe.hip).
template <class P>
VK_HD f30<P> opq30(const f30<P>& in) {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) {
        int32_t x = in.v[j];
#ifdef __HIP_DEVICE_COMPILE__
        asm("" : "+v"(x));
#endif
        r.v[j] = x;
    }
    return r;
}

// parallel centred carry pass: r_j = x_j - 2^30 c_j + c_{j-1}, c_j = round(x_j / 2^30);
// inputs |x_j| < 2^31 - 2^29 -> near limbs
template <class P>
VK_HD f30<P> norm30(const f30<P>& x) {
    constexpr int L = P::L;
    int32_t c[L];
#pragma unroll
    for (int j = 0; j < L - 1; j++) c[j] = (x.v[j] + (1 << 29)) >> 30;
    f30<P> r;
    r.v[0] = x.v[0] - (int32_t)((uint32_t)c[0] << 30);
#pragma unroll
    for (int j = 1; j < L - 1; j++) r.v[j] = x.v[j] - (int32_t)((uint32_t)c[j] << 30) + c[j - 1];
    r.v[L - 1] = x.v[L - 1] + c[L - 2];
    return r;
}

// the same for wide inputs (|x_j| <= 2^31 - 1, e.g. X3 = RR - PPP - 2Q of exact limbs): the
// rounding carry without the + 2^29 that could overflow
template <class P>
VK_HD f30<P> norm30w(const f30<P>& x) {
    constexpr int L = P::L;
    int32_t c[L];
#pragma unroll
    for (int j = 0; j < L - 1; j++) c[j] = ((x.v[j] >> 29) + 1) >> 1;
    f30<P> r;
    r.v[0] = x.v[0] - (int32_t)((uint32_t)c[0] << 30);
#pragma unroll
    for (int j = 1; j < L - 1; j++) r.v[j] = x.v[j] - (int32_t)((uint32_t)c[j] << 30) + c[j - 1];
    r.v[L - 1] = x.v[L - 1] + c[L - 2];
    return r;
}

template <class P>
VK_HD f30<P> add30(const f30<P>& a, const f30<P>& b) {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] + b.v[j];
    return norm30<P>(r);
}
template <class P>
VK_HD f30<P> sub30(const f30<P>& a, const f30<P>& b) {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] - b.v[j];
    return norm30<P>(r);
}
// -b: limb-wise (exact / near limbs stay near)
template <class P>
VK_HD f30<P> neg30(const f30<P>& b) {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = -b.v[j];
    return r;
}

// the final serial centred carry of a multiply's columns: exact limbs
template <class P>
VK_HD f30<P> fin30(int64_t* t) {
    constexpr int L = P::L;
    f30<P> r;
#pragma unroll
    for (int j = 0; j < L - 1; j++) {
        r.v[j] = sext30((uint32_t)t[j]);
        t[j + 1] += (t[j] + (1 << 29)) >> 30;  // the rounding carry: t_j - r_j = 2^30 c
    }
    r.v[L - 1] = (int32_t)t[L - 1];
    return r;
}

// one CIOS reduction step on the columns: m = -t_0 / p mod 2^30 (centred), t += m p, shift down
template <class P>
VK_HD void red30(int64_t* t) {
    constexpr int L = P::L;
    const int32_t m = sext30((uint32_t)t[0] * P::inv);
#pragma unroll
    for (int j = 0; j < L; j++) t[j] += (int64_t)m * P::p(j);
    const int64_t c = t[0] >> 30;  // t_0 is a multiple of 2^30 now
#pragma unroll
    for (int j = 0; j < L - 1; j++) t[j] = t[j + 1];
    t[L - 1] = 0;
    t[0] += c;
}

// Montgomery product a b / R' (CIOS): exact output, |value| < |a b| / R' + p / 2 (1 + 2^-30)
template <class P>
VK_HD f30<P> mul30(const f30<P>& a, const f30<P>& b) {
    constexpr int L = P::L;
    int64_t t[L];
#pragma unroll
    for (int j = 0; j < L; j++) t[j] = (int64_t)a.v[j] * b.v[0];
#pragma unroll
    for (int i = 0; i < L; i++) {
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < L; j++) t[j] += (int64_t)a.v[j] * b.v[i];
        }
        red30<P>(t);
    }
    return fin30<P>(t);
}

// (a b + c d) / R' with one reduction: 3 products per row and column; after row LH - 1 a parallel
// carry pass takes every column back to [0, 2^30) + carry (LH rows x 3 x 2^58 < 2^62.4 before it,
// the rest after it)
template <class P>
VK_HD f30<P> mul2sum30(const f30<P>& a, const f30<P>& b, const f30<P>& c, const f30<P>& d) {
    constexpr int L = P::L, LH = (L + 1) / 2;
    static_assert(3 * LH <= 24 && 3 * (L - LH) <= 24, "column bound");
    int64_t t[L];
#pragma unroll
    for (int j = 0; j < L; j++) t[j] = (int64_t)a.v[j] * b.v[0] + (int64_t)c.v[j] * d.v[0];
#pragma unroll
    for (int i = 0; i < L; i++) {
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < L; j++) t[j] += (int64_t)a.v[j] * b.v[i] + (int64_t)c.v[j] * d.v[i];
        }
        red30<P>(t);
        if (i == LH - 1) {
            int64_t cy[L];
#pragma unroll
            for (int j = 0; j < L - 1; j++) {
                cy[j] = t[j] >> 30;
                t[j] = (int64_t)((uint32_t)t[j] & M30);
            }
#pragma unroll
            for (int j = 1; j < L; j++) t[j] += cy[j - 1];
        }
    }
    return fin30<P>(t);
}

// a^2 / R': the product half by symmetry (a_i * 2 a_j, |.| <= 2^59, <= L/2 per column, plus the
// diagonal), then L reduction rows (separated operand scanning)
template <class P>
VK_HD f30<P> sqr30(const f30<P>& a) {
    constexpr int L = P::L;
    int32_t d[L];
#pragma unroll
    for (int j = 0; j < L; j++) d[j] = a.v[j] * 2;
    int64_t T[2 * L];
#pragma unroll
    for (int k = 0; k < 2 * L; k++) T[k] = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {
        T[2 * i] += (int64_t)a.v[i] * a.v[i];
#pragma unroll
        for (int j = i + 1; j < L; j++) T[i + j] += (int64_t)a.v[i] * d[j];
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
        const int32_t m = sext30((uint32_t)T[i] * P::inv);
#pragma unroll
        for (int j = 0; j < L; j++) T[i + j] += (int64_t)m * P::p(j);
        T[i + 1] += T[i] >> 30;
    }
    return fin30<P>(T + L);
}

template <class P>
VK_HD f30<P> const30(int32_t (*f)(int)) {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = f(j);
    return r;
}
template <class P>
VK_HD f30<P> one30() {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = P::one(j);
    return r;
}
template <class P>
VK_HD f30<P> zero30() {
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = 0;
    return r;
}

// a product output is 0 mod p iff it is 0 (|value| < p)
template <class P>
VK_HD bool is_zero_mo30(const f30<P>& x) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < P::L; j++) o |= (uint32_t)x.v[j];
    return o == 0;
}

// canonical residue in unsigned 30-bit limbs of a value with |value| < 8 p: add 8 p, then take
// off 8p, 4p, 2p, p where they fit
template <class P>
VK_HD void canon30(const f30<P>& x, uint32_t* out) {
    constexpr int L = P::L;
    int64_t c = 0;
    uint32_t u[L];
#pragma unroll
    for (int j = 0; j < L; j++) {  // x + 8 p, serial carry into unsigned limbs
        const int64_t s = (int64_t)x.v[j] + 8 * (int64_t)P::pu(j) + c;
        if (j < L - 1) {
            u[j] = (uint32_t)s & M30;
            c = s >> 30;
        } else {
            u[j] = (uint32_t)s;
        }
    }
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        uint32_t d[L];
        int32_t br = 0;
#pragma unroll
        for (int j = 0; j < L; j++) {
            // the limbs of (p << k) in radix 2^30 (p's top limb < 2^21: no spill out of the top)
            const uint64_t pk = ((uint64_t)P::pu(j) << k) & (j < L - 1 ? M30 : 0xffffffffu);
            const uint32_t in = j > 0 ? (uint32_t)(((uint64_t)P::pu(j - 1) << k) >> 30) : 0u;
            const int64_t s = (int64_t)u[j] - (int64_t)pk - in - br;
            br = s < 0 ? 1 : 0;
            d[j] = j < L - 1 ? ((uint32_t)s & M30) : (uint32_t)s;
        }
        if (!br) {
#pragma unroll
            for (int j = 0; j < L; j++) u[j] = d[j];
        }
    }
#pragma unroll
    for (int j = 0; j < L; j++) out[j] = u[j];
}

// canonical 32-bit words (x R mod p, the ec.hpp form) <-> signed limbs of x R' (R = 2^(32 N))
template <class P>
VK_HD f30<P> unpack30(const uint32_t* w) {  // the plain value in centred limbs (< p)
    f30<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) {
        const int b = 30 * j, q = b >> 5, s = b & 31;
        const uint32_t lo = q < P::N ? w[q] : 0u;
        const uint32_t hi = q + 1 < P::N ? w[q + 1] : 0u;
        const uint32_t v = s == 0 ? lo : ((lo >> s) | (hi << (32 - s)));
        r.v[j] = (int32_t)(j < P::L - 1 ? (v & M30) : v);
    }
    return norm30<P>(r);
}
template <class P, class F>
VK_HD f30<P> from_mont32_30(const fe<F>& a) {
    return mul30<P>(unpack30<P>(a.v), const30<P>(P::kin));
}
// unsigned 30-bit limbs of a canonical value -> N 32-bit words
template <class P>
VK_HD void pack30(const uint32_t* u, uint32_t* w) {
#pragma unroll
    for (int k = 0; k < P::N; k++) {
        const int b = 32 * k, j = b / 30, s = b - 30 * j;
        uint64_t acc = (uint64_t)u[j] >> s;
        int got = 30 - s;
        if (j + 1 < P::L) acc |= (uint64_t)u[j + 1] << got;
        got += 30;
        if (got < 32 && j + 2 < P::L) acc |= (uint64_t)u[j + 2] << got;
        w[k] = (uint32_t)acc;
    }
}
template <class P, class F>
VK_HD fe<F> to_mont32_30(const f30<P>& a) {
    uint32_t u[P::L];
    canon30<P>(mul30<P>(a, const30<P>(P::kout)), u);
    fe<F> r;
    pack30<P>(u, r.v);
    return r;
}

}  // namespace vk
