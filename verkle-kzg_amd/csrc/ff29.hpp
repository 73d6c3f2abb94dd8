// Radix-2^29 Montgomery arithmetic for the VALU-bound inner loops (bucket accumulation,
// fixed-base commits). Constants: ff29_consts.hpp (tools/gen_ff29.py).
//
// Why: on gfx950 a 64-bit v_mad_u64_u32 and every VCC add-with-carry issue at 4 cycles per
// wave64 instruction, while plain 32-bit VALU (v_add_u32, v_and_b32, shifts) issue at 2 once
// two waves share a SIMD (tools/issueprobe.hip). The 32-bit-limb CIOS multiply (mul_asm.hpp)
// spends ~300 of its ~650 instructions on carry chains. With 29-bit limbs a row's 2L products
// accumulate straight into 64-bit columns (one mad each, 64-bit addend, no carries), only the
// lowest column shifts a carry per row, and additions/subtractions are limb-wise plain adds
// plus one parallel carry pass. Measured (tools/latprobe.hip): BLS12-381 Fq 14 x 29 limbs 2176
// cycles per dependent multiply vs 2776 (asm 12 x 32), 64-70 vs 57 Gmul/s chip-wide; Fr
// 9 x 29 limbs 1080 vs 1312 cycles.
//
// Representation: f29<P> holds L limbs, value = sum v_j 2^(29 j); elements are Montgomery
// residues x R' with R' = 2^(29 L). Values are kept only "loosely reduced": every result of
// mul29 is fully normalised (limbs < 2^29 except the top) and below a*b/R' + p; add/sub
// results are "almost normalised" (limbs <= 2^29 + 7) and their value is bounded by the
// caller's choice of the subtraction constant subK (K p in redundant limbs, see the
// generator). Products then stay below 2^58.0001 and a column of 2L products below 2^63.
// Nothing here is canonical except the outputs of canon() / pack().
#pragma once
#include <stdint.h>

#include "ff.hpp"
#include "ff29_consts.hpp"

namespace vk {

constexpr uint32_t M29 = (1u << 29) - 1;

template <class P>
struct f29 {
    uint32_t v[P::L];
};

// parallel carry pass: r_j = (x_j & M) + (x_{j-1} >> 29); inputs < 2^32 -> limbs <= 2^29 + 6
template <class P>
VK_HD f29<P> norm29(const f29<P>& x) {
    f29<P> r;
    r.v[0] = x.v[0] & M29;
#pragma unroll
    for (int j = 1; j < P::L - 1; j++) r.v[j] = (x.v[j] & M29) + (x.v[j - 1] >> 29);
    r.v[P::L - 1] = x.v[P::L - 1] + (x.v[P::L - 2] >> 29);
    return r;
}

template <class P>
VK_HD f29<P> add29(const f29<P>& a, const f29<P>& b) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] + b.v[j];
    return norm29<P>(r);
}

// a + b without the carry pass: limbs <= 2^30 + 14 (inputs almost normalised). Only as a mul29
// operand (or the subtrahend of sub29, whose subK limbs cover 2^30 + 8 -- not the sum of two
// raw values), and only where the column bound holds: one raw operand keeps L products of
// 2^59 + L of 2^58 below 2^63.4 up to L = 14; two raw operands (products < 2^60.01) need L <= 9
// (9 x 2^60.01 + 9 x 2^58 < 2^63.5).
template <class P>
VK_HD f29<P> add29_raw(const f29<P>& a, const f29<P>& b) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] + b.v[j];
    return r;
}

// a - b + K p (K = 2..32, a constant of the generator): b's value must be below (K - 1) p
// and its limbs (after an add) below 2^30 + 8
template <class P, int K>
VK_HD uint32_t subk(int j) {
    if constexpr (K == 2) return P::sub2(j);
    else if constexpr (K == 4) return P::sub4(j);
    else if constexpr (K == 8) return P::sub8(j);
    else if constexpr (K == 16) return P::sub16(j);
    else return P::sub32(j);
}
template <class P, int K>
VK_HD f29<P> sub29(const f29<P>& a, const f29<P>& b) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] + subk<P, K>(j) - b.v[j];
    return norm29<P>(r);
}
template <class P, int K>
VK_HD f29<P> neg29(const f29<P>& b) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = subk<P, K>(j) - b.v[j];
    return norm29<P>(r);
}
// a - b - c + K p
template <class P, int K>
VK_HD f29<P> sub2_29(const f29<P>& a, const f29<P>& b, const f29<P>& c) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = a.v[j] + subk<P, K>(j) - b.v[j] - c.v[j];
    return norm29<P>(r);
}

// Montgomery product a b / R' (CIOS, rows of 2L independent 64-bit mads). Output fully
// normalised, value < a b / R' + p.
template <class P>
VK_HD f29<P> mul29(const f29<P>& a, const f29<P>& b) {
    constexpr int L = P::L;
    uint64_t t[L];
#pragma unroll
    for (int j = 0; j < L; j++) t[j] = (uint64_t)a.v[j] * b.v[0];
#pragma unroll
    for (int i = 0; i < L; i++) {
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < L; j++) t[j] += (uint64_t)a.v[j] * b.v[i];
        }
        const uint32_t m = ((uint32_t)t[0] * P::inv) & M29;
#pragma unroll
        for (int j = 0; j < L; j++) t[j] += (uint64_t)m * P::p(j);
        const uint64_t c = t[0] >> 29;
#pragma unroll
        for (int j = 0; j < L - 1; j++) t[j] = t[j + 1];
        t[L - 1] = 0;
        t[0] += c;
    }
    f29<P> r;
#pragma unroll
    for (int j = 0; j < L - 1; j++) {
        t[j + 1] += t[j] >> 29;
        r.v[j] = (uint32_t)t[j] & M29;
    }
    r.v[L - 1] = (uint32_t)t[L - 1];
    return r;
}
// Montgomery sum of two products (a b + c d) / R' with ONE reduction (lazy reduction): every
// row takes a b_i and c d_i before its reduction step, so the pair costs 2L^2 + L^2 mads
// instead of 2 x 2L^2. A column (absolute position k) collects at most L rows x 3 products
// (a b, c d, m p) of < 2^58.0001 plus the row carry: < 2^63.4 at L = 14. Output fully
// normalised, value < (a b + c d) / R' + p.
template <class P>
VK_HD f29<P> mul2sum29(const f29<P>& a, const f29<P>& b, const f29<P>& c, const f29<P>& d) {
    constexpr int L = P::L;
    static_assert(3 * L <= 42, "column bound");
    uint64_t t[L];
#pragma unroll
    for (int j = 0; j < L; j++) t[j] = (uint64_t)a.v[j] * b.v[0] + (uint64_t)c.v[j] * d.v[0];
#pragma unroll
    for (int i = 0; i < L; i++) {
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < L; j++) t[j] += (uint64_t)a.v[j] * b.v[i] + (uint64_t)c.v[j] * d.v[i];
        }
        const uint32_t m = ((uint32_t)t[0] * P::inv) & M29;
#pragma unroll
        for (int j = 0; j < L; j++) t[j] += (uint64_t)m * P::p(j);
        const uint64_t cy = t[0] >> 29;
#pragma unroll
        for (int j = 0; j < L - 1; j++) t[j] = t[j + 1];
        t[L - 1] = 0;
        t[0] += cy;
    }
    f29<P> r;
#pragma unroll
    for (int j = 0; j < L - 1; j++) {
        t[j + 1] += t[j] >> 29;
        r.v[j] = (uint32_t)t[j] & M29;
    }
    r.v[L - 1] = (uint32_t)t[L - 1];
    return r;
}

// Montgomery square a^2 / R': the product half by symmetry (L(L+1)/2 mads: a_i * 2a_j for i < j
// plus the diagonal, into 2L - 1 columns), then L reduction rows (separated operand scanning);
// the L result limbs are columns L .. 2L - 1.
// Columns stay below 2^63 (<= L/2 cross products of 2^59, L reduction products of 2^58).
template <class P>
VK_HD f29<P> sqr29(const f29<P>& a) {
    constexpr int L = P::L;
    uint32_t d[L];
#pragma unroll
    for (int j = 0; j < L; j++) d[j] = a.v[j] << 1;
    uint64_t T[2 * L];
#pragma unroll
    for (int k = 0; k < 2 * L; k++) T[k] = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {
        T[2 * i] += (uint64_t)a.v[i] * a.v[i];
#pragma unroll
        for (int j = i + 1; j < L; j++) T[i + j] += (uint64_t)a.v[i] * d[j];
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
        const uint32_t m = ((uint32_t)T[i] * P::inv) & M29;
#pragma unroll
        for (int j = 0; j < L; j++) T[i + j] += (uint64_t)m * P::p(j);
        T[i + 1] += T[i] >> 29;
    }
    f29<P> r;
#pragma unroll
    for (int j = L; j < 2 * L - 1; j++) {
        T[j + 1] += T[j] >> 29;
        r.v[j - L] = (uint32_t)T[j] & M29;
    }
    r.v[L - 1] = (uint32_t)T[2 * L - 1];
    return r;
}

template <class P>
VK_HD f29<P> const29(uint32_t (*f)(int)) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = f(j);
    return r;
}
template <class P>
VK_HD f29<P> one29() {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = P::one(j);
    return r;
}
template <class P>
VK_HD f29<P> zero29() {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) r.v[j] = 0;
    return r;
}

// fully normalise (serial carry): limbs < 2^29 except the top
template <class P>
VK_HD f29<P> carry29(const f29<P>& x) {
    f29<P> r;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < P::L - 1; j++) {
        const uint32_t s = x.v[j] + c;
        r.v[j] = s & M29;
        c = s >> 29;
    }
    r.v[P::L - 1] = x.v[P::L - 1] + c;
    return r;
}

// x - p if x >= p (x fully normalised)
template <class P>
VK_HD f29<P> csub29(const f29<P>& x) {
    f29<P> d;
    int32_t br = 0;
#pragma unroll
    for (int j = 0; j < P::L; j++) {
        int32_t s = (int32_t)x.v[j] - (int32_t)P::p(j) - br;
        br = s < 0 ? 1 : 0;
        d.v[j] = j < P::L - 1 ? ((uint32_t)s & M29) : (uint32_t)s;
    }
    return br ? x : d;
}

// canonical residue (< p) of a value below 4p (every mul29 output of the kernels here)
template <class P>
VK_HD f29<P> canon29(const f29<P>& x) {
    f29<P> r = carry29<P>(x);
    r = csub29<P>(r);
    r = csub29<P>(r);
    return csub29<P>(r);
}

// x == 0 mod p for a value below 4p
template <class P>
VK_HD bool is_zero29(const f29<P>& x) {
    const f29<P> c = canon29<P>(x);
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < P::L; j++) o |= c.v[j];
    return o == 0;
}

// x == 0 mod p for a FULLY normalised product output below 2p: x is 0 or p limb for limb
template <class P>
VK_HD bool is_zero_mo29(const f29<P>& x) {
    uint32_t o0 = 0, o1 = 0;
#pragma unroll
    for (int j = 0; j < P::L; j++) {
        o0 |= x.v[j];
        o1 |= x.v[j] ^ P::p(j);
    }
    return o0 == 0 || o1 == 0;
}

// ---- packed form: N 32-bit words of a canonical residue (tables / buckets in HBM)
template <class P>
VK_HD f29<P> unpack29(const uint32_t* w) {
    f29<P> r;
#pragma unroll
    for (int j = 0; j < P::L; j++) {
        const int b = 29 * j, q = b >> 5, s = b & 31;
        uint32_t lo = q < P::N ? w[q] : 0u;
        uint32_t hi = q + 1 < P::N ? w[q + 1] : 0u;
        uint32_t v = s == 0 ? lo : ((lo >> s) | (hi << (32 - s)));
        r.v[j] = j < P::L - 1 ? (v & M29) : v;
    }
    return r;
}
template <class P>
VK_HD void pack29(const f29<P>& x, uint32_t* w) {  // x canonical
#pragma unroll
    for (int k = 0; k < P::N; k++) {
        const int b = 32 * k, j = b / 29, s = b - 29 * j;
        uint64_t acc = (uint64_t)x.v[j] >> s;
        int got = 29 - s;
        if (j + 1 < P::L) acc |= (uint64_t)x.v[j + 1] << got;
        got += 29;
        if (got < 32 && j + 2 < P::L) acc |= (uint64_t)x.v[j + 2] << got;
        w[k] = (uint32_t)acc;
    }
}

// x R (the 32-bit-limb Montgomery form of ff.hpp, canonical) <-> x R' (this form)
template <class P, class F>
VK_HD f29<P> from_mont32(const fe<F>& a) {
    static_assert(F::N == P::N, "");
    f29<P> k;
#pragma unroll
    for (int j = 0; j < P::L; j++) k.v[j] = P::kin(j);
    return mul29<P>(unpack29<P>(a.v), k);
}
template <class P, class F>
VK_HD fe<F> to_mont32(const f29<P>& a) {
    static_assert(F::N == P::N, "");
    f29<P> k;
#pragma unroll
    for (int j = 0; j < P::L; j++) k.v[j] = P::kout(j);
    const f29<P> c = canon29<P>(mul29<P>(a, k));
    fe<F> r;
    pack29<P>(c, r.v);
    return r;
}

// field of ff.hpp -> its radix-2^29 parameters
template <class F>
struct F29Of;
template <>
struct F29Of<BLS381Fq> {
    using type = F29BLS381Fq;
};
template <>
struct F29Of<BN254Fq> {
    using type = F29BN254Fq;
};
template <>
struct F29Of<BLS381Fr> {
    using type = F29BLS381Fr;
};
template <>
struct F29Of<BN254Fr> {
    using type = F29BN254Fr;
};

}  // namespace vk
