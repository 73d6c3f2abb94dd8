// Prime-field arithmetic for gfx950 (and host, for conversions): Montgomery form over
// 32-bit limbs. The VALU has no 64x64 multiply; the native wide product is
// v_mad_u64_u32 (32x32+64 -> 64), so limbs are 32 bits and every product is one mad.
//
// Multiplication is "no-carry" CIOS (valid because every modulus here has its top limb
// < 2^31 - 1: BN254 Fq/Fr, BLS12-381 Fq/Fr, Bandersnatch Fr), fully unrolled so the
// modulus limbs become instruction literals.
//
// Field parameter structs (N, p(i), inv, r2(i), one(i)) are at the bottom.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#define VK_HD __host__ __device__ __forceinline__
// occupancy targets for the two VALU-heavy kernels (waves per SIMD; 0 = compiler's choice).
// Default 2 (<= 256 VGPRs + AGPRs): the 13-limb BLS12-381 commit loop otherwise takes 264 and
// runs one wave per SIMD
#ifndef VK_COMMIT_WPE
#define VK_COMMIT_WPE 2
#endif
#ifndef VK_ACC_WPE
#define VK_ACC_WPE 2
#endif
#if defined(VK_COMMIT_WPE) && VK_COMMIT_WPE > 0
#define VK_COMMIT_OCC __attribute__((amdgpu_waves_per_eu(VK_COMMIT_WPE)))
#else
#define VK_COMMIT_OCC
#endif
#if defined(VK_ACC_WPE) && VK_ACC_WPE > 0
#define VK_ACC_OCC __attribute__((amdgpu_waves_per_eu(VK_ACC_WPE)))
#else
#define VK_ACC_OCC
#endif

namespace vk {

template <class F>
struct fe {
    uint32_t v[F::N];
};

// ---------------------------------------------------------------- helpers
template <class F>
VK_HD fe<F> fe_zero() {
    fe<F> r;
#pragma unroll
    for (int i = 0; i < F::N; i++) r.v[i] = 0;
    return r;
}
template <class F>
VK_HD fe<F> fe_one() {
    fe<F> r;
#pragma unroll
    for (int i = 0; i < F::N; i++) r.v[i] = F::one(i);
    return r;
}
template <class F>
VK_HD bool fe_is_zero(const fe<F>& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) o |= a.v[i];
    return o == 0;
}
template <class F>
VK_HD bool fe_eq(const fe<F>& a, const fe<F>& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) o |= a.v[i] ^ b.v[i];
    return o == 0;
}

// r = a - p if a >= p (a < 2p)
template <class F>
VK_HD fe<F> fe_reduce_once(const fe<F>& a) {
    fe<F> t;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t d = (uint64_t)a.v[i] - F::p(i) - borrow;
        t.v[i] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
    }
    fe<F> r;
#pragma unroll
    for (int i = 0; i < F::N; i++) r.v[i] = borrow ? a.v[i] : t.v[i];
    return r;
}

template <class F>
VK_HD fe<F> fe_add(const fe<F>& a, const fe<F>& b) {
    fe<F> s;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t t = (uint64_t)a.v[i] + b.v[i] + c;
        s.v[i] = (uint32_t)t;
        c = (uint32_t)(t >> 32);
    }
    return fe_reduce_once<F>(s);  // a+b < 2p < 2^(32N): no carry out
}

template <class F>
VK_HD fe<F> fe_sub(const fe<F>& a, const fe<F>& b) {
    fe<F> d;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t t = (uint64_t)a.v[i] - b.v[i] - borrow;
        d.v[i] = (uint32_t)t;
        borrow = (uint32_t)(t >> 63);
    }
    // add back p masked by borrow
    uint32_t mask = 0u - borrow;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t t = (uint64_t)d.v[i] + (F::p(i) & mask) + c;
        d.v[i] = (uint32_t)t;
        c = (uint32_t)(t >> 32);
    }
    return d;
}

template <class F>
VK_HD fe<F> fe_dbl(const fe<F>& a) {
    return fe_add<F>(a, a);
}

template <class F>
VK_HD fe<F> fe_neg(const fe<F>& a) {
    return fe_sub<F>(fe_zero<F>(), a);
}

// no-carry CIOS Montgomery multiplication: r = a*b*2^(-32N) mod p.
// On the device it is an out-of-line call: a fully inlined 12-limb multiply is ~600
// instructions, and an EC add holds 10-16 of them -- inlining every one blows the
// instruction cache (and compile time) for no gain.
#ifndef __HIP_DEVICE_COMPILE__
// Host build of the same multiply on 64-bit limbs (unsigned __int128): for even N the
// Montgomery form is identical (R = 2^(32N) = 2^(64 N/2)), so host and device share bytes.
template <class F>
constexpr uint64_t host_inv64() {
    uint64_t p0 = (uint64_t)F::p(0) | ((uint64_t)F::p(1) << 32);
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p0 * x;
    return (uint64_t)0 - x;
}
template <class F>
struct HostP64 {
    uint64_t v[F::N / 2];
    constexpr HostP64() : v() {
        for (int i = 0; i < F::N / 2; i++) v[i] = (uint64_t)F::p(2 * i) | ((uint64_t)F::p(2 * i + 1) << 32);
    }
};
// no-carry CIOS on 64-bit limbs (every modulus leaves spare top bits), fully unrolled, with a
// branchless final subtraction; the 32-bit limb array is read as 64-bit limbs (little-endian
// host). 26 ns for BLS12-381 Fq on the GPU box's EPYC vs 38 ns for the looped version
// (tools/hostmul.cpp): it carries the MSM's host Horner pass.
template <class F>
inline fe<F> fe_mul_host64(const fe<F>& a, const fe<F>& b) {
    constexpr int M = F::N / 2;
    constexpr uint64_t inv = host_inv64<F>();
    static constexpr HostP64<F> P{};
    typedef unsigned __int128 u128;
    uint64_t pa[M], pb[M], t[M + 1] = {0};
    memcpy(pa, a.v, sizeof pa);
    memcpy(pb, b.v, sizeof pb);
#pragma unroll
    for (int i = 0; i < M; i++) {
        uint64_t C = 0;
#pragma unroll
        for (int j = 0; j < M; j++) {
            u128 s = (u128)pa[j] * pb[i] + t[j] + C;
            t[j] = (uint64_t)s;
            C = (uint64_t)(s >> 64);
        }
        t[M] += C;
        const uint64_t m = t[0] * inv;
        u128 s = (u128)m * P.v[0] + t[0];
        C = (uint64_t)(s >> 64);
#pragma unroll
        for (int j = 1; j < M; j++) {
            s = (u128)m * P.v[j] + t[j] + C;
            t[j - 1] = (uint64_t)s;
            C = (uint64_t)(s >> 64);
        }
        t[M - 1] = t[M] + C;
        t[M] = 0;
    }
    uint64_t d[M], o[M];
    uint64_t br = 0;
#pragma unroll
    for (int j = 0; j < M; j++) {
        u128 s = (u128)t[j] - P.v[j] - br;
        d[j] = (uint64_t)s;
        br = (uint64_t)(s >> 64) & 1;
    }
    const uint64_t mask = (uint64_t)0 - br;  // borrow: t < p, keep t
#pragma unroll
    for (int j = 0; j < M; j++) o[j] = (t[j] & mask) | (d[j] & ~mask);
    fe<F> r;
    memcpy(r.v, o, sizeof o);
    return r;
}
#endif

template <class F>
VK_HD fe<F> fe_mul_body(const fe<F>& a, const fe<F>& b) {
#ifndef __HIP_DEVICE_COMPILE__
    if constexpr (F::N % 2 == 0) return fe_mul_host64<F>(a, b);
#endif
    constexpr int N = F::N;
    uint32_t t[N];
#pragma unroll
    for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint64_t A = (uint64_t)a.v[0] * b.v[i] + t[0];
        t[0] = (uint32_t)A;
        uint32_t m = t[0] * F::inv;
        uint64_t C = (uint64_t)m * F::p(0) + t[0];
#pragma unroll
        for (int j = 1; j < N; j++) {
            A = (uint64_t)a.v[j] * b.v[i] + t[j] + (A >> 32);
            C = (uint64_t)m * F::p(j) + (uint32_t)A + (C >> 32);
            t[j - 1] = (uint32_t)C;
        }
        t[N - 1] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
    }
    fe<F> r;
#pragma unroll
    for (int j = 0; j < N; j++) r.v[j] = t[j];
    return fe_reduce_once<F>(r);
}
}  // namespace vk
#include "mul_asm.hpp"
namespace vk {

// Device multiply: the generated inline-asm CIOS (mul_asm.hpp) for 8- and 12-limb fields --
// 1.5x the throughput of the compiler-built CIOS above, whose carries cost ~620 zero-extension
// moves per 12-limb multiply (tools/mulvariants.hip). Host: 64-bit limbs.
template <class F>
VK_HD fe<F> fe_mul(const fe<F>& a, const fe<F>& b) {
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr (F::N == 12) return fe_mul_asm12<F>(a, b);
    else if constexpr (F::N == 8) return fe_mul_asm8<F>(a, b);
    else return fe_mul_body<F>(a, b);
#else
    return fe_mul_body<F>(a, b);
#endif
}
// policy switch kept for the curve templates (both policies use the same multiply now)
template <class F, bool IL>
VK_HD fe<F> fmul(const fe<F>& a, const fe<F>& b) {
    return fe_mul<F>(a, b);
}

template <class F>
VK_HD fe<F> fe_sqr(const fe<F>& a) {
    return fe_mul<F>(a, a);
}

// canonical -> Montgomery
template <class F>
VK_HD fe<F> fe_to_mont(const fe<F>& a) {
    fe<F> r2;
#pragma unroll
    for (int i = 0; i < F::N; i++) r2.v[i] = F::r2(i);
    return fe_mul<F>(a, r2);
}
// Montgomery -> canonical
template <class F>
VK_HD fe<F> fe_from_mont(const fe<F>& a) {
    fe<F> one = fe_zero<F>();
    one.v[0] = 1;
    // compiler multiply: with b = 1 it folds to a plain Montgomery reduction and does not pin
    // the asm multiply's fixed VGPR block (keeps e.g. the digit kernel at high occupancy)
    return fe_mul_body<F>(a, one);
}

// a^(p-2) (slow; only for rare normalisations)
template <class F>
VK_HD fe<F> fe_inv(const fe<F>& a) {
    // exponent p - 2 with the borrow propagated (BLS12-381 Fr has p[0] == 1)
    uint32_t e_limbs[F::N];
    uint32_t borrow = 2;
    for (int i = 0; i < F::N; i++) {
        uint64_t d = (uint64_t)F::p(i) - borrow;
        e_limbs[i] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
    }
    fe<F> acc = fe_one<F>();
    for (int i = F::N - 1; i >= 0; i--) {
        uint32_t e = e_limbs[i];
        for (int b = 31; b >= 0; b--) {
            acc = fe_sqr<F>(acc);
            if ((e >> b) & 1) acc = fe_mul<F>(acc, a);
        }
    }
    return acc;
}

// Montgomery inverse by the binary extended Euclidean algorithm (variable time; latency
// ~50x lower than the Fermat chain above, which matters in latency-bound tails):
// for aR (Montgomery form of a != 0) returns a^-1 R.
template <class F>
VK_HD void fe_shr1(fe<F>& a, uint32_t top) {
#pragma unroll
    for (int i = 0; i < F::N - 1; i++) a.v[i] = (a.v[i] >> 1) | (a.v[i + 1] << 31);
    a.v[F::N - 1] = (a.v[F::N - 1] >> 1) | (top << 31);
}
template <class F>
VK_HD uint32_t fe_add_p_raw(fe<F>& a) {  // a += p, returns carry
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t t = (uint64_t)a.v[i] + F::p(i) + c;
        a.v[i] = (uint32_t)t;
        c = (uint32_t)(t >> 32);
    }
    return c;
}
template <class F>
VK_HD bool fe_geq_raw(const fe<F>& a, const fe<F>& b) {
    for (int i = F::N - 1; i >= 0; i--) {
        if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
    }
    return true;
}
template <class F>
VK_HD void fe_sub_raw(fe<F>& a, const fe<F>& b) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < F::N; i++) {
        uint64_t t = (uint64_t)a.v[i] - b.v[i] - br;
        a.v[i] = (uint32_t)t;
        br = (uint32_t)(t >> 63);
    }
}
template <class F>
VK_HD bool fe_is_one_raw(const fe<F>& a) {
    uint32_t o = a.v[0] ^ 1u;
#pragma unroll
    for (int i = 1; i < F::N; i++) o |= a.v[i];
    return o == 0;
}
#ifndef __HIP_DEVICE_COMPILE__
// Host inverse by Bernstein-Yang divsteps (variable time), 62 at a time on signed 62-bit limbs:
// each batch is found from the low 64 bits of f and g alone (a 2x2 transition matrix with entries
// below 2^62), then applied to the full-size f, g (exact division by 2^62) and to the Bezout
// coefficients d, e (kept in (-2p, p); a multiple of p added so the division by 2^62 is exact).
// ~12-18 batches for a 381-bit modulus. It is the last serial step of every MSM call
// (acc_to_affine) and of every IPA round's normalisation: on the GPU box's host the 64-bit binary
// Euclid it replaces took ~8 us for BLS12-381 Fq (tools/hostinv.cpp; tests/cpp/inv_check.cpp
// checks both against a^(p-2)).
template <class F>
struct Sg62 {
    static constexpr int M = F::N / 2;                      // 64-bit words of the field
    static constexpr int L = (64 * M + 2 + 61) / 62;        // signed 62-bit limbs (value and sign)
    static constexpr uint64_t M62 = ~(uint64_t)0 >> 2;
    int64_t mod[L];
    uint64_t inv62;                                         // p^-1 mod 2^62
    constexpr Sg62() : mod(), inv62(0) {
        uint64_t w[M] = {};
        for (int i = 0; i < M; i++) w[i] = (uint64_t)F::p(2 * i) | ((uint64_t)F::p(2 * i + 1) << 32);
        for (int k = 0; k < L; k++) {
            const int o = 62 * k, wi = o / 64, sh = o % 64;
            uint64_t x = wi < M ? w[wi] >> sh : 0;
            if (sh > 2 && wi + 1 < M) x |= w[wi + 1] << (64 - sh);
            mod[k] = (int64_t)(x & M62);
        }
        uint64_t x = 1;
        for (int i = 0; i < 7; i++) x *= 2 - w[0] * x;  // p^-1 mod 2^64 (Newton)
        inv62 = x & M62;
    }
};
struct SgT {
    int64_t u, v, q, r;
};
// 62 divsteps on the low bits: returns the new eta (= -delta), the matrix in t
inline int64_t sg_divsteps62(int64_t eta, uint64_t f, uint64_t g, SgT& t) {
    uint64_t u = 1, v = 0, q = 0, r = 1;
    int i = 62;
    for (;;) {
        const int zeros = __builtin_ctzll(g | (~(uint64_t)0 << i));  // sentinel at bit i
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= zeros;
        i -= zeros;
        if (i == 0) break;
        uint64_t w;
        int limit;
        if (eta < 0) {  // swap: (f, g) <- (g, -f)
            eta = -eta;
            uint64_t tmp = f;
            f = g;
            g = 0 - tmp;
            tmp = u;
            u = q;
            q = 0 - tmp;
            tmp = v;
            v = r;
            r = 0 - tmp;
            limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
            const uint64_t m = (~(uint64_t)0 >> (64 - limit)) & 63u;
            w = (f * g * (f * f - 2)) & m;  // -g / f mod 2^6 (f (2 - f^2) = f^-1 mod 64)
        } else {
            limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
            const uint64_t m = (~(uint64_t)0 >> (64 - limit)) & 15u;
            w = f + (((f + 1) & 4) << 1);  // f^-1 mod 16
            w = (0 - w * g) & m;
        }
        g += f * w;
        q += u * w;
        r += v * w;
    }
    t.u = (int64_t)u;
    t.v = (int64_t)v;
    t.q = (int64_t)q;
    t.r = (int64_t)r;
    return eta;
}
// canonical a (not Montgomery; 0 < a < p) -> a^-1 mod p, canonical
template <class F>
inline fe<F> fe_inv_canon_host(const fe<F>& a) {
    typedef __int128 i128;
    static constexpr Sg62<F> S{};
    constexpr int L = Sg62<F>::L, M = Sg62<F>::M;
    constexpr int64_t M62 = (int64_t)Sg62<F>::M62;
    int64_t d[L] = {}, e[L] = {}, f[L], g[L] = {};
    e[0] = 1;
    for (int k = 0; k < L; k++) f[k] = S.mod[k];
    {
        uint64_t w[M];
        memcpy(w, a.v, sizeof w);
        for (int k = 0; k < L; k++) {
            const int o = 62 * k, wi = o / 64, sh = o % 64;
            uint64_t x = wi < M ? w[wi] >> sh : 0;
            if (sh > 2 && wi + 1 < M) x |= w[wi + 1] << (64 - sh);
            g[k] = (int64_t)(x & (uint64_t)M62);
        }
    }
    int len = L;
    int64_t eta = -1;
    for (;;) {
        SgT t;
        eta = sg_divsteps62(eta, (uint64_t)f[0], (uint64_t)g[0], t);
        // (d, e) <- (t [d, e] + p [md, me]) / 2^62
        {
            const int64_t sd = d[L - 1] >> 63, se = e[L - 1] >> 63;
            int64_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
            i128 cd = (i128)t.u * d[0] + (i128)t.v * e[0], ce = (i128)t.q * d[0] + (i128)t.r * e[0];
            md -= (int64_t)((S.inv62 * (uint64_t)cd + (uint64_t)md) & (uint64_t)M62);
            me -= (int64_t)((S.inv62 * (uint64_t)ce + (uint64_t)me) & (uint64_t)M62);
            cd += (i128)S.mod[0] * md;
            ce += (i128)S.mod[0] * me;
            cd >>= 62;
            ce >>= 62;
            for (int i = 1; i < L; i++) {
                cd += (i128)t.u * d[i] + (i128)t.v * e[i] + (i128)S.mod[i] * md;
                ce += (i128)t.q * d[i] + (i128)t.r * e[i] + (i128)S.mod[i] * me;
                d[i - 1] = (int64_t)cd & M62;
                cd >>= 62;
                e[i - 1] = (int64_t)ce & M62;
                ce >>= 62;
            }
            d[L - 1] = (int64_t)cd;
            e[L - 1] = (int64_t)ce;
        }
        // (f, g) <- t [f, g] / 2^62 over the live limbs
        {
            i128 cf = (i128)t.u * f[0] + (i128)t.v * g[0], cg = (i128)t.q * f[0] + (i128)t.r * g[0];
            cf >>= 62;
            cg >>= 62;
            for (int i = 1; i < len; i++) {
                cf += (i128)t.u * f[i] + (i128)t.v * g[i];
                cg += (i128)t.q * f[i] + (i128)t.r * g[i];
                f[i - 1] = (int64_t)cf & M62;
                cf >>= 62;
                g[i - 1] = (int64_t)cg & M62;
                cg >>= 62;
            }
            f[len - 1] = (int64_t)cf;
            g[len - 1] = (int64_t)cg;
        }
        if (g[0] == 0) {
            int64_t c = 0;
            for (int j = 1; j < len; j++) c |= g[j];
            if (c == 0) break;  // g = 0: f = +-1
        }
        // shorten when the top limbs of f and g are both 0 or -1
        const int64_t fn = f[len - 1], gn = g[len - 1];
        if (len > 1 && (fn ^ (fn >> 63)) == 0 && (gn ^ (gn >> 63)) == 0) {
            f[len - 2] |= (int64_t)((uint64_t)fn << 62);
            g[len - 2] |= (int64_t)((uint64_t)gn << 62);
            len--;
        }
    }
    // d in (-2p, p) -> d sign(f) in [0, p)
    {
        int64_t c = d[L - 1] >> 63;
        for (int i = 0; i < L; i++) d[i] += S.mod[i] & c;
        const int64_t neg = f[len - 1] >> 63;
        for (int i = 0; i < L; i++) d[i] = (d[i] ^ neg) - neg;
        for (int i = 0; i < L - 1; i++) {
            d[i + 1] += d[i] >> 62;
            d[i] &= M62;
        }
        c = d[L - 1] >> 63;
        for (int i = 0; i < L; i++) d[i] += S.mod[i] & c;
        for (int i = 0; i < L - 1; i++) {
            d[i + 1] += d[i] >> 62;
            d[i] &= M62;
        }
    }
    uint64_t w[M] = {};
    for (int k = 0; k < L; k++) {  // 62-bit limbs back to 64-bit words
        const int o = 62 * k, wi = o / 64, sh = o % 64;
        const uint64_t x = (uint64_t)d[k];
        if (wi < M) w[wi] |= x << sh;
        if (sh > 2 && wi + 1 < M) w[wi + 1] |= x >> (64 - sh);
    }
    fe<F> r;
    memcpy(r.v, w, sizeof w);
    return r;
}
// for aR (Montgomery form of a != 0) returns a^-1 R
template <class F>
inline fe<F> fe_inv_host(const fe<F>& a_mont) {
    fe<F> r = fe_inv_canon_host<F>(a_mont), r2;  // (aR)^-1
    for (int i = 0; i < F::N; i++) r2.v[i] = F::r2(i);
    return fe_mul<F>(fe_mul<F>(r, r2), r2);  // (aR)^-1 R^2 = a^-1 R
}
#endif

template <class F>
VK_HD fe<F> fe_inv_bin(const fe<F>& a_mont) {
#ifndef __HIP_DEVICE_COMPILE__
    if constexpr (F::N % 2 == 0) return fe_is_zero<F>(a_mont) ? fe_zero<F>() : fe_inv_host<F>(a_mont);
#endif
    fe<F> u = a_mont, v, x1 = fe_zero<F>(), x2 = fe_zero<F>();
#pragma unroll
    for (int i = 0; i < F::N; i++) v.v[i] = F::p(i);
    x1.v[0] = 1;
    if (fe_is_zero<F>(u)) return fe_zero<F>();
    while (!fe_is_one_raw<F>(u) && !fe_is_one_raw<F>(v)) {
        while ((u.v[0] & 1) == 0) {
            fe_shr1<F>(u, 0);
            uint32_t c = (x1.v[0] & 1) ? fe_add_p_raw<F>(x1) : 0u;
            fe_shr1<F>(x1, c);
        }
        while ((v.v[0] & 1) == 0) {
            fe_shr1<F>(v, 0);
            uint32_t c = (x2.v[0] & 1) ? fe_add_p_raw<F>(x2) : 0u;
            fe_shr1<F>(x2, c);
        }
        if (fe_geq_raw<F>(u, v)) {
            fe_sub_raw<F>(u, v);
            x1 = fe_sub<F>(x1, x2);
        } else {
            fe_sub_raw<F>(v, u);
            x2 = fe_sub<F>(x2, x1);
        }
    }
    fe<F> r = fe_is_one_raw<F>(u) ? x1 : x2;  // (aR)^-1
    fe<F> r2;
#pragma unroll
    for (int i = 0; i < F::N; i++) r2.v[i] = F::r2(i);
    return fe_mul<F>(fe_mul<F>(r, r2), r2);  // (aR)^-1 R^2 = a^-1 R
}

// small-constant multiple (k <= 8) via additions
template <class F, int K>
VK_HD fe<F> fe_mul_small(const fe<F>& a) {
    static_assert(K >= 1 && K <= 8, "");
    if (K == 1) return a;
    if (K == 2) return fe_dbl<F>(a);
    if (K == 3) return fe_add<F>(fe_dbl<F>(a), a);
    if (K == 4) return fe_dbl<F>(fe_dbl<F>(a));
    if (K == 5) return fe_add<F>(fe_dbl<F>(fe_dbl<F>(a)), a);
    if (K == 8) return fe_dbl<F>(fe_dbl<F>(fe_dbl<F>(a)));
    fe<F> r = a;
    for (int i = 1; i < K; i++) r = fe_add<F>(r, a);
    return r;
}

// ---------------------------------------------------------------- parameter sets
#define VK_LIMBS(...)                                  \
    {                                                  \
        constexpr uint32_t v[] = {__VA_ARGS__};        \
        return v[i];                                   \
    }

struct BN254Fq {
    static constexpr int N = 8;
    static constexpr uint32_t inv = 0xe4866389u;
    VK_HD static constexpr uint32_t p(int i) VK_LIMBS(0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u, 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u)
    VK_HD static constexpr uint32_t r2(int i) VK_LIMBS(0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u, 0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u)
    VK_HD static constexpr uint32_t one(int i) VK_LIMBS(0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u, 0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u)
};
struct BN254Fr {
    static constexpr int N = 8;
    static constexpr int BITS = 254;
    static constexpr uint32_t inv = 0xefffffffu;
    VK_HD static constexpr uint32_t p(int i) VK_LIMBS(0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u, 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u)
    VK_HD static constexpr uint32_t r2(int i) VK_LIMBS(0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u, 0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u)
    VK_HD static constexpr uint32_t one(int i) VK_LIMBS(0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u, 0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u)
};
struct BLS381Fq {
    static constexpr int N = 12;
    static constexpr uint32_t inv = 0xfffcfffdu;
    VK_HD static constexpr uint32_t p(int i) VK_LIMBS(0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau)
    VK_HD static constexpr uint32_t r2(int i) VK_LIMBS(0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u, 0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u, 0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u)
    VK_HD static constexpr uint32_t one(int i) VK_LIMBS(0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu, 0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u, 0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u)
};
// BLS12-381 Fr == Bandersnatch base field
struct BLS381Fr {
    static constexpr int N = 8;
    static constexpr int BITS = 255;
    static constexpr uint32_t inv = 0xffffffffu;
    VK_HD static constexpr uint32_t p(int i) VK_LIMBS(0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u, 0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u)
    VK_HD static constexpr uint32_t r2(int i) VK_LIMBS(0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu, 0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u)
    VK_HD static constexpr uint32_t one(int i) VK_LIMBS(0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau, 0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u)
};
struct BandFr {
    static constexpr int N = 8;
    static constexpr int BITS = 253;
    static constexpr uint32_t inv = 0x5cc063dfu;
    VK_HD static constexpr uint32_t p(int i) VK_LIMBS(0x2876e7e1u, 0x74fd06b5u, 0x74190471u, 0xff8f8700u, 0x02687600u, 0x0cce7602u, 0xca675f52u, 0x1cfb69d4u)
    VK_HD static constexpr uint32_t r2(int i) VK_LIMBS(0x58db47cbu, 0xdbb4f5d6u, 0x7fecb938u, 0x40fa7ca2u, 0xc0055ceau, 0xaa9e6daeu, 0xb14aec7du, 0x0ae793ddu)
    VK_HD static constexpr uint32_t one(int i) VK_LIMBS(0xbc48c0f8u, 0x5817ca56u, 0x5f37dc74u, 0x0383c7fcu, 0xecbc4ff8u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u)
};
#undef VK_LIMBS

}  // namespace vk
