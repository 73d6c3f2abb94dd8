// Host-side BN254 scalar/base-field helpers for the protocol layer (Montgomery fe<> from
// ff.hpp, compiled for the host). Canonical values cross the C ABI as 4 LE u64 limbs.
#pragma once
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../ec.hpp"

namespace vk {

using Fr = fe<BN254Fr>;
using Fq = fe<BN254Fq>;
using G1 = BN254G1;

template <class F>
inline fe<F> from_words(const uint64_t* w) {  // canonical words -> raw limbs (no conversion)
    fe<F> r;
    memcpy(r.v, w, F::N * 4);
    return r;
}
template <class F>
inline void to_words(const fe<F>& a, uint64_t* w) {
    memcpy(w, a.v, F::N * 4);
}
template <class F>
inline fe<F> canon_to_mont(const uint64_t* w) {
    return fe_to_mont<F>(from_words<F>(w));
}
template <class F>
inline void mont_to_canon(const fe<F>& a, uint64_t* w) {
    to_words<F>(fe_from_mont<F>(a), w);
}
template <class F>
inline fe<F> mont_from_u64(uint64_t v) {
    fe<F> r = fe_zero<F>();
    r.v[0] = (uint32_t)v;
    r.v[1] = (uint32_t)(v >> 32);
    return fe_to_mont<F>(r);
}
// canonical compare a < b (limbs of equal length)
template <class F>
inline int canon_cmp(const fe<F>& a, const fe<F>& b) {
    for (int i = F::N - 1; i >= 0; i--) {
        if (a.v[i] < b.v[i]) return -1;
        if (a.v[i] > b.v[i]) return 1;
    }
    return 0;
}
// Montgomery a -> compare canonical values a <= b (b given as small integer)
inline bool fr_le_u64(const Fr& a_mont, uint64_t b) {
    Fr c = fe_from_mont<BN254Fr>(a_mont);
    for (int i = 2; i < 8; i++)
        if (c.v[i]) return false;
    uint64_t lo = (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
    return lo <= b;
}
inline uint64_t fr_low_u64(const Fr& a_mont) {  // utils::to_usize (utils.rs:72-74)
    Fr c = fe_from_mont<BN254Fr>(a_mont);
    return (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
}
template <class F>
inline fe<F> fe_pow_u64(fe<F> a, uint64_t e) {
    fe<F> r = fe_one<F>();
    while (e) {
        if (e & 1) r = fe_mul<F>(r, a);
        a = fe_sqr<F>(a);
        e >>= 1;
    }
    return r;
}
// a^e for a multi-limb exponent given as canonical fe words (LE u32)
template <class F, class E>
inline fe<F> fe_pow_fe(const fe<F>& a, const fe<E>& e) {
    fe<F> r = fe_one<F>();
    for (int i = E::N - 1; i >= 0; i--)
        for (int b = 31; b >= 0; b--) {
            r = fe_sqr<F>(r);
            if ((e.v[i] >> b) & 1) r = fe_mul<F>(r, a);
        }
    return r;
}

// integer (little-endian bytes, up to 64 bytes) mod p, returned in Montgomery form
template <class F>
inline fe<F> fe_from_le_bytes_mod(const uint8_t* b, size_t len) {
    // Horner over 32-bit words from the top: acc = acc * 2^32 + w (all Montgomery)
    fe<F> acc = fe_zero<F>();
    fe<F> base = mont_from_u64<F>(1ull << 32);
    size_t nw = (len + 3) / 4;
    for (size_t k = nw; k-- > 0;) {
        uint32_t w = 0;
        for (int j = 3; j >= 0; j--) {
            size_t idx = 4 * k + j;
            w = (w << 8) | (idx < len ? b[idx] : 0);
        }
        acc = fe_add<F>(fe_mul<F>(acc, base), mont_from_u64<F>(w));
    }
    return acc;
}
template <class F>
inline fe<F> fe_from_be_bytes_mod(const uint8_t* b, size_t len) {
    std::vector<uint8_t> le(b, b + len);
    for (size_t i = 0; i < len / 2; i++) std::swap(le[i], le[len - 1 - i]);
    return fe_from_le_bytes_mod<F>(le.data(), len);
}

// domain generator w_n = 5^((r-1)/n) (GeneralEvaluationDomain radix-2)
inline Fr bn254_group_gen_uncached(uint64_t n) {
    // (r - 1) / n for power-of-two n <= 2^28: shift r - 1 right by log2 n
    Fr e;
    for (int i = 0; i < 8; i++) e.v[i] = BN254Fr::p(i);
    e.v[0] -= 1;  // r is odd
    int lg = 0;
    while ((1ull << lg) < n) lg++;
    for (int s = 0; s < lg; s++) {
        for (int i = 0; i < 7; i++) e.v[i] = (e.v[i] >> 1) | (e.v[i + 1] << 31);
        e.v[7] >>= 1;
    }
    return fe_pow_fe<BN254Fr, BN254Fr>(mont_from_u64<BN254Fr>(5), e);
}
// the same, one exponentiation per domain size and process (~7 us each: every IPA prove / verify
// and multiproof finish asked for it)
inline Fr bn254_group_gen(uint64_t n) {
    int lg = 0;
    while ((1ull << lg) < n) lg++;
    if (lg > 28) return bn254_group_gen_uncached(n);
    static std::mutex mu;
    static Fr cache[29];
    static bool have[29] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (!have[lg]) {
        cache[lg] = bn254_group_gen_uncached(n);
        have[lg] = true;
    }
    return cache[lg];
}

}  // namespace vk
