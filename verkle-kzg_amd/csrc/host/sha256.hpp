// SHA-256 (FIPS 180-4), host only. Used by the Fiat-Shamir transcript
// (reference transcript.rs:28-62 via DefaultFieldHasher<Sha256>) and the IPA CRS
// generator (ipa_point_generator.rs:96-108).
#pragma once
#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace vk {

static const uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// x86 SHA extensions (SHA-NI): 4 rounds per sha256rnds2 pair, message schedule by
// sha256msg1/msg2. Used when the host CPU has them (the multiproof transcript hashes ~5 MB at
// Q = 2^16 -- 4x faster than the portable rounds); same digest, checked in tests/test_abi.py.
__attribute__((target("sha,sse4.1"))) static inline void sha256_blocks_shani(uint32_t st[8], const uint8_t* data,
                                                                             size_t nblocks) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i TMP = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[0]));
    __m128i S1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[4]));
    TMP = _mm_shuffle_epi32(TMP, 0xB1);
    S1 = _mm_shuffle_epi32(S1, 0x1B);
    __m128i S0 = _mm_alignr_epi8(TMP, S1, 8);
    S1 = _mm_blend_epi16(S1, TMP, 0xF0);
    while (nblocks--) {
        const __m128i A0 = S0, C0 = S1;
        __m128i M[4];
        // fully unrolled (M[] stays in registers): without the pragma, hipcc's host pass kept the
        // 16 groups as a loop over a stack array -- 2x slower on the multiproof transcript
#pragma unroll
        for (int k = 0; k < 4; k++)
            M[k] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * k)), MASK);
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const __m128i cur = M[g & 3];
            __m128i MSG = _mm_add_epi32(cur, _mm_loadu_si128(reinterpret_cast<const __m128i*>(&kSha256K[4 * g])));
            S1 = _mm_sha256rnds2_epu32(S1, S0, MSG);
            if (g >= 3 && g <= 14) {
                __m128i& nx = M[(g + 1) & 3];
                nx = _mm_add_epi32(nx, _mm_alignr_epi8(cur, M[(g + 3) & 3], 4));
                nx = _mm_sha256msg2_epu32(nx, cur);
            }
            MSG = _mm_shuffle_epi32(MSG, 0x0E);
            S0 = _mm_sha256rnds2_epu32(S0, S1, MSG);
            if (g >= 1 && g <= 12) M[(g + 3) & 3] = _mm_sha256msg1_epu32(M[(g + 3) & 3], cur);
        }
        S0 = _mm_add_epi32(S0, A0);
        S1 = _mm_add_epi32(S1, C0);
        data += 64;
    }
    TMP = _mm_shuffle_epi32(S0, 0x1B);
    S1 = _mm_shuffle_epi32(S1, 0xB1);
    S0 = _mm_blend_epi16(TMP, S1, 0xF0);
    S1 = _mm_alignr_epi8(S1, TMP, 8);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[0]), S0);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[4]), S1);
}

inline bool sha256_have_shani() {
    static const int have = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") ? 1 : 0;
    return have != 0;
}

class Sha256 {
   public:
    Sha256() { reset(); }
    void reset() {
        static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                       0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
        memcpy(h_, iv, sizeof h_);
        len_ = 0;
        nbuf_ = 0;
    }
    void update(const void* data, size_t n) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        len_ += n;
        while (n > 0) {
            if (nbuf_ == 0 && n >= 64) {  // whole blocks straight from the input
                size_t nb = n / 64;
                blocks(p, nb);
                p += nb * 64;
                n -= nb * 64;
                continue;
            }
            size_t take = 64 - nbuf_;
            if (take > n) take = n;
            memcpy(buf_ + nbuf_, p, take);
            nbuf_ += take;
            p += take;
            n -= take;
            if (nbuf_ == 64) {
                blocks(buf_, 1);
                nbuf_ = 0;
            }
        }
    }
    void final(uint8_t out[32]) {
        uint64_t bits = len_ * 8;
        uint8_t pad = 0x80;
        update(&pad, 1);
        uint8_t z = 0;
        while (nbuf_ != 56) update(&z, 1);
        uint8_t lb[8];
        for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(lb, 8);
        for (int i = 0; i < 8; i++) {
            out[4 * i] = (uint8_t)(h_[i] >> 24);
            out[4 * i + 1] = (uint8_t)(h_[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h_[i] >> 8);
            out[4 * i + 3] = (uint8_t)h_[i];
        }
        reset();
    }

    // force the portable rounds (tests compare both paths)
    bool portable = false;

   private:
    void blocks(const uint8_t* b, size_t nb) {
        if (!portable && sha256_have_shani()) {
            sha256_blocks_shani(h_, b, nb);
            return;
        }
        for (size_t i = 0; i < nb; i++) block(b + 64 * i);
    }
    static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t* b) {
        const uint32_t* K = kSha256K;
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h_[0], bb = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6], h = h_[7];
        for (int i = 0; i < 64; i++) {
            uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = h + S1 + ch + K[i] + w[i];
            uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
            uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
            uint32_t t2 = S0 + mj;
            h = g;
            g = f;
            f = e;
            e = d + t1;
            d = c;
            c = bb;
            bb = a;
            a = t1 + t2;
        }
        h_[0] += a; h_[1] += bb; h_[2] += c; h_[3] += d;
        h_[4] += e; h_[5] += f; h_[6] += g; h_[7] += h;
    }
    uint32_t h_[8];
    uint64_t len_;
    uint8_t buf_[64];
    size_t nbuf_;
};

}  // namespace vk
