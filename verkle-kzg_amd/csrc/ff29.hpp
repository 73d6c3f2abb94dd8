// Radix-2^29 Montgomery field arithmetic (probe). Elements are L limbs of 29 bits in u32
// (top limb may carry a few extra bits); R' = 2^(29 L). A row of the CIOS multiply adds
// 2L 58-bit products into 64-bit column accumulators, so no 32-bit carry chains are needed:
// every product is one v_mad_u64_u32 with a 64-bit addend.
#pragma once
#include <stdint.h>

namespace vk {

struct Q29 {  // BLS12-381 Fq
    static constexpr int L = 14;
    static constexpr uint32_t inv = 0x1ffcfffdu;
    __host__ __device__ static constexpr uint32_t p(int j) {
        constexpr uint32_t v[L] = {0x1fffaaabu, 0xff7ffffu,  0x14ffffeeu, 0x17fffd62u, 0xf6241eau,
                                   0x9507b58u,  0xafd9cc3u,  0x109e70a2u, 0x1764774bu, 0x121a5d66u,
                                   0x12c6e9edu, 0x12ffcd34u, 0x111ea3u,   0xdu};
        return v[j];
    }
};
struct R29 {  // BLS12-381 Fr (Bandersnatch base field)
    static constexpr int L = 9;
    static constexpr uint32_t inv = 0x1fffffffu;
    __host__ __device__ static constexpr uint32_t p(int j) {
        constexpr uint32_t v[L] = {0x1u, 0x1ffffff8u, 0x1f96ffbfu, 0x1b4805ffu, 0x1d80553bu,
                                   0xc0404d0u, 0x1520cce7u, 0xa6533afu, 0x73eda7u};
        return v[j];
    }
};

template <class P>
struct f29 {
    uint32_t v[P::L];
};

template <class P>
__host__ __device__ __forceinline__ f29<P> mul29(const f29<P>& a, const f29<P>& b) {
    constexpr int L = P::L;
    constexpr uint32_t MASK = (1u << 29) - 1;
    uint64_t t[L];
#pragma unroll
    for (int j = 0; j < L; j++) t[j] = (uint64_t)a.v[j] * b.v[0];
#pragma unroll
    for (int i = 0; i < L; i++) {
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < L; j++) t[j] += (uint64_t)a.v[j] * b.v[i];
        }
        const uint32_t m = ((uint32_t)t[0] * P::inv) & MASK;
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
        r.v[j] = (uint32_t)t[j] & MASK;
    }
    r.v[L - 1] = (uint32_t)t[L - 1];
    return r;
}

}  // namespace vk
