// Launchers of the latency-bound Pippenger tail kernels (msm_tail.hip).
#pragma once
#include "ctx.hpp"
#include "ec.hpp"

namespace vk {
// items per lane of the bit-sum stage: as many as keep >= 1024 waves (one per SIMD) busy,
// within [2, 8]: each wave also pays a 6-add butterfly, so K = 1 doubles the waves for one
// add less per lane (measured: 2-window slices of 2^20, K = 1 -> 2 cut the stage ~2x)
inline uint32_t msm_bitsum_k(uint32_t S, uint32_t W, uint32_t J) {
    const uint64_t items = (uint64_t)W * ((uint64_t)J * (S / 2) + S);
    uint64_t k = items / (1024ull * 64);
    return (uint32_t)(k < 2 ? 2 : (k > 8 ? 8 : k));
}
// partial slots per (window, bit) sum of the bit-sum stage (K items per lane, 64 lanes)
inline uint32_t msm_bitsum_pw(uint32_t S, uint32_t K) { return (S + 64 * K - 1) / (64 * K); }
template <class C>
int msm_tail_fixup(vc_ctx* ctx, uint32_t T, const uint32_t* Lp, uint32_t M, typename C::Acc* buckets,
                   typename C::Acc* carry, const uint8_t* through, const typename C::Acc* owner,
                   const uint32_t* owner_b, const uint32_t* d_chain_max);
template <class C>
int msm_tail_reduce(vc_ctx* ctx, const typename C::Acc* buckets, const uint32_t* offsets, uint32_t NB, int W,
                    uint32_t Lseg, uint32_t S, uint32_t J, typename C::Acc* accs, typename C::Acc* Rs,
                    typename C::Acc* partial, typename C::Acc* out);
}  // namespace vk
