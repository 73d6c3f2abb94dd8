// Launchers of the latency-bound Pippenger tail kernels (msm_tail.hip).
#pragma once
#include "ctx.hpp"
#include "ec.hpp"

namespace vk {
// partial slots per (window, bit) sum of the bit-sum stage (K = 8 items per lane, 64 lanes)
inline uint32_t msm_bitsum_pw(uint32_t S) { return (S + 511) / 512; }
template <class C>
int msm_tail_fixup(vc_ctx* ctx, uint32_t T, const uint32_t* Lp, uint32_t M, typename C::Acc* buckets, const typename C::Acc* carry,
                   const uint8_t* through, const typename C::Acc* owner, const uint32_t* owner_b);
template <class C>
int msm_tail_reduce(vc_ctx* ctx, const typename C::Acc* buckets, const uint32_t* offsets, uint32_t NB, int W,
                    uint32_t Lseg, uint32_t S, uint32_t J, typename C::Acc* accs, typename C::Acc* Rs,
                    typename C::Acc* partial, typename C::Acc* out);
}  // namespace vk
