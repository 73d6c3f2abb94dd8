// Launchers of the latency-bound Pippenger tail kernels (msm_tail.hip).
#pragma once
#include <stdlib.h>

#include <algorithm>

#include "ctx.hpp"
#include "ec.hpp"
#include "ec29.hpp"

namespace vk {
// items per lane of the bit-sum stage: the smallest K in [2, 32] whose busy waves (a wave per
// `lanes` K items of each of the W (J + 1) sums) fit one wave per SIMD (1024): a wave costs K +
// log2(lanes) serial adds (its butterfly included) and a SIMD's second wave doubles its time, so
// fewer, longer waves win until every SIMD has one (measured: 1192 busy waves at K = 7 took 2x the
// 960 of K = 8 on a GLV 2^20 MSM). lanes = logical lanes per wave (64; 16 for quads of the
// cooperative add, SW29::add_quad -- not used here: with every SIMD busy the stage is issue-bound,
// and quads' 2.1x shorter adds lose to their 4x fewer lanes)
inline uint32_t msm_bitsum_k(uint32_t S, uint32_t W, uint32_t J, uint32_t lanes = 64, uint32_t nU = 1) {
    for (uint32_t k = 2; k < 32; k++) {
        const uint64_t per = (uint64_t)lanes * k;
        const uint64_t busy = (uint64_t)W * ((uint64_t)J * ((S / 2 + per - 1) / per) + nU * ((S + per - 1) / per));
        if (busy <= 1024) return k;
    }
    return 32;
}
// waves (= partial slots) of one bit-stage sum over `items` items (K per logical lane)
inline uint32_t msm_bitsum_pw(uint32_t items, uint32_t K, uint32_t lanes = 64) {
    return (items + lanes * K - 1) / (lanes * K);
}
// Geometry of the bit stage. Bit form (h = 0): J sums T_j over S/2 items each (nb1 waves per
// sum) + nU sums U over S items (nb2 waves). Marginal form (h > 0, J >= 12): with s = G hi + lo
// (G = 2^h, Hn = 2^(J-h) high values) the stage instead makes the G column sums L_lo = sum_hi
// R_(G hi + lo) (Hn items) and the Hn row sums H_hi = sum_lo R_(G hi + lo) (G items), each by one
// wave, plus the U sums as before; the final stage then reads T_j = sum over lo with bit j of L_lo
// (j < h) or over hi with bit j - h of H_hi (j >= h) -- the same T_j from 2 S + ~S adds instead of
// J S / 2. per_w = partial slots per set (the WS_WIN layout).
// Row-derived total (urow, marginal form with nU = 1 and Lseg = 1, where U = sum_s R_s is the
// total of the row sums): no U waves; the final stage sums X = the H_hi of even hi (Hn / 2 items, as
// every T_j >= h) and the host adds T_h (the odd hi) to it. The column sums may then take pL waves
// each (Hn / pL items per wave, pL <= Hn / G, so the T_j < h sums still read <= Hn / 2 partials).
// Packed marginal waves (gL, gH > 1, several sets on quads): a wave makes gL column sums (or gH row
// sums) on 64 / g lanes each, so the column / row waves carry as many items per lane as the U waves
// and leave room for them in one round (the one-call KZG's two radix sets: 2 x (64 + 64 + 5 x 64)
// waves of 8 items instead of the bit form's 13). Partial slots stay one per sum (`slots` per set;
// per_w counts waves).
struct TailPlan {
    uint32_t h = 0, K = 0, nb1 = 0, nb2 = 0, per_w = 0, pL = 1, gL = 1, gH = 1, slots = 0;
    bool urow = false;
};
// Chosen by a cost model in full-add times: a wave costs its K serial adds plus the in-wave
// butterfly (7 quad adds ~ 3.5 full adds; 6 full adds without quads), and a stage whose waves fit
// one round (<= 1024, a wave per SIMD) takes its longest wave. The marginal form is taken only
// within one round and when shorter: measured on one MI355X, the 2^20 radix MSM's one set 10.5 ->
// 7.5 units, 0.165 -> 0.118 ms; the 8-way window slice 8.5 -> 7.5, 0.121 -> 0.107 ms. Stacked
// rounds do not follow the model (8 and 16 windows of 2^13 segments, 1744+ waves of 1-5 items
// per lane: 0.170 -> 0.198 and 0.139 -> 0.179 ms), so several sets keep the bit form.
inline TailPlan msm_tail_plan(uint32_t S, uint32_t W, uint32_t J, uint32_t nU, bool quad = true,
                              bool u_total = false) {
    static const int marg_env = getenv("VKZG_TAIL_MARGINAL") ? atoi(getenv("VKZG_TAIL_MARGINAL")) : 1;  // A/B probe
    static const int urow_env = getenv("VKZG_TAIL_UROW") ? atoi(getenv("VKZG_TAIL_UROW")) : 1;          // A/B probe
    const double bf = quad ? 3.5 : 6.0;
    TailPlan p;
    p.K = msm_bitsum_k(S, W, J, 64, nU);
    p.nb1 = msm_bitsum_pw(S / 2, p.K);
    p.nb2 = msm_bitsum_pw(S, p.K);
    p.per_w = J * p.nb1 + nU * p.nb2;
    p.slots = p.per_w;
    if (!(marg_env && J >= 12 && S == (1u << J))) return p;
    if ((uint64_t)W * p.per_w > 1024) return p;
    const uint32_t h = J / 2, G = 1u << h, Hn = 1u << (J - h), kl = Hn / 64;  // Hn >= G >= 64
    double best = p.K + bf;
    for (uint32_t k = kl; k <= 32; k++) {  // U sums: no fewer items per lane than the L waves
        const uint32_t nb = msm_bitsum_pw(S, k);
        if ((uint64_t)W * (G + Hn + nU * nb) > 1024) continue;
        const double t = k + bf;  // one round: the longest wave (k >= kl >= G / 64)
        if (t < best - 1e-9) {
            best = t;
            p.h = h;
            p.K = k;
            p.nb1 = 0;
            p.nb2 = nb;
            p.per_w = G + Hn + nU * nb;
            p.slots = p.per_w;
        }
    }
    static const int pack_env = getenv("VKZG_TAIL_PACK") ? atoi(getenv("VKZG_TAIL_PACK")) : 1;  // A/B probe
    if (pack_env && quad && W > 1) {  // several sets: pack 2-4 column / row sums per wave
        for (uint32_t k = kl; k <= 32; k++) {
            uint32_t gL = 1, gH = 1;
            while (gL < 16 && Hn * (gL * 2) / 64 <= k) gL *= 2;  // items per lane of a column wave <= k
            while (gH < 16 && G * (gH * 2) / 64 <= k) gH *= 2;
            if (gL == 1 && gH == 1) continue;  // the plain marginal form above
            const uint32_t nb = msm_bitsum_pw(S, k);
            const uint32_t waves = G / gL + Hn / gH + nU * nb;
            if ((uint64_t)W * waves > 1024) continue;
            const double t = k + bf;
            if (t < best - 1e-9) {
                best = t;
                p.h = h;
                p.K = k;
                p.nb1 = 0;
                p.nb2 = nb;
                p.gL = gL;
                p.gH = gH;
                p.per_w = waves;
                p.slots = G + Hn + nU * nb;
            }
        }
    }
    if (urow_env && u_total && nU == 1) {  // U from the row sums (u_total: the U items are the R_s)
        for (uint32_t pl = 1; pl <= Hn / G; pl *= 2) {
            if ((uint64_t)W * (G * pl + Hn) > 1024) break;
            const uint32_t k = std::max(Hn / (64 * pl), G / 64);
            const double t = k + bf;
            if (t < best + 1e-9) {  // ties too: no U waves, and X reads half the U sum's partials
                best = t;
                p.h = h;
                p.K = k;
                p.nb1 = 0;
                p.nb2 = 0;
                p.pL = pl;
                p.gL = p.gH = 1;
                p.urow = true;
                p.per_w = G * pl + Hn;
                p.slots = p.per_w;
            }
        }
    }
    return p;
}
// guarded = 0: read the longest chain back (host sync) and run exactly the rounds it needs;
// guarded = r > 0: r device-guarded rounds, no sync (chains up to 2^r threads; longer ones are
// finished by msm_tail_fixup_more once the caller has read chain_max with its results)
// raw radix-29 accumulator of curve C (what k_msm_accumulate writes)
template <class C>
using FAcc = typename Fast29<C>::type::Acc;
template <class C>
int msm_tail_fixup(vc_ctx* ctx, Lane L, uint32_t T, const uint32_t* Lp, uint32_t M, FAcc<C>* buckets, FAcc<C>* carry,
                   const uint8_t* through, const FAcc<C>* owner, const uint32_t* owner_b,
                   const uint32_t* d_chain_max, uint32_t guarded = 0);
template <class C>
int msm_tail_fixup_more(vc_ctx* ctx, Lane L, uint32_t T, const uint32_t* Lp, uint32_t M, FAcc<C>* buckets,
                        FAcc<C>* carry, const uint8_t* through, const FAcc<C>* owner, const uint32_t* owner_b,
                        uint32_t guarded, uint32_t Lmax);
template <class C>
int msm_tail_fixup_walk(vc_ctx* ctx, Lane L, const uint32_t* offsets, uint32_t NBtot, uint32_t M, FAcc<C>* buckets,
                        const FAcc<C>* carry, const FAcc<C>* owner, uint32_t limit, const uint32_t* owner_b = nullptr,
                        const uint8_t* through = nullptr, uint32_t Tmax = 0);
// guarded rounds for nv entries over NB buckets per window at M entries per thread: covers a
// bucket of 4x the mean load (the top window of a GLV split uses half its buckets: 2x)
inline uint32_t msm_fixup_guard_rounds(size_t nv, uint32_t NB, uint32_t M) {
    const size_t chain = 4 * nv / ((size_t)NB * M) + 2;
    uint32_t r = 1;
    while ((1ull << r) < chain && r < 6) r++;
    return r;
}
// Direct completion of the reduction: `out` is the device address of fine-grained page-locked
// memory, each final-stage block writes its point there, block 0 also copies *chain_src (the
// accumulate's longest chain) to *chain_dst, and then the block's flag takes `epoch` (system-scope
// release). The host polls the flags instead of a read-back copy and a stream wait.
struct TailDirect {
    uint32_t* flags = nullptr;
    uint32_t epoch = 0;
    const uint32_t* chain_src = nullptr;
    uint32_t* chain_dst = nullptr;
};
template <class C>
int msm_tail_reduce(vc_ctx* ctx, Lane L, const FAcc<C>* buckets, const uint32_t* offsets, uint32_t NB, int W,
                    uint32_t Lseg, uint32_t S, uint32_t J, FAcc<C>* accs, FAcc<C>* Rs, FAcc<C>* partial,
                    typename C::Acc* out, bool residue = false, const TailDirect* direct = nullptr);
}  // namespace vk
