// Variable-base Pippenger MSM for gfx950 -- the engine behind utils::inner_product
// (/root/reference/vector-commit/src/utils.rs:16-19) at large n (configs 2 and 4).
//
// Pipeline (all on the ctx stream, one host sync at the end):
//   k_msm_digits     scalar -> W signed c-bit digits (|d| <= 2^(c-1)), bucket histogram
//   hipcub scan      bucket counts -> bucket offsets (all windows concatenated)
//   k_msm_scatter    (w, i) -> sorted[offset[w,|d|] + k] = i | sign<<31  (counting sort)
//   k_msm_accumulate every thread sums exactly M consecutive sorted entries (mixed adds
//                    of affine bases gathered from HBM), writing complete buckets directly
//                    and bucket pieces that straddle a thread boundary to side slots
//   k_msm_fixup      owner thread of a straddling bucket folds the pieces
//   k_msm_reduce     per window, segments of Lseg buckets: running sums -> sum_b b*B_b
//   k_msm_winsum     per window, LDS tree over segments
//   host             Horner over windows (c doublings per window) -> projective result
// Load balance does not depend on the scalar distribution: the accumulate work per
// thread is fixed (M entries) even when every scalar hits one bucket.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "ec.hpp"
#include "msm_tail.hpp"

namespace vk {

constexpr uint32_t NONE = 0xffffffffu;

template <class Fr>
__device__ __forceinline__ fe<Fr> load_scalar(const uint32_t* __restrict__ sc, size_t i) {
    const uint4* p = reinterpret_cast<const uint4*>(sc + 8 * i);
    uint4 a = p[0], b = p[1];
    fe<Fr> s;
    s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
    s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
    return s;
}

// ------------------------------------------------------------------ digits + histogram
template <class Fr>
__global__ void __launch_bounds__(256) k_msm_digits(const uint32_t* __restrict__ sc,
                                                   const uint8_t* __restrict__ inf, uint32_t n,
                                                   int c, int W, int mont,
                                                   int32_t* __restrict__ digits,
                                                   uint32_t* __restrict__ counts, uint32_t NB) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe<Fr> s = load_scalar<Fr>(sc, i);
    if (mont) s = fe_from_mont<Fr>(s);
    bool skip = inf != nullptr && inf[i];
    const uint32_t mask = (1u << c) - 1, half = 1u << (c - 1);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
        uint32_t raw = (s.v[0] & mask) + carry;
        // s >>= c (c < 32)
#pragma unroll
        for (int k = 0; k < 7; k++) s.v[k] = (s.v[k] >> c) | (s.v[k + 1] << (32 - c));
        s.v[7] >>= c;
        int32_t d;
        if (raw > half) {
            d = (int32_t)raw - (int32_t)(1u << c);
            carry = 1;
        } else {
            d = (int32_t)raw;
            carry = 0;
        }
        if (skip) d = 0;
        digits[(size_t)w * n + i] = d;
        if (d != 0) atomicAdd(&counts[(size_t)w * NB + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
    }
}

__global__ void __launch_bounds__(256) k_msm_scatter(const int32_t* __restrict__ digits, uint32_t n,
                                                    int W, uint32_t NB,
                                                    uint32_t* __restrict__ cursor,
                                                    uint32_t* __restrict__ sorted) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // 4 windows at a time: issue the returning atomics back to back, then the stores
    for (int w0 = 0; w0 < W; w0 += 4) {
        int32_t d[4];
        uint32_t pos[4];
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = (w0 + k < W) ? digits[(size_t)(w0 + k) * n + i] : 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t b = (uint32_t)(d[k] < 0 ? -d[k] : d[k]) - 1;
            pos[k] = d[k] ? atomicAdd(&cursor[(size_t)(w0 + k) * NB + b], 1u) : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (d[k]) sorted[pos[k]] = i | (d[k] < 0 ? 0x80000000u : 0u);
    }
}

// ------------------------------------------------------------------ bucket accumulation
template <class C>
__global__ void __launch_bounds__(256) k_msm_accumulate(
    const typename C::Aff* __restrict__ bases, const uint32_t* __restrict__ sorted,
    const uint32_t* __restrict__ offsets, uint32_t NBtot, uint32_t k_begin, uint32_t L, uint32_t M,
    typename C::Acc* __restrict__ buckets, typename C::Acc* __restrict__ carry_in,
    uint8_t* __restrict__ through, typename C::Acc* __restrict__ owner_piece,
    uint32_t* __restrict__ owner_bucket) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t k = k_begin + t * M;  // this launch covers sorted entries [k_begin, L)
    if (k >= L) return;
    uint32_t e = min(k + M, L);
    owner_bucket[t] = NONE;
    through[t] = 0;
    // bucket b with offsets[b] <= k < offsets[b+1]
    uint32_t lo = 0, hi = NBtot;  // invariant offsets[lo] <= k < offsets[hi]
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (offsets[mid] <= k) lo = mid;
        else hi = mid;
    }
    uint32_t b = lo;
    uint32_t bend = offsets[b + 1];
    bool left_open = offsets[b] < k;
    Acc acc = C::zero();
    uint32_t idx = sorted[k];
    Aff P = bases[idx & 0x7fffffffu];
    while (true) {
        uint32_t cur = idx;
        Aff Q = P;
        if (k + 1 < e) {  // prefetch next base
            idx = sorted[k + 1];
            P = bases[idx & 0x7fffffffu];
        }
        acc = C::madd(acc, Q, (cur >> 31) != 0);
        k++;
        if (k == bend || k == e) {
            bool right_open = (k == e) && (bend > e);
            if (!left_open && !right_open) {
                buckets[b] = acc;
            } else if (left_open) {
                carry_in[t] = acc;
                through[t] = right_open ? 1 : 0;
            } else {
                owner_piece[t] = acc;
                owner_bucket[t] = b;
            }
            if (k == e) break;
            left_open = false;
            acc = C::zero();
            do {
                b++;
                bend = offsets[b + 1];
            } while (bend <= k);
        }
    }
}

// ------------------------------------------------------------------ host side
static int choose_window(size_t n) {
    if (n >= (1u << 19)) return 16;
    if (n >= (1u << 17)) return 15;
    if (n >= (1u << 15)) return 13;
    if (n >= (1u << 12)) return 11;
    if (n >= (1u << 9)) return 9;
    if (n >= 64) return 7;
    return 5;
}

template <class C, class Fr>
static int msm_run_t(vc_ctx* ctx, Table* t, size_t offset, const uint32_t* d_sc, size_t n,
                     int mont, uint32_t* out_acc) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    if (n == 0) {
        Acc z = C::zero();
        memcpy(out_acc, &z, sizeof(Acc));
        return VC_OK;
    }
    if (n >= 0x7fffffffu) return VC_E_INVALID;
    const int c = choose_window(n);
    const int W = (Fr::BITS + 1 + c - 1) / c;  // one spare bit absorbs the final carry
    const uint32_t NB = 1u << (c - 1);
    const uint32_t NBtot = NB * W;
    const uint32_t M = 32;                 // sorted entries per accumulate thread
    const uint32_t Lseg = NB >= 256 ? 8 : (NB >= 4 ? 2 : 1);
    const uint32_t S = NB / Lseg;  // power of two
    uint32_t J = 0;
    while ((1u << J) < S) J++;
    const size_t maxL = n * (size_t)W;
    const uint32_t Tmax = (uint32_t)((maxL + M - 1) / M);
    hipStream_t st = ctx->stream;

    VK_TRY(ctx->ws[WS_DIGITS].ensure(maxL * 4));
    VK_TRY(ctx->ws[WS_COUNTS].ensure((size_t)(NBtot + 1) * 4));
    VK_TRY(ctx->ws[WS_OFFSETS].ensure((size_t)(NBtot + 1) * 4));
    VK_TRY(ctx->ws[WS_CURSOR].ensure((size_t)(NBtot + 1) * 4));
    VK_TRY(ctx->ws[WS_SORTED].ensure(maxL * 4));
    VK_TRY(ctx->ws[WS_BUCKETS].ensure((size_t)NBtot * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_CARRY].ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_THROUGH].ensure((size_t)(Tmax + 8)));
    VK_TRY(ctx->ws[WS_OWNER].ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_OWNER_B].ensure((size_t)(Tmax + 8) * 4));
    VK_TRY(ctx->ws[WS_SEG].ensure((size_t)S * W * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_TREE].ensure((size_t)S * W * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_WIN].ensure((size_t)W * (J + 1) * msm_bitsum_pw(S) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_TAIL].ensure((size_t)W * (J + 1) * sizeof(Acc)));

    int32_t* digits = ctx->ws[WS_DIGITS].as<int32_t>();
    uint32_t* counts = ctx->ws[WS_COUNTS].as<uint32_t>();
    uint32_t* offsets = ctx->ws[WS_OFFSETS].as<uint32_t>();
    uint32_t* cursor = ctx->ws[WS_CURSOR].as<uint32_t>();
    uint32_t* sorted = ctx->ws[WS_SORTED].as<uint32_t>();
    Acc* buckets = ctx->ws[WS_BUCKETS].as<Acc>();
    Acc* carry = ctx->ws[WS_CARRY].as<Acc>();
    uint8_t* through = ctx->ws[WS_THROUGH].as<uint8_t>();
    Acc* owner = ctx->ws[WS_OWNER].as<Acc>();
    uint32_t* owner_b = ctx->ws[WS_OWNER_B].as<uint32_t>();
    Acc* seg = ctx->ws[WS_SEG].as<Acc>();
    Acc* rs = ctx->ws[WS_TREE].as<Acc>();
    Acc* part = ctx->ws[WS_WIN].as<Acc>();
    Acc* tail = ctx->ws[WS_TAIL].as<Acc>();

    const Aff* bases = t->bases.as<Aff>() + offset;
    const uint8_t* inf = t->inf.as<uint8_t>() + offset;

    VK_CHECK_HIP(hipMemsetAsync(counts, 0, (size_t)(NBtot + 1) * 4, st));
    const uint32_t nb = (uint32_t)((n + 255) / 256);
    VK_LAUNCH(ctx, "msm_digits", (k_msm_digits<Fr>), nb, 256, 0, d_sc, inf, (uint32_t)n, c, W, mont,
              digits, counts, NB);
    size_t tmp_bytes = 0;
    VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, offsets, NBtot + 1, st));
    VK_TRY(ctx->ws[WS_SCAN_TMP].ensure(tmp_bytes));
    {
        hipEvent_t ev = nullptr;
        if (ctx->timing) ctx->timer_begin("msm_scan", &ev);
        VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(ctx->ws[WS_SCAN_TMP].p, tmp_bytes, counts,
                                                      offsets, NBtot + 1, st));
        if (ctx->timing) ctx->timer_end("msm_scan", ev);
    }
    VK_CHECK_HIP(hipMemcpyAsync(cursor, offsets, (size_t)(NBtot + 1) * 4, hipMemcpyDeviceToDevice, st));
    VK_LAUNCH(ctx, "msm_scatter", k_msm_scatter, nb, 256, 0, digits, (uint32_t)n, W, NB, cursor,
              sorted);
    // total entries L = offsets[NBtot]
    uint32_t L = 0;
    VK_CHECK_HIP(hipMemcpyAsync(&L, offsets + NBtot, 4, hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));
    if (L > 0) {
        const uint32_t T = (L + M - 1) / M;
        VK_LAUNCH(ctx, "msm_accumulate", (k_msm_accumulate<C>), (T + 255) / 256, 256, 0, bases, sorted, offsets,
                  NBtot, 0u, L, M, buckets, carry, through, owner, owner_b);
        VK_TRY(msm_tail_fixup<C>(ctx, T, buckets, carry, through, owner, owner_b));
    }
    VK_TRY(msm_tail_reduce<C>(ctx, buckets, offsets, NB, W, Lseg, S, J, seg, rs, part, tail));
    std::vector<Acc> ht((size_t)W * (J + 1));
    VK_CHECK_HIP(hipMemcpyAsync(ht.data(), tail, ht.size() * sizeof(Acc), hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));
    // MSM = sum_w 2^(c w) (A_w + Lseg sum_j 2^j T_wj): Horner over bit positions (host, 64-bit limbs)
    int lg_seg = 0;
    while ((1u << lg_seg) < Lseg) lg_seg++;
    const int maxpos = c * (W - 1) + lg_seg + (int)J;
    std::vector<std::vector<int>> at(maxpos + 1);
    for (int w = 0; w < W; w++) {
        at[c * w].push_back(w * (int)(J + 1) + (int)J);
        for (uint32_t j = 0; j < J; j++) at[c * w + lg_seg + (int)j].push_back(w * (int)(J + 1) + (int)j);
    }
    Acc res = C::zero();
    for (int pos = maxpos; pos >= 0; pos--) {
        if (!C::is_zero(res)) res = C::dbl(res);
        for (int idx : at[pos]) res = C::add(res, ht[idx]);
    }
    memcpy(out_acc, &res, sizeof(Acc));
    return VC_OK;
}

int msm_run(vc_ctx* ctx, Table* t, size_t offset, const void* d_scalars, size_t n, int mont,
            uint32_t* out_acc) {
    const uint32_t* sc = reinterpret_cast<const uint32_t*>(d_scalars);
    switch (t->curve) {
        case VC_CURVE_BN254: return msm_run_t<BN254G1, BN254Fr>(ctx, t, offset, sc, n, mont, out_acc);
        case VC_CURVE_BLS12_381: return msm_run_t<BLS381G1, BLS381Fr>(ctx, t, offset, sc, n, mont, out_acc);
        case VC_CURVE_BANDERSNATCH: return msm_run_t<Bandersnatch, BandFr>(ctx, t, offset, sc, n, mont, out_acc);
    }
    return VC_E_INVALID;
}

}  // namespace vk
