// Variable-base Pippenger MSM for gfx950 -- the engine behind utils::inner_product
// (/root/reference/vector-commit/src/utils.rs:16-19) at large n (configs 2 and 4).
//
// Pipeline (all on the ctx stream, one host sync at the end):
//   k_sort_*         scalar -> W signed c-bit digits (|d| <= 2^(c-1)); two-pass LDS counting
//                    sort of the (window, bucket) keys: sorted[] = i | sign<<31 grouped by
//                    bucket, offsets[] = bucket starts (all windows concatenated)
//   k_msm_accumulate every thread sums exactly M consecutive sorted entries (mixed adds
//                    of affine bases gathered from HBM), writing complete buckets directly
//                    and bucket pieces that straddle a thread boundary to side slots
//   k_msm_fixup      owner thread of a straddling bucket folds the pieces
//   msm_tail.hip     segment sums, bit sums (window sum = sum_b b B_b without a serial
//                    running sum over all buckets), then host Horner over bit positions
// Load balance does not depend on the scalar distribution: the accumulate work per
// thread is fixed (M entries) even when every scalar hits one bucket.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <immintrin.h>
#include <cstdio>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "ctx.hpp"
#include "host/pool.hpp"
#include "ec.hpp"
#include "msm_tail.hpp"
#include "ec29.hpp"

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

// ------------------------------------------------------------------ bucket sort
// Signed c-bit digits of one scalar, least significant window first: d_w in (-2^(c-1), 2^(c-1)],
// carry into the next window; W windows have one spare bit, so the last carry is absorbed.
template <class Fr, class Fn>
__device__ __forceinline__ void for_each_digit(fe<Fr> s, int c, int W, Fn&& f) {
    const uint32_t mask = (1u << c) - 1, half = 1u << (c - 1);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
        uint32_t raw = (s.v[0] & mask) + carry;
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
        f(w, d);
    }
}

// Digits of a 4-limb magnitude (GLV halves, < 2^127), same recoding.
template <class Fn>
__device__ __forceinline__ void for_each_digit4(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, int c, int W,
                                                Fn&& f) {
    const uint32_t mask = (1u << c) - 1, half = 1u << (c - 1);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
        uint32_t raw = (s0 & mask) + carry;
        s0 = (s0 >> c) | (s1 << (32 - c));
        s1 = (s1 >> c) | (s2 << (32 - c));
        s2 = (s2 >> c) | (s3 << (32 - c));
        s3 >>= c;
        int32_t d;
        if (raw > half) {
            d = (int32_t)raw - (int32_t)(1u << c);
            carry = 1;
        } else {
            d = (int32_t)raw;
            carry = 0;
        }
        f(w, d);
    }
}

// Digit sources of the sort: entry i of the MSM -> its signed digits (nothing for an identity base).
// Every digit source maps its term i to the point index of the shared-window copies (Table::win,
// [w][2N] for a table of N points): the identity for a whole-table MSM; a point range [off, off + n)
// of the table (RadixDigits with half = n, gap = N - n) puts k1 term i < n at off + i and k2 term
// n + j at N + off + j.
template <class Fr>
struct ScalarDigits {  // plain scalars, canonical or Montgomery
    const uint32_t* sc;
    const uint8_t* inf;
    int mont;
    __device__ __forceinline__ uint32_t pt(uint32_t i) const { return i; }
    template <class Fn>
    __device__ __forceinline__ void operator()(uint32_t i, int c, int W, Fn&& f) const {
        if (inf != nullptr && inf[i]) return;
        fe<Fr> s = load_scalar<Fr>(sc, i);
        if (mont) s = fe_from_mont<Fr>(s);
        for_each_digit<Fr>(s, c, W, f);
    }
};
// GLV halves (k_glv_split): entry i < n is k1 of scalar i against P_i, entry n + i is k2 against
// phi(P_i); magnitude in bits 0..126, sign in bit 127 (a negative half negates every digit).
// Shared windows with a short top window (tw >= 0): its digits are scaled by 2^ts -- the window
// copy of that window holds 2^(c tw - ts) P -- so they spread over the whole bucket range
// instead of piling into the lowest 2^-ts of it.
struct GlvDigits {
    const uint4* k;
    const uint8_t* inf;
    uint32_t n;
    int tw = -1, ts = 0;
    __device__ __forceinline__ uint32_t pt(uint32_t i) const { return i; }
    template <class Fn>
    __device__ __forceinline__ void operator()(uint32_t i, int c, int W, Fn&& f) const {
        if (inf != nullptr && inf[i < n ? i : i - n]) return;
        const uint4 v = k[i];
        const bool neg = (v.w >> 31) != 0;
        for_each_digit4(v.x, v.y, v.z, v.w & 0x7fffffffu, c, W, [&](int w, int32_t d) {
            if (w == tw) d *= (1 << ts);
            f(w, neg ? -d : d);
        });
    }
};

// Radix-B digits made by k_glv_radix ([W][nv] signed, zero for identity bases): entry i of the
// (2n-term) MSM has digit dig[w * nv + i] in window w.
struct RadixDigits {
    const int32_t* dig;
    uint32_t nv;
    int w0 = 0;  // first window read (a per-set coarse pass of several bucket sets starts at its set)
    uint32_t off = 0, half = 0xffffffffu, gap = 0;  // point range of the table (see above)
    __device__ __forceinline__ uint32_t pt(uint32_t i) const { return i + off + (i >= half ? gap : 0u); }
    template <class Fn>
    __device__ __forceinline__ void operator()(uint32_t i, int, int W, Fn&& f) const {
        for (int w = w0; w < W; w++) f(w, dig[(size_t)w * nv + i]);
    }
};

// Two-pass MSD counting sort of the n*W (window, bucket) keys, all in LDS -- no global atomics
// (global atomics execute memory-side on CDNA4, ~26 G/s for scattered words, which made the
// one-pass global-histogram sort cost 2.2 ms at 2^20 x 16 windows).
//   coarse bin g = w * NBC + (b >> FB)          (NBC = NB >> FB coarse bins per window)
//   k_sort_hist     block = CHUNK entries: LDS histogram of coarse bins -> counts[g][block]
//   hipcub scan     counts -> base[g][block] (global position of the block's run in bin g)
//   k_sort_coarse   same digits again, LDS cursors from base: tmp[pos] = fine<<32 | i | sign<<31
//   k_sort_fine     block = coarse bin: LDS histogram of the 2^FB fine buckets -> bucket
//                   offsets (written directly), then scatter into sorted[]
// Order inside a bucket is arbitrary (EC addition is commutative and exact).
// Shared windows (stride != 0): every window's digits go to ONE set of buckets and the entry
// names the point 2^(c w) P_i by its index w * stride + i in the window copies (Table::win).
#ifndef VK_SORT_CHUNK
#define VK_SORT_CHUNK 1024
#endif
constexpr uint32_t SORT_CHUNK = VK_SORT_CHUNK;

// XCD-aware run order: blocks are dispatched round-robin over the 8 XCDs (block b on XCD b % 8),
// each with its own L2. A block's run inside every coarse bin sits at its slot in this order, so
// the runs of one XCD's blocks are adjacent and the partial-line writes of the scatter merge in
// ONE L2 instead of being written back as masked partial lines by several.
__device__ __forceinline__ uint32_t sort_slot(uint32_t b, uint32_t nblk) {
    const uint32_t q = nblk / 8, rem = nblk % 8, x = b % 8;
    return x * q + min(x, rem) + b / 8;
}

template <class Src>
__global__ void __launch_bounds__(1024) k_sort_hist(Src src, uint32_t n, int c, int wb, int we, uint32_t FB,
                                                   uint32_t NBC, uint32_t nblk, uint32_t stride, uint32_t wps,
                                                   uint32_t chunk, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t hist[];
    // shared windows: windows [s wps, (s + 1) wps) fill bucket set s (several MSMs over one table)
    const uint32_t bins = (stride ? ((uint32_t)we + wps - 1) / wps : (uint32_t)(we - wb)) * NBC;
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const uint32_t lo = blockIdx.x * chunk, hi = min(lo + chunk, n);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        src(i, c, we, [&](int w, int32_t d) {
            if (d != 0 && w >= wb)
                atomicAdd(&hist[(stride ? (uint32_t)w / wps : (uint32_t)(w - wb)) * NBC +
                                (((uint32_t)(d < 0 ? -d : d) - 1) >> FB)],
                          1u);
        });
    }
    __syncthreads();
    const uint32_t slot = sort_slot(blockIdx.x, nblk);
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) counts[(size_t)k * nblk + slot] = hist[k];
    if (blockIdx.x == 0 && threadIdx.x == 0) counts[(size_t)bins * nblk] = 0;  // the scan's terminal slot
}

// Coarse entries: u64 = fine << 32 | e | sign << 31, or -- when e < 2^(31 - FB), e.g. the
// shared-window 2^20 MSM (e < 2^24, FB = 5) -- u32 = fine << (31 - FB) | e | sign << 31, which
// halves the scatter's and the fine pass's traffic.
template <class T>
__device__ __forceinline__ T sort_pack(uint32_t fine, uint32_t e, bool neg, uint32_t FB) {
    if constexpr (sizeof(T) == 8) return ((uint64_t)fine << 32) | e | (neg ? 0x80000000u : 0u);
    else return (fine << (31 - FB)) | e | (neg ? 0x80000000u : 0u);
}
template <class T>
__device__ __forceinline__ uint32_t sort_fine_of(T x, uint32_t FB) {
    if constexpr (sizeof(T) == 8) return (uint32_t)(x >> 32);
    else return (x & 0x7fffffffu) >> (31 - FB);
}
template <class T>
__device__ __forceinline__ uint32_t sort_entry_of(T x, uint32_t FB) {
    if constexpr (sizeof(T) == 8) return (uint32_t)x;
    else return x & (0x80000000u | ((1u << (31 - FB)) - 1));
}

template <class Src, class T>
__global__ void __launch_bounds__(1024) k_sort_coarse(Src src, uint32_t n, int c, int wb, int we, uint32_t FB,
                                                     uint32_t NBC, uint32_t nblk, uint32_t stride, uint32_t wps,
                                                     uint32_t chunk, const uint32_t* __restrict__ base,
                                                     T* __restrict__ tmp) {
    extern __shared__ uint32_t cur[];
    const uint32_t bins = (stride ? ((uint32_t)we + wps - 1) / wps : (uint32_t)(we - wb)) * NBC;
    const uint32_t slot = sort_slot(blockIdx.x, nblk);
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) cur[k] = base[(size_t)k * nblk + slot];
    __syncthreads();
    const uint32_t fmask = (1u << FB) - 1;
    const uint32_t lo = blockIdx.x * chunk, hi = min(lo + chunk, n);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        src(i, c, we, [&](int w, int32_t d) {
            if (d != 0 && w >= wb) {
                uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
                uint32_t pos = atomicAdd(&cur[(stride ? (uint32_t)w / wps : (uint32_t)(w - wb)) * NBC + (b >> FB)], 1u);
                const uint32_t e = stride ? src.pt(i) + ((uint32_t)w % wps) * stride : i;
                tmp[pos] = sort_pack<T>(b & fmask, e, d < 0, FB);
            }
        });
    }
}

// Staged coarse scatter over precomputed radix digits (RadixDigits, narrow entries): the block's
// entries are counting-sorted by coarse bin in LDS (local offsets from its own per-bin counts,
// written by k_sort_hist), then every bin's run is written in one burst by one wave. The direct
// scatter wrote each run one 4-B entry at a time over the block's whole life; with 1280 bins x 32
// blocks per XCD of open runs the partly written lines left L2 repeatedly (PMC WRITE_SIZE ~6x
// the entries). LDS: 2 bins + 1 + chunk * we words (<= 160 KB: chunk 4096 at 7 windows).
template <class Src>
__global__ void __launch_bounds__(1024) k_sort_coarse_st(Src src, uint32_t n, int c, int wb, int we, uint32_t FB,
                                                        uint32_t NBC, uint32_t nblk, uint32_t stride, uint32_t wps,
                                                        uint32_t chunk, const uint32_t* __restrict__ counts,
                                                        const uint32_t* __restrict__ base,
                                                        uint32_t* __restrict__ tmp, uint32_t bin0, uint32_t bins) {
    extern __shared__ uint32_t sm[];
    __shared__ uint32_t part[1024];
    // this launch's coarse bins [bin0, bin0 + bins): all of them, or one bucket set's (windows
    // [wb, we) of a several-set sort, one launch per set so a block's entries fit LDS)
    uint32_t* loff = sm;             // bins + 1 local run starts
    uint32_t* lcur = sm + bins + 1;  // bins cursors
    uint32_t* stage = lcur + bins;   // the block's entries, bin-major
    const uint32_t t = threadIdx.x, slot = sort_slot(blockIdx.x, nblk);
    // local exclusive scan of the block's per-bin counts: ceil(bins / 1024) bins per thread
    const uint32_t per = (bins + blockDim.x - 1) / blockDim.x, b0 = t * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < bins) s += counts[(size_t)(bin0 + b0 + k) * nblk + slot];
    part[t] = s;
    __syncthreads();
    for (uint32_t o = 1; o < blockDim.x; o <<= 1) {
        const uint32_t a = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += a;
        __syncthreads();
    }
    uint32_t run = part[t] - s;  // exclusive prefix of this thread's first bin
    for (uint32_t k = 0; k < per; k++)
        if (b0 + k < bins) {
            loff[b0 + k] = run;
            lcur[b0 + k] = run;
            run += counts[(size_t)(bin0 + b0 + k) * nblk + slot];
        }
    if (t == blockDim.x - 1) loff[bins] = part[t];
    __syncthreads();
    const uint32_t fmask = (1u << FB) - 1;
    const uint32_t lo = blockIdx.x * chunk, hi = min(lo + chunk, n);
    auto put = [&](uint32_t i, int w, int32_t d) {
        if (d != 0 && w >= wb) {
            const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
            const uint32_t p = atomicAdd(
                &lcur[(stride ? (uint32_t)w / wps : (uint32_t)(w - wb)) * NBC + (b >> FB) - bin0], 1u);
            stage[p] = sort_pack<uint32_t>(b & fmask, stride ? src.pt(i) + ((uint32_t)w % wps) * stride : i, d < 0, FB);
        }
    };
    if constexpr (std::is_same<Src, RadixDigits>::value) {
        // radix digits: the digits of PRE iterations (<= 8 windows each) loaded before their LDS
        // atomics (one load, one atomic at a time left the waves waiting on memory 71 % of their
        // cycles: profiles/r04/tail_pmc/sq_summary.txt)
        constexpr int PRE = 4, WMAX = 8;
        if (we - src.w0 <= WMAX) {
            for (uint32_t i0 = lo + t; i0 < hi; i0 += PRE * blockDim.x) {
                int32_t dg[PRE][WMAX];
#pragma unroll
                for (int k = 0; k < PRE; k++) {
                    const uint32_t i = i0 + (uint32_t)k * blockDim.x;
#pragma unroll
                    for (int j = 0; j < WMAX; j++)
                        dg[k][j] = (i < hi && src.w0 + j < we) ? src.dig[(size_t)(src.w0 + j) * src.nv + i] : 0;
                }
#pragma unroll
                for (int k = 0; k < PRE; k++) {
                    const uint32_t i = i0 + (uint32_t)k * blockDim.x;
                    if (i >= hi) break;
#pragma unroll
                    for (int j = 0; j < WMAX; j++)
                        if (src.w0 + j < we) put(i, src.w0 + j, dg[k][j]);
                }
            }
        } else {
            for (uint32_t i = lo + t; i < hi; i += blockDim.x) src(i, c, we, [&](int w, int32_t d) { put(i, w, d); });
        }
    } else {
        for (uint32_t i = lo + t; i < hi; i += blockDim.x) src(i, c, we, [&](int w, int32_t d) { put(i, w, d); });
    }
    __syncthreads();
    // every bin's run in one burst: 16 lanes per bin (runs are ~10-25 entries: a whole wave per bin
    // left most lanes idle), 4 bins per wave at a time
    const uint32_t grp = t >> 4, sub = t & 15, ngrp = blockDim.x >> 4;
    for (uint32_t g = grp; g < bins; g += ngrp) {
        const uint32_t l0 = loff[g], len = loff[g + 1] - l0;
        const uint32_t gb = base[(size_t)(bin0 + g) * nblk + slot];
        for (uint32_t j = sub; j < len; j += 16) tmp[gb + j] = stage[l0 + j];
    }
}

// one block per coarse bin; offsets[g * 2^FB + f] = start of fine bucket f of bin g. Block 0
// also clears the accumulate's chain_max word (no separate memset in the pipeline). Blocks of
// 256 or 1024 threads (large bins): the 256 fine counters are scanned by the first 256.
// cap > 0: a bin of at most cap entries is scattered into LDS (dynamic, cap words) and written
// out in one coalesced pass -- the direct scatter wrote each bucket's 4-B entries one at a time
// over the block's life, and the partly written lines left L2 several times (PMC WRITE_SIZE
// ~4x the entries); larger bins scatter directly.
template <class T>
__global__ void __launch_bounds__(1024) k_sort_fine(const T* __restrict__ tmp, const uint32_t* __restrict__ base,
                                                   uint32_t nblk, uint32_t bins, uint32_t FB,
                                                   uint32_t* __restrict__ offsets, uint32_t* __restrict__ sorted,
                                                   uint32_t* __restrict__ zero_word, uint32_t cap, uint32_t regs_ok) {
    __shared__ uint32_t h[256], x[256];
    extern __shared__ uint32_t stage[];
    const uint32_t g = blockIdx.x, F = 1u << FB, t = threadIdx.x;
    const bool cnt_lane = t < 256;
    if (zero_word != nullptr && g == 0 && t == 0) *zero_word = 0;
    const uint32_t start = base[(size_t)g * nblk];
    const uint32_t end = base[(size_t)(g + 1) * nblk];  // base has bins*nblk + 1 entries
    if (cnt_lane) h[t] = 0;
    __syncthreads();
    // a staged bin of at most RMAX entries per thread keeps its entries in registers from the
    // counting pass to the scatter: the bin is read from HBM once, not twice (uniform per block)
    constexpr uint32_t RMAX = 16;
    T er[RMAX];
    const bool regs = regs_ok != 0 && cap != 0 && end - start <= cap && end - start <= RMAX * blockDim.x;
    if (regs) {
#pragma unroll
        for (uint32_t k = 0; k < RMAX; k++) {
            const uint32_t p = start + t + k * blockDim.x;
            er[k] = p < end ? tmp[p] : T(0);
        }
#pragma unroll
        for (uint32_t k = 0; k < RMAX; k++)
            if (start + t + k * blockDim.x < end) atomicAdd(&h[sort_fine_of<T>(er[k], FB)], 1u);
    } else {  // RH loads in flight per thread before their counter atomics
        constexpr uint32_t RH = 4;
        for (uint32_t p0 = start + t; p0 < end; p0 += RH * blockDim.x) {
            T e[RH];
#pragma unroll
            for (uint32_t k = 0; k < RH; k++) {
                const uint32_t p = p0 + k * blockDim.x;
                e[k] = p < end ? tmp[p] : T(0);
            }
#pragma unroll
            for (uint32_t k = 0; k < RH; k++)
                if (p0 + k * blockDim.x < end) atomicAdd(&h[sort_fine_of<T>(e[k], FB)], 1u);
        }
    }
    __syncthreads();
    // inclusive Hillis-Steele scan over 256 counters
    const uint32_t v = cnt_lane ? h[t] : 0u;
    if (cnt_lane) x[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t a = (cnt_lane && t >= o) ? x[t - o] : 0u;
        __syncthreads();
        if (cnt_lane) x[t] += a;
        __syncthreads();
    }
    const uint32_t excl = cnt_lane ? x[t] - v : 0u;
    if (t < F) offsets[(size_t)g * F + t] = start + excl;
    if (g == bins - 1 && t == 0) offsets[(size_t)bins * F] = end;
    __syncthreads();
    if (cnt_lane) h[t] = excl;  // cursors
    __syncthreads();
    // the scatter RS entries at a time (loads, then LDS cursor atomics, then stores: RS atomics in
    // flight per thread)
    constexpr uint32_t RS = 4;
    if (regs) {
#pragma unroll
        for (uint32_t k = 0; k < RMAX; k++)
            if (start + t + k * blockDim.x < end) stage[atomicAdd(&h[sort_fine_of<T>(er[k], FB)], 1u)] = sort_entry_of<T>(er[k], FB);
        __syncthreads();
        for (uint32_t p = t; p < end - start; p += blockDim.x) sorted[start + p] = stage[p];
        return;
    }
    if (end - start <= cap) {  // uniform over the block
        for (uint32_t p0 = start + t; p0 < end; p0 += RS * blockDim.x) {
            T e[RS];
            uint32_t pos[RS];
#pragma unroll
            for (uint32_t k = 0; k < RS; k++) {
                const uint32_t p = p0 + k * blockDim.x;
                e[k] = p < end ? tmp[p] : T(0);
            }
#pragma unroll
            for (uint32_t k = 0; k < RS; k++)
                if (p0 + k * blockDim.x < end) pos[k] = atomicAdd(&h[sort_fine_of<T>(e[k], FB)], 1u);
#pragma unroll
            for (uint32_t k = 0; k < RS; k++)
                if (p0 + k * blockDim.x < end) stage[pos[k]] = sort_entry_of<T>(e[k], FB);
        }
        __syncthreads();
        for (uint32_t p = t; p < end - start; p += blockDim.x) sorted[start + p] = stage[p];
        return;
    }
    for (uint32_t p0 = start + t; p0 < end; p0 += RS * blockDim.x) {
        T e[RS];
        uint32_t pos[RS];
#pragma unroll
        for (uint32_t k = 0; k < RS; k++) {
            const uint32_t p = p0 + k * blockDim.x;
            e[k] = p < end ? tmp[p] : T(0);
        }
#pragma unroll
        for (uint32_t k = 0; k < RS; k++)
            if (p0 + k * blockDim.x < end) pos[k] = start + atomicAdd(&h[sort_fine_of<T>(e[k], FB)], 1u);
#pragma unroll
        for (uint32_t k = 0; k < RS; k++)
            if (p0 + k * blockDim.x < end) sorted[pos[k]] = sort_entry_of<T>(e[k], FB);
    }
}

// ------------------------------------------------------------------ bucket accumulation
// The bases / phi / fixed-base tables read here are in the packed-29 form (x R', ec29.hpp)
// and the adds run in radix-2^29 arithmetic. Buckets and pieces are stored raw (radix-29) for
// the fix-up and the reduction (msm_tail.hip), which run the same arithmetic; converting them
// to the ec.hpp form at the three store sites (4 multiplies each) put ~50 KB of rarely-run code
// into the loop and cost 7 % of the kernel.
// BT: the base entry type -- packed-29 C::Aff (tables), the limb form of the fixed-base tables
// the sparse commits read (ec29.hpp FbE: the limbs in a 128-B entry), or the signed limb form of the
// shared-window copies (SW29::AffN: x, y, -y -- the entry's sign picks the y to load)
template <class FC, class BT, class = void>
struct is_affn : std::false_type {};
template <class FC, class BT>
struct is_affn<FC, BT, std::void_t<typename FC::AffN>> : std::is_same<BT, typename FC::AffN> {};
template <class FC, class BT, class = void>
struct is_affp : std::false_type {};
template <class FC, class BT>
struct is_affp<FC, BT, std::void_t<typename FC::AffP>> : std::is_same<BT, typename FC::AffP> {};
// a fixed-base table entry (FbE: the limbs in .u, padded to a 128-B line)
template <class C, class BT>
struct is_fbe : std::is_same<BT, FbE<C>> {};

// straddle merge inside the accumulate (A/B knob VKZG_ACC_MERGE in a -DVKZG_ACC_MERGE_BUILD build;
// the default build leaves the code out: it grew the kernel to 237 VGPRs and 18,441 instructions).
// Measured slower: accumulate +0.087 ms, the remaining fix-up 0.083 -> 0.158 ms (profiles/r04/merge_ab/)
static uint32_t acc_merge() {
    static const uint32_t v = getenv("VKZG_ACC_MERGE") ? (uint32_t)atoi(getenv("VKZG_ACC_MERGE")) : 0u;
    return v;
}

// one lane's value from lane + 1 of the wave (word by word through ds_bpermute)
template <class T>
__device__ __forceinline__ T shfl_down1(const T& v) {
    static_assert(sizeof(T) % 4 == 0, "");
    constexpr int NW = (int)(sizeof(T) / 4);
    uint32_t w[NW];
    __builtin_memcpy(w, &v, sizeof w);
#pragma unroll
    for (int k = 0; k < NW; k++) w[k] = (uint32_t)__shfl_down((int)w[k], 1);
    T r;
    __builtin_memcpy(&r, w, sizeof w);
    return r;
}

// merge: the owner piece of a straddling bucket whose only carry piece is in the next lane of the
// same wave is added here, after the loop (one general add per lane, all lanes together), and its
// bucket written: owner_bucket[t] is cleared so the fix-up kernels skip it. Left for the fix-up:
// lane 63's straddles (the next lane is in another wave) and chains over three or more threads.
template <class C, class BT = typename C::Aff>
__global__ void __launch_bounds__(256) VK_ACC_OCC k_msm_accumulate(
    const BT* __restrict__ bases, const BT* __restrict__ phi, uint32_t nphi,
    const uint32_t* __restrict__ sorted, const uint32_t* __restrict__ offsets, uint32_t NBtot, uint32_t M,
    typename Fast29<C>::type::Acc* __restrict__ buckets, typename Fast29<C>::type::Acc* __restrict__ carry_in,
    uint8_t* __restrict__ through, typename Fast29<C>::type::Acc* __restrict__ owner_piece,
    uint32_t* __restrict__ owner_bucket, uint32_t* __restrict__ chain_max, uint32_t merge,
    unsigned long long* __restrict__ clk) {
    using FC = typename Fast29<C>::type;
    using Aff = BT;
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t L = offsets[NBtot];  // entry count, read on the device: no host round trip
    uint32_t k = t * M;                 // grid sized for the n*W upper bound
    if (k >= L) return;
    // clock stamp (timing passes only: clk is null otherwise): shader cycles and 100 MHz ticks
    const bool stamp = clk != nullptr && t == 0;
    if (stamp) {
        clk[0] = __builtin_amdgcn_s_memtime();
        clk[1] = __builtin_amdgcn_s_memrealtime();
    }
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
    typename FC::Acc acc = FC::zero();
    // entry j < nphi: bases[j]; j >= nphi: phi[j - nphi] (the GLV endomorphism images)
    auto base_of = [&](uint32_t j) -> const Aff* { return j < nphi ? bases + j : phi + (j - nphi); };
    constexpr bool SN = is_affn<FC, BT>::value;
    constexpr bool SP = is_affp<FC, BT>::value;  // pair layout: the sign picks the record
    constexpr bool FBE = is_fbe<C, BT>::value;   // fixed-base entries: the limbs, not the padding
    using Pre = std::conditional_t<SN || SP || FBE, typename FC::Aff, Aff>;  // the prefetched entry
    auto fetch = [&](uint32_t id) -> Pre {
        if constexpr (FBE) {
            return base_of(id & 0x7fffffffu)->u;
        } else if constexpr (SP) {
            const Aff* r = bases + 2 * (size_t)(id & 0x7fffffffu) + (id >> 31);
            typename FC::Aff a;
            a.x = r->x;
            a.y = r->y;
            return a;
        } else {
            const Aff* b = base_of(id & 0x7fffffffu);
            if constexpr (SN) {
                typename FC::Aff a;
                a.x = b->x;
                // y or -y through the address (a select of values would load both)
                a.y = *reinterpret_cast<const decltype(a.y)*>(reinterpret_cast<const char*>(&b->y) +
                                                              ((id >> 31) ? sizeof(a.y) : 0u));
                return a;
            } else {
                return *b;
            }
        }
    };
    uint32_t idx = sorted[k];
    Pre P = fetch(idx);
    uint32_t my_through = 0, own_b = NONE;  // for the merge after the loop
    while (true) {
        uint32_t cur = idx;
        typename FC::Aff Q;
        if constexpr (SN || SP || FBE) Q = P;
        else Q = FC::load(&P);
        if (k + 1 < e) {  // prefetch next base
            idx = sorted[k + 1];
            P = fetch(idx);
        }
        acc = FC::madd(acc, Q, !SN && !SP && (cur >> 31) != 0);
        k++;
        if (k == bend || k == e) {
            bool right_open = (k == e) && (bend > e);
            if (!left_open && !right_open) {
                buckets[b] = acc;
            } else if (left_open) {
                carry_in[t] = acc;
                my_through = right_open ? 2 : 1;
                through[t] = (uint8_t)my_through;  // 1: carry piece ending here, 2: bucket continues
                if (!right_open) {  // chain end: chain length = carry threads of this bucket
                    const uint32_t L = t - offsets[b] / M;
                    if (L >= 2) atomicMax(chain_max, L);
                }
            } else {
                owner_piece[t] = acc;
                owner_bucket[t] = b;
                own_b = b;  // acc keeps the owner piece: it is the thread's last bucket
            }
            if (k == e) break;
            left_open = false;
            acc = FC::zero();
            do {
                b++;
                bend = offsets[b + 1];
            } while (bend <= k);
        }
    }
    if (stamp) {
        clk[2] = __builtin_amdgcn_s_memtime();
        clk[3] = __builtin_amdgcn_s_memrealtime();
    }
#ifdef VKZG_ACC_MERGE_BUILD
    if (merge) {  // uniform
        // the next lane's carry piece (its own store, read back by the thread that wrote it)
        const typename FC::Acc mine = my_through == 1 ? carry_in[t] : FC::zero();
        const typename FC::Acc nxt = shfl_down1(mine);
        const uint32_t nth = (uint32_t)__shfl_down((int)my_through, 1);
        if (own_b != NONE && (threadIdx.x & 63u) != 63u && nth == 1) {
            buckets[own_b] = FC::add(acc, nxt);
            owner_bucket[t] = NONE;
        }
    }
#else
    (void)merge;
    (void)my_through;
    (void)own_b;
#endif
}

// radix-29 bucket accumulators -> ec.hpp form, non-empty buckets only (empty ones keep what the
// caller put there)
template <class C>
__global__ void __launch_bounds__(256) k_fast_store(const FAcc<C>* __restrict__ a, uint32_t n,
                                                   const uint32_t* __restrict__ offsets, typename C::Acc* __restrict__ o) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && offsets[i + 1] > offsets[i]) o[i] = Fast29<C>::type::store(a[i]);
}

// ec.hpp affine points -> packed-29 form (the tables the accumulate / commit loops read)
template <class C>
__global__ void __launch_bounds__(256) k_to_fast(const typename C::Aff* __restrict__ in, size_t n,
                                                typename C::Aff* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fast29<C>::type::pack_aff(in[i], out + i);
}
// ... or straight to radix-2^29 limbs (the shared-window copies: the accumulate reads them with
// no unpacking, 112 instead of 96 B per BLS12-381 point)
template <class C>
__global__ void __launch_bounds__(256) k_to_limbs(const typename C::Aff* __restrict__ in, size_t n,
                                                 typename Fast29<C>::type::Aff* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Aff packed;
    FC::pack_aff(in[i], &packed);
    out[i] = FC::load(&packed);
}

// ... and to the signed limb form (x, y, -y) of the shared-window copies
template <class C>
__global__ void __launch_bounds__(256) k_to_limbs_n(const typename C::Aff* __restrict__ in, size_t n,
                                                   typename Fast29<C>::type::AffN* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Aff a = in[i], packed;
    FC::pack_aff(a, &packed);
    const typename FC::Aff l = FC::load(&packed);
    a.y = fe_neg<typename C::F>(a.y);
    FC::pack_aff(a, &packed);
    typename FC::AffN o;
    o.x = l.x;
    o.y = l.y;
    o.ny = FC::load(&packed).y;
    out[i] = o;
}

// ... and to the pair layout (x, y) | (x, -y), one 128-B record each
template <class C>
__global__ void __launch_bounds__(256) k_to_limbs_p(const typename C::Aff* __restrict__ in, size_t n,
                                                   typename Fast29<C>::type::AffP* __restrict__ out) {
    using FC = typename Fast29<C>::type;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Aff a = in[i], packed;
    FC::pack_aff(a, &packed);
    const typename FC::Aff l = FC::load(&packed);
    a.y = fe_neg<typename C::F>(a.y);
    FC::pack_aff(a, &packed);
    typename FC::AffP o;
#pragma unroll
    for (int k = 0; k < FC::PADW; k++) o.pad[k] = 0;
    o.x = l.x;
    o.y = l.y;
    out[2 * i] = o;
    o.y = FC::load(&packed).y;
    out[2 * i + 1] = o;
}

// ------------------------------------------------------------------ GLV endomorphism (BLS12-381 G1)
// phi(x, y) = (beta x, y) acts on the prime-order subgroup as multiplication by
// lambda = z^2 - 1 (z = -0xd201000000010000), and r = lambda^2 + lambda + 1. A scalar splits as
// k = k1 + lambda k2 with |k1|, |k2| <= lambda/2 + 1 < 2^127, so an n-term MSM is a 2n-term MSM
// of 127-bit scalars over (P_i, phi(P_i)): the same number of accumulate entries (2n x 8
// windows instead of n x 16 at c = 16) but half the buckets, half the bucket reduction and
// half the Horner doublings. Used only when every base of the table is in the subgroup
// (checked once per table: phi^2(P) = -z^2 P, which non-subgroup points fail), so the result
// is the same group element as the reference's sum of k_i P_i for any input.
struct GlvK {
    uint64_t lam[2];
    uint64_t mu[3];  // floor(2^256 / lambda)
    uint64_t r[4];
};
constexpr size_t GLV_MIN_N = 4096;
constexpr int GLV_BITS = 128;  // |k1|, |k2| < 2^127, plus the recoding's spare bit

typedef unsigned __int128 u128;

// k = k1 + lambda k2 (k < 2^256, canonical or not): |k1| = rem (negative when nr), |k2| = q (nq)
__device__ __forceinline__ void glv_decompose(uint64_t s[4], const GlvK& K, u128& rem, bool& nr, u128& q, bool& nq) {
    // s mod r (inputs are < 2^256 < 3r)
    for (int rep = 0; rep < 2; rep++) {
        bool ge = true;
        for (int k = 3; k >= 0; k--)
            if (s[k] != K.r[k]) {
                ge = s[k] > K.r[k];
                break;
            }
        if (!ge) break;
        uint64_t br = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            u128 d = (u128)s[k] - K.r[k] - br;
            s[k] = (uint64_t)d;
            br = (uint64_t)(d >> 64) & 1;
        }
    }
    // q = floor(s mu / 2^256): floor(s / lambda) or up to 2 less
    uint64_t p[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < 4; a++) {
        uint64_t carry = 0;
#pragma unroll
        for (int b = 0; b < 3; b++) {
            u128 t = (u128)s[a] * K.mu[b] + p[a + b] + carry;
            p[a + b] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        p[a + 3] = carry;
    }
    q = ((u128)p[5] << 64) | p[4];
    const u128 lam = ((u128)K.lam[1] << 64) | K.lam[0];
    // rem = s - q lambda (< 3 lambda: 3 limbs)
    uint64_t ql[4] = {0, 0, 0, 0};
    const uint64_t qv[2] = {(uint64_t)q, (uint64_t)(q >> 64)};
#pragma unroll
    for (int a = 0; a < 2; a++) {
        uint64_t carry = 0;
#pragma unroll
        for (int b = 0; b < 2; b++) {
            u128 t = (u128)qv[a] * K.lam[b] + ql[a + b] + carry;
            ql[a + b] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        ql[a + 2] = carry;
    }
    uint64_t rm[3];
    {
        uint64_t br = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            u128 d = (u128)s[k] - ql[k] - br;
            rm[k] = (uint64_t)d;
            br = (uint64_t)(d >> 64) & 1;
        }
    }
    for (int it = 0; it < 4; it++) {  // at most 2 corrections
        const u128 lo = ((u128)rm[1] << 64) | rm[0];
        if (rm[2] == 0 && lo < lam) break;
        const u128 d = lo - lam;
        if (lo < lam) rm[2] -= 1;
        rm[0] = (uint64_t)d;
        rm[1] = (uint64_t)(d >> 64);
        q += 1;
    }
    rem = ((u128)rm[1] << 64) | rm[0];
    // balance: k = rem + lambda q with rem in [0, lambda), q in [0, lambda + 1]
    //   q > lambda/2:   (rem - 1) + lambda (q - lambda - 1)   (= k - r)
    //   rem > lambda/2: (rem - lambda) + lambda (q + 1)
    const u128 half = lam >> 1;
    nq = false;
    nr = false;
    if (q > half) {
        q = lam + 1 - q;  // magnitude of q - lambda - 1
        nq = true;
        if (rem == 0) {
            rem = 1;
            nr = true;
        } else {
            rem -= 1;
        }
    }
    if (!nr && rem > half) {
        rem = lam - rem;
        nr = true;
        if (!nq) {
            q += 1;
        } else if (q == 0) {
            q = 1;
            nq = false;
        } else {
            q -= 1;
        }
    }
}

template <class Fr>
__device__ __forceinline__ void glv_load(const uint32_t* __restrict__ sc, uint32_t i, int mont, uint64_t s[4]) {
    fe<Fr> f = load_scalar<Fr>(sc, i);
    if (mont) f = fe_from_mont<Fr>(f);
#pragma unroll
    for (int k = 0; k < 4; k++) s[k] = (uint64_t)f.v[2 * k] | ((uint64_t)f.v[2 * k + 1] << 32);
}

template <class Fr>
__global__ void __launch_bounds__(256) k_glv_split(const uint32_t* __restrict__ sc, uint32_t n, int mont, GlvK K,
                                                  uint4* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[4];
    glv_load<Fr>(sc, i, mont, s);
    u128 rem, q;
    bool nr, nq;
    glv_decompose(s, K, rem, nr, q, nq);
    out[i] = make_uint4((uint32_t)rem, (uint32_t)(rem >> 32), (uint32_t)(rem >> 64),
                        (uint32_t)(rem >> 96) | (nr ? 0x80000000u : 0u));
    out[n + i] = make_uint4((uint32_t)q, (uint32_t)(q >> 32), (uint32_t)(q >> 64),
                            (uint32_t)(q >> 96) | (nq ? 0x80000000u : 0u));
}

// Mixed-radix digits of a GLV half for the radix-B shared-window MSM (B = MUL 2^C0, not a power
// of two): |k| < 2^127 = sum_w d_w B^w with signed d_w in (-B/2, B/2] (carry recoding as
// for_each_digit), W digits (B^W / 2 > 2^127: the top digit is below B/2 and never carries).
// k mod B = (k mod 2^C0) + 2^C0 ((k >> C0) mod MUL); the division by MUL runs over the four
// 32-bit limbs from the top. A negative half negates every digit.
// (rem 2^32 + x) / MUL for rem < MUL, in 32-bit steps (2^32 = MUL Q + 1 for MUL | 2^32 - 1):
// x = MUL q0 + x0 with q0 by a multiply-high, then rem + x0 < 2 MUL carries at most one
template <uint32_t MUL>
__device__ __forceinline__ uint32_t div_step(uint32_t x, uint32_t& rem) {
    static_assert(MUL == 5 || MUL == 3, "2^32 = 1 mod MUL");
    constexpr uint32_t Q = (uint32_t)(0xffffffffull / MUL);  // (2^32 - 1) / MUL
    const uint32_t q0 = MUL == 5 ? __umulhi(x, 0xCCCCCCCDu) >> 2 : __umulhi(x, 0xAAAAAAABu) >> 1;
    const uint32_t t = rem + (x - q0 * MUL);
    const uint32_t ge = t >= MUL ? 1u : 0u;
    const uint32_t q = rem * Q + q0 + ge;
    rem = t - ge * MUL;
    return q;
}

template <uint32_t MUL, int C0, class Fn>
__device__ __forceinline__ void radix_digits(u128 k, bool neg, int W, Fn&& f) {
    constexpr uint32_t B = MUL << C0, H = B / 2, LO = (1u << C0) - 1;
    uint32_t x0 = (uint32_t)k, x1 = (uint32_t)(k >> 32), x2 = (uint32_t)(k >> 64), x3 = (uint32_t)(k >> 96);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
        const uint32_t lo = x0 & LO;
        x0 = (x0 >> C0) | (x1 << (32 - C0));
        x1 = (x1 >> C0) | (x2 << (32 - C0));
        x2 = (x2 >> C0) | (x3 << (32 - C0));
        x3 >>= C0;
        uint32_t rem = 0;
        x3 = div_step<MUL>(x3, rem);
        x2 = div_step<MUL>(x2, rem);
        x1 = div_step<MUL>(x1, rem);
        x0 = div_step<MUL>(x0, rem);
        const uint32_t raw = lo + (rem << C0) + carry;
        int32_t d;
        if (raw > H) {
            d = (int32_t)raw - (int32_t)B;
            carry = 1;
        } else {
            d = (int32_t)raw;
            carry = 0;
        }
        f(w, neg ? -d : d);
    }
}

// GLV split straight to radix-B digits: dig[w][i] (k1 of scalar i against P_i) and dig[w][n + i]
// (k2 against phi(P_i)); identity bases get zero digits (no entries)
template <class Fr, uint32_t MUL, int C0>
__global__ void __launch_bounds__(256) k_glv_radix(const uint32_t* __restrict__ sc, const uint8_t* __restrict__ inf,
                                                  uint32_t n, int mont, GlvK K, int W, int32_t* __restrict__ dig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t nv = 2 * (size_t)n;
    if (inf != nullptr && inf[i]) {
        for (int w = 0; w < W; w++) dig[(size_t)w * nv + i] = dig[(size_t)w * nv + n + i] = 0;
        return;
    }
    uint64_t s[4];
    glv_load<Fr>(sc, i, mont, s);
    u128 rem, q;
    bool nr, nq;
    glv_decompose(s, K, rem, nr, q, nq);
    radix_digits<MUL, C0>(rem, nr, W, [&](int w, int32_t d) { dig[(size_t)w * nv + i] = d; });
    radix_digits<MUL, C0>(q, nq, W, [&](int w, int32_t d) { dig[(size_t)w * nv + n + i] = d; });
}

// k_glv_radix fused with k_sort_hist for one shared bucket set (windows [0, W) into one set of
// m 2^(c-1) buckets): a block takes `chunk` scalars, i.e. the entries of sort blocks blockIdx.x
// (k1 terms, entries i) and n / chunk + blockIdx.x (k2 terms, entries n + i), and writes both
// blocks' coarse-bin counts where k_sort_hist would (n % chunk == 0). Saves the hist pass's
// re-read of the W x 2n digits and one launch. Several sets (several MSMs over one table): one
// launch per set, its coarse bins at [bin0, bin0 + NBC) of bins_total.
template <class Fr, uint32_t MUL, int C0>
__global__ void __launch_bounds__(1024) k_glv_radix_hist(const uint32_t* __restrict__ sc,
                                                        const uint8_t* __restrict__ inf, uint32_t n, int mont,
                                                        GlvK K, int W, int32_t* __restrict__ dig, uint32_t FB,
                                                        uint32_t NBC, uint32_t nblk, uint32_t chunk,
                                                        uint32_t* __restrict__ counts, uint32_t bin0,
                                                        uint32_t bins_total) {
    extern __shared__ uint32_t hist[];  // [2][NBC]: k1 block, k2 block
    for (uint32_t k = threadIdx.x; k < 2 * NBC; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const size_t nv = 2 * (size_t)n;
    const uint32_t lo = blockIdx.x * chunk, hi = lo + chunk;
    // a thread's scalars are loaded up front, PRE at a time (the loads of one scalar after the
    // previous one's digits left the waves waiting on memory 52 % of their cycles:
    // profiles/r04/tail_pmc/sq_summary.txt)
    constexpr int PRE = 4;
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += PRE * blockDim.x) {
        fe<Fr> f[PRE];
        bool skip[PRE];
#pragma unroll
        for (int k = 0; k < PRE; k++) {
            const uint32_t i = i0 + (uint32_t)k * blockDim.x;
            skip[k] = i >= hi || (inf != nullptr && inf[i]);
            f[k] = i < hi ? load_scalar<Fr>(sc, i) : fe_zero<Fr>();
        }
        // unrolled (no break): f[k] / skip[k] stay in registers -- a rolled loop indexed them
        // dynamically, i.e. through scratch memory
#pragma unroll
        for (int k = 0; k < PRE; k++) {
            const uint32_t i = i0 + (uint32_t)k * blockDim.x;
            if (i >= hi) continue;
            if (skip[k]) {
                for (int w = 0; w < W; w++) dig[(size_t)w * nv + i] = dig[(size_t)w * nv + n + i] = 0;
                continue;
            }
            if (mont) f[k] = fe_from_mont<Fr>(f[k]);
            uint64_t s[4];
#pragma unroll
            for (int j = 0; j < 4; j++) s[j] = (uint64_t)f[k].v[2 * j] | ((uint64_t)f[k].v[2 * j + 1] << 32);
            u128 rem, q;
            bool nr, nq;
            glv_decompose(s, K, rem, nr, q, nq);
            radix_digits<MUL, C0>(rem, nr, W, [&](int w, int32_t d) {
                dig[(size_t)w * nv + i] = d;
                if (d != 0) atomicAdd(&hist[((uint32_t)(d < 0 ? -d : d) - 1) >> FB], 1u);
            });
            radix_digits<MUL, C0>(q, nq, W, [&](int w, int32_t d) {
                dig[(size_t)w * nv + n + i] = d;
                if (d != 0) atomicAdd(&hist[NBC + (((uint32_t)(d < 0 ? -d : d) - 1) >> FB)], 1u);
            });
        }
    }
    __syncthreads();
    const uint32_t s1 = sort_slot(blockIdx.x, nblk), s2 = sort_slot(blockIdx.x + n / chunk, nblk);
    for (uint32_t k = threadIdx.x; k < NBC; k += blockDim.x) {
        counts[(size_t)(bin0 + k) * nblk + s1] = hist[k];
        counts[(size_t)(bin0 + k) * nblk + s2] = hist[NBC + k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) counts[(size_t)bins_total * nblk] = 0;  // the scan's terminal slot
}

template <class C>
__global__ void __launch_bounds__(256) k_glv_phi(const typename C::Aff* __restrict__ bases, uint32_t n,
                                                fe<typename C::F> beta, typename C::Aff* __restrict__ phi) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Aff p = bases[i];
    p.x = fe_mul<typename C::F>(p.x, beta);
    phi[i] = p;
}

// bad |= some base with phi^2(P) + z^2 P != 0 (phi^2 = (beta^2 x, y) has eigenvalue lambda^2 = -z^2)
template <class C>
__global__ void __launch_bounds__(256) k_glv_check(const typename C::Aff* __restrict__ bases,
                                                  const uint8_t* __restrict__ inf, uint32_t n,
                                                  fe<typename C::F> beta2, uint64_t z2lo, uint64_t z2hi,
                                                  uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || inf[i]) return;
    typename C::Aff p = bases[i];
    typename C::Acc acc = C::zero();
    for (int b = 127; b >= 0; b--) {
        acc = C::dbl(acc);
        const uint64_t w = b >= 64 ? z2hi : z2lo;
        if ((w >> (b & 63)) & 1) acc = C::madd(acc, p, false);
    }
    p.x = fe_mul<typename C::F>(p.x, beta2);
    acc = C::madd(acc, p, false);
    if (!C::is_zero(acc)) atomicOr(bad, 1u);
}

static GlvK glv_consts() {
    return GlvK{{0x00000000ffffffffull, 0xac45a4010001a402ull},
                {0x63f6e522f6cfee30ull, 0x7c6becf1e01faaddull, 0x1ull},
                {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull, 0x73eda753299d7d48ull}};
}
static const uint64_t GLV_BETA[6] = {0x8bfd00000000aaacull, 0x409427eb4f49fffdull, 0x897d29650fb85f9bull,
                                     0xaa0d857d89759ad4ull, 0xec02408663d4de85ull, 0x1a0111ea397fe699ull};
static const uint64_t GLV_BETA2[6] = {0x2e01fffffffefffeull, 0xde17d813620a0002ull, 0xddb3a93be6f89688ull,
                                      0xba69c6076a0f77eaull, 0x5f19672fdf76ce51ull, 0x0ull};
static fe<BLS381Fq> bls_fq_mont(const uint64_t* w) {
    fe<BLS381Fq> r;
    memcpy(r.v, w, sizeof(r.v));
    return fe_to_mont<BLS381Fq>(r);
}
static const uint64_t GLV_Z2[2] = {0x0000000100000000ull, 0xac45a4010001a402ull};  // z^2 = lambda + 1

// is every base of t in the prime-order subgroup? (checked once per table, cached)
static int glv_table_ok(vc_ctx* ctx, Table* t, bool* ok) {
    using C = BLS381G1;
    if (t->subgroup < 0) {
        VK_TRY(ctx->ws[WS_GLV_FLAG].ensure(4));
        uint32_t* d_bad = ctx->ws[WS_GLV_FLAG].as<uint32_t>();
        VK_CHECK_HIP(hipMemsetAsync(d_bad, 0, 4, ctx->stream));
        if (t->n > 0)
            VK_LAUNCH(ctx, "glv_check", (k_glv_check<C>), (t->n + 255) / 256, 256, 0, t->bases.as<C::Aff>(),
                      t->inf.as<uint8_t>(), (uint32_t)t->n, bls_fq_mont(GLV_BETA2), GLV_Z2[0], GLV_Z2[1],
                      d_bad);
        uint32_t bad = 0;
        VK_CHECK_HIP(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        t->subgroup = bad ? 0 : 1;
    }
    *ok = t->subgroup == 1;
    return VC_OK;
}

// the packed-29 copies of a table's bases (and of phi(bases) for GLV MSMs), made once
template <class C>
static int fast_tables(vc_ctx* ctx, Table* t, bool with_phi) {
    using Aff = typename C::Aff;
    const size_t need = (with_phi ? 2 : 1) * std::max<size_t>(t->n, 1) * sizeof(Aff);
    if (t->fast.cap < need) {
        t->fast_ok = t->phi_ok = 0;
        t->fast.release();
        VK_TRY(t->fast.ensure(need));
    }
    if (!t->fast_ok && t->n > 0) {
        VK_LAUNCH(ctx, "to_fast", (k_to_fast<C>), (t->n + 255) / 256, 256, 0, t->bases.as<Aff>(), t->n,
                  t->fast.as<Aff>());
        t->fast_ok = 1;
    }
    if constexpr (std::is_same<C, BLS381G1>::value) {
        if (with_phi && !t->phi_ok && t->n > 0) {
            DevBuf phi;
            VK_TRY(phi.ensure(t->n * sizeof(Aff)));
            VK_LAUNCH(ctx, "glv_phi", (k_glv_phi<C>), (t->n + 255) / 256, 256, 0, t->bases.as<Aff>(), (uint32_t)t->n,
                      bls_fq_mont(GLV_BETA), phi.as<Aff>());
            VK_LAUNCH(ctx, "to_fast", (k_to_fast<C>), (t->n + 255) / 256, 256, 0, phi.as<Aff>(), t->n,
                      t->fast.as<Aff>() + t->n);
            VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // before phi's buffer is freed
            t->phi_ok = 1;
        }
    }
    return VC_OK;
}

// out[i] = mul 2^c in[i] (mul odd and small; identity bases stay the identity)
template <class C>
__global__ void __launch_bounds__(256) k_win_next(const typename C::Aff* __restrict__ in,
                                                 const uint8_t* __restrict__ inf, uint32_t n, int c, uint32_t mul,
                                                 typename C::Acc* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    typename C::Acc a = inf[i] ? C::zero() : C::from_aff(in[i], false);
    if (!inf[i] && mul > 1) {  // double-and-add; k P != +-P for 1 < k < r, so no exceptional add
        const typename C::Aff p = in[i];
        for (int b = 30 - __builtin_clz(mul); b >= 0; b--) {
            a = C::dbl(a);
            if ((mul >> b) & 1) a = C::madd(a, p, false);
        }
    }
    for (int k = 0; k < c; k++) a = C::dbl(a);
    out[i] = a;
}

// Shared-window copies of a GLV table (Table::win): for w < W, 2^(c w) P_i at [w][i] and
// 2^(c w) phi(P_i) at [w][n + i], packed-29. A GLV MSM over the whole table then sends every
// window's digits to one set of 2^(c-1) buckets -- the same mixed adds, but one bucket reduction
// instead of W and no doublings in the host fold. 2 W n points (1.6 GB at n = 2^20, c = 16),
// built once per table and window size: W - 1 steps of c doublings + a batch normalisation.
// mul > 1: radix B = mul 2^c (the radix-B shared windows): the copy of window w holds B^w P.
template <class C>
static int win_tables(vc_ctx* ctx, Table* t, int c, int W, int ts, uint32_t mul = 1, bool pair = false) {
    using Aff = typename C::Aff;
    using Acc = typename C::Acc;
    if (t->win_ok && t->win_c == c && t->win_W == W && t->win_ts == ts && t->win_m == (int)mul &&
        t->win_pair == (pair ? 1 : 0))
        return VC_OK;
    const size_t n = t->n;
    t->win_ok = 0;
    using FA = typename Fast29<C>::type::AffN;  // signed limb form (k_to_limbs_n)
    using FP = typename Fast29<C>::type::AffP;  // pair layout (k_to_limbs_p)
    // VKZG_WIN_PACKED=1 keeps the packed-29 form (A/B probe: unpacking costs the accumulate ~84 of
    // 5,044 instructions per add, the limb form 16 B more per gather); the limb form holds
    // x, y and -y (168 B) so the accumulate never negates
    static const bool packed = getenv("VKZG_WIN_PACKED") != nullptr;
    t->win_limbs = packed ? 0 : 1;
    t->win_pair = (pair && !packed) ? 1 : 0;
    VK_TRY(t->win.ensure((size_t)W * 2 * n * (packed ? sizeof(Aff) : t->win_pair ? 2 * sizeof(FP) : sizeof(FA))));
    Table cur;  // 2^(c w) P (affine, Montgomery): normalised by table_from_acc (commit.hip)
    DevBuf nxt, acc;
    VK_TRY(nxt.ensure(n * sizeof(Aff)));
    VK_TRY(acc.ensure(n * sizeof(Acc)));
    FA* win = t->win.as<FA>();
    const unsigned g = (unsigned)((n + 255) / 256);
    for (int w = 0; w < W; w++) {
        const Aff* src = t->bases.as<Aff>();
        if (w > 0) {
            // the top window's copy is 2^(c w - ts) P (its digits are scaled by 2^ts, GlvDigits)
            VK_LAUNCH(ctx, "win_next", (k_win_next<C>), g, 256, 0, w == 1 ? t->bases.as<Aff>() : cur.bases.as<Aff>(),
                      t->inf.as<uint8_t>(), (uint32_t)n, w == W - 1 ? c - ts : c, mul, acc.as<Acc>());
            VK_TRY(table_from_acc(ctx, &cur, acc.p, n));
            src = cur.bases.as<Aff>();
        }
        VK_LAUNCH(ctx, "glv_phi", (k_glv_phi<C>), g, 256, 0, src, (uint32_t)n, bls_fq_mont(GLV_BETA), nxt.as<Aff>());
        if (packed) {
            Aff* wp = t->win.as<Aff>();
            VK_LAUNCH(ctx, "to_fast", (k_to_fast<C>), g, 256, 0, src, n, wp + (size_t)w * 2 * n);
            VK_LAUNCH(ctx, "to_fast", (k_to_fast<C>), g, 256, 0, nxt.as<Aff>(), n, wp + (size_t)w * 2 * n + n);
        } else if (t->win_pair) {
            FP* wp = t->win.as<FP>();
            VK_LAUNCH(ctx, "to_limbs", (k_to_limbs_p<C>), g, 256, 0, src, n, wp + 2 * ((size_t)w * 2 * n));
            VK_LAUNCH(ctx, "to_limbs", (k_to_limbs_p<C>), g, 256, 0, nxt.as<Aff>(), n, wp + 2 * ((size_t)w * 2 * n + n));
        } else {
            VK_LAUNCH(ctx, "to_limbs", (k_to_limbs_n<C>), g, 256, 0, src, n, win + (size_t)w * 2 * n);
            VK_LAUNCH(ctx, "to_limbs", (k_to_limbs_n<C>), g, 256, 0, nxt.as<Aff>(), n, win + (size_t)w * 2 * n + n);
        }
    }
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // before the staging buffers are freed
    t->win_ok = 1;
    t->win_c = c;
    t->win_W = W;
    t->win_ts = ts;
    t->win_m = (int)mul;
    return VC_OK;
}

// hipFuncAttributeMaxDynamicSharedMemorySize is per device: set it once per (kernel, device), so
// a process driving several GPUs (one vc_ctx each, or a vc_group) has it on every device it launches on
static int coarse_st_lds_attr(const void* fn, int device) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({fn, device})) return VC_OK;
    VK_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
    done.insert({fn, device});
    return VC_OK;
}

template <class Src>
static int sort_entries(vc_ctx* ctx, Lane L, Src src, uint32_t nv, int c, int wb, int we, uint32_t FB,
                        uint32_t NBC, uint32_t nblk, uint32_t chunk, uint32_t stride, uint32_t wps, size_t ncnt,
                        uint32_t* counts, uint32_t* base, void* tmp, uint32_t* offsets, uint32_t* sorted,
                        uint32_t* zero_word, bool coarse_stage = false, bool counts_ready = false,
                        uint32_t sets_split = 1) {
    hipStream_t st = L.st;
    if (stride && wps == 0) return VC_E_INVALID;
    const uint32_t bins = (stride ? ((uint32_t)we + wps - 1) / wps : (uint32_t)(we - wb)) * NBC;
    const size_t lds = (size_t)bins * 4;
    if (lds > 64 * 1024) return VC_E_INVALID;  // c <= 16 keeps bins <= W * 128
    if (ncnt != (size_t)bins * nblk + 1) return VC_E_INVALID;
    // largest entry index e: i < nv, or w * stride + i with shared windows
    const uint64_t emax = stride ? (uint64_t)std::min<uint32_t>((uint32_t)we, wps) * stride : (uint64_t)nv;
    const bool narrow = emax <= (1ull << (31 - FB));
    // scalars per hist / coarse block: runs of a block inside a coarse bin are chunk * W / bins
    // entries long, so a big bucket set (many coarse bins) takes bigger blocks to keep the
    // scatter's runs near a cache line
    const uint32_t sblk = chunk >= 4096 ? 1024 : 256;
    if (!counts_ready)  // else written by k_glv_radix_hist
        VK_LAUNCH_ON(ctx, st, "msm_sort_hist", (k_sort_hist<Src>), nblk, sblk, lds, src, nv, c, wb, we, FB, NBC,
                     nblk, stride, wps, chunk, counts);
    size_t tmp_bytes = 0;
    VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, base, ncnt, st));
    VK_TRY(L.ws[WS_SCAN_TMP].ensure(tmp_bytes));
    {
        hipEvent_t ev = nullptr;
        if (ctx->timing) ctx->timer_begin("msm_scan", &ev, st);
        VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(L.ws[WS_SCAN_TMP].p, tmp_bytes, counts, base, ncnt, st));
        if (ctx->timing) ctx->timer_end("msm_scan", ev, st);
    }
    // fine-pass block: 1024 threads once bins average >= 2^15 entries (one block per bin)
    static const int fine_env = getenv("VKZG_SORT_FINE_BLOCK") ? atoi(getenv("VKZG_SORT_FINE_BLOCK")) : 0;  // probe
    const uint64_t total = (uint64_t)nv * (uint32_t)(we - wb);
    int fblk = fine_env == 256 || fine_env == 1024 ? fine_env : (total / bins >= (1u << 15) ? 1024 : 256);
    // LDS staging of the fine scatter (16K entries, 64 KB: two blocks per CU, 1024 threads) when the
    // mean bin leaves it ~40 % headroom (radix 2^20: 11.5K); a bin beyond it scatters directly
    static const int stage_env = getenv("VKZG_SORT_STAGE") ? atoi(getenv("VKZG_SORT_STAGE")) : 1;  // A/B probe
    // staged bins of <= 16 entries per thread keep their entries in registers (k_sort_fine);
    // VKZG_SORT_FINE_REGS=0: A/B probe
    static const uint32_t fine_regs = !(getenv("VKZG_SORT_FINE_REGS") && atoi(getenv("VKZG_SORT_FINE_REGS")) == 0);
    uint32_t cap = 0;
    if (stage_env && total / bins <= 12000) {
        cap = 16384;
        if (fine_env == 0) fblk = 1024;
    }
    // staged coarse scatter (k_sort_coarse_st): narrow entries, the block's entries in LDS; with
    // several shared bucket sets (windows [s wps, (s + 1) wps) -> set s) one launch per set, so a
    // block holds one set's chunk x wps entries (the KZG commit + open's two sets keep 4096-scalar
    // blocks, as one set does)
    const uint32_t nsplit = (stride && sets_split > 1 && wb == 0 && (uint32_t)we == sets_split * wps) ? sets_split : 1;
    const uint32_t bins_l = bins / nsplit;
    const uint32_t wl = (uint32_t)(we - wb) / nsplit;
    const size_t st_lds = ((size_t)2 * bins_l + 1 + (size_t)chunk * wl) * 4;
    const bool staged = coarse_stage && narrow && st_lds <= 152 * 1024;
    if (staged) {
        VK_TRY(coarse_st_lds_attr(reinterpret_cast<const void*>(&k_sort_coarse_st<Src>), ctx->device));
        for (uint32_t s = 0; s < nsplit; s++) {
            Src ss = src;
            const int wbs = nsplit > 1 ? (int)(s * wps) : wb, wes = nsplit > 1 ? (int)((s + 1) * wps) : we;
            if constexpr (std::is_same<Src, RadixDigits>::value) ss.w0 = wbs;
            VK_LAUNCH_ON(ctx, st, "msm_sort_coarse", k_sort_coarse_st<Src>, nblk, 1024, st_lds, ss, nv, c, wbs, wes, FB,
                         NBC, nblk, stride, wps, chunk, counts, base, static_cast<uint32_t*>(tmp), s * bins_l, bins_l);
        }
        VK_LAUNCH_ON(ctx, st, "msm_sort_fine", k_sort_fine<uint32_t>, bins, fblk, cap * 4,
                     static_cast<const uint32_t*>(tmp), base, nblk, bins, FB, offsets, sorted, zero_word, cap, fine_regs);
    } else if (narrow) {
        VK_LAUNCH_ON(ctx, st, "msm_sort_coarse", (k_sort_coarse<Src, uint32_t>), nblk, sblk, lds, src, nv, c, wb, we,
                     FB, NBC, nblk, stride, wps, chunk, base, static_cast<uint32_t*>(tmp));
        VK_LAUNCH_ON(ctx, st, "msm_sort_fine", k_sort_fine<uint32_t>, bins, fblk, cap * 4,
                     static_cast<const uint32_t*>(tmp), base, nblk, bins, FB, offsets, sorted, zero_word, cap, fine_regs);
    } else {
        VK_LAUNCH_ON(ctx, st, "msm_sort_coarse", (k_sort_coarse<Src, uint64_t>), nblk, sblk, lds, src, nv, c, wb, we,
                     FB, NBC, nblk, stride, wps, chunk, base, static_cast<uint64_t*>(tmp));
        VK_LAUNCH_ON(ctx, st, "msm_sort_fine", k_sort_fine<uint64_t>, bins, fblk, cap * 4,
                     static_cast<const uint64_t*>(tmp), base, nblk, bins, FB, offsets, sorted, zero_word, cap, fine_regs);
    }
    return VC_OK;
}

// ------------------------------------------------------------------ host side
// GLV halves are < 2^127: window sizes whose top window still spans most of its digit range
// (16 -> 8 windows, top 15 of 16 bits; 13 -> 10, top 10; 10 -> 13, top 7). A nearly empty
// top window (c = 15 leaves 7 bits, c = 14 one) piles all its entries into a few buckets:
// one fine-sort block and long fix-up chains (measured 0.25 + 0.23 ms at 2^16 with c = 15).
// the radix shared-window copies in the pair layout (SW29::AffP: one aligned 128-B record per
// signed copy, 3.76 GB at 2^20 instead of 2.47). Default on: the 2^20 accumulate 2.15 ms against
// 2.17-2.38 with the (x, y, -y) records (profiles/r04/pair_ab.txt); VKZG_WIN_PAIR=0 for the A/B
static bool win_pair_on() {
    static const int env = getenv("VKZG_WIN_PAIR") ? atoi(getenv("VKZG_WIN_PAIR")) : 1;
    return env != 0;
}

static int glv_window(size_t nv) {
    if (nv >= (1u << 19)) return 16;
    if (nv >= (1u << 15)) return 13;
    return 10;
}
// shared windows (msm_run_t): a short top window's digits are scaled to span the bucket range
// (GlvDigits::ts), so c need not divide 128. Measured at 2^21 terms: c = 19 (7 windows) cuts
// the accumulate by 0.3-0.45 ms but its 2^18-bucket reduction, the top window's hot buckets in
// the fix-up and the sort give it all back (3.61 vs 3.60 ms) -- c = 16 stays.
static int glv_window_shared(size_t nv) {
    static const int env = getenv("VKZG_MSM_C") ? atoi(getenv("VKZG_MSM_C")) : 0;  // tuning probe
    if (env >= 8 && env <= 20) return env;
    return glv_window(nv);
}
// bits of the top window of `total` digit bits cut into c-bit windows, as a shortfall: the top
// window's digits fall into 2^-(shortfall) of its bucket set
static int top_shortfall(int c, int total) {
    const int W = (total + c - 1) / c;
    return c - (total - c * (W - 1));
}
// window bits of a per-window (non-GLV) MSM of n terms whose signed digits cover `total` bits
// (scalar bits + 1). The size rule alone gave BN254 (255 bits) top windows of 2 bits at c = 11
// and 8 of 13 at c = 13: a 4096-term MSM piled all its top digits into 2 of 1,024 buckets,
// chains of ~256 pieces, so every call redid its fix-up by pointer jumping and the reduction
// (+0.37 ms of a 0.7 ms MSM, the multiproof verifier's). A size whose top window is short by more
// than 2 bits is replaced by the cheapest of c - 5 .. c + 2 (W n mixed adds + 2 W 2^(c-1)
// reduction adds) that is not.
static int choose_window(size_t n, int total) {
    int c0 = 5;
    if (n >= (1u << 19)) c0 = 16;
    else if (n >= (1u << 17)) c0 = 15;
    else if (n >= (1u << 15)) c0 = 13;
    else if (n >= (1u << 12)) c0 = 11;
    else if (n >= (1u << 9)) c0 = 9;
    else if (n >= 64) c0 = 7;
    static const int env = getenv("VKZG_MSM_TOPFIT") ? atoi(getenv("VKZG_MSM_TOPFIT")) : 1;  // A/B probe
    if (!env || top_shortfall(c0, total) <= 2) return c0;
    int best = c0;
    double best_cost = 0.0;
    for (int c = std::max(4, c0 - 5); c <= std::min(16, c0 + 2); c++) {
        if (top_shortfall(c, total) > 2) continue;
        const double W = (total + c - 1) / c;
        const double cost = W * (double)n + 2.0 * W * (double)(1u << (c - 1));
        if (best == c0 || cost < best_cost) best = c, best_cost = cost;
    }
    return best;
}

// One window slice [wb, we) of an MSM enqueued on a lane: sort, accumulate, fix-up, reduction and
// the read-back of its W (J + 1) reduced points; slice_finish waits for it and folds them by
// Horner over bit positions. msm_run_t can run two slices of a (rank's) window range on the two
// lanes, staggered: slice 1's sort beside slice 0's accumulate, slice 1's accumulate after slice
// 0's (an event), beside slice 0's latency-bound fix-up and reduction (off by default, see below).
template <class C>
struct MsmSlice {
    using Acc = typename C::Acc;
    Lane L{};
    int c = 0, wb = 0, we = 0, W = 0;
    bool shared = false;  // all windows into one bucket set (Table::win copies)
    int top_f = 0;        // per-window buckets: the top window's shortfall (top_shortfall), if in the slice
    uint32_t m = 1;       // > 1: radix m 2^c digits (RadixDigits), m 2^(c-1) buckets
    int sets = 1;         // shared windows: bucket sets = MSMs over the table in this slice
    uint32_t wps = 0;     // shared windows: windows per set (the window copies' count)
    uint32_t stride = 0;  // shared windows: points per window copy (2N for a table of N); 0 = the terms
    int Wr = 0;           // bucket sets reduced: `sets` shared, W otherwise
    uint32_t NB = 0, NBtot = 0, Tmax = 0, M = 0, Lseg = 0, S = 0, J = 0, guard = 0;
    uint32_t nU = 1;  // sums per set after the J bit sums: A (1), or the Lseg residue sums U_r
    uint32_t* offsets = nullptr;
    uint32_t* chain_max = nullptr;  // in the WS_TAIL buffer, tail_bytes after the tail points
    size_t tail_bytes = 0;
    uint8_t* through = nullptr;
    uint32_t* owner_b = nullptr;
    FAcc<C>* buckets = nullptr;
    FAcc<C>* carry = nullptr;
    FAcc<C>* owner = nullptr;
    FAcc<C>* seg = nullptr;
    FAcc<C>* rs = nullptr;
    FAcc<C>* bsum_part = nullptr;
    Acc* tail = nullptr;
    std::vector<Acc> ht;
    uint32_t Lmax = 0;
    // chunked MSMs (msm_run_host_chunks_t): the accumulate writes these buckets instead of the
    // workspace's, the chain word is this one, and the reduction is left to the caller
    FAcc<C>* bucket_dst = nullptr;
    uint32_t* chain_dst = nullptr;
    bool skip_reduce = false;
    // direct completion (TailDirect): the final stage wrote the points and the chain word into the
    // lane's fine-grained page-locked buffer, then `nflags` flags at flag_off took `epoch`
    bool direct = false;
    uint32_t epoch = 0, nflags = 0;
    size_t flag_off = 0;
    double t_launch0 = 0.0;  // VKZG_HOST_TIMING: when the slice's first kernel was launched (us)
    // BLS12-381 radix digits still to be made (msm_run_t leaves the GLV split to slice_enqueue,
    // which fuses the sort histogram into it when the geometry allows): sc == nullptr otherwise
    struct {
        std::vector<const uint32_t*> sc;  // one scalar set per bucket set (empty: digits made already)
        std::vector<int> mont;
        const uint8_t* inf = nullptr;
        uint32_t n = 0;
        int32_t* dig = nullptr;  // set s at dig + s W 2n
    } radix;
};

template <class C, class BT, class Src>
static int slice_enqueue(vc_ctx* ctx, MsmSlice<C>& sl, Src src, size_t nv, const BT* bases, const BT* phi,
                         uint32_t nphi, hipEvent_t acc_wait, hipEvent_t acc_done) {
    using Acc = typename C::Acc;
    using RAcc = FAcc<C>;  // raw radix-29 accumulators of the accumulate / fix-up / reduction
    const Lane L = sl.L;
    const int c = sl.c, W = sl.W;  // shared: W = sets x windows per set
    const int Wr = sl.shared ? sl.sets : W;
    sl.Wr = Wr;
    const uint32_t NB = sl.m << (c - 1);
    const uint32_t NBtot = NB * (uint32_t)Wr;
    const size_t maxL = nv * (size_t)W;
    const size_t load = maxL / Wr;  // entries per bucket set
    // sorted entries per accumulate thread: 64 at 2^20 x 16 windows (2 rounds of 2048 waves),
    // fewer for window slices / small MSMs so the grid still fills the chip
    // (not below 16: a bucket then straddles more threads and the fix-up's serial merge chain
    // costs more than the emptier accumulate rounds -- measured at 2 windows of 2^20)
    uint32_t M = (uint32_t)std::min<size_t>(64, std::max<size_t>(16, maxL / 131072));
    // ... and at least twice the mean bucket load, so few buckets straddle more than two
    // threads (the GLV 2^20 MSM has 64 entries per bucket: M = 128 drops the fix-up's
    // pointer-jumping rounds, 0.23 -> 0.06 ms, for 0.1 ms more accumulate)
    if (load / NB > M / 2 && M < 128) M *= 2;
    // shared windows: the fix-up is a lane per bucket, so M just fills one round of two waves
    // per SIMD (131072 lanes)
    if (sl.shared) M = (uint32_t)std::max<size_t>(16, (maxL + 131071) / 131072);
    if (const char* em = getenv("VKZG_MSM_M")) M = (uint32_t)std::max(1, atoi(em));  // tuning probe
    // buckets per reduction segment (the segment sum is a serial chain of 2*Lseg adds): 4, or 2
    // when the segments (one lane each) would not give every SIMD a wave (GLV 2^20: 4 at 8
    // windows, 2 for the 1-4 window slices of multi-GPU runs; 8 measured 0.1-0.15 ms slower)
    uint32_t Lseg = NB >= 64 ? 4 : (NB >= 4 ? 2 : 1);
    if (Lseg == 4 && (size_t)(NB / Lseg) * Wr < 65536) Lseg = 2;
    // one bucket set: the bit sums straight over 2^15 buckets (measured), segments of 4 at 2^18;
    // radix m 2^c: segments of m buckets (S = 2^(c-1) segments)
    if (sl.shared) Lseg = sl.m > 1 ? sl.m : (NB >= (1u << 17) ? 4 : 1);
    if (const char* el = getenv("VKZG_MSM_LSEG")) Lseg = (uint32_t)std::max(1, atoi(el));  // tuning probe
    const uint32_t S = NB / Lseg;  // power of two
    uint32_t J = 0;
    while ((1u << J) < S) J++;
    // shared windows with segments: the residue form of the reduction (msm_tail.hip k_msm_segr)
    static const int resid_env = getenv("VKZG_TAIL_RESIDUE") ? atoi(getenv("VKZG_TAIL_RESIDUE")) : 1;  // A/B probe
    // per-window bucket sets too, up to 8 of them (VKZG_TAIL_RESIDUE=2: shared windows only -- A/B
    // probe): the segment stage's 2 Lseg dependent adds become Lseg - 1 for Lseg more U sums in the bit
    // stage. Measured (`profiles/r03/probes/residue_perwin/`): the GLV variable-base 2^20 MSM (8 sets)
    // tail 0.436 -> 0.38 ms; 16-20 sets (BN254, Bandersnatch) 0.05-0.16 ms slower, so they keep acc_s
    const bool resid_sets = sl.shared || Wr <= 8;
    const uint32_t nU = (Lseg > 1 && resid_sets && (resid_env == 1 || (resid_env == 2 && sl.shared))) ? Lseg : 1;
    const uint32_t Tmax = (uint32_t)((maxL + M - 1) / M);
    hipStream_t st = L.st;

    // bucket sort geometry (k_sort_*): 2^FB fine buckets per coarse bin
    const uint32_t lgNB = (uint32_t)c - 1;  // NB = m 2^lgNB
    uint32_t FB = lgNB < 8 ? lgNB : 8;
    uint32_t chunk = SORT_CHUNK;
    if (sl.m > 1) {
        // radix buckets (5 x 2^15 at 2^21 x 7 entries): FB = 7 keeps the coarse entries narrow
        // (entry index < 7 x 2^21 < 2^24), i.e. 1280 coarse bins; blocks of 8192 scalars keep a
        // block's runs ~45 entries long
        FB = lgNB < 7 ? lgNB : 7;
        chunk = 8192;
    }
    static const int chunk_env = getenv("VKZG_SORT_CHUNK") ? atoi(getenv("VKZG_SORT_CHUNK")) : 0;  // tuning probe
    static const int fb_env = getenv("VKZG_SORT_FB") ? atoi(getenv("VKZG_SORT_FB")) : 0;           // tuning probe
    // radix buckets: the staged coarse scatter (k_sort_coarse_st) holds a block's chunk x W entries in
    // LDS, so the chunk is the largest power of two that fits 152 KB beside the 2 x bins counters
    static const int cstage_env = getenv("VKZG_SORT_CSTAGE") ? atoi(getenv("VKZG_SORT_CSTAGE")) : 1;  // A/B probe
    bool cstage = false;
    if (sl.m > 1 && sl.shared && cstage_env) {
        // one coarse launch per bucket set (sort_entries): a block stages one set's windows
        const uint64_t bins_l = (uint64_t)(NB >> FB);
        const uint32_t Wl = (uint32_t)W / (uint32_t)Wr;
        const uint64_t room = (152u * 1024 / 4 > 2 * bins_l + 1) ? 152u * 1024 / 4 - 2 * bins_l - 1 : 0;
        uint32_t ch = 1u << 12;
        while (ch > 1024 && (uint64_t)ch * Wl > room) ch >>= 1;
        if ((uint64_t)ch * Wl <= room) {  // 4096 scalars for one set and for each of several
            chunk = ch;
            cstage = true;
        }
    }
    // per-window buckets: one more coarse bit when the fine bins would be too big to stage in LDS
    // (GLV variable-base 2^21 x 8: 16K -> 8K entries; fine pass 0.118 -> 0.041 ms)
    if (sl.m == 1 && !sl.shared && cstage_env && FB > 1 && load / (NB >> FB) > 12000) FB--;
    if (chunk_env >= 256) chunk = (uint32_t)chunk_env;
    // shared windows: ~64K entries per coarse bin (one 1024-thread k_sort_fine block each) but at
    // least 256 bins (a fine block per CU). Measured at 2^21 x 8 entries (hist + coarse + fine):
    // 0.233 ms at 2^14 entries per bin (256-thread fine blocks), 0.222 at 2^15, 0.204 at 2^16,
    // 0.295 at 2^17 -- bigger bins shorten the scatter's partial-line writes
    static const int bin_lg = getenv("VKZG_SORT_BIN_LG") ? atoi(getenv("VKZG_SORT_BIN_LG")) : 16;  // tuning probe
    while (sl.shared && sl.m == 1 && FB > 1 && (load >> bin_lg) > (size_t)(NB >> FB)) FB--;
    while (sl.shared && sl.m == 1 && FB > 1 && (NB >> FB) < 256) FB--;
    if (fb_env >= 1 && fb_env <= (int)std::min<uint32_t>(lgNB, 8)) FB = (uint32_t)fb_env;
    const uint32_t NBC = NB >> FB;
    const uint32_t nblk = (uint32_t)((nv + chunk - 1) / chunk);
    // the staged coarse pass pays for its LDS sort and write-out with >= 4096 entries per block and
    // either runs of >= 10 entries per bin (radix: 22, or 11 with two sets) or LDS <= 64 KB (two or
    // more blocks per CU: GLV variable-base 2^21 x 8, 4-entry runs, 0.129 -> 0.106 ms). Measured
    // slower: BN254 2^20 (16 windows, 98 KB, 0.119 -> 0.169 ms) and the 8-way window slice (1024
    // entries per block, 0.016 -> 0.029 ms)
    if (sl.m == 1 && cstage_env) {
        const uint64_t per_blk = (uint64_t)chunk * (uint32_t)(sl.we - sl.wb), bins_all = (uint64_t)Wr * NBC;
        const uint64_t lds_b = (2 * bins_all + 1 + per_blk) * 4;
        cstage = per_blk >= 4096 && (per_blk >= 10 * bins_all || lds_b <= 64 * 1024);
    }
    const size_t ncnt = (size_t)Wr * NBC * nblk + 1;

    DevBuf* ws = L.ws;
    VK_TRY(ws[WS_DIGITS].ensure(maxL * 8));
    VK_TRY(ws[WS_COUNTS].ensure(ncnt * 4));
    VK_TRY(ws[WS_CURSOR].ensure(ncnt * 4));
    VK_TRY(ws[WS_OFFSETS].ensure((size_t)(NBtot + 1) * 4));
    VK_TRY(ws[WS_SORTED].ensure(maxL * 4));
    VK_TRY(ws[WS_BUCKETS].ensure((size_t)NBtot * sizeof(RAcc)));
    VK_TRY(ws[WS_CARRY].ensure((size_t)(Tmax + 8) * sizeof(RAcc)));
    VK_TRY(ws[WS_THROUGH].ensure((size_t)(Tmax + 8)));
    VK_TRY(ws[WS_OWNER].ensure((size_t)(Tmax + 8) * sizeof(RAcc)));
    VK_TRY(ws[WS_OWNER_B].ensure((size_t)(Tmax + 8) * 4));
    VK_TRY(ws[WS_SEG].ensure((size_t)S * Wr * sizeof(RAcc)));
    VK_TRY(ws[WS_TREE].ensure((size_t)S * Wr * sizeof(RAcc)));
    VK_TRY(ws[WS_WIN].ensure((size_t)Wr * msm_tail_plan(S, (uint32_t)Wr, J, nU, Fast29<C>::type::quad, Lseg == 1).slots *
                             sizeof(RAcc)));
    // tail points, then the chain_max word: one read-back
    const size_t tail_bytes = ((size_t)Wr * (J + nU) * sizeof(Acc) + 15) & ~(size_t)15;
    VK_TRY(ws[WS_TAIL].ensure(tail_bytes + 16));

    sl.NB = NB;
    sl.NBtot = NBtot;
    sl.Tmax = Tmax;
    sl.M = M;
    sl.Lseg = Lseg;
    sl.S = S;
    sl.J = J;
    sl.nU = nU;
    sl.offsets = ws[WS_OFFSETS].as<uint32_t>();
    sl.tail_bytes = tail_bytes;
    sl.chain_max = sl.chain_dst ? sl.chain_dst : reinterpret_cast<uint32_t*>(ws[WS_TAIL].as<uint8_t>() + tail_bytes);
    sl.through = ws[WS_THROUGH].as<uint8_t>();
    sl.owner_b = ws[WS_OWNER_B].as<uint32_t>();
    sl.buckets = sl.bucket_dst ? sl.bucket_dst : ws[WS_BUCKETS].as<RAcc>();
    sl.carry = ws[WS_CARRY].as<RAcc>();
    sl.owner = ws[WS_OWNER].as<RAcc>();
    sl.seg = ws[WS_SEG].as<RAcc>();
    sl.rs = ws[WS_TREE].as<RAcc>();
    sl.bsum_part = ws[WS_WIN].as<RAcc>();
    sl.tail = ws[WS_TAIL].as<Acc>();

    bool counts_ready = false;
    static const bool timing = getenv("VKZG_HOST_TIMING") && atoi(getenv("VKZG_HOST_TIMING")) != 0;
    if (timing)
        sl.t_launch0 =
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    if constexpr (std::is_same<C, BLS381G1>::value) {
        if (!sl.radix.sc.empty()) {
            // whole bucket sets over all their windows, whole sort blocks of scalars: the GLV split
            // of set s writes the sort histogram of its bins [s NBC, (s + 1) NBC) itself
            static const int fuse_env = getenv("VKZG_RADIX_HIST") ? atoi(getenv("VKZG_RADIX_HIST")) : 1;  // A/B
            const uint32_t rn = sl.radix.n;
            const int ns = (int)sl.radix.sc.size();
            counts_ready = fuse_env && sl.shared && Wr == ns && sl.wb == 0 && (uint32_t)sl.we == sl.wps * (uint32_t)ns &&
                           nv == 2 * (size_t)rn && rn % chunk == 0 && (size_t)2 * NBC * 4 <= 64 * 1024;
            for (int s2 = 0; s2 < ns; s2++) {
                int32_t* dig = sl.radix.dig + (size_t)s2 * sl.wps * nv;
                if (counts_ready)
                    VK_LAUNCH_ON(ctx, st, "glv_split", (k_glv_radix_hist<BLS381Fr, 5, 16>), rn / chunk, 1024,
                                 (size_t)2 * NBC * 4, sl.radix.sc[s2], sl.radix.inf, rn, sl.radix.mont[s2], glv_consts(),
                                 (int)sl.wps, dig, FB, NBC, nblk, chunk, ws[WS_COUNTS].as<uint32_t>(),
                                 (uint32_t)s2 * NBC, (uint32_t)Wr * NBC);
                else
                    VK_LAUNCH_ON(ctx, st, "glv_split", (k_glv_radix<BLS381Fr, 5, 16>), (rn + 255) / 256, 256, 0,
                                 sl.radix.sc[s2], sl.radix.inf, rn, sl.radix.mont[s2], glv_consts(), (int)sl.wps, dig);
            }
        }
    }
    VK_TRY(sort_entries(ctx, L, src, (uint32_t)nv, c, sl.wb, sl.we, FB, NBC, nblk, chunk, sl.shared ? (sl.stride ? sl.stride : (uint32_t)nv) : 0u,
                        sl.wps, ncnt,
                        ws[WS_COUNTS].as<uint32_t>(),
                        ws[WS_CURSOR].as<uint32_t>(), ws[WS_DIGITS].p, sl.offsets,
                        ws[WS_SORTED].as<uint32_t>(), sl.chain_max, cstage, counts_ready,
                        sl.shared ? (uint32_t)Wr : 1u));
    // entry count L = offsets[NBtot] stays on the device; grids are sized for L <= nv*W;
    // chain_max was cleared by k_sort_fine
    if (acc_wait) VK_CHECK_HIP(hipStreamWaitEvent(st, acc_wait, 0));
    VK_LAUNCH_ON(ctx, st, "msm_accumulate", (k_msm_accumulate<C, BT>), (Tmax + 255) / 256, 256, 0, bases, phi, nphi,
                 ws[WS_SORTED].as<uint32_t>(), sl.offsets, NBtot, M, sl.buckets, sl.carry, sl.through, sl.owner,
                 sl.owner_b, sl.chain_max, acc_merge(), (unsigned long long*)ctx->clk_slot());
    if (acc_done) VK_CHECK_HIP(hipEventRecord(acc_done, st));
    // chains up to 2^guard carry pieces are walked serially by their owners; longer ones
    // (adversarial scalars) take the pointer-jumping path in slice_finish
    // (a top window short by f bits loads its buckets 2^f times the mean)
    sl.guard = msm_fixup_guard_rounds(sl.shared ? load : load << sl.top_f, NB, M);
    // shared windows: a short top window's digits load 2^-tb of the buckets several times the
    // mean (c = 19: ~310 entries vs 56), so the walk takes chains of up to 16 pieces
    if (sl.shared) sl.guard = std::max<uint32_t>(sl.guard, 4);
    static const int fix_env = getenv("VKZG_MSM_FIXUP") ? atoi(getenv("VKZG_MSM_FIXUP")) : 0;  // tuning probe
    if (fix_env == 1)  // guarded pointer-jumping rounds instead of the owner walk
        VK_TRY(msm_tail_fixup<C>(ctx, L, Tmax, sl.offsets + NBtot, M, sl.buckets, sl.carry, sl.through, sl.owner,
                                 sl.owner_b, sl.chain_max, sl.guard));
    else
        VK_TRY(msm_tail_fixup_walk<C>(ctx, L, sl.offsets, NBtot, M, sl.buckets, sl.carry, sl.owner, 1u << sl.guard,
                                      sl.owner_b, sl.through, Tmax));
    if (sl.skip_reduce) return VC_OK;
    // direct completion: the final stage writes its W (J + nU) points and the chain word straight
    // into the lane's fine-grained page-locked buffer and flags each block; the host polls the flags
    // (slice_finish) -- no read-back copy (a ~4-us blit plus its dispatch) and no stream wake-up
    // (~10-20 us). VKZG_TAIL_POLL=0 (A/B probe): copy and wait.
    static const bool poll_env = !(getenv("VKZG_TAIL_POLL") && atoi(getenv("VKZG_TAIL_POLL")) == 0);
    TailDirect td;
    Acc* out = sl.tail;
    sl.direct = false;
    if (poll_env && L.pin->flags == hipHostMallocCoherent) {
        sl.nflags = (uint32_t)Wr * (J + nU);
        sl.flag_off = tail_bytes + 16;
        VK_TRY(L.pin->ensure(sl.flag_off + (size_t)sl.nflags * 4));
        // (fresh page-locked memory holds anything: no stale flag may match)
        volatile uint32_t* hf = reinterpret_cast<volatile uint32_t*>(static_cast<uint8_t*>(L.pin->p) + sl.flag_off);
        for (uint32_t k = 0; k < sl.nflags; k++) hf[k] = 0;
        sl.epoch = ++ctx->tail_epoch == 0 ? ++ctx->tail_epoch : ctx->tail_epoch;  // never 0
        uint8_t* dbase = static_cast<uint8_t*>(L.pin->dp);
        td.flags = reinterpret_cast<uint32_t*>(dbase + sl.flag_off);
        td.epoch = sl.epoch;
        td.chain_src = sl.chain_max;
        td.chain_dst = reinterpret_cast<uint32_t*>(dbase + tail_bytes);
        out = reinterpret_cast<Acc*>(dbase);
        sl.direct = true;
    }
    VK_TRY(msm_tail_reduce<C>(ctx, L, sl.buckets, sl.offsets, NB, Wr, Lseg, S, J, sl.seg, sl.rs, sl.bsum_part, out,
                              nU > 1, sl.direct ? &td : nullptr));
    return VC_OK;
}

// read back (after every slice has been enqueued: a copy into pageable memory may block the host)
template <class C>
static int slice_fetch(MsmSlice<C>& sl) {
    sl.ht.resize((size_t)sl.Wr * (sl.J + sl.nU));
    if (sl.direct) return VC_OK;  // written in place by the final stage
    VK_TRY(sl.L.pin->ensure(sl.tail_bytes + 16));
    VK_CHECK_HIP(hipMemcpyAsync(sl.L.pin->p, sl.tail, sl.tail_bytes + 4, hipMemcpyDeviceToHost, sl.L.st));
    return VC_OK;
}

// the wait for a slice's results: its flags at this epoch (direct completion), bounded -- past
// 20 ms (a first launch loading its code, or a fault) the stream wait, which also reports errors
template <class C>
static int slice_wait(const MsmSlice<C>& sl) {
    if (sl.direct) {
        const volatile uint32_t* hf =
            reinterpret_cast<const volatile uint32_t*>(static_cast<const uint8_t*>(sl.L.pin->p) + sl.flag_off);
        const auto w0 = std::chrono::steady_clock::now();
        for (uint32_t spins = 0;; spins++) {
            uint32_t k = 0;
            while (k < sl.nflags && hf[k] == sl.epoch) k++;
            if (k == sl.nflags) {
                std::atomic_thread_fence(std::memory_order_acquire);
                return VC_OK;
            }
            if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(20)) break;
            _mm_pause();
        }
    }
    VK_CHECK_HIP(hipStreamSynchronize(sl.L.st));
    return VC_OK;
}

template <class C>
static int slice_finish(vc_ctx* ctx, MsmSlice<C>& sl, typename C::Acc* res);

// the reduced points of bucket set `set` (shared windows: one MSM each) -> its sum
//   Lseg sum_j 2^j T_j + A,  A = sum_r (r + 1) U_r = sum_k (U_k + ... + U_{nU-1}) (suffix sums)
template <class C>
static typename C::Acc shared_set_sum(const MsmSlice<C>& sl, int set) {
    using Acc = typename C::Acc;
    const uint32_t J = sl.J;
    const Acc* ht = sl.ht.data() + (size_t)set * (J + sl.nU);
    Acc x = C::zero();  // sum_j 2^j T_j
    for (int j = (int)J - 1; j >= 0; j--) {
        if (!C::is_zero(x)) x = C::dbl(x);
        x = C::add(x, ht[j]);
    }
    Acc r = C::zero();  // Lseg x by double-and-add (Lseg = m for the radix buckets)
    for (int b = 31 - __builtin_clz(sl.Lseg); b >= 0; b--) {
        if (!C::is_zero(r)) r = C::dbl(r);
        if ((sl.Lseg >> b) & 1) r = C::add(r, x);
    }
    Acc suf = C::zero();
    for (int k = (int)sl.nU - 1; k >= 0; k--) {
        suf = C::add(suf, ht[J + k]);
        r = C::add(r, suf);
    }
    return r;
}

template <class C>
static int slice_finish(vc_ctx* ctx, MsmSlice<C>& sl, typename C::Acc* res) {
    using Acc = typename C::Acc;
    VK_TRY(slice_wait<C>(sl));
    memcpy(sl.ht.data(), sl.L.pin->p, sl.ht.size() * sizeof(Acc));
    memcpy(&sl.Lmax, static_cast<const uint8_t*>(sl.L.pin->p) + sl.tail_bytes, 4);
    if (sl.Lmax > (1u << sl.guard)) {  // rare (heavily repeated scalars): pointer jumping, redo the tail
        VK_TRY(msm_tail_fixup<C>(ctx, sl.L, sl.Tmax, sl.offsets + sl.NBtot, sl.M, sl.buckets, sl.carry, sl.through,
                                 sl.owner, sl.owner_b, sl.chain_max, 0));
        VK_TRY(msm_tail_reduce<C>(ctx, sl.L, sl.buckets, sl.offsets, sl.NB, sl.Wr, sl.Lseg, sl.S, sl.J, sl.seg,
                                  sl.rs, sl.bsum_part, sl.tail, sl.nU > 1));
        VK_CHECK_HIP(hipMemcpyAsync(sl.ht.data(), sl.tail, sl.ht.size() * sizeof(Acc), hipMemcpyDeviceToHost,
                                    sl.L.st));
        VK_CHECK_HIP(hipStreamSynchronize(sl.L.st));
    }
    // row-derived totals (TailPlan::urow): the final stage left X = sum of the even-hi row sums in
    // each set's U slot; U = X + T_h (the odd-hi rows)
    const TailPlan tp = msm_tail_plan(sl.S, (uint32_t)sl.Wr, sl.J, sl.nU, Fast29<C>::type::quad, sl.Lseg == 1);
    if (tp.urow)
        for (int w = 0; w < sl.Wr; w++) {
            Acc* u = &sl.ht[(size_t)w * (sl.J + sl.nU) + sl.J];
            *u = C::add(*u, sl.ht[(size_t)w * (sl.J + sl.nU) + tp.h]);
        }
    // slice = sum_w 2^(c w) (A_w + Lseg sum_j 2^j T_wj): Horner over bit positions (host); with
    // shared windows the one bucket set already holds the 2^(c w) factors: A + Lseg sum_j 2^j T_j
    const uint32_t J = sl.J;
    if (sl.shared && sl.sets > 1) {  // several MSMs: res[k] = set k's sum
        for (int k = 0; k < sl.sets; k++) res[k] = shared_set_sum<C>(sl, k);
        return VC_OK;
    }
    if (sl.shared) {  // one bucket set: Lseg x (radix buckets: Lseg = m is odd) and the U_r weights
        *res = shared_set_sum<C>(sl, 0);
        return VC_OK;
    }
    int lg_seg = 0;
    while ((1u << lg_seg) < sl.Lseg) lg_seg++;
    const int maxpos = (sl.shared ? 0 : sl.c * (sl.we - 1)) + lg_seg + (int)J;
    std::vector<std::vector<int>> at(maxpos + 1);
    const int st = (int)(J + sl.nU);  // reduced points per window: T_0 .. T_{J-1}, then the U sums
    std::vector<Acc> aw(sl.Wr);       // A_w = sum_r (r + 1) U_r by suffix sums (nU = 1: the sum A)
    for (int w = 0; w < sl.Wr; w++) {
        const int p0 = sl.shared ? 0 : sl.c * (sl.wb + w);  // absolute bit position of window wb + w
        Acc a = C::zero(), suf = C::zero();
        for (int k = (int)sl.nU - 1; k >= 0; k--) {
            suf = C::add(suf, sl.ht[(size_t)w * st + J + k]);
            a = C::add(a, suf);
        }
        aw[w] = a;
        at[p0].push_back(-1 - w);  // < 0: A_w
        for (uint32_t j = 0; j < J; j++) at[p0 + lg_seg + (int)j].push_back(w * st + (int)j);
    }
    Acc r = C::zero();
    for (int pos = maxpos; pos >= 0; pos--) {
        if (!C::is_zero(r)) r = C::dbl(r);
        for (int idx : at[pos]) r = C::add(r, idx < 0 ? aw[-1 - idx] : sl.ht[idx]);
    }
    *res = r;
    return VC_OK;
}

// VKZG_HOST_TIMING=1: host-side phases of each MSM on stderr (probe; tools/msm_probe.py)
static bool host_timing() {
    static const bool on = getenv("VKZG_HOST_TIMING") && atoi(getenv("VKZG_HOST_TIMING")) != 0;
    return on;
}
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class C, class Fr>
static int msm_run_t(vc_ctx* ctx, Table* t, size_t offset, const uint32_t* d_sc, size_t n,
                     int mont, int part, int parts, uint32_t* out_acc) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    const double t_entry = host_timing() ? now_us() : 0.0;
    if (n == 0) {
        Acc z = C::zero();
        memcpy(out_acc, &z, sizeof(Acc));
        return VC_OK;
    }
    if (n >= 0x7fffffffu) return VC_E_INVALID;
    if (parts < 1 || part < 0 || part >= parts) return VC_E_INVALID;
    bool glv = false;
    if constexpr (std::is_same<C, BLS381G1>::value) {
        if (n >= GLV_MIN_N && n < (1u << 30)) VK_TRY(glv_table_ok(ctx, t, &glv));
    }
    const size_t nv = glv ? 2 * n : n;  // MSM terms after the endomorphism split
    VK_TRY(fast_tables<C>(ctx, t, glv));
    const Aff* bases = t->fast.as<Aff>() + offset;  // packed-29 copies (ec29.hpp)
    // shared windows (GLV MSM over the whole table): every window into one bucket set through
    // the 2^(c w) copies of the bases (Table::win, built once; up to 8 GB of HBM). The window
    // size then only trades mixed adds (W per term) against one bucket reduction: c = 19 at
    // 2^21 terms (7 windows instead of 8). VKZG_MSM_SHARED=0 keeps per-window buckets (probe).
    bool shared = false;
    int top_shift = 0;
    uint32_t radix_m = 1;  // > 1: radix-B shared windows, B = radix_m 2^c
    int c = glv ? glv_window(nv) : choose_window(nv, Fr::BITS + 1);
    if constexpr (std::is_same<C, BLS381G1>::value) {
        const bool shared_env = ctx->opt_shared_windows != 0;  // vc_ctx_set_option(VC_OPT_MSM_SHARED_WINDOWS)
        // Radix-B shared windows (B = 5 x 2^16 ~ 2^18.3, one MSM on one GPU): 7 uniformly loaded
        // windows instead of 8 (B^7 / 2 > 2^127, the GLV halves' bound) -- 12.5 % fewer mixed
        // adds -- into 5 x 2^15 buckets. The power-of-two c = 19 (7 windows) left a 14-bit top
        // window whose digits hit 1 bucket in 16 (chains in the fix-up) and 2^18 buckets to
        // reduce. Window-sliced (multi-GPU) parts keep c = 16: a one-window slice would reduce
        // the whole bucket set for 1/7 of the adds. VKZG_MSM_RADIX=1: power-of-two windows (probe).
        static const int radix_env = getenv("VKZG_MSM_RADIX") ? atoi(getenv("VKZG_MSM_RADIX")) : 5;
        // a point range [offset, offset + n) of >= 2^18 points (one GPU's share of a point-split
        // MSM, vc_msm_device_partial) reads the same whole-table copies, its entries at their table
        // positions (RadixDigits::pt): one copy layout serves whole-table and point-range MSMs
        static const int range_env = getenv("VKZG_MSM_RANGE") ? atoi(getenv("VKZG_MSM_RANGE")) : 1;  // A/B
        const bool whole = offset == 0 && n == t->n;
        // ranges down to 2^16 points of a >= 2^18-point table: an eighth of 2^20 on the copies (the
        // 163,840-bucket tail is a fixed cost, but a standalone 2^17-term plan took 1.8 ms against
        // ~0.6: profiles/r04/split_probe*.txt)
        const bool big = whole ? nv >= (1u << 19) : (2 * (size_t)t->n >= (1u << 19) && nv >= (1u << 17));
        if (glv && shared_env && (whole || range_env) && parts == 1 && big && radix_env == 5 &&
            !getenv("VKZG_MSM_C") && !getenv("VKZG_WIN_PACKED")) {
            const size_t win_bytes = (size_t)7 * 2 * t->n *
                                     (win_pair_on() ? 2 * sizeof(typename Fast29<C>::type::AffP)
                                                    : sizeof(typename Fast29<C>::type::AffN));
            if (win_bytes <= (8ull << 30)) {
                const int st = win_tables<C>(ctx, t, 16, 7, 0, 5, win_pair_on());
                if (st == VC_OK) {
                    shared = true;
                    c = 16;
                    radix_m = 5;
                } else if (st != VC_E_OOM) {
                    return st;
                } else {
                    t->win.release();
                }
            }
        }
        const int cs = glv_window_shared(nv);
        const int Ws = (GLV_BITS + cs - 1) / cs;
        // top window: GLV_BITS - cs (Ws - 1) bits -> digits up to 2^tb; scaled to fill 2^(cs-1)
        const int tb = GLV_BITS - cs * (Ws - 1);
        const int ts = std::max(0, (cs - 1) - tb);
        const size_t win_bytes = (size_t)Ws * 2 * t->n * sizeof(typename Fast29<C>::type::AffN);
        if (!shared && glv && shared_env && offset == 0 && n == t->n && win_bytes <= (8ull << 30)) {
            const int st = win_tables<C>(ctx, t, cs, Ws, ts);
            if (st == VC_OK) {
                shared = true;
                c = cs;
                top_shift = ts;
            } else if (st != VC_E_OOM) {
                return st;
            } else {
                t->win.release();  // out of memory: per-window buckets instead
            }
        }
    }
    // one spare bit absorbs the final carry of the signed recoding
    const int Wfull = radix_m > 1 ? 7 : glv ? (GLV_BITS + c - 1) / c : (Fr::BITS + 1 + c - 1) / c;
    ctx->plan = {c, Wfull, glv ? 2 : 1, (int)radix_m, shared ? 1 : 0};  // vc_msm_last_plan
    // window slice [wb, we) of this call (parts > 1: the MSM split by windows across GPUs;
    // the slices' results add up to the whole MSM)
    const int wb = part * Wfull / parts, we = (part + 1) * Wfull / parts;
    const int W = we - wb;
    // entry counts, offsets, scan counts and sorted positions are u32: nv * W must fit (msm_run
    // cuts larger MSMs into chunks of ctx->opt_msm_chunk points, so this only guards misuse)
    if ((uint64_t)nv * (uint64_t)Wfull >= 0xffffffffull) return VC_E_RANGE;
    if (W == 0) {
        Acc z = C::zero();
        memcpy(out_acc, &z, sizeof(Acc));
        return VC_OK;
    }
    const uint8_t* inf = t->inf.as<uint8_t>() + offset;
    // VKZG_MSM_SLICES=2 runs two staggered slices on the two lanes (tuning probe): measured no
    // faster at 2^20 BLS12-381 (4.09-4.29 vs 3.98-4.06 ms) -- a 4-window slice's accumulate fills
    // one wave per SIMD (6-13 % below two), and the overlapped tail shares the same SIMDs
    static const int slices_env = getenv("VKZG_MSM_SLICES") ? atoi(getenv("VKZG_MSM_SLICES")) : 1;
    const int nsl = (slices_env == 2 && W >= 2 && nv * (size_t)W >= (1u << 22)) ? 2 : 1;
    MsmSlice<C> sl[2];
    for (int k = 0; k < nsl; k++) {
        sl[k].L = ctx->lane(k);
        sl[k].c = c;
        sl[k].wb = wb + k * W / nsl;
        sl[k].we = wb + (k + 1) * W / nsl;
        sl[k].W = sl[k].we - sl[k].wb;
        sl[k].shared = shared;
        sl[k].m = radix_m;
        sl[k].wps = (uint32_t)Wfull;
        if (!shared && radix_m == 1 && sl[k].we == Wfull)
            sl[k].top_f = top_shortfall(c, glv ? GLV_BITS : Fr::BITS + 1);
    }
    hipEvent_t fork = nullptr, join = nullptr, acc0 = nullptr;
    if (nsl == 2) acc0 = ctx->get_event();
    if (glv) {
        if constexpr (std::is_same<C, BLS381G1>::value) {
            VK_TRY(ctx->ws[WS_GLV_SC].ensure(radix_m > 1 ? nv * 4 * (size_t)Wfull : nv * 16));
            uint4* halves = ctx->ws[WS_GLV_SC].as<uint4>();
            const Aff* dphi = t->fast.as<Aff>() + t->n + offset;
            if (radix_m > 1 && nsl == 1) {  // the split runs in slice_enqueue (sort histogram fused)
                sl[0].radix.sc = {d_sc};
                sl[0].radix.mont = {mont};
                sl[0].radix.inf = inf;
                sl[0].radix.n = (uint32_t)n;
                sl[0].radix.dig = ctx->ws[WS_GLV_SC].as<int32_t>();
            }
            else if (radix_m > 1)
                VK_LAUNCH(ctx, "glv_split", (k_glv_radix<Fr, 5, 16>), (n + 255) / 256, 256, 0, d_sc, inf, (uint32_t)n,
                          mont, glv_consts(), Wfull, ctx->ws[WS_GLV_SC].as<int32_t>());
            else
                VK_LAUNCH(ctx, "glv_split", (k_glv_split<Fr>), (n + 255) / 256, 256, 0, d_sc, (uint32_t)n, mont,
                          glv_consts(), halves);
            if (nsl == 2) {
                fork = ctx->get_event();
                VK_CHECK_HIP(hipEventRecord(fork, ctx->stream));
                VK_CHECK_HIP(hipStreamWaitEvent(ctx->side_stream, fork, 0));
            }
            // [w][2n] limb-form copies: entry w * 2n + i (sort_entries' stride)
            const auto* win = t->win.as<typename Fast29<C>::type::AffN>();
            GlvDigits src{halves, inf, (uint32_t)n};
            if (shared && top_shift > 0) {
                src.tw = Wfull - 1;
                src.ts = top_shift;
            }
            for (int k = 0; k < nsl; k++) {
                if (radix_m > 1) {
                    RadixDigits rd{ctx->ws[WS_GLV_SC].as<int32_t>(), (uint32_t)nv};
                    rd.off = (uint32_t)offset;  // the point range inside the table's copies
                    rd.half = (uint32_t)n;
                    rd.gap = (uint32_t)(t->n - n);
                    sl[k].stride = (uint32_t)(2 * t->n);
                    if (t->win_pair) {
                        const auto* wp = t->win.as<typename Fast29<C>::type::AffP>();
                        VK_TRY(slice_enqueue<C>(ctx, sl[k], rd, nv, wp, wp, 0xffffffffu, k == 1 ? acc0 : nullptr,
                                                k == 0 ? acc0 : nullptr));
                    } else {
                        VK_TRY(slice_enqueue<C>(ctx, sl[k], rd, nv, win, win, 0xffffffffu, k == 1 ? acc0 : nullptr,
                                                k == 0 ? acc0 : nullptr));
                    }
                }
                else if (shared && !t->win_limbs)  // (power-of-two shared windows: whole tables only)
                    VK_TRY(slice_enqueue<C>(ctx, sl[k], src, nv, t->win.as<Aff>(), t->win.as<Aff>(), 0xffffffffu,
                                            k == 1 ? acc0 : nullptr, k == 0 ? acc0 : nullptr));
                else if (shared)
                    VK_TRY(slice_enqueue<C>(ctx, sl[k], src, nv, win, win, 0xffffffffu, k == 1 ? acc0 : nullptr,
                                            k == 0 ? acc0 : nullptr));
                else
                    VK_TRY(slice_enqueue<C>(ctx, sl[k], src, nv, bases, dphi, (uint32_t)n, k == 1 ? acc0 : nullptr,
                                            k == 0 ? acc0 : nullptr));
            }
        }
    } else {
        if (nsl == 2) {
            fork = ctx->get_event();
            VK_CHECK_HIP(hipEventRecord(fork, ctx->stream));
            VK_CHECK_HIP(hipStreamWaitEvent(ctx->side_stream, fork, 0));
        }
        for (int k = 0; k < nsl; k++)
            VK_TRY(slice_enqueue<C>(ctx, sl[k], ScalarDigits<Fr>{d_sc, inf, mont}, nv, bases, bases, 0xffffffffu,
                                    k == 1 ? acc0 : nullptr, k == 0 ? acc0 : nullptr));
    }
    for (int k = 0; k < nsl; k++) VK_TRY(slice_fetch<C>(sl[k]));
    const double t_enq = host_timing() ? now_us() : 0.0;
    if (host_timing()) VK_CHECK_HIP(hipStreamSynchronize(sl[nsl - 1].L.st));
    const double t_sync = host_timing() ? now_us() : 0.0;
    Acc res = C::zero();
    for (int k = 0; k < nsl; k++) {
        Acc r;
        VK_TRY(slice_finish<C>(ctx, sl[k], &r));
        res = C::add(res, r);
    }
    if (host_timing())
        fprintf(stderr, "msm_host n=%zu first_launch_us=%.1f enqueue_us=%.1f wait_us=%.1f fold_us=%.1f\n", n,
                sl[0].t_launch0 - t_entry, t_enq - t_entry, t_sync - t_enq, now_us() - t_sync);
    if (nsl == 2) {  // later work on the context's stream stays ordered after lane 1
        join = ctx->get_event();
        VK_CHECK_HIP(hipEventRecord(join, ctx->side_stream));
        VK_CHECK_HIP(hipStreamWaitEvent(ctx->stream, join, 0));
        ctx->event_pool.push_back(fork);  // a wait binds the record it saw: safe to re-record
        ctx->event_pool.push_back(join);
        ctx->event_pool.push_back(acc0);
    }
    memcpy(out_acc, &res, sizeof(Acc));
    return VC_OK;
}

// K MSMs over one whole table (e.g. a KZG commitment and its opening proof over the Lagrange
// SRS): one pipeline for all K -- the radix digits of every scalar set, ONE sort into K bucket
// sets (bucket set k of entry (k, w, i) names the same window copy B^w P_i), one accumulate
// launch, one fix-up and one reduction over the K sets -- so the latency-bound tail and the
// launch gaps are paid once, not K times. Only the radix shared-window geometry (BLS12-381, GLV,
// whole table from 2^18 points) batches; other tables run the K MSMs one by one.
template <class C, class Fr>
static int msm_run_many_t(vc_ctx* ctx, Table* t, const void* const* d_sc, const int* mont, size_t n, size_t K,
                          uint32_t* out_accs) {
    using Acc = typename C::Acc;
    bool batched = false;
    if constexpr (std::is_same<C, BLS381G1>::value) {
        bool glv = false;
        if (K > 1 && n == t->n && n >= (1u << 18) && n < (1u << 30) && ctx->opt_shared_windows != 0 &&
            !getenv("VKZG_MSM_RADIX") && !getenv("VKZG_MSM_C") && !getenv("VKZG_WIN_PACKED") &&
            (uint64_t)2 * n * 7 * std::min<size_t>(K, 8) < 0xffffffffull)
            VK_TRY(glv_table_ok(ctx, t, &glv));
        if (glv) {
            VK_TRY(fast_tables<C>(ctx, t, true));
            const int st = win_tables<C>(ctx, t, 16, 7, 0, 5, win_pair_on());
            if (st == VC_E_OOM) t->win.release();
            else if (st != VC_OK) return st;
            batched = st == VC_OK;
        }
        if (batched) {
            const size_t nv = 2 * n;
            const int Ws = 7;
            // up to 8 bucket sets per pipeline (the sort's LDS histogram holds 8 x 1280 coarse bins)
            for (size_t k0 = 0; k0 < K; k0 += 8) {
                const size_t Kb = std::min<size_t>(8, K - k0);
                if (Kb == 1) {
                    VK_TRY(msm_run(ctx, t, 0, d_sc[k0], n, mont[k0], out_accs + k0 * (sizeof(Acc) / 4)));
                    continue;
                }
                VK_TRY(ctx->ws[WS_GLV_SC].ensure(nv * 4 * (size_t)Ws * Kb));
                MsmSlice<C> sl;
                sl.L = ctx->lane(0);
                sl.c = 16;
                sl.m = 5;
                sl.shared = true;
                sl.sets = (int)Kb;
                sl.wps = (uint32_t)Ws;
                sl.wb = 0;
                sl.we = Ws * (int)Kb;
                sl.W = sl.we;
                sl.radix.inf = t->inf.as<uint8_t>();
                sl.radix.n = (uint32_t)n;
                sl.radix.dig = ctx->ws[WS_GLV_SC].as<int32_t>();
                for (size_t k = k0; k < k0 + Kb; k++) {  // the GLV split of every set runs in slice_enqueue
                    sl.radix.sc.push_back(static_cast<const uint32_t*>(d_sc[k]));
                    sl.radix.mont.push_back(mont[k]);
                }
                if (t->win_pair) {
                    const auto* wp = t->win.as<typename Fast29<C>::type::AffP>();
                    VK_TRY(slice_enqueue<C>(ctx, sl, RadixDigits{sl.radix.dig, (uint32_t)nv}, nv, wp, wp, 0xffffffffu,
                                            nullptr, nullptr));
                } else {
                    const auto* win = t->win.as<typename Fast29<C>::type::AffN>();
                    VK_TRY(slice_enqueue<C>(ctx, sl, RadixDigits{sl.radix.dig, (uint32_t)nv}, nv, win, win,
                                            0xffffffffu, nullptr, nullptr));
                }
                VK_TRY(slice_fetch<C>(sl));
                std::vector<Acc> res(Kb);
                VK_TRY(slice_finish<C>(ctx, sl, res.data()));
                memcpy(out_accs + k0 * (sizeof(Acc) / 4), res.data(), Kb * sizeof(Acc));
            }
            ctx->plan = {16, Ws, 2, 5, 1};
            return VC_OK;
        }
    }
    for (size_t k = 0; k < K; k++)
        VK_TRY(msm_run(ctx, t, 0, d_sc[k], n, mont[k], out_accs + k * (sizeof(Acc) / 4)));
    return VC_OK;
}

int msm_run_many(vc_ctx* ctx, Table* t, const void* const* d_sc, const int* mont, size_t n, size_t K, uint32_t* out) {
    switch (t->curve) {
        case VC_CURVE_BN254:
            return msm_run_many_t<BN254G1, BN254Fr>(ctx, t, d_sc, mont, n, K, out);
        case VC_CURVE_BLS12_381:
            return msm_run_many_t<BLS381G1, BLS381Fr>(ctx, t, d_sc, mont, n, K, out);
        case VC_CURVE_BANDERSNATCH:
            return msm_run_many_t<Bandersnatch, BandFr>(ctx, t, d_sc, mont, n, K, out);
    }
    return VC_E_INVALID;
}

// ------------------------------------------------------------------ sparse batched commits
// Rows of a CSR matrix (row g = commit g: non-zero (column i, scalar s) pairs) against the
// fixed-base window tables of a table: every non-zero expands to its non-zero signed window
// digits, each a table point T[i][w][|d|-1] -- so the entries of a row are contiguous and the
// rows play the buckets of the Pippenger accumulate: the same balanced k_msm_accumulate (M
// entries per thread, rows straddling threads merged by the fix-up) sums them. For verkle
// nodes (~5 non-zeros of 256 per internal node, 2 of N per extension row) this replaces
// dense width-256 rows.
// the signed digits of a scalar over a fixed-base table's windows (widths g.width(w), ctx.hpp)
template <class Fr, class Fn>
__device__ __forceinline__ void for_each_digit_fb(fe<Fr> s, const FbGeom& g, Fn&& f) {
    uint32_t carry = 0;
    for (int w = 0; w < g.W; w++) {
        const int c = g.width(w);
        const uint32_t raw = (s.v[0] & ((1u << c) - 1)) + carry;
#pragma unroll
        for (int k = 0; k < 7; k++) s.v[k] = (s.v[k] >> c) | (s.v[k + 1] << (32 - c));
        s.v[7] >>= c;
        carry = raw > (1u << (c - 1)) ? 1u : 0u;
        f(w, carry ? (int32_t)raw - (int32_t)(1u << c) : (int32_t)raw);
    }
}

template <class Fr>
__global__ void k_sparse_count(const uint32_t* __restrict__ sc, size_t nnz, int mont, FbGeom g,
                               uint32_t* __restrict__ cnt) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    fe<Fr> s = load_scalar<Fr>(sc, j);
    if (mont) s = fe_from_mont<Fr>(s);
    uint32_t k = 0;
    for_each_digit_fb<Fr>(s, g, [&](int, int32_t d) { k += d != 0; });
    cnt[j] = k;
}

template <class Fr>
__global__ void k_sparse_expand(const uint32_t* __restrict__ sc, const uint32_t* __restrict__ cols, size_t nnz,
                                int mont, FbGeom g, const uint32_t* __restrict__ eoff,
                                uint32_t* __restrict__ entries) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    fe<Fr> s = load_scalar<Fr>(sc, j);
    if (mont) s = fe_from_mont<Fr>(s);
    const uint32_t base = cols[j] * (uint32_t)g.stride();
    uint32_t pos = eoff[j];
    for_each_digit_fb<Fr>(s, g, [&](int w, int32_t d) {
        if (d != 0)
            entries[pos++] = (base + (uint32_t)g.off(w) + (uint32_t)(d < 0 ? -d : d) - 1) | (d < 0 ? 0x80000000u : 0u);
    });
}

// Fused form of count + scan + expand + rows (round 6): two launches instead of six (the hipcub
// scan's two, the count, the expand, the row offsets and a fill) -- each tiny launch costs ~4.5 us
// of GPU time even when the host is ahead (profiles/r06/verkle/norm_early/timeline_full_and_update.txt).
// K1: elements [256 b, 256 b + 256) of block b (j <= nnz: the grid has nnz / 256 + 1 blocks, so
// j = nnz is always some block's element, with count 0) -> local[j] = the exclusive count prefix
// inside the block, bsum[b] = its total; the last block to arrive scans the block totals into
// boff[0 .. nb] (boff[nb] = all entries) and resets the arrival counter for the next launch.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < wv; k++) before += s_w[k];
    *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return before + x - v;
}
template <class Fr>
__global__ void __launch_bounds__(256) k_sparse_count_scan(const uint32_t* __restrict__ sc, size_t nnz, int mont,
                                                          FbGeom g, uint32_t* __restrict__ local,
                                                          uint64_t* __restrict__ bsum, uint32_t* __restrict__ boff,
                                                          uint32_t* __restrict__ counter, uint32_t* __restrict__ chain_max,
                                                          uint32_t epoch) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_last;
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t k = 0;
    if (j < nnz) {
        fe<Fr> s = load_scalar<Fr>(sc, j);
        if (mont) s = fe_from_mont<Fr>(s);
        for_each_digit_fb<Fr>(s, g, [&](int, int32_t d) { k += d != 0; });
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan256(k, s_w, &tot);
    if (j <= nnz) local[j] = ex;
    if (chain_max && blockIdx.x == 0 && threadIdx.x == 0) *chain_max = 0;
    const uint32_t nb = gridDim.x;
    const uint64_t tag = (uint64_t)epoch << 32;
    // the block total as one (epoch << 32 | total) word and no fence before the arrival: the last
    // block polls the words until they carry this launch's epoch (a fence per block writes back its
    // XCD's whole L2: ~28 us for the 1,025 blocks of a 262,144-non-zero level)
    if (threadIdx.x == 0) {
        __hip_atomic_store(&bsum[blockIdx.x], tag | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = atomicAdd(counter, 1u) == nb - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    auto total_of = [&](uint32_t b) -> uint32_t {  // (bounded: 10 ms)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const uint64_t w = __hip_atomic_load(&bsum[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((w & 0xffffffff00000000ull) == tag || __builtin_amdgcn_s_memrealtime() - t0 > 1000000ull)
                return (uint32_t)w;
        }
    };
    // the last block: exclusive scan of the nb block totals, ceil(nb / 256) consecutive per thread
    // (the loads of a thread's totals go out together: one after another they cost ~1-2 us each,
    // 30 us for the 1,025 blocks of a 262,144-non-zero level)
    const uint32_t per = (nb + 255) / 256, b0 = min(threadIdx.x * per, nb), b1 = min(b0 + per, nb);
    constexpr uint32_t PR = 8;
    uint32_t v[PR];
    uint32_t seg = 0;
    if (per <= PR) {
#pragma unroll
        for (uint32_t q = 0; q < PR; q++) v[q] = b0 + q < b1 ? total_of(b0 + q) : 0u;
#pragma unroll
        for (uint32_t q = 0; q < PR; q++) seg += v[q];
    } else {
        for (uint32_t b = b0; b < b1; b++) seg += total_of(b);
    }
    uint32_t all;
    uint32_t run = block_excl_scan256(seg, s_w, &all);
    if (per <= PR) {
#pragma unroll
        for (uint32_t q = 0; q < PR; q++) {
            if (b0 + q < b1) boff[b0 + q] = run;
            run += v[q];
        }
    } else {
        for (uint32_t b = b0; b < b1; b++) {
            boff[b] = run;
            run += total_of(b);
        }
    }
    if (threadIdx.x == 0) {
        boff[nb] = all;
        *counter = 0;  // for the next launch (stream-ordered after this one)
    }
}
// K2: thread i < nnz expands element i's digits at boff[i / 256] + local[i]; thread i <= nch sets
// chunk i's entry offset (rp[i] is an element index <= nnz) and, for an empty chunk, its identity
template <class Fr, class C>
__global__ void __launch_bounds__(256) k_sparse_expand_rows(const uint32_t* __restrict__ sc,
                                                           const uint32_t* __restrict__ cols, size_t nnz, int mont,
                                                           FbGeom g, const uint32_t* __restrict__ local,
                                                           const uint32_t* __restrict__ boff,
                                                           uint32_t* __restrict__ entries,
                                                           const uint64_t* __restrict__ rp, size_t nch,
                                                           uint32_t* __restrict__ offsets,
                                                           typename C::Acc* __restrict__ chunks) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nnz) {
        fe<Fr> s = load_scalar<Fr>(sc, i);
        if (mont) s = fe_from_mont<Fr>(s);
        const uint32_t base = cols[i] * (uint32_t)g.stride();
        uint32_t pos = boff[i >> 8] + local[i];
        for_each_digit_fb<Fr>(s, g, [&](int w, int32_t d) {
            if (d != 0)
                entries[pos++] = (base + (uint32_t)g.off(w) + (uint32_t)(d < 0 ? -d : d) - 1) | (d < 0 ? 0x80000000u : 0u);
        });
    }
    if (i <= nch) {
        auto at = [&](uint64_t e) { return boff[e >> 8] + local[e]; };
        const uint32_t o = at(rp[i]);
        offsets[i] = o;
        if (i < nch && at(rp[i + 1]) == o) chunks[i] = C::zero();
    }
}

// row offsets in entry space; empty rows get the identity (the accumulate never writes them)
template <class C>
__global__ void k_sparse_rows(const uint64_t* __restrict__ row_ptr, const uint32_t* __restrict__ eoff, size_t batch,
                              uint32_t* __restrict__ offsets, typename C::Acc* __restrict__ rows) {
    size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g > batch) return;
    offsets[g] = eoff[row_ptr[g]];
    if (g < batch && eoff[row_ptr[g + 1]] == eoff[row_ptr[g]]) rows[g] = C::zero();
}

// row g = sum of its chunks [rc[g], rc[g+1]) -- one wave per row: lanes load chunk sums (a
// strided loop when a row has more than 64), then an xor butterfly over the used lanes
template <class C>
__global__ void __launch_bounds__(64) k_sparse_combine(const typename C::Acc* __restrict__ chunks,
                                                      const uint32_t* __restrict__ rc, typename C::Acc* __restrict__ rows) {
    using Acc = typename C::Acc;
    const uint32_t g = blockIdx.x, lane = threadIdx.x;
    const uint32_t b = rc[g], n = rc[g + 1] - b;
    if (n == 1) {  // uniform per wave
        if (lane == 0) rows[g] = chunks[b];
        return;
    }
    uint32_t span = 1, lg = 0;
    while (span < n && span < 64) {
        span <<= 1;
        lg++;
    }
    const uint32_t nk = (n + 63) / 64;
    Acc v = C::zero();
    for (uint32_t it = 0; it < nk + lg; it++) {  // one add call site (see msm_tail.hip)
        Acc o;
        if (it < nk) {
            const uint32_t k = lane + it * 64;
            o = k < n ? chunks[b + k] : C::zero();
        } else {
            const uint32_t m = 1u << (it - nk);
            const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
            uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
            for (int k = 0; k < C::ACC_WORDS; k++) dst[k] = __shfl_xor(src[k], m, 64);
        }
        v = C::add(v, o);
    }
    if (lane == 0) rows[g] = v;
}

__global__ void k_iota(uint32_t* __restrict__ o, uint32_t n);

// Chunk lists of a CSR row structure (host): rows are cut into chunks of <= CHNZ non-zeros (the
// accumulate's buckets), so a long row (e.g. a verkle root: 256 children x W windows) does not
// become one bucket straddling hundreds of threads -- whose pieces the fix-up would add serially;
// chunk sums are folded per row by k_sparse_combine. rc[g] = first chunk of row g (an empty row
// gets one empty chunk), cptr = chunk ends. When every row has 1..CHNZ non-zeros the chunks are
// the rows (identity: rc = 0..batch, cptr = row_ptr; nothing is built).
constexpr size_t SPARSE_CHNZ = 4;
struct SparseChunks {
    const uint32_t* rc = nullptr;    // row g's chunks are [rc[g], rc[g + 1])
    const uint64_t* cptr = nullptr;  // chunk k's non-zeros are [cptr[k], cptr[k + 1])
    size_t nch = 0;
    bool identity = false;
};
// The chunk lists in one serial pass, straight into page-locked staging (one upload each): the two
// pooled passes into fresh vectors they replace cost ~0.1 ms of idle GPU on a 17k-row verkle level
// (the pool's wake-ups and page faults; profiles/r05/verkle/sparse_norm_vk/). The previous call's
// uploads from the staging have completed: every sparse commit ends in a normalisation that saw its
// first kernel finish (or waited for the stream).
static int sparse_chunks(vc_ctx* ctx, const uint64_t* row_ptr, size_t batch, bool rows_fit, SparseChunks* out) {
    const size_t CHNZ = SPARSE_CHNZ;
    if (rows_fit) {  // the caller knows every row has 1..CHNZ non-zeros
        out->identity = true;
        out->nch = batch;
        return VC_OK;
    }
    // max(1, ceil(len / CHNZ)) <= 1 + floor(len / CHNZ) chunks per row
    const size_t cap = batch + row_ptr[batch] / CHNZ;
    VK_TRY(ctx->pin_sparse_ch.ensure((cap + 1) * 8 + (batch + 1) * 4));
    uint64_t* cptr = ctx->pin_sparse_ch.as<uint64_t>();
    uint32_t* rc = reinterpret_cast<uint32_t*>(cptr + cap + 1);
    size_t run = 0;
    cptr[0] = 0;
    for (size_t g = 0; g < batch; g++) {
        rc[g] = (uint32_t)run;
        const uint64_t lo = row_ptr[g], hi = row_ptr[g + 1];
        if (lo == hi) {  // an empty row is one empty chunk (the identity)
            cptr[++run] = lo;
            continue;
        }
        for (uint64_t j = lo; j < hi; j += CHNZ) cptr[++run] = std::min<uint64_t>(j + CHNZ, hi);
    }
    rc[batch] = (uint32_t)run;
    out->rc = rc;
    out->cptr = cptr;
    out->nch = run;
    return VC_OK;
}

// The sparse commit on the device: columns d_cols (u32) and scalars d_sc (4 u64, canonical unless
// mont) already in device memory, the row structure row_ptr on the host (the chunk lists; rows_fit:
// every row has 1..CHNZ non-zeros). Outputs on the device: canonical affine rows d_xy / d_inf and,
// with d_items (BN254), their to_data_item values. Enqueued on ctx->stream; the normalisation's
// host step synchronises it once (normalize_split), nothing else waits.
// row g += the canonical affine point (cxy[id], cinf[id]) of id = add_ids[g] (none: 0xffffffff)
template <class C>
__global__ void k_rows_add_base(typename C::Acc* __restrict__ rows, size_t batch, const uint32_t* __restrict__ add_ids,
                                const uint64_t* __restrict__ cxy, const uint8_t* __restrict__ cinf) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= batch) return;
    const uint32_t id = add_ids[g];
    if (id == 0xffffffffu || cinf[id]) return;
    using F = typename C::F;
    typename C::Aff a;
    memcpy(a.x.v, cxy + (size_t)id * 2 * (F::N / 2), F::N * 4);
    memcpy(a.y.v, cxy + (size_t)id * 2 * (F::N / 2) + F::N / 2, F::N * 4);
    a.x = fe_to_mont<F>(a.x);
    a.y = fe_to_mont<F>(a.y);
    rows[g] = C::madd(rows[g], a, false);
}

template <class C, class Fr>
static int sparse_commit_dev(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, bool rows_fit,
                             const uint32_t* d_cols_in, const void* d_sc_in, int mont, void* d_xy, uint8_t* d_inf,
                             void* d_items, const uint32_t* d_add_ids = nullptr, const uint64_t* d_add_xy = nullptr,
                             const uint8_t* d_add_inf = nullptr, const uint32_t* d_dst = nullptr,
                             const std::function<void()>* overlap = nullptr, const uint64_t* d_row_ptr = nullptr) {
    using Acc = typename C::Acc;
    if (batch == 0) return VC_OK;
    const size_t nnz = row_ptr[batch];
    static const bool verbose = getenv("VKZG_VERBOSE") != nullptr;
    auto tic = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!verbose) return;
        (void)hipStreamSynchronize(ctx->stream);
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[sparse %zu rows %zu nnz] %s %.3f ms\n", batch, nnz, what,
                std::chrono::duration<double, std::milli>(now - tic).count());
        tic = now;
    };
    if (t->fb_c == 0) VK_TRY(fixed_base_precompute(ctx, t, 8));
    const FbGeom fg = t->fb_geom();
    const int W = fg.W;
    SparseChunks ch;
    VK_TRY(sparse_chunks(ctx, row_ptr, batch, rows_fit, &ch));
    const size_t nch = ch.nch;
    if ((uint64_t)t->n * fg.stride() >= (1ull << 31)) return VC_E_RANGE;  // entry index + sign bit
    const size_t maxL = nnz * (size_t)W;
    if (maxL >= 0xffffffffull) return VC_E_RANGE;
    hipStream_t st = ctx->stream;
    // grow-only ctx workspaces (the MSM's own slots for entries / carries / scan scratch: the
    // two paths never run concurrently on one ctx)
    DevBuf& d_rp = ctx->ws[WS_SP_RP];
    DevBuf& d_cnt = ctx->ws[WS_SP_CNT];
    DevBuf& d_eoff = ctx->ws[WS_SP_EOFF];
    DevBuf& d_ent = ctx->ws[WS_SORTED];
    DevBuf& d_off = ctx->ws[WS_SP_OFF];
    DevBuf& d_rows = ctx->ws[WS_SP_ROWS];
    DevBuf& d_carry = ctx->ws[WS_CARRY];
    DevBuf& d_thr = ctx->ws[WS_THROUGH];
    DevBuf& d_own = ctx->ws[WS_OWNER];
    DevBuf& d_ownb = ctx->ws[WS_OWNER_B];
    DevBuf& d_tmp = ctx->ws[WS_SCAN_TMP];
    uint32_t M = (uint32_t)std::min<size_t>(64, std::max<size_t>(16, maxL / 131072));
    if (const char* em = getenv("VKZG_SPARSE_M")) M = (uint32_t)std::max(1, atoi(em));  // tuning probe (read per call)
    const uint32_t Tmax = (uint32_t)((maxL + M - 1) / M);
    DevBuf& d_rc = ctx->ws[WS_SP_RC];
    DevBuf& d_chunks = ctx->ws[WS_SP_CHUNKS];
    // chunk lists: cptr and rc lie back to back in the page-locked staging (sparse_chunks), so they
    // go up in one copy into d_rp (rc at the same offset); identity rows use d_rc for their iota
    const size_t rc_off = ch.identity ? 0 : (size_t)(reinterpret_cast<const uint8_t*>(ch.rc) -
                                                     reinterpret_cast<const uint8_t*>(ch.cptr));
    VK_TRY(d_rp.ensure(ch.identity ? (nch + 1) * 8 : rc_off + (batch + 1) * 4));
    VK_TRY(d_rc.ensure((batch + 1) * 4));
    VK_TRY(d_chunks.ensure(nch * sizeof(Acc)));
    VK_TRY(d_cnt.ensure((nnz + 1) * 4));
    VK_TRY(d_eoff.ensure((nnz + 1) * 4));
    VK_TRY(d_ent.ensure(std::max<size_t>(maxL, 1) * 4));
    VK_TRY(d_off.ensure((nch + 1) * 4));
    VK_TRY(d_rows.ensure(batch * sizeof(Acc)));
    VK_TRY(d_carry.ensure((size_t)(Tmax + 8) * sizeof(FAcc<C>)));
    VK_TRY(d_thr.ensure((size_t)(Tmax + 8)));
    VK_TRY(d_own.ensure((size_t)(Tmax + 8) * sizeof(FAcc<C>)));
    VK_TRY(d_ownb.ensure((size_t)(Tmax + 8) * 4));
    lap("host chunk lists");
    // rows as chunks: the row pointers are the chunk pointers -- the caller's device copy when it
    // has one (d_row_ptr: the verkle extension rows upload theirs with the rows, or make them on the
    // device), else one upload
    const uint64_t* rp_dev = d_rp.as<uint64_t>();
    const uint32_t* rc_dev = d_rc.as<uint32_t>();
    if (ch.identity) {  // (no chunk lists: the combine, their only reader, is skipped)
        if (d_row_ptr) rp_dev = d_row_ptr;
        else VK_CHECK_HIP(hipMemcpyAsync(d_rp.p, row_ptr, (batch + 1) * 8, hipMemcpyHostToDevice, st));
    } else {
        VK_CHECK_HIP(hipMemcpyAsync(d_rp.p, ch.cptr, rc_off + (batch + 1) * 4, hipMemcpyHostToDevice, st));
        rc_dev = reinterpret_cast<const uint32_t*>(d_rp.as<uint8_t>() + rc_off);
    }
    const uint32_t* d_cols = d_cols_in;
    const uint32_t* d_sc = static_cast<const uint32_t*>(d_sc_in);
    VK_TRY(ctx->ws[WS_CHAIN].ensure(4));
    uint32_t* chain_max = ctx->ws[WS_CHAIN].as<uint32_t>();
    // VKZG_SPARSE_FUSED=0 (read per call, A/B): the count, the hipcub scan, the expand and the row
    // offsets as separate launches
    const char* fe_env = getenv("VKZG_SPARSE_FUSED");
    const bool fused = !(fe_env && atoi(fe_env) == 0);
    if (fused) {
        // the arrival counter: a word of the normalisation's zeroed counter buffer (commit.hip)
        DevBuf& cntb = ctx->ws[WS_NORM_CNT];
        if (cntb.p == nullptr) {
            VK_TRY(cntb.ensure(256));
            VK_CHECK_HIP(hipMemsetAsync(cntb.p, 0, 256, st));
        }
        const size_t nb = nnz / 256 + 1;  // elements 0 .. nnz
        VK_TRY(d_eoff.ensure(nb * 8 + (nb + 1) * 4));
        uint64_t* bsum = d_eoff.as<uint64_t>();
        uint32_t* boff = reinterpret_cast<uint32_t*>(bsum + nb);
        const uint32_t epoch = ++ctx->small_epoch == 0 ? ++ctx->small_epoch : ctx->small_epoch;  // never 0
        VK_LAUNCH(ctx, "sparse_count_scan", (k_sparse_count_scan<Fr>), (unsigned)nb, 256, 0, d_sc, nnz, mont, fg,
                  d_cnt.as<uint32_t>(), bsum, boff, cntb.as<uint32_t>() + 16, Tmax > 0 ? chain_max : (uint32_t*)nullptr,
                  epoch);
        VK_LAUNCH(ctx, "sparse_expand_rows", (k_sparse_expand_rows<Fr, C>), (unsigned)((std::max(nnz, nch + 1) + 255) / 256),
                  256, 0, d_sc, d_cols, nnz, mont, fg, d_cnt.as<uint32_t>(), boff, d_ent.as<uint32_t>(), rp_dev, nch,
                  d_off.as<uint32_t>(), d_chunks.as<Acc>());
    } else {
        VK_CHECK_HIP(hipMemsetAsync(d_cnt.as<uint32_t>() + nnz, 0, 4, st));
        if (nnz)
            VK_LAUNCH(ctx, "sparse_count", (k_sparse_count<Fr>), (nnz + 255) / 256, 256, 0, d_sc, nnz, mont, fg,
                      d_cnt.as<uint32_t>());
        size_t tmp_bytes = 0;
        VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_cnt.as<uint32_t>(), d_eoff.as<uint32_t>(),
                                                      nnz + 1, st));
        VK_TRY(d_tmp.ensure(std::max<size_t>(tmp_bytes, 1)));
        VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp.p, tmp_bytes, d_cnt.as<uint32_t>(), d_eoff.as<uint32_t>(),
                                                      nnz + 1, st));
        if (nnz)
            VK_LAUNCH(ctx, "sparse_expand", (k_sparse_expand<Fr>), (nnz + 255) / 256, 256, 0, d_sc, d_cols, nnz, mont, fg,
                      d_eoff.as<uint32_t>(), d_ent.as<uint32_t>());
        VK_LAUNCH(ctx, "sparse_rows", (k_sparse_rows<C>), (nch + 1 + 255) / 256, 256, 0, rp_dev,
                  d_eoff.as<uint32_t>(), nch, d_off.as<uint32_t>(), d_chunks.as<Acc>());
        if (Tmax > 0) VK_CHECK_HIP(hipMemsetAsync(chain_max, 0, 4, st));
    }
    // the fixed-base tables hold radix-2^29 limbs in 128-B entries (ec29.hpp FbE): the accumulate
    // reads the entries' limbs (is_fbe)
    using FA = FbE<C>;
    const FA* tab = t->fb.as<FA>();
    if (Tmax > 0) {  // all-zero rows only: the row offsets already set every chunk to the identity
        using RAcc = FAcc<C>;
        DevBuf& d_raw = ctx->ws[WS_RAW_B];
        VK_TRY(d_raw.ensure(nch * sizeof(RAcc)));
        VK_LAUNCH(ctx, "sparse_accumulate", (k_msm_accumulate<C, FA>), (Tmax + 255) / 256, 256, 0, tab, tab, 0xffffffffu,
                  d_ent.as<uint32_t>(), d_off.as<uint32_t>(), (uint32_t)nch, M, d_raw.as<RAcc>(), d_carry.as<RAcc>(),
                  d_thr.as<uint8_t>(), d_own.as<RAcc>(), d_ownb.as<uint32_t>(), chain_max, acc_merge(),
                  (unsigned long long*)nullptr);
        // straddling chunks merged by the serial walk of their owners, no chain limit: a chunk holds at
        // most CHNZ x W entries, so it spans at most CHNZ W / M + 2 threads. (The pointer-jumping rounds
        // used before read the longest chain back first -- a host sync per level -- and ran ~3 guarded
        // launches: 0.6 ms of the 65,536-key full commitment's kernels.)
        VK_TRY(msm_tail_fixup_walk<C>(ctx, ctx->lane(0), d_off.as<uint32_t>(), (uint32_t)nch, M, d_raw.as<RAcc>(),
                                      d_carry.as<RAcc>(), d_own.as<RAcc>(), 0xffffffffu, d_ownb.as<uint32_t>(),
                                      d_thr.as<uint8_t>(), Tmax));
        VK_LAUNCH(ctx, "sparse_store", (k_fast_store<C>), (nch + 255) / 256, 256, 0, d_raw.as<RAcc>(), (uint32_t)nch,
                  d_off.as<uint32_t>(), d_chunks.as<Acc>());
    }
    // one chunk per row (identity): the chunk sums are the rows -- no combine launch (a one-wave
    // block per row only copied them: ~60 us for the 131,072 extension c1 / c2 rows)
    Acc* rows_p = d_rows.as<Acc>();
    if (ch.identity)
        rows_p = d_chunks.as<Acc>();
    else
        VK_LAUNCH(ctx, "sparse_combine", (k_sparse_combine<typename C::Inl>), batch, 64, 0, d_chunks.as<Acc>(),
                  rc_dev, rows_p);
    if constexpr (std::is_same<C, BN254G1>::value) {
        // BN254 rows with items (the verkle levels): the old-commitment adds, the canonical points,
        // their items and the placement at d_dst in normalize_rows_items' two kernels, the block
        // products polled from page-locked memory (no copies, no stream wait, no separate item /
        // scatter launches: ~40 us of idle GPU per level before, profiles/r05/verkle/)
        if (d_items) {
            lap("kernels");
            return normalize_rows_items(ctx, rows_p, batch, d_add_ids, d_add_xy, d_add_inf, d_dst,
                                        static_cast<uint64_t*>(d_xy), d_inf, static_cast<uint64_t*>(d_items), overlap);
        }
    }
    if (d_dst || overlap) return VC_E_INVALID;  // (BN254 with items only)
    if (d_add_ids)  // rows that update a previous commitment: C_old + sum (delta_k) L_k
        VK_LAUNCH(ctx, "sparse_add_base", (k_rows_add_base<C>), (unsigned)((batch + 255) / 256), 256, 0,
                  rows_p, batch, d_add_ids, d_add_xy, d_add_inf);
    lap("kernels");
    VK_TRY(normalize_to_canon(ctx, ctx->curve, rows_p, batch, d_xy, d_inf));
    lap("normalise");
    if (d_items) VK_TRY(to_data_item_device(ctx, d_xy, d_inf, batch, d_items));
    return VC_OK;
}

template <class C, class Fr>
static int msm_batch_sparse_t(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                              const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf,
                              uint64_t* out_items = nullptr) {
    if (batch == 0) return VC_OK;
    const size_t nnz = row_ptr[batch];
    // argument checks on the host pool (verkle levels: 10^5 rows / non-zeros)
    std::vector<uint8_t> bad_part(host_pool().size(), 0);
    host_pool().run([&](unsigned k) {
        const unsigned T = host_pool().size();
        uint8_t b = 0;
        for (size_t g = batch * k / T; g < batch * (k + 1) / T; g++) b |= row_ptr[g + 1] < row_ptr[g] ? 1 : 0;
        for (size_t j = nnz * k / T; j < nnz * (k + 1) / T; j++) b |= cols[j] >= t->n ? 2 : 0;
        bad_part[k] = b;
    });
    uint8_t bad = 0;
    for (uint8_t b : bad_part) bad |= b;
    if (bad & 1) return VC_E_INVALID;
    if (bad & 2) return VC_E_RANGE;
    hipStream_t st = ctx->stream;
    DevBuf& d_cols = ctx->ws[WS_SP_COLS];
    DevBuf& d_sc = ctx->ws[WS_SP_SC];
    DevBuf& d_xy = ctx->ws[WS_SP_XY];
    DevBuf& d_inf = ctx->ws[WS_SP_INF];
    DevBuf& d_it = ctx->ws[WS_SP_ITEMS];
    VK_TRY(d_cols.ensure(std::max<size_t>(nnz, 1) * 4));
    VK_TRY(d_sc.ensure(std::max<size_t>(nnz, 1) * 32));
    VK_TRY(d_xy.ensure(batch * 2 * C::F::N * 4));
    VK_TRY(d_inf.ensure(batch));
    if (out_items) VK_TRY(d_it.ensure(batch * 32));
    if (nnz) {
        VK_CHECK_HIP(hipMemcpyAsync(d_cols.p, cols, nnz * 4, hipMemcpyHostToDevice, st));
        VK_CHECK_HIP(hipMemcpyAsync(d_sc.p, scalars, nnz * 32, hipMemcpyHostToDevice, st));
    }
    VK_TRY((sparse_commit_dev<C, Fr>(ctx, t, batch, row_ptr, false, d_cols.as<uint32_t>(), d_sc.p, mont, d_xy.p,
                                     d_inf.as<uint8_t>(), out_items ? d_it.p : nullptr)));
    VK_CHECK_HIP(hipMemcpyAsync(out_xy, d_xy.p, batch * 2 * C::F::N * 4, hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipMemcpyAsync(out_inf, d_inf.p, batch, hipMemcpyDeviceToHost, st));
    if (out_items) VK_CHECK_HIP(hipMemcpyAsync(out_items, d_it.p, batch * 32, hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));  // host staging vectors die on return
    return VC_OK;
}

// ---- latency path of the sparse commits (verkle levels of a few thousand non-zeros). The
// sort-based path above is a chain of ~10 launches whose accumulate runs M = 16 serial mixed adds
// per thread and whose fix-up walks straddles serially: ~0.2 ms of kernels for a level of 1,000
// non-zeros, whatever its size (profiles/r05/verkle/). Here a wave takes a chunk of <= 64 of a
// row's (non-zero, window) pairs -- two non-zeros at W = 32 --, every lane adds its one table
// point (a load: the accumulator starts at the identity) and the wave folds on quad-cooperative
// adds (7 dependent ones); rows of several chunks are folded by k_sparse_combine.
// MODE 0: scalars vals[j] (4 canonical words); 1: 16-byte values (2 words: the leaf halves of
// an extension's c1 / c2 rows); 2: item[child[j]] - (sidx[j] < 0 ? 0 : snap[sidx[j]]) mod r (a
// verkle level's children's items from the mirror, minus the old item of a delta row's slot).
struct SmallChunk {
    uint32_t j0, npairs, p0, pad;  // the row's first non-zero, its pair count, this chunk's first pair
};
template <class C, class Fr, int MODE, int NT>
__global__ void __launch_bounds__(NT) k_fb_sparse_small(const FbE<C>* __restrict__ tab, const uint8_t* __restrict__ inf,
                                                       FbGeom fg, const SmallChunk* __restrict__ ck,
                                                       const uint32_t* __restrict__ cols, const uint64_t* __restrict__ vals,
                                                       const uint64_t* __restrict__ item, const uint32_t* __restrict__ child,
                                                       const int32_t* __restrict__ sidx, const uint64_t* __restrict__ snap,
                                                       typename C::Acc* __restrict__ part) {
    using FC = typename Fast29<C>::type;
    const SmallChunk c = ck[blockIdx.x];
    const uint32_t p = c.p0 + threadIdx.x, W = (uint32_t)fg.W;
    typename FC::Acc fa = FC::zero();
    if (p < c.npairs) {
        const size_t j = (size_t)c.j0 + p / W;
        const int w = (int)(p % W);
        const uint32_t col = cols[j];
        fe<Fr> s = fe_zero<Fr>();
        if constexpr (MODE == 0) {
            memcpy(s.v, vals + 4 * j, 32);
        } else if constexpr (MODE == 1) {
            memcpy(s.v, vals + 2 * j, 16);
        } else {
            memcpy(s.v, item + 4 * (size_t)child[j], 32);
            const int32_t k = sidx ? sidx[j] : -1;
            if (k >= 0) {
                fe<Fr> o;
                memcpy(o.v, snap + 4 * (size_t)k, 32);
                s = fe_sub<Fr>(s, o);  // canonical in, canonical out
            }
        }
        int32_t d = 0;
        for_each_digit_fb<Fr>(s, fg, [&](int ww, int32_t dd) {
            if (ww == w) d = dd;
        });
        if (d != 0 && !inf[col])
            fa = FC::madd(fa, tab[(size_t)col * fg.stride() + fg.off(w) + (uint32_t)(d < 0 ? -d : d) - 1].u, d < 0);
    }
    fb_block_sum_store<C, NT>(fa, &part[blockIdx.x]);
}

size_t sparse_small_pairs(const Table* t, size_t nnz) {
    const int W = t->fb_c ? t->fb_geom().W : 32;
    return nnz * (size_t)W;
}

int sparse_small_items_dev(vc_ctx* ctx, Table* t, const SmallRows& in, const std::function<void()>* overlap) {
    using C = BN254G1;
    using Fr = BN254Fr;
    using Acc = C::Acc;
    if (t->curve != VC_CURVE_BN254) return VC_E_INVALID;
    const size_t batch = in.batch;
    if (batch == 0) return VC_OK;
    if (t->fb_c == 0) VK_TRY(fixed_base_precompute(ctx, t, 8));
    const FbGeom fg = t->fb_geom();
    const uint64_t W = (uint64_t)fg.W;
    const uint64_t* rp = in.row_ptr;
    if (rp[batch] * W >= (1ull << 32)) return VC_E_RANGE;
    // chunks of NT pairs: a wave (7 dependent quad adds) while every row fits one (<= 2 non-zeros at
    // W = 32: the extension c1 / c2 rows), else 256 threads (9 adds; rows of <= 8 non-zeros -- the
    // extension rows [1, stem, c1, c2], an update's delta rows -- need no k_sparse_combine, whose
    // one full add per level costs ~30 us, profiles/r05/verkle/)
    uint64_t maxp = 0;
    for (size_t g = 0; g < batch; g++) maxp = std::max<uint64_t>(maxp, (rp[g + 1] - rp[g]) * W);
    const uint32_t NT = maxp <= 64 ? 64 : 256;
    // chunk table (host, page-locked: one upload) and, when a row has several chunks, rc
    size_t nch = 0;
    bool multi = false;
    for (size_t g = 0; g < batch; g++) {
        const uint64_t np = (rp[g + 1] - rp[g]) * W;
        const size_t k = np == 0 ? 1 : (size_t)((np + NT - 1) / NT);
        multi |= k > 1;
        nch += k;
    }
    const size_t ck_bytes = nch * sizeof(SmallChunk), rc_bytes = multi ? (batch + 1) * 4 : 0;
    VK_TRY(ctx->pin_sparse_ck.ensure(ck_bytes + rc_bytes));
    SmallChunk* hck = ctx->pin_sparse_ck.as<SmallChunk>();
    uint32_t* hrc = reinterpret_cast<uint32_t*>(ctx->pin_sparse_ck.as<uint8_t>() + ck_bytes);
    size_t b = 0;
    for (size_t g = 0; g < batch; g++) {
        const uint32_t np = (uint32_t)((rp[g + 1] - rp[g]) * W);
        if (multi) hrc[g] = (uint32_t)b;
        uint32_t p0 = 0;
        do {
            hck[b++] = SmallChunk{(uint32_t)rp[g], np, p0, 0};
            p0 += NT;
        } while (p0 < np);
    }
    if (multi) hrc[batch] = (uint32_t)b;
    hipStream_t st = ctx->stream;
    DevBuf d_ck(ctx), d_part(ctx), d_rows(ctx);
    VK_TRY(d_ck.ensure(ck_bytes + rc_bytes));
    VK_TRY(d_part.ensure(nch * sizeof(Acc)));
    if (multi) VK_TRY(d_rows.ensure(batch * sizeof(Acc)));
    VK_CHECK_HIP(hipMemcpyAsync(d_ck.p, hck, ck_bytes + rc_bytes, hipMemcpyHostToDevice, st));
    using FA = FbE<C>;
    const FA* tab = t->fb.as<FA>();
    const uint8_t* tinf = t->inf.as<uint8_t>();
    const SmallChunk* dck = d_ck.as<SmallChunk>();
#define VK_SMALL_(MODE, NTV)                                                                                  \
    VK_LAUNCH(ctx, "sparse_small", (k_fb_sparse_small<C, Fr, MODE, NTV>), nch, NTV, 0, tab, tinf, fg, dck, in.d_cols, \
              in.d_vals, in.d_item, in.d_child, in.d_sidx, in.d_snap, d_part.as<Acc>())
    if (NT == 64) {
        if (in.mode == 0) VK_SMALL_(0, 64);
        else if (in.mode == 1) VK_SMALL_(1, 64);
        else VK_SMALL_(2, 64);
    } else {
        if (in.mode == 0) VK_SMALL_(0, 256);
        else if (in.mode == 1) VK_SMALL_(1, 256);
        else VK_SMALL_(2, 256);
    }
#undef VK_SMALL_
    Acc* rows = d_part.as<Acc>();
    if (multi) {
        VK_LAUNCH(ctx, "sparse_combine", (k_sparse_combine<C::Inl>), batch, 64, 0, d_part.as<Acc>(),
                  reinterpret_cast<const uint32_t*>(d_ck.as<uint8_t>() + ck_bytes), d_rows.as<Acc>());
        rows = d_rows.as<Acc>();
    }
    return normalize_rows_items(ctx, rows, batch, in.d_add_ids, in.d_add_xy, in.d_add_inf, in.d_dst, in.d_out_xy,
                                in.d_out_inf, in.d_out_item, overlap);
}

// BN254 sparse commits with device inputs and outputs (the verkle tree's device-resident levels)
int sparse_commit_items_dev(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, bool rows_fit,
                            const uint32_t* d_cols, const void* d_sc, void* d_xy, uint8_t* d_inf, void* d_items,
                            const uint32_t* d_add_ids, const uint64_t* d_add_xy, const uint8_t* d_add_inf,
                            const uint32_t* d_dst, const std::function<void()>* overlap, const uint64_t* d_row_ptr) {
    if (t->curve != VC_CURVE_BN254 || !d_items) return VC_E_INVALID;
    return sparse_commit_dev<BN254G1, BN254Fr>(ctx, t, batch, row_ptr, rows_fit, d_cols, d_sc, 0, d_xy, d_inf, d_items,
                                               d_add_ids, d_add_xy, d_add_inf, d_dst, overlap, d_row_ptr);
}

int msm_batch_sparse_items(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                           const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_items) {
    if (t->curve != VC_CURVE_BN254 || (batch && !out_items)) return VC_E_INVALID;
    return msm_batch_sparse_t<BN254G1, BN254Fr>(ctx, t, batch, row_ptr, cols, scalars, mont, out_xy, out_inf,
                                                 out_items);
}

int msm_batch_sparse(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                     const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf) {
    switch (t->curve) {
        case VC_CURVE_BN254:
            return msm_batch_sparse_t<BN254G1, BN254Fr>(ctx, t, batch, row_ptr, cols, scalars, mont, out_xy, out_inf);
        case VC_CURVE_BLS12_381:
            return msm_batch_sparse_t<BLS381G1, BLS381Fr>(ctx, t, batch, row_ptr, cols, scalars, mont, out_xy,
                                                           out_inf);
        case VC_CURVE_BANDERSNATCH:
            return msm_batch_sparse_t<Bandersnatch, BandFr>(ctx, t, batch, row_ptr, cols, scalars, mont, out_xy,
                                                             out_inf);
    }
    return VC_E_INVALID;
}

int msm_windows(int curve, size_t n, int* c, int* W, int* terms) {
    int bits = curve == VC_CURVE_BN254 ? BN254Fr::BITS : curve == VC_CURVE_BLS12_381 ? BLS381Fr::BITS : BandFr::BITS;
    // BLS12-381 tables of subgroup points take the GLV split (2n terms of 127-bit scalars)
    const bool glv = curve == VC_CURVE_BLS12_381 && n >= GLV_MIN_N && n < (1u << 30);
    // (a GLV MSM over a whole table takes the shared-window size, msm_run_t)
    *c = glv ? glv_window_shared(2 * n) : choose_window(n, bits + 1);
    *W = glv ? (GLV_BITS + *c - 1) / *c : (bits + 1 + *c - 1) / *c;
    if (terms) *terms = glv ? 2 : 1;
    return VC_OK;
}

// MSMs of more than ctx->opt_msm_chunk points (default 2^27: nv * W then stays below 2^31 on
// every curve, so the u32 entry space of the sort cannot wrap) run as consecutive point chunks
// whose accumulators are added on the host; each chunk is an ordinary partial-table MSM.
template <class C, class Fr>
static int msm_run_chunked(vc_ctx* ctx, Table* t, size_t offset, const uint32_t* sc, size_t n, int mont,
                           int part, int parts, uint32_t* out_acc) {
    using Acc = typename C::Acc;
    const size_t chunk = std::max<size_t>(ctx->opt_msm_chunk, 1);
    if (n <= chunk) return msm_run_t<C, Fr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
    Acc res = C::zero();
    for (size_t lo = 0; lo < n; lo += chunk) {
        const size_t m = std::min(chunk, n - lo);
        Acc r;
        VK_TRY((msm_run_t<C, Fr>(ctx, t, offset + lo, sc + 8 * lo, m, mont, part, parts,
                                 reinterpret_cast<uint32_t*>(&r))));
        res = C::add(res, r);
    }
    memcpy(out_acc, &res, sizeof(Acc));
    return VC_OK;
}

// chunked host-scalar MSM: chunk j's buckets added into the running set (first: empty buckets
// set to the identity, so the one reduction after the last chunk reads every bucket as live)
template <class A>
__global__ void __launch_bounds__(256) k_bucket_merge(typename A::Acc* __restrict__ acc,
                                                     const typename A::Acc* __restrict__ add,
                                                     const uint32_t* __restrict__ offsets, uint32_t NBtot,
                                                     uint32_t first) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= NBtot) return;
    const bool ne = offsets[b + 1] > offsets[b];
    if (first) {
        if (!ne) acc[b] = A::zero();
    } else if (ne) {
        acc[b] = A::add(acc[b], add[b]);
    }
}
__global__ void k_iota(uint32_t* __restrict__ o, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) o[i] = i;
}

// vc_msm with host scalars (the drop-in `commit` of INTEGRATION.md over utils.rs:16-19): the
// 32 n bytes cross PCIe in K chunks on the side stream while the context's stream runs the
// previous chunk -- each chunk a point-range MSM on the table's radix shared-window copies (GLV
// split + histogram, sort, accumulate, fix-up) whose buckets add into one set -- and ONE
// reduction + host fold finish it. Only for that geometry (BLS12-381, GLV, radix copies);
// *done = false otherwise (the caller copies and runs msm_run). A chunk whose fix-up chains
// exceed its walk (adversarial scalars) sends the whole MSM to msm_run_t once the scalars are in.
template <class C, class Fr>
static int msm_run_host_chunks_t(vc_ctx* ctx, Table* t, size_t offset, const uint64_t* host_sc, size_t n, int mont,
                                 int K, uint32_t* out_acc, bool* done) {
    *done = false;
    if constexpr (!std::is_same<C, BLS381G1>::value) {
        return VC_OK;
    } else {
        using Acc = typename C::Acc;
        using A = typename Fast29<C>::type;
        using RAcc = FAcc<C>;
        static const int radix_env = getenv("VKZG_MSM_RADIX") ? atoi(getenv("VKZG_MSM_RADIX")) : 5;
        static const int range_env = getenv("VKZG_MSM_RANGE") ? atoi(getenv("VKZG_MSM_RANGE")) : 1;
        if (K < 2 || K > 4 || n >= (1u << 30) || !ctx->opt_shared_windows || radix_env != 5 || !range_env ||
            getenv("VKZG_MSM_C") || getenv("VKZG_WIN_PACKED") || 2 * (size_t)t->n < (1u << 19))
            return VC_OK;
        // chunks of whole 8192-scalar sort blocks, each >= 2^16 points (a point range on the copies)
        const size_t blk = 8192, nb = (n + blk - 1) / blk;
        if (nb < (size_t)K || n / K < (1u << 16)) return VC_OK;
        bool glv = false;
        VK_TRY(glv_table_ok(ctx, t, &glv));
        if (!glv) return VC_OK;
        VK_TRY(fast_tables<C>(ctx, t, true));
        {
            const size_t win_bytes = (size_t)7 * 2 * t->n *
                                     (win_pair_on() ? 2 * sizeof(typename A::AffP) : sizeof(typename A::AffN));
            if (win_bytes > (8ull << 30)) return VC_OK;
            const int st = win_tables<C>(ctx, t, 16, 7, 0, 5, win_pair_on());
            if (st == VC_E_OOM) {
                t->win.release();
                return VC_OK;
            }
            VK_TRY(st);
        }
        ctx->plan = {16, 7, 2, 5, 1};
        const uint32_t NB = 5u << 15;
        std::vector<size_t> lo(K + 1);
        for (int j = 0; j <= K; j++) lo[j] = std::min(n, (nb * j / K) * blk);
        size_t nmax = 0;
        for (int j = 0; j < K; j++) nmax = std::max(nmax, lo[j + 1] - lo[j]);
        VK_TRY(ctx->ws[WS_SCALARS].ensure(n * 32));
        VK_TRY(ctx->ws[WS_GLV_SC].ensure(2 * nmax * 4 * 7));
        VK_TRY(ctx->ws[WS_BUCKETS].ensure((size_t)NB * sizeof(RAcc)));
        VK_TRY(ctx->ws2[WS_BUCKETS].ensure((size_t)NB * sizeof(RAcc)));
        VK_TRY(ctx->ws2[WS_CHAIN].ensure(16));
        VK_TRY(ctx->ws2[WS_OFFSETS].ensure(((size_t)NB + 1) * 4));
        uint8_t* d_sc = ctx->ws[WS_SCALARS].as<uint8_t>();
        RAcc* bA = ctx->ws[WS_BUCKETS].as<RAcc>();
        RAcc* bB = ctx->ws2[WS_BUCKETS].as<RAcc>();
        uint32_t* chain = ctx->ws2[WS_CHAIN].as<uint32_t>();
        std::vector<hipEvent_t> ev(K);
        for (int j = 0; j < K; j++) ev[j] = ctx->get_event();
        // on every exit (errors included): no copy still reading the caller's buffer, events back
        struct Done {
            vc_ctx* ctx;
            std::vector<hipEvent_t>& ev;
            ~Done() {
                (void)hipStreamSynchronize(ctx->side_stream);
                for (hipEvent_t e : ev) ctx->event_pool.push_back(e);
            }
        } done_guard{ctx, ev};
        MsmSlice<C> sl;
        std::vector<uint32_t> guard(K);
        for (int j = 0; j < K; j++) {
            const size_t nj = lo[j + 1] - lo[j];
            // chunk j's scalars on the side stream, issued after chunk j - 1's kernels are queued (a
            // pageable copy can block the host until its data is staged)
            VK_CHECK_HIP(hipMemcpyAsync(d_sc + lo[j] * 32, host_sc + lo[j] * 4, nj * 32, hipMemcpyHostToDevice,
                                        ctx->side_stream));
            VK_CHECK_HIP(hipEventRecord(ev[j], ctx->side_stream));
            VK_CHECK_HIP(hipStreamWaitEvent(ctx->stream, ev[j], 0));
            sl = MsmSlice<C>();
            sl.L = ctx->lane(0);
            sl.c = 16;
            sl.wb = 0;
            sl.we = 7;
            sl.W = 7;
            sl.shared = true;
            sl.m = 5;
            sl.wps = 7;
            sl.bucket_dst = j == 0 ? bA : bB;
            sl.chain_dst = chain + j;
            sl.skip_reduce = true;
            sl.radix.sc = {reinterpret_cast<const uint32_t*>(d_sc + lo[j] * 32)};
            sl.radix.mont = {mont};
            sl.radix.inf = t->inf.as<uint8_t>() + offset + lo[j];
            sl.radix.n = (uint32_t)nj;
            sl.radix.dig = ctx->ws[WS_GLV_SC].as<int32_t>();
            RadixDigits rd{ctx->ws[WS_GLV_SC].as<int32_t>(), (uint32_t)(2 * nj)};
            rd.off = (uint32_t)(offset + lo[j]);
            rd.half = (uint32_t)nj;
            rd.gap = (uint32_t)(t->n - nj);
            sl.stride = (uint32_t)(2 * t->n);
            if (t->win_pair) {
                const auto* wp = t->win.as<typename A::AffP>();
                VK_TRY(slice_enqueue<C>(ctx, sl, rd, 2 * nj, wp, wp, 0xffffffffu, nullptr, nullptr));
            } else {
                const auto* wn = t->win.as<typename A::AffN>();
                VK_TRY(slice_enqueue<C>(ctx, sl, rd, 2 * nj, wn, wn, 0xffffffffu, nullptr, nullptr));
            }
            guard[j] = sl.guard;
            VK_LAUNCH(ctx, "msm_merge", (k_bucket_merge<A>), (NB + 255) / 256, 256, 0, bA, bB, sl.offsets, NB,
                      j == 0 ? 1u : 0u);
        }
        // one reduction over the merged set: every bucket live (empty ones hold the identity)
        uint32_t* iota = ctx->ws2[WS_OFFSETS].as<uint32_t>();
        VK_LAUNCH(ctx, "msm_iota", k_iota, (NB + 1 + 255) / 256, 256, 0, iota, NB);
        VK_TRY(msm_tail_reduce<C>(ctx, sl.L, bA, iota, sl.NB, sl.Wr, sl.Lseg, sl.S, sl.J, sl.seg, sl.rs, sl.bsum_part,
                                  sl.tail, sl.nU > 1));
        // the tail buffer's own chain word (read by slice_finish) was not used by the chunks
        VK_CHECK_HIP(hipMemsetAsync(reinterpret_cast<uint8_t*>(sl.tail) + sl.tail_bytes, 0, 4, ctx->stream));
        VK_TRY(slice_fetch<C>(sl));
        uint32_t hchain[4] = {0, 0, 0, 0};
        VK_CHECK_HIP(hipMemcpyAsync(hchain, chain, 4 * K, hipMemcpyDeviceToHost, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        for (int j = 0; j < K; j++)
            if (hchain[j] > (1u << guard[j])) {  // long chains: the unchunked MSM over the copied scalars
                *done = true;
                return msm_run_t<C, Fr>(ctx, t, offset, reinterpret_cast<const uint32_t*>(d_sc), n, mont, 0, 1,
                                        out_acc);
            }
        Acc res;
        VK_TRY(slice_finish<C>(ctx, sl, &res));
        memcpy(out_acc, &res, sizeof(Acc));
        *done = true;
        return VC_OK;
    }
}

// vc_msm: host scalars
int msm_run_host(vc_ctx* ctx, Table* t, size_t offset, const uint64_t* host_sc, size_t n, int mont,
                 uint32_t* out_acc) {
    if (t->curve == VC_CURVE_BLS12_381 && ctx->opt_host_chunks > 1 && ctx->opt_msm_chunk >= n) {
        bool done = false;
        VK_TRY((msm_run_host_chunks_t<BLS381G1, BLS381Fr>(ctx, t, offset, host_sc, n, mont, ctx->opt_host_chunks,
                                                          out_acc, &done)));
        if (done) return VC_OK;
    }
    if (n > 0) {
        VK_TRY(ctx->ws[WS_SCALARS].ensure(n * 32));
        VK_CHECK_HIP(hipMemcpyAsync(ctx->ws[WS_SCALARS].p, host_sc, n * 32, hipMemcpyHostToDevice, ctx->stream));
    }
    return msm_run(ctx, t, offset, ctx->ws[WS_SCALARS].p, n, mont, out_acc, 0, 1);
}

int msm_run(vc_ctx* ctx, Table* t, size_t offset, const void* d_scalars, size_t n, int mont,
            uint32_t* out_acc, int part, int parts) {
    const uint32_t* sc = reinterpret_cast<const uint32_t*>(d_scalars);
    switch (t->curve) {
        case VC_CURVE_BN254:
            return msm_run_chunked<BN254G1, BN254Fr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
        case VC_CURVE_BLS12_381:
            return msm_run_chunked<BLS381G1, BLS381Fr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
        case VC_CURVE_BANDERSNATCH:
            return msm_run_chunked<Bandersnatch, BandFr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
    }
    return VC_E_INVALID;
}

}  // namespace vk
