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

// Two-pass MSD counting sort of the n*W (window, bucket) keys, all in LDS -- no global atomics
// (global atomics execute memory-side on CDNA4, ~26 G/s for scattered words, which made the
// one-pass global-histogram sort cost 2.2 ms at 2^20 x 16 windows).
//   coarse bin g = w * NBC + (b >> FB)          (NBC = NB >> FB coarse bins per window)
//   k_sort_hist     block = CHUNK scalars: LDS histogram of coarse bins -> counts[g][block]
//   hipcub scan     counts -> base[g][block] (global position of the block's run in bin g)
//   k_sort_coarse   same digits again, LDS cursors from base: tmp[pos] = fine<<32 | i | sign<<31
//   k_sort_fine     block = coarse bin: LDS histogram of the 2^FB fine buckets -> bucket
//                   offsets (written directly), then scatter into sorted[]
// Order inside a bucket is arbitrary (EC addition is commutative and exact).
constexpr uint32_t SORT_CHUNK = 1024;

template <class Fr>
__global__ void __launch_bounds__(256) k_sort_hist(const uint32_t* __restrict__ sc, const uint8_t* __restrict__ inf,
                                                  uint32_t n, int c, int wb, int we, int mont, uint32_t FB,
                                                  uint32_t NBC, uint32_t nblk, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t hist[];
    const uint32_t bins = (uint32_t)(we - wb) * NBC;
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const uint32_t lo = blockIdx.x * SORT_CHUNK, hi = min(lo + SORT_CHUNK, n);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        if (inf != nullptr && inf[i]) continue;
        fe<Fr> s = load_scalar<Fr>(sc, i);
        if (mont) s = fe_from_mont<Fr>(s);
        for_each_digit<Fr>(s, c, we, [&](int w, int32_t d) {
            if (d != 0 && w >= wb)
                atomicAdd(&hist[(uint32_t)(w - wb) * NBC + (((uint32_t)(d < 0 ? -d : d) - 1) >> FB)], 1u);
        });
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) counts[(size_t)k * nblk + blockIdx.x] = hist[k];
}

template <class Fr>
__global__ void __launch_bounds__(256) k_sort_coarse(const uint32_t* __restrict__ sc, const uint8_t* __restrict__ inf,
                                                    uint32_t n, int c, int wb, int we, int mont, uint32_t FB,
                                                    uint32_t NBC, uint32_t nblk, const uint32_t* __restrict__ base,
                                                    uint64_t* __restrict__ tmp) {
    extern __shared__ uint32_t cur[];
    const uint32_t bins = (uint32_t)(we - wb) * NBC;
    for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) cur[k] = base[(size_t)k * nblk + blockIdx.x];
    __syncthreads();
    const uint32_t fmask = (1u << FB) - 1;
    const uint32_t lo = blockIdx.x * SORT_CHUNK, hi = min(lo + SORT_CHUNK, n);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        if (inf != nullptr && inf[i]) continue;
        fe<Fr> s = load_scalar<Fr>(sc, i);
        if (mont) s = fe_from_mont<Fr>(s);
        for_each_digit<Fr>(s, c, we, [&](int w, int32_t d) {
            if (d != 0 && w >= wb) {
                uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
                uint32_t pos = atomicAdd(&cur[(uint32_t)(w - wb) * NBC + (b >> FB)], 1u);
                tmp[pos] = ((uint64_t)(b & fmask) << 32) | i | (d < 0 ? 0x80000000u : 0u);
            }
        });
    }
}

// one block per coarse bin; offsets[g * 2^FB + f] = start of fine bucket f of bin g
__global__ void __launch_bounds__(256) k_sort_fine(const uint64_t* __restrict__ tmp, const uint32_t* __restrict__ base,
                                                  uint32_t nblk, uint32_t bins, uint32_t FB,
                                                  uint32_t* __restrict__ offsets, uint32_t* __restrict__ sorted) {
    __shared__ uint32_t h[256], x[256];
    const uint32_t g = blockIdx.x, F = 1u << FB, t = threadIdx.x;
    const uint32_t start = base[(size_t)g * nblk];
    const uint32_t end = base[(size_t)(g + 1) * nblk];  // base has bins*nblk + 1 entries
    h[t] = 0;
    __syncthreads();
    for (uint32_t p = start + t; p < end; p += blockDim.x) atomicAdd(&h[(uint32_t)(tmp[p] >> 32)], 1u);
    __syncthreads();
    // inclusive Hillis-Steele scan over 256 counters
    uint32_t v = h[t];
    x[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        uint32_t a = t >= o ? x[t - o] : 0u;
        __syncthreads();
        x[t] += a;
        __syncthreads();
    }
    const uint32_t excl = x[t] - v;
    if (t < F) offsets[(size_t)g * F + t] = start + excl;
    if (g == bins - 1 && t == 0) offsets[(size_t)bins * F] = end;
    __syncthreads();
    h[t] = excl;  // cursors
    __syncthreads();
    for (uint32_t p = start + t; p < end; p += blockDim.x) {
        uint64_t e = tmp[p];
        uint32_t pos = start + atomicAdd(&h[(uint32_t)(e >> 32)], 1u);
        sorted[pos] = (uint32_t)e;
    }
}

// ------------------------------------------------------------------ bucket accumulation
template <class C>
__global__ void __launch_bounds__(256) k_msm_accumulate(
    const typename C::Aff* __restrict__ bases, const uint32_t* __restrict__ sorted,
    const uint32_t* __restrict__ offsets, uint32_t NBtot, uint32_t M,
    typename C::Acc* __restrict__ buckets, typename C::Acc* __restrict__ carry_in,
    uint8_t* __restrict__ through, typename C::Acc* __restrict__ owner_piece,
    uint32_t* __restrict__ owner_bucket, uint32_t* __restrict__ chain_max) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t L = offsets[NBtot];  // entry count, read on the device: no host round trip
    uint32_t k = t * M;                 // grid sized for the n*W upper bound
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
                through[t] = right_open ? 2 : 1;  // 1: carry piece ending here, 2: bucket continues
                if (!right_open) {  // chain end: chain length = carry threads of this bucket
                    const uint32_t L = t - offsets[b] / M;
                    if (L >= 2) atomicMax(chain_max, L);
                }
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
                     int mont, int part, int parts, uint32_t* out_acc) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    if (n == 0) {
        Acc z = C::zero();
        memcpy(out_acc, &z, sizeof(Acc));
        return VC_OK;
    }
    if (n >= 0x7fffffffu) return VC_E_INVALID;
    if (parts < 1 || part < 0 || part >= parts) return VC_E_INVALID;
    const int c = choose_window(n);
    const int Wfull = (Fr::BITS + 1 + c - 1) / c;  // one spare bit absorbs the final carry
    // window slice [wb, we) of this call (parts > 1: the MSM split by windows across GPUs;
    // the slices' results add up to the whole MSM)
    const int wb = part * Wfull / parts, we = (part + 1) * Wfull / parts;
    const int W = we - wb;
    if (W == 0) {
        Acc z = C::zero();
        memcpy(out_acc, &z, sizeof(Acc));
        return VC_OK;
    }
    const uint32_t NB = 1u << (c - 1);
    const uint32_t NBtot = NB * W;
    const size_t maxL = n * (size_t)W;
    // sorted entries per accumulate thread: 64 at 2^20 x 16 windows (2 rounds of 2048 waves),
    // fewer for window slices / small MSMs so the grid still fills the chip
    // (not below 16: a bucket then straddles more threads and the fix-up's serial merge chain
    // costs more than the emptier accumulate rounds -- measured at 2 windows of 2^20)
    const uint32_t M = (uint32_t)std::min<size_t>(64, std::max<size_t>(16, maxL / 131072));
    // buckets per reduction segment (the segment sum is a serial chain of 2*Lseg adds): 8, or
    // 4 when the segments (one lane each) would not give every SIMD a wave
    uint32_t Lseg = NB >= 64 ? 8 : (NB >= 4 ? 2 : 1);
    if (Lseg == 8 && (size_t)(NB / Lseg) * W < 65536) Lseg = 4;
    const uint32_t S = NB / Lseg;  // power of two
    uint32_t J = 0;
    while ((1u << J) < S) J++;
    const uint32_t Tmax = (uint32_t)((maxL + M - 1) / M);
    hipStream_t st = ctx->stream;

    // bucket sort geometry (k_sort_*): 2^FB fine buckets per coarse bin
    uint32_t lgNB = (uint32_t)c - 1;
    const uint32_t FB = lgNB < 8 ? lgNB : 8;
    const uint32_t NBC = NB >> FB, bins = (uint32_t)W * NBC;
    const uint32_t nblk = (uint32_t)((n + SORT_CHUNK - 1) / SORT_CHUNK);
    const size_t ncnt = (size_t)bins * nblk + 1;

    VK_TRY(ctx->ws[WS_DIGITS].ensure(maxL * 8));
    VK_TRY(ctx->ws[WS_COUNTS].ensure(ncnt * 4));
    VK_TRY(ctx->ws[WS_CURSOR].ensure(ncnt * 4));
    VK_TRY(ctx->ws[WS_OFFSETS].ensure((size_t)(NBtot + 1) * 4));
    VK_TRY(ctx->ws[WS_SORTED].ensure(maxL * 4));
    VK_TRY(ctx->ws[WS_BUCKETS].ensure((size_t)NBtot * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_CARRY].ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_THROUGH].ensure((size_t)(Tmax + 8)));
    VK_TRY(ctx->ws[WS_OWNER].ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_OWNER_B].ensure((size_t)(Tmax + 8) * 4));
    VK_TRY(ctx->ws[WS_SEG].ensure((size_t)S * W * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_TREE].ensure((size_t)S * W * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_WIN].ensure((size_t)W * (J + 1) * msm_bitsum_pw(S, msm_bitsum_k(S, (uint32_t)W, J)) * sizeof(Acc)));
    VK_TRY(ctx->ws[WS_TAIL].ensure((size_t)W * (J + 1) * sizeof(Acc)));

    uint64_t* tmp = ctx->ws[WS_DIGITS].as<uint64_t>();
    uint32_t* counts = ctx->ws[WS_COUNTS].as<uint32_t>();
    uint32_t* base = ctx->ws[WS_CURSOR].as<uint32_t>();
    uint32_t* offsets = ctx->ws[WS_OFFSETS].as<uint32_t>();
    uint32_t* sorted = ctx->ws[WS_SORTED].as<uint32_t>();
    Acc* buckets = ctx->ws[WS_BUCKETS].as<Acc>();
    Acc* carry = ctx->ws[WS_CARRY].as<Acc>();
    uint8_t* through = ctx->ws[WS_THROUGH].as<uint8_t>();
    Acc* owner = ctx->ws[WS_OWNER].as<Acc>();
    uint32_t* owner_b = ctx->ws[WS_OWNER_B].as<uint32_t>();
    Acc* seg = ctx->ws[WS_SEG].as<Acc>();
    Acc* rs = ctx->ws[WS_TREE].as<Acc>();
    Acc* bsum_part = ctx->ws[WS_WIN].as<Acc>();
    Acc* tail = ctx->ws[WS_TAIL].as<Acc>();

    const Aff* bases = t->bases.as<Aff>() + offset;
    const uint8_t* inf = t->inf.as<uint8_t>() + offset;

    const size_t lds = (size_t)bins * 4;
    if (lds > 64 * 1024) return VC_E_INVALID;  // c <= 16 keeps bins <= W * 128
    VK_CHECK_HIP(hipMemsetAsync(counts + ncnt - 1, 0, 4, st));
    VK_LAUNCH(ctx, "msm_sort_hist", (k_sort_hist<Fr>), nblk, 256, lds, d_sc, inf, (uint32_t)n, c, wb, we, mont, FB,
              NBC, nblk, counts);
    size_t tmp_bytes = 0;
    VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, base, ncnt, st));
    VK_TRY(ctx->ws[WS_SCAN_TMP].ensure(tmp_bytes));
    {
        hipEvent_t ev = nullptr;
        if (ctx->timing) ctx->timer_begin("msm_scan", &ev);
        VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(ctx->ws[WS_SCAN_TMP].p, tmp_bytes, counts, base, ncnt, st));
        if (ctx->timing) ctx->timer_end("msm_scan", ev);
    }
    VK_LAUNCH(ctx, "msm_sort_coarse", (k_sort_coarse<Fr>), nblk, 256, lds, d_sc, inf, (uint32_t)n, c, wb, we, mont,
              FB, NBC, nblk, base, tmp);
    VK_LAUNCH(ctx, "msm_sort_fine", k_sort_fine, bins, 256, 0, tmp, base, nblk, bins, FB, offsets, sorted);
    // entry count L = offsets[NBtot] stays on the device; grids are sized for L <= n*W
    VK_TRY(ctx->ws[WS_CHAIN].ensure(4));
    uint32_t* chain_max = ctx->ws[WS_CHAIN].as<uint32_t>();
    VK_CHECK_HIP(hipMemsetAsync(chain_max, 0, 4, st));
    VK_LAUNCH(ctx, "msm_accumulate", (k_msm_accumulate<C>), (Tmax + 255) / 256, 256, 0, bases, sorted, offsets,
              NBtot, M, buckets, carry, through, owner, owner_b, chain_max);
    VK_TRY(msm_tail_fixup<C>(ctx, Tmax, offsets + NBtot, M, buckets, carry, through, owner, owner_b, chain_max));
    VK_TRY(msm_tail_reduce<C>(ctx, buckets, offsets, NB, W, Lseg, S, J, seg, rs, bsum_part, tail));
    std::vector<Acc> ht((size_t)W * (J + 1));
    VK_CHECK_HIP(hipMemcpyAsync(ht.data(), tail, ht.size() * sizeof(Acc), hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));
    // MSM = sum_w 2^(c w) (A_w + Lseg sum_j 2^j T_wj): Horner over bit positions (host, 64-bit limbs)
    int lg_seg = 0;
    while ((1u << lg_seg) < Lseg) lg_seg++;
    const int maxpos = c * (we - 1) + lg_seg + (int)J;
    std::vector<std::vector<int>> at(maxpos + 1);
    for (int w = 0; w < W; w++) {
        const int p0 = c * (wb + w);  // absolute bit position of window wb + w
        at[p0].push_back(w * (int)(J + 1) + (int)J);
        for (uint32_t j = 0; j < J; j++) at[p0 + lg_seg + (int)j].push_back(w * (int)(J + 1) + (int)j);
    }
    Acc res = C::zero();
    for (int pos = maxpos; pos >= 0; pos--) {
        if (!C::is_zero(res)) res = C::dbl(res);
        for (int idx : at[pos]) res = C::add(res, ht[idx]);
    }
    memcpy(out_acc, &res, sizeof(Acc));
    return VC_OK;
}

// ------------------------------------------------------------------ sparse batched commits
// Rows of a CSR matrix (row g = commit g: non-zero (column i, scalar s) pairs) against the
// fixed-base window tables of a table: every non-zero expands to its non-zero signed window
// digits, each a table point T[i][w][|d|-1] -- so the entries of a row are contiguous and the
// rows play the buckets of the Pippenger accumulate: the same balanced k_msm_accumulate (M
// entries per thread, rows straddling threads merged by the fix-up) sums them. For verkle
// nodes (~5 non-zeros of 256 per internal node, 2 of N per extension row) this replaces
// dense width-256 rows.
template <class Fr>
__global__ void k_sparse_count(const uint32_t* __restrict__ sc, size_t nnz, int mont, int c, int W,
                               uint32_t* __restrict__ cnt) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    fe<Fr> s = load_scalar<Fr>(sc, j);
    if (mont) s = fe_from_mont<Fr>(s);
    uint32_t k = 0;
    for_each_digit<Fr>(s, c, W, [&](int, int32_t d) { k += d != 0; });
    cnt[j] = k;
}

template <class Fr>
__global__ void k_sparse_expand(const uint32_t* __restrict__ sc, const uint32_t* __restrict__ cols, size_t nnz,
                                int mont, int c, int W, const uint32_t* __restrict__ eoff,
                                uint32_t* __restrict__ entries) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz) return;
    fe<Fr> s = load_scalar<Fr>(sc, j);
    if (mont) s = fe_from_mont<Fr>(s);
    const uint32_t NBk = 1u << (c - 1), i = cols[j];
    uint32_t pos = eoff[j];
    for_each_digit<Fr>(s, c, W, [&](int w, int32_t d) {
        if (d != 0)
            entries[pos++] = (((uint32_t)i * (uint32_t)W + (uint32_t)w) * NBk + (uint32_t)(d < 0 ? -d : d) - 1) |
                             (d < 0 ? 0x80000000u : 0u);
    });
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

template <class C, class Fr>
static int msm_batch_sparse_t(vc_ctx* ctx, Table* t, size_t batch, const uint64_t* row_ptr, const uint32_t* cols,
                              const uint64_t* scalars, int mont, uint64_t* out_xy, uint8_t* out_inf) {
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    if (batch == 0) return VC_OK;
    const size_t nnz = row_ptr[batch];
    for (size_t g = 0; g < batch; g++)
        if (row_ptr[g + 1] < row_ptr[g]) return VC_E_INVALID;
    for (size_t j = 0; j < nnz; j++)
        if (cols[j] >= t->n) return VC_E_RANGE;
    if (t->fb_c == 0) VK_TRY(fixed_base_precompute(ctx, t, 8));
    const int c = t->fb_c, W = t->fb_W;
    // rows are cut into chunks of <= CHNZ non-zeros (the accumulate's buckets), so a long row
    // (e.g. a verkle root: 256 children x W windows) does not become one bucket straddling
    // hundreds of threads -- whose pieces the fix-up would add serially; chunk sums are folded
    // per row by k_sparse_combine
    const size_t CHNZ = 4;
    std::vector<uint64_t> cptr{0};
    std::vector<uint32_t> rc(batch + 1);
    for (size_t g = 0; g < batch; g++) {
        rc[g] = (uint32_t)(cptr.size() - 1);
        if (row_ptr[g + 1] == row_ptr[g]) cptr.push_back(row_ptr[g]);  // empty row -> one empty chunk
        for (uint64_t j = row_ptr[g]; j < row_ptr[g + 1]; j += CHNZ) cptr.push_back(std::min<uint64_t>(j + CHNZ, row_ptr[g + 1]));
    }
    rc[batch] = (uint32_t)(cptr.size() - 1);
    const size_t nch = cptr.size() - 1;
    if ((uint64_t)t->n * W << (c - 1) >= (1ull << 31)) return VC_E_RANGE;  // entry index + sign bit
    const size_t maxL = nnz * (size_t)W;
    if (maxL >= 0xffffffffull) return VC_E_RANGE;
    hipStream_t st = ctx->stream;
    // grow-only ctx workspaces (the MSM's own slots for entries / carries / scan scratch: the
    // two paths never run concurrently on one ctx)
    DevBuf& d_rp = ctx->ws[WS_SP_RP];
    DevBuf& d_cols = ctx->ws[WS_SP_COLS];
    DevBuf& d_sc = ctx->ws[WS_SP_SC];
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
    DevBuf& d_xy = ctx->ws[WS_SP_XY];
    DevBuf& d_inf = ctx->ws[WS_SP_INF];
    const uint32_t M = (uint32_t)std::min<size_t>(64, std::max<size_t>(16, maxL / 131072));
    const uint32_t Tmax = (uint32_t)((maxL + M - 1) / M);
    DevBuf& d_rc = ctx->ws[WS_SP_RC];
    DevBuf& d_chunks = ctx->ws[WS_SP_CHUNKS];
    VK_TRY(d_rp.ensure((nch + 1) * 8));
    VK_TRY(d_rc.ensure((batch + 1) * 4));
    VK_TRY(d_chunks.ensure(nch * sizeof(Acc)));
    VK_TRY(d_cols.ensure(std::max<size_t>(nnz, 1) * 4));
    VK_TRY(d_sc.ensure(std::max<size_t>(nnz, 1) * 32));
    VK_TRY(d_cnt.ensure((nnz + 1) * 4));
    VK_TRY(d_eoff.ensure((nnz + 1) * 4));
    VK_TRY(d_ent.ensure(std::max<size_t>(maxL, 1) * 4));
    VK_TRY(d_off.ensure((nch + 1) * 4));
    VK_TRY(d_rows.ensure(batch * sizeof(Acc)));
    VK_TRY(d_carry.ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(d_thr.ensure((size_t)(Tmax + 8)));
    VK_TRY(d_own.ensure((size_t)(Tmax + 8) * sizeof(Acc)));
    VK_TRY(d_ownb.ensure((size_t)(Tmax + 8) * 4));
    VK_TRY(d_xy.ensure(batch * 2 * C::F::N * 4));
    VK_TRY(d_inf.ensure(batch));
    VK_CHECK_HIP(hipMemcpyAsync(d_rp.p, cptr.data(), (nch + 1) * 8, hipMemcpyHostToDevice, st));
    VK_CHECK_HIP(hipMemcpyAsync(d_rc.p, rc.data(), (batch + 1) * 4, hipMemcpyHostToDevice, st));
    if (nnz) {
        VK_CHECK_HIP(hipMemcpyAsync(d_cols.p, cols, nnz * 4, hipMemcpyHostToDevice, st));
        VK_CHECK_HIP(hipMemcpyAsync(d_sc.p, scalars, nnz * 32, hipMemcpyHostToDevice, st));
    }
    VK_CHECK_HIP(hipMemsetAsync(d_cnt.as<uint32_t>() + nnz, 0, 4, st));
    if (nnz)
        VK_LAUNCH(ctx, "sparse_count", (k_sparse_count<Fr>), (nnz + 255) / 256, 256, 0, d_sc.as<uint32_t>(), nnz, mont,
                  c, W, d_cnt.as<uint32_t>());
    size_t tmp_bytes = 0;
    VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_cnt.as<uint32_t>(), d_eoff.as<uint32_t>(),
                                                  nnz + 1, st));
    VK_TRY(d_tmp.ensure(std::max<size_t>(tmp_bytes, 1)));
    VK_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp.p, tmp_bytes, d_cnt.as<uint32_t>(), d_eoff.as<uint32_t>(),
                                                  nnz + 1, st));
    if (nnz)
        VK_LAUNCH(ctx, "sparse_expand", (k_sparse_expand<Fr>), (nnz + 255) / 256, 256, 0, d_sc.as<uint32_t>(),
                  d_cols.as<uint32_t>(), nnz, mont, c, W, d_eoff.as<uint32_t>(), d_ent.as<uint32_t>());
    VK_LAUNCH(ctx, "sparse_rows", (k_sparse_rows<C>), (nch + 1 + 255) / 256, 256, 0, d_rp.as<uint64_t>(),
              d_eoff.as<uint32_t>(), nch, d_off.as<uint32_t>(), d_chunks.as<Acc>());
    const Aff* tab = t->fb.as<Aff>();
    if (Tmax > 0) {  // all-zero rows only: k_sparse_rows already set every chunk to the identity
        VK_TRY(ctx->ws[WS_CHAIN].ensure(4));
        uint32_t* chain_max = ctx->ws[WS_CHAIN].as<uint32_t>();
        VK_CHECK_HIP(hipMemsetAsync(chain_max, 0, 4, st));
        VK_LAUNCH(ctx, "sparse_accumulate", (k_msm_accumulate<C>), (Tmax + 255) / 256, 256, 0, tab,
                  d_ent.as<uint32_t>(), d_off.as<uint32_t>(), (uint32_t)nch, M, d_chunks.as<Acc>(),
                  d_carry.as<Acc>(), d_thr.as<uint8_t>(), d_own.as<Acc>(), d_ownb.as<uint32_t>(), chain_max);
        VK_TRY(msm_tail_fixup<C>(ctx, Tmax, d_off.as<uint32_t>() + nch, M, d_chunks.as<Acc>(), d_carry.as<Acc>(),
                                 d_thr.as<uint8_t>(), d_own.as<Acc>(), d_ownb.as<uint32_t>(), chain_max));
    }
    VK_LAUNCH(ctx, "sparse_combine", (k_sparse_combine<typename C::Inl>), batch, 64, 0, d_chunks.as<Acc>(),
              d_rc.as<uint32_t>(), d_rows.as<Acc>());
    VK_TRY(normalize_to_canon(ctx, ctx->curve, d_rows.p, batch, d_xy.p, d_inf.as<uint8_t>()));
    VK_CHECK_HIP(hipMemcpyAsync(out_xy, d_xy.p, batch * 2 * C::F::N * 4, hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipMemcpyAsync(out_inf, d_inf.p, batch, hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));  // host staging vectors die on return
    return VC_OK;
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

int msm_windows(int curve, size_t n, int* c, int* W) {
    int bits = curve == VC_CURVE_BN254 ? BN254Fr::BITS : curve == VC_CURVE_BLS12_381 ? BLS381Fr::BITS : BandFr::BITS;
    *c = choose_window(n);
    *W = (bits + 1 + *c - 1) / *c;
    return VC_OK;
}

int msm_run(vc_ctx* ctx, Table* t, size_t offset, const void* d_scalars, size_t n, int mont,
            uint32_t* out_acc, int part, int parts) {
    const uint32_t* sc = reinterpret_cast<const uint32_t*>(d_scalars);
    switch (t->curve) {
        case VC_CURVE_BN254: return msm_run_t<BN254G1, BN254Fr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
        case VC_CURVE_BLS12_381:
            return msm_run_t<BLS381G1, BLS381Fr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
        case VC_CURVE_BANDERSNATCH:
            return msm_run_t<Bandersnatch, BandFr>(ctx, t, offset, sc, n, mont, part, parts, out_acc);
    }
    return VC_E_INVALID;
}

}  // namespace vk
