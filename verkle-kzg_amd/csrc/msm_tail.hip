// Latency-bound tail of the Pippenger MSM (split from msm.hip to keep rebuilds short). The
// kernels run the radix-2^29 point arithmetic of ec29.hpp on the raw accumulators of
// k_msm_accumulate (A = Fast29<C>::type): a serial add chain in one wave is bound by its
// instruction count (~4.4 cycles per wave64 instruction alone on a SIMD), and the radix-29
// add is ~20 % shorter than the 32-bit-limb one. Only the W x (J + 1) outputs are converted
// back to the ec.hpp form (for the host Horner pass).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "ctx.hpp"
#include "ec.hpp"
#include "ec29.hpp"
#include "msm_tail.hpp"

namespace vk {

constexpr uint32_t NONE_T = 0xffffffffu;

// Diagnostic build only (-DVKZG_TAIL_TRACE, tools/tail_trace.py): every lane of the tail kernels
// records its entry and exit on the 100 MHz s_memrealtime clock, its wave's hardware slot (HW_ID,
// XCC_ID) and a kernel-specific word (the fix-up's chain length, the bit sums' kind and item count)
// into g_tail_trace[kernel][global thread] (4 x u64, vector stores); the default build has none.
#ifdef VKZG_TAIL_TRACE
constexpr uint32_t TT_KERNELS = 4, TT_MAXT = 1u << 18;
__device__ unsigned long long g_tail_trace[(size_t)TT_KERNELS * TT_MAXT * 4];
struct TTLane {
    unsigned long long t0;
    uint32_t kid, info = 0;
    __device__ explicit TTLane(uint32_t k) : t0(__builtin_amdgcn_s_memrealtime()), kid(k) {}
    __device__ ~TTLane() {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
        if (g >= TT_MAXT) return;
        unsigned long long* p = g_tail_trace + ((size_t)kid * TT_MAXT + g) * 4;
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        p[0] = t0;
        p[1] = t1;
        p[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        p[3] = (unsigned long long)info | (1ull << 63);
    }
};
#define TT_BEGIN(k) TTLane tt_lane_(k)
#define TT_INFO(x) (tt_lane_.info = (uint32_t)(x))
#else
#define TT_BEGIN(k) ((void)0)
#define TT_INFO(x) ((void)0)
#endif

// ---- fix-up of buckets that straddle accumulate threads. Thread u's carry piece (through[u]
// = 1: the bucket ends in u; 2: it continues into u + 1) belongs to the bucket whose owner
// thread t0 < u holds the first piece. The carry pieces of one bucket form a chain u0 = t0+1
// .. u1; its sum is built by pointer jumping -- round r adds the piece 2^r threads ahead --
// so a bucket spanning L threads costs ceil(log2 L) parallel rounds, not L serial adds (an
// all-equal-scalar 2^20 MSM has one 2^20-entry bucket per window: L = 16k threads). The
// accumulate reports the longest chain (chain_max, only when >= 2), read back once.
template <class C>
__global__ void __launch_bounds__(256) k_fixup_init(const uint8_t* __restrict__ through, uint32_t Tmax,
                                                   const uint32_t* __restrict__ Lp, uint32_t M,
                                                   uint32_t* __restrict__ nxt) {
    uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = (*Lp + M - 1) / M;  // accumulate threads that ran
    if (u >= T || u >= Tmax) return;
    nxt[u] = through[u] == 2 && u + 1 < T ? u + 1 : NONE_T;
}

template <class A>
__global__ void __launch_bounds__(256) k_fixup_jump(const typename A::Acc* __restrict__ val_in,
                                                   const uint32_t* __restrict__ nxt_in,
                                                   const uint8_t* __restrict__ through, uint32_t Tmax,
                                                   const uint32_t* __restrict__ Lp, uint32_t M,
                                                   typename A::Acc* __restrict__ val_out,
                                                   uint32_t* __restrict__ nxt_out, uint32_t span,
                                                   const uint32_t* __restrict__ chain_max) {
    uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = (*Lp + M - 1) / M;
    if (u >= T || u >= Tmax || through[u] == 0) return;  // no carry piece in thread u
    // device-guarded round (launched before the host knows the longest chain): a round the
    // chains do not need passes its input through unchanged
    const uint32_t n = (chain_max && span >= *chain_max) ? NONE_T : nxt_in[u];
    if (n == NONE_T) {
        val_out[u] = val_in[u];
        nxt_out[u] = NONE_T;
        return;
    }
    val_out[u] = A::add(val_in[u], val_in[n]);
    nxt_out[u] = nxt_in[n];
}

template <class A>
__global__ void __launch_bounds__(256) k_msm_fixup(typename A::Acc* __restrict__ buckets,
                                                  const typename A::Acc* __restrict__ chain_sum,
                                                  const typename A::Acc* __restrict__ owner_piece,
                                                  const uint32_t* __restrict__ owner_bucket,
                                                  uint32_t Tmax, const uint32_t* __restrict__ Lp, uint32_t M) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = (*Lp + M - 1) / M;
    if (t >= T || t >= Tmax) return;
    uint32_t b = owner_bucket[t];
    if (b == NONE_T) return;
    // an owner piece exists only when the bucket continues into t + 1 (< T by construction)
    buckets[b] = A::add(owner_piece[t], chain_sum[t + 1]);
}

// Common case: a lane per bucket. A bucket b over accumulate threads t0 < t1 (t = entry / M)
// has its owner piece in t0 and carry pieces in t0 + 1 .. t1; the lane adds them serially (at
// most `limit` carry pieces): one kernel, one add call site, every lane of a wave busy (a lane
// per accumulate thread left 3 of 4 lanes idle at 512 entries per bucket and ran the waves in
// two rounds). A longer bucket is left unwritten here; the accumulate's chain_max tells the
// host, which then runs the pointer-jumping path (msm_tail_fixup with the known Lmax) from the
// untouched carry pieces and redoes the reduction.
template <class A>
__global__ void __launch_bounds__(256) k_msm_fixup_walk(typename A::Acc* __restrict__ buckets,
                                                       const typename A::Acc* __restrict__ carry,
                                                       const typename A::Acc* __restrict__ owner_piece,
                                                       const uint32_t* __restrict__ offsets, uint32_t NBtot,
                                                       uint32_t M, uint32_t limit, const uint32_t* __restrict__ owner_b) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= NBtot) return;
    const uint32_t lo = offsets[b], hi = offsets[b + 1];
    if (hi <= lo) return;  // empty
    const uint32_t t0 = lo / M, t1 = (hi - 1) / M;
    if (t0 == t1 || t1 - t0 > limit) return;  // inside one thread (written) / long chain (host path)
    if (owner_b && owner_b[t0] == NONE_T) return;  // merged inside the accumulate (written)
    typename A::Acc acc = owner_piece[t0];
    for (uint32_t u = t0 + 1; u <= t1; u++) acc = A::add(acc, carry[u]);
    buckets[b] = acc;
}
// the same with a quad per bucket (SW curves: SW29::add_quad, ~half the latency of an add): the
// walk is bound by its longest chains -- the top window's hot buckets at the multi-GPU window
// slices, up to 16 pieces -- and leaves most SIMDs idle with a lane per bucket
template <class A>
__global__ void __launch_bounds__(256) k_msm_fixup_walk_q(typename A::Acc* __restrict__ buckets,
                                                         const typename A::Acc* __restrict__ carry,
                                                         const typename A::Acc* __restrict__ owner_piece,
                                                         const uint32_t* __restrict__ offsets, uint32_t NBtot,
                                                         uint32_t M, uint32_t limit, const uint32_t* __restrict__ owner_b) {
    TT_BEGIN(0);
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, b = gid >> 2, role = gid & 3;
    if (b >= NBtot) return;  // whole quads (NBtot * 4 threads)
    const uint32_t lo = offsets[b], hi = offsets[b + 1];
    if (hi <= lo) return;
    const uint32_t t0 = lo / M, t1 = (hi - 1) / M;
    if (t0 == t1 || t1 - t0 > limit) return;  // uniform over the quad
    if (owner_b && owner_b[t0] == NONE_T) return;  // merged inside the accumulate (written)
    TT_INFO(t1 - t0);
    typename A::Acc acc = owner_piece[t0];
    for (uint32_t u = t0 + 1; u <= t1; u++) {
        const typename A::Acc o = carry[u];
        acc = A::add_quad(acc, o, role);
    }
    if (role == 0) buckets[b] = acc;
}

// The same walk with a lane per accumulate THREAD: the owner thread t of a straddling bucket
// (owner_bucket[t] != NONE) adds the carry pieces of t + 1 .. u1 (through == 2 continues, 1 ends).
// Denser than a lane per bucket when there are fewer threads than buckets -- the radix
// shared-window MSM has ~90 entries per bucket and 112 per thread: 131K lanes, every one an
// owner, two waves per SIMD in one round, where the 164K lanes per bucket took 2.5 waves per
// SIMD, i.e. two rounds. Chains longer than `limit` are left to the host path, as above.
template <class A>
__global__ void __launch_bounds__(256) k_msm_fixup_own(typename A::Acc* __restrict__ buckets,
                                                      const typename A::Acc* __restrict__ carry,
                                                      const typename A::Acc* __restrict__ owner_piece,
                                                      const uint32_t* __restrict__ owner_bucket,
                                                      const uint8_t* __restrict__ through, uint32_t Tmax,
                                                      const uint32_t* __restrict__ Lp, uint32_t M, uint32_t limit) {
    TT_BEGIN(0);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = (*Lp + M - 1) / M;
    if (t >= T || t >= Tmax) return;
    // the owner's piece, the next thread's carry piece and its through flag are loaded with the
    // owner word, not after it: one memory latency instead of a chain of three (the kernel waited
    // on loads 37 % of its wave cycles: profiles/r04/tail_pmc/). Threads t < T - 1 have a slot
    // t + 1 in the through / carry arrays (written or zeroed by the accumulate's threads < T).
    const bool nx = t + 1 < T;
    const uint32_t b = owner_bucket[t];
    const uint8_t th1 = nx ? through[t + 1] : (uint8_t)0;
    typename A::Acc acc = owner_piece[t];
    typename A::Acc c1 = nx ? carry[t + 1] : A::zero();
    if (b == NONE_T) return;
    // an owner piece exists only when the bucket continues into t + 1, so the chain ends in a
    // thread u1 < T with through[u1] == 1
    uint32_t u1 = t + 1;
    if (th1 == 2) {  // longer chains (rare)
        u1++;
        while (through[u1] == 2) {
            if (u1 - t >= limit) return;  // longer than the walk takes: host path
            u1++;
        }
    }
    TT_INFO(u1 - t);
    // one add call site (an inlined add is ~34 KB of code: two would not share the I-cache)
    for (uint32_t u = t + 1;; u++) {
        acc = A::add(acc, c1);
        if (u == u1) break;
        c1 = carry[u + 1];
    }
    buckets[b] = acc;
}

// c ? a : b word by word through masks: a plain select of two aggregates becomes a load through a
// selected address, which keeps both in scratch memory for the whole loop
template <class T>
__device__ __forceinline__ T mask_select(bool c, const T& a, const T& b) {
    static_assert(sizeof(T) % 4 == 0, "");
    constexpr int NW = (int)(sizeof(T) / 4);
    uint32_t wa[NW], wb[NW];
    __builtin_memcpy(wa, &a, sizeof wa);
    __builtin_memcpy(wb, &b, sizeof wb);
    const uint32_t m = 0u - (uint32_t)c;
#pragma unroll
    for (int k = 0; k < NW; k++) wa[k] = (wa[k] & m) | (wb[k] & ~m);
    T r;
    __builtin_memcpy(&r, wa, sizeof wa);
    return r;
}

// ------------------------------------------------------------------ bucket reduction
// Window sum  V_w = sum_b (b + 1) B_b  over NB buckets, in two shallow GPU stages and a host pass:
//  (1) k_msm_segsum: segment s of Lseg buckets -> acc_s = sum (b - lo + 1) B_b, R_s = sum B_b
//      (2 Lseg serial adds);  V_w = sum_s acc_s + Lseg * sum_s s R_s
//  (2) k_msm_bitsum: sum_s s R_s = sum_j 2^j T_j with T_j = sum_{s: bit j of s} R_s, and
//      A = sum_s acc_s: J + 1 plain sums per window (8 serial adds per lane + wave butterflies)
//  (3) host: MSM = sum_w 2^(c w) (A_w + Lseg sum_j 2^j T_wj) -- every term is a point at a
//      bit position, so one Horner pass over positions (msm.hip).
// Serial GPU depth 2 Lseg + 13 EC adds instead of 2 Lseg + ~22 (lo * R by double-and-add)
// + 24 (per-window reduction) before.
// I-cache note: an inlined BLS12-381 EC add is ~34 KB of straight-line code (14 asm multiplies),
// so a kernel with two add call sites in its loop streams ~70 KB per iteration through a 64 KB
// instruction cache. Every kernel below has ONE add call site: operands are selected first.
template <class A>
__global__ void __launch_bounds__(256) k_msm_segsum(const typename A::Acc* __restrict__ buckets,
                                                   const uint32_t* __restrict__ offsets, uint32_t NB, int W,
                                                   uint32_t Lseg, uint32_t S, typename A::Acc* __restrict__ accs,
                                                   typename A::Acc* __restrict__ Rs) {
    using Acc = typename A::Acc;
    uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t w = gid / S, s = gid % S;
    if (w >= (uint32_t)W) return;
    uint32_t lo = s * Lseg, hi = min(lo + Lseg, NB);
    Acc R = A::zero(), acc = A::zero();
    // buckets from the top: R += B_j, then acc += R (2 (hi - lo) adds through one call site)
    for (uint32_t it = 0; it < 2 * (hi - lo); it++) {
        const bool second = (it & 1) != 0;
        Acc y;
        if (second) {
            y = R;
        } else {
            const size_t g = (size_t)w * NB + (hi - 1 - it / 2);
            y = offsets[g + 1] > offsets[g] ? buckets[g] : A::zero();
        }
        const Acc r = A::add(mask_select(second, acc, R), y);
        acc = mask_select(second, r, acc);
        R = mask_select(second, R, r);
    }
    accs[gid] = acc;
    Rs[gid] = R;
}

// the same on quads (SW curves, SW29::add_quad: about half the latency of an add): a segment
// chain is 2 Lseg dependent adds and the 5 x 2^15 radix buckets give 2^15 segments, one wave per
// SIMD on half the SIMDs with a lane each -- a quad each fills every SIMD twice
template <class A>
__global__ void __launch_bounds__(256) k_msm_segsum_q(const typename A::Acc* __restrict__ buckets,
                                                     const uint32_t* __restrict__ offsets, uint32_t NB, int W,
                                                     uint32_t Lseg, uint32_t S, typename A::Acc* __restrict__ accs,
                                                     typename A::Acc* __restrict__ Rs) {
    using Acc = typename A::Acc;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, q = gid >> 2, role = gid & 3;
    const uint32_t w = q / S, s = q % S;
    if (w >= (uint32_t)W) return;  // whole quads
    const uint32_t lo = s * Lseg, hi = min(lo + Lseg, NB);
    Acc R = A::zero(), acc = A::zero();
    for (uint32_t it = 0; it < 2 * (hi - lo); it++) {
        const bool second = (it & 1) != 0;
        Acc y;
        if (second) {
            y = R;
        } else {
            const size_t g = (size_t)w * NB + (hi - 1 - it / 2);
            y = offsets[g + 1] > offsets[g] ? buckets[g] : A::zero();
        }
        const Acc r = A::add_quad(mask_select(second, acc, R), y, role);
        acc = mask_select(second, r, acc);
        R = mask_select(second, R, r);
    }
    if (role == 0) {
        accs[q] = acc;
        Rs[q] = R;
    }
}

// Residue form of the reduction (the radix shared-window MSM, Lseg = m = 5): with b = Lseg s + r,
//   V = sum_b (b + 1) B_b = Lseg sum_s s R_s + sum_r (r + 1) U_r,   U_r = sum_s B_{Lseg s + r},
// so the segment stage only needs R_s = sum_r B_{Lseg s + r} (Lseg - 1 dependent adds instead of
// the 2 Lseg of acc_s and R_s), and the bit stage adds the Lseg sums U_r (bucket columns of S
// items) beside its J sums T_j; the host weighs U_r by r + 1 (shared_set_sum).
template <class A>
__global__ void __launch_bounds__(256) k_msm_segr(const typename A::Acc* __restrict__ buckets,
                                                 const uint32_t* __restrict__ offsets, uint32_t NB, int W,
                                                 uint32_t Lseg, uint32_t S, typename A::Acc* __restrict__ Rs) {
    using Acc = typename A::Acc;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t w = gid / S, s = gid % S;
    if (w >= (uint32_t)W) return;
    const size_t g0 = (size_t)w * NB + (size_t)s * Lseg;
    Acc R = A::zero();
    for (uint32_t r = 0; r < Lseg; r++) {
        const size_t g = g0 + r;
        const Acc y = offsets[g + 1] > offsets[g] ? buckets[g] : A::zero();
        R = A::add(R, y);
    }
    Rs[gid] = R;
}
template <class A>
__global__ void __launch_bounds__(256) k_msm_segr_q(const typename A::Acc* __restrict__ buckets,
                                                   const uint32_t* __restrict__ offsets, uint32_t NB, int W,
                                                   uint32_t Lseg, uint32_t S, typename A::Acc* __restrict__ Rs) {
    using Acc = typename A::Acc;
    TT_BEGIN(1);
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, q = gid >> 2, role = gid & 3;
    const uint32_t w = q / S, s = q % S;
    if (w >= (uint32_t)W) return;  // whole quads
    TT_INFO(Lseg);
    const size_t g0 = (size_t)w * NB + (size_t)s * Lseg;
    Acc R = A::zero();
    for (uint32_t r = 0; r < Lseg; r++) {
        const size_t g = g0 + r;
        const Acc y = offsets[g + 1] > offsets[g] ? buckets[g] : A::zero();
        R = A::add_quad(R, y, role);
    }
    if (role == 0) Rs[q] = R;
}

template <class A>
__device__ __forceinline__ typename A::Acc shfl_acc(const typename A::Acc& v, uint32_t m) {
    static_assert(sizeof(typename A::Acc) % 4 == 0, "");
    typename A::Acc o;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(typename A::Acc) / 4); k++) dst[k] = __shfl_xor(src[k], m, 64);
    return o;
}

// stage 1: lane sums K (msm_bitsum_k) selected items of one (w, q) sum serially, then the wave
// folds its 64 lane sums (xor butterfly) -- K + 6 iterations of one add:
//   q < J: T_q = R_s over s with bit q set (S/2 items of tsrc, nb1 waves);
//   q = J + u (u < nU): U_u = item nU m + u of usrc over m < S (S items, nb2 waves) -- nU = 1 with
//   usrc = acc_s is the sum A = sum_s acc_s, nU = Lseg with usrc = the buckets the residue sums.
// tsrc / usrc item liveness from toff / uoff (bucket offsets: an empty bucket was never written)
// when they are buckets, none otherwise.
// Waves are laid out compactly (window by window: J x nb1 bit-sum waves, then nb2), so the grid
// holds only busy waves and every CU gets at most one block (a grid with idle waves let the
// dispatcher stack two busy blocks on some CUs: their SIMDs ran two waves, twice as long).
// Marginal form (h > 0, msm_tail_plan): per set, waves [0, G) make the column sums L_lo (Hn items
// lo + G m), waves [G, G + Hn) the row sums H_hi (G items G hi + m) -- one wave and one partial
// slot each, Hn / 64 or G / 64 items per lane -- and the rest the U partials as in the bit form.
template <class A>
__global__ void __launch_bounds__(256) k_msm_bitsum(const typename A::Acc* __restrict__ usrc,
                                                   const typename A::Acc* __restrict__ tsrc, uint32_t S, uint32_t J,
                                                   uint32_t h, uint32_t nU, uint32_t K, uint32_t nb1, uint32_t nb2,
                                                   uint32_t pL, uint32_t gL, uint32_t gH, uint32_t n_waves,
                                                   const uint32_t* __restrict__ toff,
                                                   const uint32_t* __restrict__ uoff,
                                                   typename A::Acc* __restrict__ partial) {
    using Acc = typename A::Acc;
    TT_BEGIN(2);
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
    if (gw >= n_waves) return;  // grid rounded up to whole blocks (uniform per wave)
    const uint32_t G = h ? 1u << h : 0u, Hn = h ? 1u << (J - h) : 0u;
    // waves of the T side per set: a column sum takes pL waves, or a wave makes gL column sums (gH row
    // sums) on 64 / g lanes each; partial slots stay one per sum (pL per column sum)
    const uint32_t nLw = h ? G * pL / gL : 0u, nT = h ? nLw + Hn / gH : J * nb1;
    const uint32_t nTs = h ? G * pL + Hn : J * nb1;  // partial slots of the T side per set
    const uint32_t per_w = nT + nU * nb2;            // urow: nb2 = 0, no U waves
    const uint32_t w = gw / per_w, r = gw % per_w;
    // kind: 0 = T_q (bit form), 1 = L_lo, 2 = H_hi, 3 = U_u; sel = q, lo, hi or u
    const uint32_t kind = r >= nT ? 3u : h == 0 ? 0u : r < nLw ? 1u : 2u;
    const uint32_t g = kind == 1 ? gL : kind == 2 ? gH : 1u;  // sums per wave
    const uint32_t lanes = 64 / g, gi = lane / lanes, li = lane % lanes;
    const uint32_t sel = kind == 0 ? r / nb1 : kind == 1 ? (gL > 1 ? r * gL + gi : r / pL)
                         : kind == 2 ? (r - nLw) * gH + gi : (r - nT) / nb2;
    const uint32_t wv = kind == 0 ? r % nb1 : kind == 1 ? (gL > 1 ? 0u : r % pL) : kind == 3 ? (r - nT) % nb2 : 0u;
    const uint32_t n_items = kind == 0 ? S / 2 : kind == 1 ? Hn : kind == 2 ? G : S;
    const uint32_t Kw = kind == 1 ? Hn / (lanes * pL) : kind == 2 ? G / lanes : K;
    const uint32_t base = wv * lanes * Kw;
    const uint32_t slot = kind == 0 ? sel * nb1 + wv : kind == 1 ? sel * pL + wv : kind == 2 ? G * pL + sel
                                                                                 : nTs + sel * nb2 + wv;
    const size_t set0 = kind < 3 ? (size_t)w * S : (size_t)w * S * nU;
    const Acc* src = (kind < 3 ? tsrc : usrc) + set0;
    const uint32_t* off = (kind < 3 ? toff : uoff);
    if (off) off += set0;
    // item m of this sum -> its index in src (T_q: the m-th s with bit q set; L_lo: G m + lo;
    // H_hi: G hi + m; U_u: nU m + u)
    auto item = [&](uint32_t m) -> uint32_t {
        return kind == 0   ? (((m >> sel) << (sel + 1)) | (1u << sel) | (m & ((1u << sel) - 1)))
               : kind == 1 ? m * G + sel
               : kind == 2 ? sel * G + m
                           : m * nU + sel;
    };
    uint32_t lg_lanes = 0;  // xor levels of the fold inside a sum's lane group
    while ((1u << lg_lanes) < lanes) lg_lanes++;
    const size_t out = (size_t)w * (nTs + nU * nb2) + slot;
    TT_INFO(kind << 24 | Kw);
    Acc v = A::zero();
    if constexpr (A::quad) {
        // Kw serial full adds per lane (every SIMD busy: issue-bound), then the wave's 64 lane sums
        // on 4-lane cooperative adds: each quad first folds its own 4 lanes (3 rounds), then the
        // 16 quads by xor (4) -- 7 adds of ~14.6k cycles instead of the 6-level butterfly of full
        // adds (~30k cycles each)
        for (uint32_t it = 0; it < Kw; it++) {
            const uint32_t m = base + it * lanes + li;
            const uint32_t idx = item(m);
            const bool live = m < n_items && (!off || off[idx + 1] > off[idx]);
            const Acc o = live ? src[idx] : A::zero();
            v = A::add(v, o);
        }
        const uint32_t role = lane & 3, q0 = lane & ~3u;
        Acc s = shfl_idx_pod(v, q0);
        for (uint32_t it = 0; it < 3 + (lg_lanes - 2); it++) {  // xor levels stay inside the group
            const Acc o = it < 3 ? shfl_idx_pod(v, q0 + it + 1) : shfl_acc<A>(s, 4u << (it - 3));
            s = A::add_quad(s, o, role);
        }
        if (li == 0) partial[out] = s;
        return;
    }
    for (uint32_t it = 0; it < Kw + lg_lanes; it++) {
        Acc o;
        if (it < Kw) {
            const uint32_t m = base + it * lanes + li;  // lane-interleaved rows
            const uint32_t idx = item(m);
            const bool live = m < n_items && (!off || off[idx + 1] > off[idx]);
            o = live ? src[idx] : A::zero();
        } else {
            o = shfl_acc<A>(v, 1u << (it - Kw));
        }
        v = A::add(v, o);
    }
    if (li == 0) partial[out] = v;
}

// where sum `sum` (= w (J + nU) + q) of the final stage finds its items in `partial`: cnt items,
// the k-th at index pos(k). Bit form: the sum's own nb1 / nb2 wave partials. Marginal form:
// T_q (q < h) = the G / 2 column sums L_lo with bit q of lo set, T_q (q >= h) = the Hn / 2 row
// sums H_hi with bit q - h of hi set, U_u = its nb2 partials.
struct PartLoc {
    size_t start;
    uint32_t cnt, bit;  // bit < 32: the items are the slots with this bit set (clear: unset), from start
    uint32_t lgp = 0;   // column sums: 2^lgp partial slots each (pL), all taken
    bool clear = false;
    __device__ PartLoc(uint32_t sum, uint32_t J, uint32_t h, uint32_t nU, uint32_t nb1, uint32_t nb2, uint32_t pL,
                       bool urow) {
        const uint32_t w = sum / (J + nU), q = sum % (J + nU);
        const uint32_t G = h ? 1u << h : 0u, Hn = h ? 1u << (J - h) : 0u;
        const uint32_t nT = h ? G * pL + Hn : J * nb1;
        const size_t set0 = (size_t)w * (nT + nU * nb2);
        bit = 32;
        if (q >= J && urow) {  // X = the row sums of even hi (the host adds T_h: U = T_h + X)
            start = set0 + (size_t)G * pL;
            cnt = Hn / 2;
            bit = 0;
            clear = true;
        } else if (q >= J) {
            start = set0 + nT + (size_t)(q - J) * nb2;
            cnt = nb2;
        } else if (h == 0) {
            start = set0 + (size_t)q * nb1;
            cnt = nb1;
        } else if (q < h) {
            start = set0;
            cnt = G / 2 * pL;
            bit = q;
            while ((1u << lgp) < pL) lgp++;
        } else {
            start = set0 + (size_t)G * pL;
            cnt = Hn / 2;
            bit = q - h;
        }
    }
    __device__ size_t pos(uint32_t k) const {
        if (bit >= 32) return start + k;
        const uint32_t i = k >> lgp, sub = k & ((1u << lgp) - 1);
        const uint32_t e = ((i >> bit) << (bit + 1)) | (clear ? 0u : 1u << bit) | (i & ((1u << bit) - 1));
        return start + ((size_t)e << lgp) + sub;
    }
};

// the final stage's completion in direct mode (TailDirect): the block's point (and, for block 0,
// the chain word) reach host memory before its flag does
__device__ __forceinline__ void tail_flag(TailDirect d, uint32_t sum) {
    if (d.flags == nullptr) return;
    if (sum == 0 && d.chain_dst) *d.chain_dst = *d.chain_src;
    __threadfence_system();
    __hip_atomic_store(&d.flags[sum], d.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// stage 2: one wave per (w, q) sum folds its partials (nb1 or nb2: ceil(n/64) per lane, then
// the butterfly)
template <class C, class A>
__global__ void __launch_bounds__(64) k_msm_sumpart(const typename A::Acc* __restrict__ partial, uint32_t J,
                                                   uint32_t h, uint32_t nU, uint32_t nb1, uint32_t nb2,
                                                   uint32_t pL, uint32_t urow, typename C::Acc* __restrict__ out,
                                                   TailDirect dir) {
    using Acc = typename A::Acc;
    const uint32_t sum = blockIdx.x, lane = threadIdx.x;
    const PartLoc loc(sum, J, h, nU, nb1, nb2, pL, urow != 0);
    const uint32_t cnt = loc.cnt;
    uint32_t span = 1, lg = 0;
    while (span < cnt && span < 64) {
        span <<= 1;
        lg++;
    }
    const uint32_t nk = (cnt + 63) / 64;
    Acc v = A::zero();
    for (uint32_t it = 0; it < nk + lg; it++) {
        Acc o;
        if (it < nk) {
            const uint32_t k = lane + it * 64;
            o = k < cnt ? partial[loc.pos(k)] : A::zero();
        } else {
            o = shfl_acc<A>(v, 1u << (it - nk));
        }
        v = A::add(v, o);
    }
    if (lane == 0) {
        out[sum] = A::store(v);
        tail_flag(dir, sum);
    }
}

// the same on quads (SW curves): 16 logical lanes per wave, each a quad running the 4-lane
// cooperative add (SW29::add_quad: ~3,100 instead of ~6,600 instructions per add). This stage is
// latency-bound -- a block per sum, W (J + 1) blocks on 1024 SIMDs -- so the shorter add pays.
// A block of SUMPART_WAVES waves per sum (64 quads at 4): a 52-partial sum is one add per quad,
// 4 butterfly levels inside each wave, then wave 0 folds the wave totals from LDS in 2 more --
// 7 dependent adds (8 for the 103-partial A sum) instead of 8 (11) with one wave per sum.
constexpr uint32_t SUMPART_WAVES = 4;
template <class C, class A>
__global__ void __launch_bounds__(64 * SUMPART_WAVES) k_msm_sumpart_q(const typename A::Acc* __restrict__ partial,
                                                                     uint32_t J, uint32_t h, uint32_t nU,
                                                                     uint32_t nb1, uint32_t nb2, uint32_t pL,
                                                                     uint32_t urow, typename C::Acc* __restrict__ out,
                                                                     TailDirect dir) {
    using Acc = typename A::Acc;
    constexpr uint32_t QPB = 16 * SUMPART_WAVES, LGW = SUMPART_WAVES == 4 ? 2 : SUMPART_WAVES == 2 ? 1 : 0;
    static_assert((1u << LGW) == SUMPART_WAVES, "SUMPART_WAVES: 1, 2 or 4");
    __shared__ Acc wave_sum[SUMPART_WAVES];
    TT_BEGIN(3);
    const uint32_t sum = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, role = lane & 3;
    const PartLoc loc(sum, J, h, nU, nb1, nb2, pL, urow != 0);
    const uint32_t cnt = loc.cnt;
    TT_INFO(cnt);
    const uint32_t nk = (cnt + QPB - 1) / QPB;
    Acc v = A::zero();
    for (uint32_t it = 0; it < nk + 4 + LGW; it++) {  // one add call site
        Acc o;
        if (it < nk) {
            const uint32_t k = (tid >> 2) + it * QPB;  // quad index within the block
            o = k < cnt ? partial[loc.pos(k)] : A::zero();
        } else if (it < nk + 4) {
            o = shfl_acc<A>(v, 4u << (it - nk));  // quad to quad inside the wave: xor of a multiple of 4
        } else {
            if (it == nk + 4) {  // every quad of a wave holds the wave's total
                if (lane == 0) wave_sum[wv] = v;
                __syncthreads();
                if (wv != 0) break;
                v = (lane >> 2) < SUMPART_WAVES ? wave_sum[lane >> 2] : A::zero();
            }
            o = shfl_acc<A>(v, 4u << (it - nk - 4));
        }
        v = A::add_quad(v, o, role);
    }
    if (tid == 0) {
        out[sum] = A::store(v);
        tail_flag(dir, sum);
    }
}

// pointer-jumping rounds r0 <= r < r1 (span 2^r) for a host-known Lmax, or -- guarded -- rounds
// whose kernels compare span with the device's chain_max: no host sync in the pipeline;
// msm_tail_fixup_more finishes the rare longer chains afterwards. The carry pieces ping-pong
// between `carry` and WS_CARRY2 (links: WS_NXT / WS_NXT2), so the parity of r0 says where the
// latest state is. Buffers hold the raw radix-29 accumulators (FAcc<C>).
template <class C>
static int fixup_rounds(vc_ctx* ctx, Lane L, uint32_t T, const uint32_t* Lp, uint32_t M, FAcc<C>* carry,
                        const uint8_t* through, uint32_t r0, uint32_t r1, const uint32_t* d_chain_max,
                        const FAcc<C>** sum) {
    using A = typename Fast29<C>::type;
    using Acc = FAcc<C>;
    VK_TRY(L.ws[WS_CARRY2].ensure((size_t)(T + 8) * sizeof(Acc)));
    VK_TRY(L.ws[WS_NXT].ensure((size_t)(T + 8) * 4));
    VK_TRY(L.ws[WS_NXT2].ensure((size_t)(T + 8) * 4));
    Acc* va = carry;
    Acc* vb = L.ws[WS_CARRY2].as<Acc>();
    uint32_t* na = L.ws[WS_NXT].as<uint32_t>();
    uint32_t* nb = L.ws[WS_NXT2].as<uint32_t>();
    if (r0 & 1) {  // continuing after an odd number of rounds: the latest state is in the second pair
        std::swap(va, vb);
        std::swap(na, nb);
    }
    if (r0 == 0) VK_LAUNCH_ON(ctx, L.st, "msm_fixup_init", (k_fixup_init<A>), (T + 255) / 256, 256, 0, through, T, Lp, M, na);
    for (uint32_t r = r0; r < r1; r++) {
        VK_LAUNCH_ON(ctx, L.st, "msm_fixup_jump", (k_fixup_jump<A>), (T + 255) / 256, 256, 0, va, na, through, T, Lp, M, vb,
                  nb, 1u << r, d_chain_max);
        std::swap(va, vb);
        std::swap(na, nb);
    }
    *sum = va;
    return VC_OK;
}

template <class C>
int msm_tail_fixup(vc_ctx* ctx, Lane L, uint32_t T, const uint32_t* Lp, uint32_t M, FAcc<C>* buckets, FAcc<C>* carry,
                   const uint8_t* through, const FAcc<C>* owner, const uint32_t* owner_b,
                   const uint32_t* d_chain_max, uint32_t guarded) {
    using A = typename Fast29<C>::type;
    const FAcc<C>* sum = carry;
    if (guarded) {
        VK_TRY(fixup_rounds<C>(ctx, L, T, Lp, M, carry, through, 0, guarded, d_chain_max, &sum));
    } else {
        uint32_t Lmax = 0;
        VK_CHECK_HIP(hipMemcpyAsync(&Lmax, d_chain_max, 4, hipMemcpyDeviceToHost, L.st));
        VK_CHECK_HIP(hipStreamSynchronize(L.st));
        uint32_t r1 = 0;
        while (Lmax >= 2 && (1u << r1) < Lmax) r1++;
        if (r1 > 0) VK_TRY(fixup_rounds<C>(ctx, L, T, Lp, M, carry, through, 0, r1, nullptr, &sum));
    }
    VK_LAUNCH_ON(ctx, L.st, "msm_fixup", (k_msm_fixup<A>), (T + 255) / 256, 256, 0, buckets, sum, owner, owner_b, T, Lp, M);
    return VC_OK;
}

// the serial walk of every owner over at most `limit` carry pieces (see k_msm_fixup_walk)
template <class C>
int msm_tail_fixup_walk(vc_ctx* ctx, Lane L, const uint32_t* offsets, uint32_t NBtot, uint32_t M, FAcc<C>* buckets,
                        const FAcc<C>* carry, const FAcc<C>* owner, uint32_t limit, const uint32_t* owner_b,
                        const uint8_t* through, uint32_t Tmax) {
    using A = typename Fast29<C>::type;
    static const int quad_env = getenv("VKZG_FIXUP_QUAD") ? atoi(getenv("VKZG_FIXUP_QUAD")) : 1;  // A/B probe
    static const int own_env = getenv("VKZG_FIXUP_OWN") ? atoi(getenv("VKZG_FIXUP_OWN")) : 1;     // A/B probe
    // fewer accumulate threads than buckets: a lane per owner thread (k_msm_fixup_own). Round 6
    // built a variant with the rare long chains compacted through LDS (one wave per block finishing
    // them) and measured it slower, 0.076 vs 0.072 ms (profiles/r06/tail_trace/; commit 9fc06f9's
    // k_msm_fixup_own_c): removed
    if (own_env && owner_b && Tmax <= NBtot) {
        VK_LAUNCH_ON(ctx, L.st, "msm_fixup", (k_msm_fixup_own<A>), (Tmax + 255) / 256, 256, 0, buckets, carry, owner,
                     owner_b, through, Tmax, offsets + NBtot, M, limit);
        return VC_OK;
    }
    // quads while their waves fit ~2 per SIMD (one bucket set: 2^15 buckets -> 2048 waves); with
    // per-window bucket sets (8 x 2^15) every SIMD already has lane-per-bucket waves and the
    // quads' ~2x instructions per add made the walk slower (0.08 -> 0.115 ms)
    if constexpr (A::quad) {
        if ((quad_env && NBtot <= 65536) || quad_env == 2) {
            VK_LAUNCH_ON(ctx, L.st, "msm_fixup", (k_msm_fixup_walk_q<A>), (uint32_t)(((size_t)NBtot * 4 + 255) / 256), 256,
                         0, buckets, carry, owner, offsets, NBtot, M, limit, owner_b);
            return VC_OK;
        }
    }
    VK_LAUNCH_ON(ctx, L.st, "msm_fixup", (k_msm_fixup_walk<A>), (NBtot + 255) / 256, 256, 0, buckets, carry, owner,
                 offsets, NBtot, M, limit, owner_b);
    return VC_OK;
}

// after `guarded` guarded rounds: chains longer than 2^guarded threads (Lmax read back with the
// results) get their remaining rounds, then the owners are rewritten (idempotent)
template <class C>
int msm_tail_fixup_more(vc_ctx* ctx, Lane L, uint32_t T, const uint32_t* Lp, uint32_t M, FAcc<C>* buckets,
                        FAcc<C>* carry, const uint8_t* through, const FAcc<C>* owner, const uint32_t* owner_b,
                        uint32_t guarded, uint32_t Lmax) {
    using A = typename Fast29<C>::type;
    uint32_t r1 = guarded;
    while ((1u << r1) < Lmax) r1++;
    const FAcc<C>* sum = carry;
    VK_TRY(fixup_rounds<C>(ctx, L, T, Lp, M, carry, through, guarded, r1, nullptr, &sum));
    VK_LAUNCH_ON(ctx, L.st, "msm_fixup", (k_msm_fixup<A>), (T + 255) / 256, 256, 0, buckets, sum, owner, owner_b, T, Lp, M);
    return VC_OK;
}

// outputs W x (J + nU) points in ec.hpp form: [w][q] = T_wq (q < J), then A_w (nU = 1) or the
// residue sums U_w,u (nU = Lseg, `residue`)
template <class C>
int msm_tail_reduce(vc_ctx* ctx, Lane L, const FAcc<C>* buckets, const uint32_t* offsets, uint32_t NB, int W,
                    uint32_t Lseg, uint32_t S, uint32_t J, FAcc<C>* accs, FAcc<C>* Rs, FAcc<C>* partial,
                    typename C::Acc* out, bool residue, const TailDirect* direct) {
    using A = typename Fast29<C>::type;
    const TailDirect dir = direct ? *direct : TailDirect{};
    const uint32_t* toff = nullptr;
    const uint32_t* uoff = nullptr;
    const FAcc<C>* usrc = accs;
    uint32_t nU = 1;
    if (Lseg == 1) {  // segments of one bucket: R_s = acc_s = B_s, read in place
        accs = Rs = const_cast<FAcc<C>*>(buckets);
        usrc = buckets;
        toff = uoff = offsets;
    } else if (residue) {
        nU = Lseg;
        usrc = buckets;
        uoff = offsets;
        static const int segrq_env = getenv("VKZG_SEGR_QUAD") ? atoi(getenv("VKZG_SEGR_QUAD")) : 1;  // A/B probe
        bool quads = false;
        if constexpr (A::quad) {
            quads = segrq_env != 0 && (size_t)S * W <= 65536;
            if (quads)
                VK_LAUNCH_ON(ctx, L.st, "msm_segsum", (k_msm_segr_q<A>), (S * (uint32_t)W * 4 + 255) / 256, 256, 0,
                             buckets, offsets, NB, W, Lseg, S, Rs);
        }
        if (!quads)
            VK_LAUNCH_ON(ctx, L.st, "msm_segsum", (k_msm_segr<A>), (S * (uint32_t)W + 255) / 256, 256, 0, buckets,
                         offsets, NB, W, Lseg, S, Rs);
    } else {
        static const int segq_env = getenv("VKZG_SEGSUM_QUAD") ? atoi(getenv("VKZG_SEGSUM_QUAD")) : 1;  // A/B probe
        bool quads = false;
        if constexpr (A::quad) {
            quads = segq_env != 0 && (size_t)S * W <= 65536;
            if (quads)
                VK_LAUNCH_ON(ctx, L.st, "msm_segsum", (k_msm_segsum_q<A>), (S * (uint32_t)W * 4 + 255) / 256, 256, 0,
                             buckets, offsets, NB, W, Lseg, S, accs, Rs);
        }
        if (!quads)
            VK_LAUNCH_ON(ctx, L.st, "msm_segsum", (k_msm_segsum<A>), (S * (uint32_t)W + 255) / 256, 256, 0, buckets,
                         offsets, NB, W, Lseg, S, accs, Rs);
    }
    const uint32_t sums = (uint32_t)W * (J + nU);
    // Lseg = 1: the U items are the R_s themselves, so U can come from the row sums (TailPlan::urow;
    // the caller's fold then adds T_h to it, msm_tail_fix_urow)
    const TailPlan tp = msm_tail_plan(S, (uint32_t)W, J, nU, A::quad, Lseg == 1);
    const uint32_t n_waves = (uint32_t)W * tp.per_w;
    VK_LAUNCH_ON(ctx, L.st, "msm_bitsum", (k_msm_bitsum<A>), (n_waves * 64 + 255) / 256, 256, 0, usrc, Rs, S, J, tp.h,
                 nU, tp.K, tp.nb1, tp.nb2, tp.pL, tp.gL, tp.gH, n_waves, toff, uoff, partial);
    if constexpr (A::quad)
        VK_LAUNCH_ON(ctx, L.st, "msm_sumpart", (k_msm_sumpart_q<C, A>), sums, 64 * SUMPART_WAVES, 0, partial, J, tp.h,
                     nU, tp.nb1, tp.nb2, tp.pL, tp.urow ? 1u : 0u, out, dir);
    else
        VK_LAUNCH_ON(ctx, L.st, "msm_sumpart", (k_msm_sumpart<C, A>), sums, 64, 0, partial, J, tp.h, nU, tp.nb1,
                     tp.nb2, tp.pL, tp.urow ? 1u : 0u, out, dir);
    return VC_OK;
}

#ifdef VKZG_TAIL_TRACE
// the trace (TT_KERNELS x TT_MAXT x 4 u64) -> host, then cleared (diagnostic build only; not part
// of the C ABI in include/)
extern "C" int vkzg_tail_trace_fetch(unsigned long long* out, size_t words) {
    const size_t all = sizeof(g_tail_trace) / sizeof(unsigned long long);
    void* dp = nullptr;
    VK_CHECK_HIP(hipGetSymbolAddress(&dp, HIP_SYMBOL(g_tail_trace)));
    VK_CHECK_HIP(hipDeviceSynchronize());
    if (out) VK_CHECK_HIP(hipMemcpy(out, dp, std::min(words, all) * 8, hipMemcpyDeviceToHost));
    VK_CHECK_HIP(hipMemset(dp, 0, sizeof(g_tail_trace)));
    VK_CHECK_HIP(hipDeviceSynchronize());
    return VC_OK;
}
#endif

#define VK_INST_TAIL(C)                                                                                      \
    template int msm_tail_fixup<C>(vc_ctx*, Lane, uint32_t, const uint32_t*, uint32_t, FAcc<C>*, FAcc<C>*,           \
                                   const uint8_t*, const FAcc<C>*, const uint32_t*, const uint32_t*, uint32_t); \
    template int msm_tail_fixup_more<C>(vc_ctx*, Lane, uint32_t, const uint32_t*, uint32_t, FAcc<C>*, FAcc<C>*,      \
                                        const uint8_t*, const FAcc<C>*, const uint32_t*, uint32_t, uint32_t);   \
    template int msm_tail_fixup_walk<C>(vc_ctx*, Lane, const uint32_t*, uint32_t, uint32_t, FAcc<C>*, const FAcc<C>*, \
                                        const FAcc<C>*, uint32_t, const uint32_t*, const uint8_t*, uint32_t);                                             \
    template int msm_tail_reduce<C>(vc_ctx*, Lane, const FAcc<C>*, const uint32_t*, uint32_t, int, uint32_t, uint32_t, \
                                    uint32_t, FAcc<C>*, FAcc<C>*, FAcc<C>*, C::Acc*, bool, const TailDirect*);
VK_INST_TAIL(BN254G1)
VK_INST_TAIL(BLS381G1)
VK_INST_TAIL(Bandersnatch)

}  // namespace vk
