// Mixed additions over the radix-2^29 fields (ff29.hpp) for the VALU-bound inner loops:
// Pippenger bucket accumulation (k_msm_accumulate) and the fixed-base commits (commit.hip).
// Points in HBM stay in the ec.hpp layouts; the tables these loops read hold x R' mod p
// ("packed 29" form, made once per table by k_to_fast), accumulators are converted back to
// the ec.hpp form (x R) when stored. Same group law and exceptional-case handling as ec.hpp.
//
// Value bounds (ff29.hpp keeps residues loosely reduced; rho = p / R'):
//  SW (XYZZ, a = 0): X < 11p, Y < 7p, ZZ, ZZZ < 1.1p between adds (BN254's rho = 2^-7.4 is
//    the tight case; BLS12-381's 2^-25 leaves every product output below 1.0001 p). The add
//    paths' Y3 = R (Q - X3) + Y1 (4p - PPP) is one lazy sum of products (mul2sum29):
//    < (17p 17p + 7p 4p) rho + p = 2.9p at BN254, 1.0001p at BLS12-381.
//  TE (extended, a = -5, Bandersnatch over BLS12-381 Fr, rho = 2^-6.1): every coordinate is
//    a product output < 1.9p (fixed point of the bounds with inputs < 2p).
#pragma once
#include "ec.hpp"
#include "ec30.hpp"
#include "ff29.hpp"

namespace vk {

template <class C, class P>
struct SW29 {
    using OAcc = typename C::Acc;
    using OAff = typename C::Aff;
    using F = typename C::F;
    struct Aff {
        f29<P> x, y;
    };
    // a base with both signs of y (the shared-window copies): the accumulate picks y or -y by
    // the entry's sign through the load address, so the mixed add has no negation in it
    struct AffN {
        f29<P> x, y, ny;
    };
    // pair layout of the same copies: one signed copy of a base per 128-B record -- record 2 i
    // holds (x, y), 2 i + 1 (x, -y) -- so the accumulate's gather is ONE aligned line (the x, y,
    // -y record straddles two or three); 256 B per base instead of 168
    static constexpr int PADW = ((2 * P::L * 4 + 127) / 128 * 128 - 2 * P::L * 4) / 4;
    static_assert(PADW > 0, "pair record padding");
    struct AffP {
        f29<P> x, y;
        uint32_t pad[PADW];
    };
    struct Acc {
        f29<P> x, y, zz, zzz;
        bool inf;
    };
    VK_HD static Acc zero() {
        Acc r;
        r.x = r.y = r.zz = r.zzz = zero29<P>();
        r.inf = true;
        return r;
    }
    // a packed-29 table point
    VK_HD static Aff load(const OAff* p) {
        Aff a;
        a.x = unpack29<P>(p->x.v);
        a.y = unpack29<P>(p->y.v);
        return a;
    }
    // a table point already in limbs (fixed-base tables, commit.hip FbE)
    VK_HD static Aff load(const Aff* p) { return *p; }
    VK_HD static Acc dbl_aff(const f29<P>& x, const f29<P>& y) {
        const f29<P> U = add29<P>(y, y);
        const f29<P> V = sqr29<P>(U);
        const f29<P> W = mul29<P>(U, V);
        const f29<P> S = mul29<P>(x, V);
        const f29<P> X2 = sqr29<P>(x);
        const f29<P> M = add29<P>(add29<P>(X2, X2), X2);
        Acc r;
        r.x = sub29<P, 8>(sqr29<P>(M), add29<P>(S, S));
        r.y = sub29<P, 4>(mul29<P>(M, sub29<P, 16>(S, r.x)), mul29<P>(W, y));
        r.zz = V;
        r.zzz = W;
        r.inf = false;
        return r;
    }
    // madd-2008-s: acc + (x2, +-y2)
    VK_HD static Acc madd(const Acc& p, const Aff& q, bool neg) {
        const f29<P> y2 = neg ? neg29<P, 2>(q.y) : q.y;
        if (p.inf) {
            Acc r;
            r.x = q.x;
            r.y = y2;
            r.zz = one29<P>();
            r.zzz = one29<P>();
            r.inf = false;
            return r;
        }
        const f29<P> U2 = mul29<P>(q.x, p.zz);
        const f29<P> S2 = mul29<P>(y2, p.zzz);
        const f29<P> Pd = sub29<P, 16>(U2, p.x);
        const f29<P> R = sub29<P, 16>(S2, p.y);
        const f29<P> PP = sqr29<P>(Pd);
        const f29<P> PPP = mul29<P>(Pd, PP);
        const f29<P> Q = mul29<P>(p.x, PP);
        Acc r;
        // X3 = R^2 - PPP - 2Q in one pass: 8p - (PPP + 2Q) per limb (product outputs: limbs < 2^29,
        // so the subtrahend's limbs stay below 3 * 2^29 < subK's 2^31 - 4), one carry pass
        {
            const f29<P> RR = sqr29<P>(R);
            f29<P> x3;
#pragma unroll
            for (int j = 0; j < P::L; j++) x3.v[j] = RR.v[j] + subk<P, 8>(j) - (PPP.v[j] + Q.v[j] + Q.v[j]);
            r.x = norm29<P>(x3);
        }
        // Y3 = R (Q - X3) + Y1 (4p - PPP) with one reduction (mul2sum29)
        r.y = mul2sum29<P>(R, sub29<P, 16>(Q, r.x), p.y, neg29<P, 4>(PPP));
        r.zz = mul29<P>(p.zz, PP);
        r.zzz = mul29<P>(p.zzz, PPP);
        r.inf = false;
        // P == 0 mod p (q = +-acc, rare). (A filter on ZZ3's lowest limb first kept more values live
        // across the branch: 268 VGPRs, one wave per SIMD, 2.24 -> 2.56 ms -- the full check stays.)
        if (is_zero_mo29<P>(r.zz)) {
            if (is_zero_mo29<P>(mul29<P>(R, one29<P>()))) return dbl_aff(q.x, y2);
            return zero();
        }
        return r;
    }
    // dbl-2008-s-1
    VK_HD static Acc dbl(const Acc& p) {
        if (p.inf) return p;
        const f29<P> U = add29<P>(p.y, p.y);
        const f29<P> V = sqr29<P>(U);
        const f29<P> W = mul29<P>(U, V);
        const f29<P> S = mul29<P>(p.x, V);
        const f29<P> X2 = sqr29<P>(p.x);
        const f29<P> M = add29<P>(add29<P>(X2, X2), X2);
        Acc r;
        r.x = sub29<P, 8>(sqr29<P>(M), add29<P>(S, S));
        r.y = sub29<P, 4>(mul29<P>(M, sub29<P, 16>(S, r.x)), mul29<P>(W, p.y));
        r.zz = mul29<P>(V, p.zz);
        r.zzz = mul29<P>(W, p.zzz);
        r.inf = is_zero_mo29<P>(r.zz);  // y == 0: 2P = O
        return r;
    }
    // add-2008-s (both operands general XYZZ accumulators)
    VK_HD static Acc add(const Acc& p, const Acc& q) {
        if (p.inf) return q;
        if (q.inf) return p;
        const f29<P> U1 = mul29<P>(p.x, q.zz);
        const f29<P> U2 = mul29<P>(q.x, p.zz);
        const f29<P> S1 = mul29<P>(p.y, q.zzz);
        const f29<P> S2 = mul29<P>(q.y, p.zzz);
        const f29<P> Pd = sub29<P, 4>(U2, U1);
        const f29<P> R = sub29<P, 4>(S2, S1);
        const f29<P> PP = sqr29<P>(Pd);
        const f29<P> PPP = mul29<P>(Pd, PP);
        const f29<P> Q = mul29<P>(U1, PP);
        Acc r;
        r.x = sub2_29<P, 8>(sqr29<P>(R), PPP, add29<P>(Q, Q));
        r.y = mul2sum29<P>(R, sub29<P, 16>(Q, r.x), S1, neg29<P, 4>(PPP));
        r.zz = mul29<P>(mul29<P>(p.zz, q.zz), PP);
        r.zzz = mul29<P>(mul29<P>(p.zzz, q.zzz), PPP);
        r.inf = false;
        if (is_zero_mo29<P>(r.zz)) {  // P == 0 mod p: q = +-p (rare)
            if (is_zero_mo29<P>(mul29<P>(R, one29<P>()))) return dbl(p);
            return zero();
        }
        return r;
    }
#ifdef __HIPCC__
    // ---- 4-lane cooperative add for the latency-bound tails (msm_tail.hip). The four lanes of a
    // quad hold the same operands and each computes a different product of the same round in ONE
    // instruction stream (operands selected by role = lane & 3), the products are broadcast inside
    // the quad with DPP quad_perm: 3 multiplies + 1 lazy pair of issue per add instead of 10 + 2
    // squares + 1 pair (~3,100 vs ~6,600 instructions per wave, the same group element as add()).
    // Every lane of a quad must call it with identical p, q.
    static constexpr bool quad = true;
    template <int K>
    __device__ static f29<P> qb(const f29<P>& x) {
        f29<P> r;
#pragma unroll
        for (int j = 0; j < P::L; j++) r.v[j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.v[j], K * 0x55, 0xf, 0xf, false);
        return r;
    }
    // operand of this lane's role, by masks: a select of the values (role ? a.v[j] : b.v[j]) lets
    // the compiler turn it into a load through a selected address, which pins the accumulators
    // in scratch memory (572 B per lane, reloaded every add)
    __device__ static f29<P> sel4(uint32_t role, const f29<P>& a0, const f29<P>& a1, const f29<P>& a2,
                                  const f29<P>& a3) {
        const uint32_t m0 = 0u - (uint32_t)(role == 0), m1 = 0u - (uint32_t)(role == 1);
        const uint32_t m2 = 0u - (uint32_t)(role == 2), m3 = 0u - (uint32_t)(role == 3);
        f29<P> r;
#pragma unroll
        for (int j = 0; j < P::L; j++) r.v[j] = (a0.v[j] & m0) | (a1.v[j] & m1) | (a2.v[j] & m2) | (a3.v[j] & m3);
        return r;
    }
    __device__ __forceinline__ static Acc add_quad(const Acc& p, const Acc& q, uint32_t role) {
        if (p.inf) return q;
        if (q.inf) return p;
        // round 1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
        const f29<P> m1 = mul29<P>(sel4(role, p.x, q.x, p.y, q.y), sel4(role, q.zz, p.zz, q.zzz, p.zzz));
        const f29<P> U1 = qb<0>(m1), U2 = qb<1>(m1), S1 = qb<2>(m1), S2 = qb<3>(m1);
        const f29<P> Pd = sub29<P, 4>(U2, U1), R = sub29<P, 4>(S2, S1);
        // round 2: PP = P^2, RR = R^2, ZZ1 ZZ2, ZZZ1 ZZZ2
        const f29<P> m2 = mul29<P>(sel4(role, Pd, R, p.zz, p.zzz), sel4(role, Pd, R, q.zz, q.zzz));
        const f29<P> PP = qb<0>(m2), RR = qb<1>(m2), ZZ12 = qb<2>(m2), ZZZ12 = qb<3>(m2);
        if (is_zero_mo29<P>(PP)) {  // P == 0 mod p: q = +-p (rare; uniform inside the quad)
            if (is_zero_mo29<P>(RR)) return dbl(p);
            return zero();
        }
        // round 3: PPP = P PP, Q = U1 PP, ZZ3 = ZZ1 ZZ2 PP (role 3 repeats role 2)
        const f29<P> m3 = mul29<P>(sel4(role, Pd, U1, ZZ12, ZZ12), PP);
        const f29<P> PPP = qb<0>(m3), Q = qb<1>(m3), ZZ3 = qb<2>(m3);
        Acc r;
        r.x = sub2_29<P, 8>(RR, PPP, add29<P>(Q, Q));
        // round 4: Y3 = R (Q - X3) + S1 (4p - PPP) (roles 0, 2); ZZZ3 = ZZZ1 ZZZ2 PPP + 0 (roles 1, 3)
        const f29<P> z = zero29<P>();
        const bool ev = (role & 1) == 0;
        const f29<P> QX = sub29<P, 16>(Q, r.x), nP = neg29<P, 4>(PPP);
        const f29<P> m4 = mul2sum29<P>(ev ? R : ZZZ12, ev ? QX : PPP, ev ? S1 : z, ev ? nP : z);
        r.y = qb<0>(m4);
        r.zz = ZZ3;
        r.zzz = qb<1>(m4);
        r.inf = false;
        return r;
    }
#endif
    // back to the ec.hpp accumulator (x R, canonical)
    VK_HD static OAcc store(const Acc& a) {
        if (a.inf) return C::zero();
        OAcc r;
        r.x = to_mont32<P, F>(a.x);
        r.y = to_mont32<P, F>(a.y);
        r.zz = to_mont32<P, F>(a.zz);
        r.zzz = to_mont32<P, F>(a.zzz);
        return r;
    }
    // ec.hpp affine point (x R) -> packed 29 (x R')
    VK_HD static void pack_aff(const OAff& a, OAff* out) {
        OAff o;
        pack29<P>(canon29<P>(from_mont32<P, F>(a.x)), o.x.v);
        pack29<P>(canon29<P>(from_mont32<P, F>(a.y)), o.y.v);
        *out = o;
    }
};

template <class C, class P>
struct TE29 {
    static constexpr bool quad = false;  // no cooperative add: the Edwards tails keep add()
    using OAcc = typename C::Acc;
    using OAff = typename C::Aff;
    using F = typename C::F;
    struct Aff {
        f29<P> x, y, kt;
    };
    struct Acc {
        f29<P> X, Y, T, Z;
    };
    VK_HD static Acc zero() {
        Acc r;
        r.X = r.T = zero29<P>();
        r.Y = r.Z = one29<P>();
        return r;
    }
    VK_HD static Aff load(const OAff* p) {
        Aff a;
        a.x = unpack29<P>(p->x.v);
        a.y = unpack29<P>(p->y.v);
        a.kt = unpack29<P>(p->kt.v);
        return a;
    }
    VK_HD static Aff load(const Aff* p) { return *p; }
    // unified mixed add (add-2008-hwcd, Z2 = 1, kt = d x2 y2): complete, no exceptions
    VK_HD static Acc madd(const Acc& p, const Aff& q, bool neg) {
        const f29<P> x2 = neg ? neg29<P, 2>(q.x) : q.x;
        const f29<P> kt = neg ? neg29<P, 2>(q.kt) : q.kt;
        static_assert(P::L <= 9, "raw x raw operands of mul29 (add29_raw) need L <= 9");
        const f29<P> A = mul29<P>(p.X, x2);
        const f29<P> B = mul29<P>(p.Y, q.y);
        const f29<P> Cc = mul29<P>(p.T, kt);
        // sums that only feed products skip the carry pass (add29_raw): X + Y and x2 + y2 are both
        // raw operands of one product, G = Z + C a raw operand of two
        const f29<P> E = sub2_29<P, 8>(mul29<P>(add29_raw<P>(p.X, p.Y), add29_raw<P>(x2, q.y)), A, B);
        const f29<P> Fv = sub29<P, 4>(p.Z, Cc);
        const f29<P> G = add29_raw<P>(p.Z, Cc);
        // H = B - a A = B + 5 A (a = -5): limb-wise < 2^31.6, one carry pass
        f29<P> H;
#pragma unroll
        for (int j = 0; j < P::L; j++) H.v[j] = B.v[j] + 5u * A.v[j];
        H = norm29<P>(H);
        Acc r;
        r.X = mul29<P>(E, Fv);
        r.Y = mul29<P>(G, H);
        r.T = mul29<P>(E, H);
        r.Z = mul29<P>(Fv, G);
        return r;
    }
    // unified add (add-2008-hwcd): 10 multiplies (d T1 T2 as two)
    VK_HD static Acc add(const Acc& p, const Acc& q) {
        f29<P> d;
#pragma unroll
        for (int j = 0; j < P::L; j++) d.v[j] = P::band_d(j);
        const f29<P> A = mul29<P>(p.X, q.X);
        const f29<P> B = mul29<P>(p.Y, q.Y);
        const f29<P> Cc = mul29<P>(mul29<P>(p.T, q.T), d);
        const f29<P> D = mul29<P>(p.Z, q.Z);
        const f29<P> E = sub2_29<P, 8>(mul29<P>(add29<P>(p.X, p.Y), add29<P>(q.X, q.Y)), A, B);
        const f29<P> Fv = sub29<P, 4>(D, Cc);
        const f29<P> G = add29<P>(D, Cc);
        const f29<P> A2 = add29<P>(A, A);
        const f29<P> H = add29<P>(B, add29<P>(add29<P>(A2, A2), A));
        Acc r;
        r.X = mul29<P>(E, Fv);
        r.Y = mul29<P>(G, H);
        r.T = mul29<P>(E, H);
        r.Z = mul29<P>(Fv, G);
        return r;
    }
    VK_HD static OAcc store(const Acc& a) {
        OAcc r;
        r.X = to_mont32<P, F>(a.X);
        r.Y = to_mont32<P, F>(a.Y);
        r.T = to_mont32<P, F>(a.T);
        r.Z = to_mont32<P, F>(a.Z);
        return r;
    }
    VK_HD static void pack_aff(const OAff& a, OAff* out) {
        OAff o;
        pack29<P>(canon29<P>(from_mont32<P, F>(a.x)), o.x.v);
        pack29<P>(canon29<P>(from_mont32<P, F>(a.y)), o.y.v);
        pack29<P>(canon29<P>(from_mont32<P, F>(a.kt)), o.kt.v);
        *out = o;
    }
};

#ifdef __HIPCC__
// xor-shuffle of a POD accumulator across the wave (word by word)
template <class T>
__device__ __forceinline__ T shfl_xor_pod(const T& v, uint32_t m) {
    static_assert(sizeof(T) % 4 == 0, "");
    T o;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = __shfl_xor(src[k], m, 64);
    return o;
}
// v of lane `src` (word by word)
template <class T>
__device__ __forceinline__ T shfl_idx_pod(const T& v, uint32_t src_lane) {
    static_assert(sizeof(T) % 4 == 0, "");
    T o;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = __shfl(src[k], (int)src_lane, 64);
    return o;
}
#endif

// curve of ec.hpp -> its mixed-add engine: radix 2^29, except BLS12-381 G1 on the signed
// radix-2^30 engine of ec30.hpp (13 limbs instead of 14: -14 % of the multiply's products;
// -DVKZG_BLS_R29 builds the radix-2^29 one for A/B runs)
template <class C>
struct Fast29;
template <>
struct Fast29<BLS381G1> {
#ifdef VKZG_BLS_R29
    using type = SW29<BLS381G1, F29BLS381Fq>;
#else
    using type = SW30<BLS381G1, F30BLS381Fq>;
#endif
};
template <>
struct Fast29<BN254G1> {
    using type = SW29<BN254G1, F29BN254Fq>;
};
template <>
struct Fast29<Bandersnatch> {
    using type = TE29<Bandersnatch, F29BLS381Fr>;
};

// Fixed-base window table entry (commit.hip; read by the sparse commits' accumulate, msm.hip).
// Table entry (kept as a type so the layout can change in one place): the radix-2^29 limbs the
// mixed add consumes (ec29.hpp Aff, 4 B per 29-bit limb: 108 B for Bandersnatch's x, y, d x y),
// so the loop reads operands with no unpacking (~53 of 2,250 instructions per Edwards add).
// (Padding the packed 96-B form -- unpacked in the loop -- to 128 B was measured slower, round 2.)
// Every entry is padded to a whole 128-B line (round 5), so a gather reads one line instead of
// straddling two: Bandersnatch's 108-B entries mostly spanned two lines (33.3M gathers per 10k
// commits at c = 19 x 13 moved 8-9.5 GB by the counters). Measured on one MI355X, 10k width-256
// commits: c = 16 3.08-3.11 -> 3.19-3.25 M/s, c = 17 (15 windows) 3.27-3.31 -> 3.40-3.41, c = 18 x 14
// 3.53 -> 3.66-3.68 (profiles/r05/commit_pad128/). -DVKZG_FB_PACKED keeps the 108-B entries (A/B).
template <class C>
struct FbEntryLimbs {
    typename Fast29<C>::type::Aff u;
#ifndef VKZG_FB_PACKED
    uint32_t pad[(128 - sizeof(typename Fast29<C>::type::Aff) % 128) % 128 / 4];
#endif
};
template <class C>
using FbE = FbEntryLimbs<C>;

#ifdef __HIPCC__
// xor butterfly over the wave on the radix-29 accumulators (the add the tails run too). The
// shuffle moves sizeof(Acc) / 4 words (shfl_xor_pod): SW29::Acc is 4 L limbs of 29 bits plus the
// `inf` flag -- 37 words at BN254 (L = 9), 57 at BLS12-381 -- not the 4 N words of the ec.hpp
// accumulator (C::ACC_WORDS = 32 / 48). An earlier version shuffled C::ACC_WORDS words of the
// radix-29 accumulator, which left zz / zzz partly and `inf` entirely lane-local: every commit
// with more than one non-identity lane came out wrong (batched-commit parity failed at the first
// non-zero commit on the GPU while the host tests of the add formulas passed).
template <class FC>
__device__ __forceinline__ typename FC::Acc fb_wave_sum29(typename FC::Acc v) {
    for (uint32_t m = 1; m < 64; m <<= 1) v = FC::add(v, shfl_xor_pod(v, m));
    return v;
}

// The sum of a block's accumulators (one per thread, NT = 256 or 64 threads), stored by thread 0
// at *out (the fixed-base latency paths: commit.hip k_fb_commit_small, msm.hip k_fb_sparse_small).
// On 4-lane cooperative adds (SW29::add_quad, ~half the latency of a full add): quad q first adds
// its own four lanes' points (3 rounds), then the 16 quads of the wave fold by xor (4), then (NT =
// 256) wave 0 folds the 4 wave sums from LDS (2): 9 dependent adds of ~6 us instead of 6 full adds
// of ~13 us plus 3 more on one thread. Every thread of the block must call it.
template <class C, int NT = 256>
__device__ __forceinline__ void fb_block_sum_store(typename Fast29<C>::type::Acc fa, typename C::Acc* out) {
    static_assert(NT == 256 || NT == 64, "a wave or four");
    using FC = typename Fast29<C>::type;
    using Acc = typename C::Acc;
    if constexpr (FC::quad) {
        __shared__ typename FC::Acc wq[NT / 64];
        const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, role = lane & 3, q0 = lane & ~3u;
        constexpr uint32_t ITS = NT == 256 ? 9 : 7;
        typename FC::Acc v = shfl_idx_pod(fa, q0);
        for (uint32_t it = 0; it < ITS; it++) {  // one add call site
            typename FC::Acc o;
            if (it < 3) {
                o = shfl_idx_pod(fa, q0 + it + 1);
            } else if (it < 7) {
                o = shfl_xor_pod(v, 4u << (it - 3));
            } else {
                if (it == 7) {
                    if (lane == 0) wq[wave] = v;
                    __syncthreads();
                    if (wave != 0) break;
                    v = (lane >> 2) < 4 ? wq[lane >> 2] : FC::zero();
                }
                o = shfl_xor_pod(v, 4u << (it - 7));
            }
            v = FC::add_quad(v, o, role);
        }
        if (threadIdx.x == 0) *out = FC::store(v);
    } else {
        Acc acc = FC::store(fb_wave_sum29<FC>(fa));
        if constexpr (NT == 64) {
            if (threadIdx.x == 0) *out = acc;
        } else {
            __shared__ Acc wsum[4];
            const int wave = threadIdx.x / 64;
            if ((threadIdx.x & 63) == 0) wsum[wave] = acc;
            __syncthreads();
            if (threadIdx.x == 0) *out = C::add(C::add(wsum[0], wsum[1]), C::add(wsum[2], wsum[3]));
        }
    }
}

#endif  // __HIPCC__

}  // namespace vk
