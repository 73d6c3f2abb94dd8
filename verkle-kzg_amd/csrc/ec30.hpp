// XYZZ additions over the signed radix-2^30 field (ff30.hpp): the SW29 engine (ec29.hpp) for
// BLS12-381 G1 in 13 limbs instead of 14 -- same interface (Aff / AffN / AffP, Acc, load,
// madd, add, dbl, add_quad, store, pack_aff), same formulas, signed values: no K p constants,
// subtraction is limb-wise. Fast29<BLS381G1> selects it (ec29.hpp; -DVKZG_BLS_R29 keeps the
// radix-2^29 engine for A/B builds).
//
// Tables ("packed 30"): canonical x R' mod p (R' = 2^390) in the N 32-bit words of the ec.hpp
// layout, made by pack_aff; the limb forms (Aff, AffN, AffP) hold near limbs.
//
// Value bounds (|.| in units of p; product outputs < 0.51, ff30.hpp): X = RR - PPP - 2Q < 2.1,
// Y (a lazy pair) < 0.52, ZZ, ZZZ < 0.51; operands: U2 - X < 2.7, S2 - Y < 1.1, Q - X3 < 2.7, the
// general add's U2 - U1 < 1.1, the doubling's M = 3 X^2 < 1.6, S - X3 < 2.7 -- every product of
// two of them far below the c_a c_b < 300 of ff30.hpp. RR - PPP - 2Q (and M^2 - 2S, 3 X^2) of
// exact limbs lie in [-2^31 + 3, 2^31 - 1]: norm30w takes them.
#pragma once
#include "ec.hpp"
#include "ff30.hpp"

namespace vk {

template <class C, class P>
struct SW30 {
    using OAcc = typename C::Acc;
    using OAff = typename C::Aff;
    using F = typename C::F;
    struct Aff {
        f30<P> x, y;
    };
    // both signs of y (shared-window copies): the entry's sign picks y or -y through the address
    struct AffN {
        f30<P> x, y, ny;
    };
    // pair layout: record 2 i holds (x, y), 2 i + 1 (x, -y), one aligned 128-B line each
    static constexpr int PADW = ((2 * P::L * 4 + 127) / 128 * 128 - 2 * P::L * 4) / 4;
    static_assert(PADW > 0, "pair record padding");
    struct AffP {
        f30<P> x, y;
        uint32_t pad[PADW];
    };
    struct Acc {
        f30<P> x, y, zz, zzz;
        bool inf;
    };
    VK_HD static Acc zero() {
        Acc r;
        r.x = r.y = r.zz = r.zzz = zero30<P>();
        r.inf = true;
        return r;
    }
    // a packed-30 table point
    VK_HD static Aff load(const OAff* p) {
        Aff a;
        a.x = unpack30<P>(p->x.v);
        a.y = unpack30<P>(p->y.v);
        return a;
    }
    VK_HD static Aff load(const Aff* p) { return *p; }
    VK_HD static Acc dbl_aff(const f30<P>& x, const f30<P>& y) {
        const f30<P> U = add30<P>(y, y);
        const f30<P> V = sqr30<P>(U);
        const f30<P> W = mul30<P>(U, V);
        const f30<P> S = mul30<P>(x, V);
        const f30<P> X2 = sqr30<P>(x);
        f30<P> M;
#pragma unroll
        for (int j = 0; j < P::L; j++) M.v[j] = 3 * X2.v[j];
        M = norm30w<P>(M);
        Acc r;
        const f30<P> MM = sqr30<P>(M);
        f30<P> x3;
#pragma unroll
        for (int j = 0; j < P::L; j++) x3.v[j] = MM.v[j] - 2 * S.v[j];
        r.x = norm30w<P>(x3);
        r.y = mul2sum30<P>(M, sub30<P>(S, r.x), W, neg30<P>(y));
        r.zz = V;
        r.zzz = W;
        r.inf = false;
        return r;
    }
    // madd-2008-s: acc + (x2, +-y2). The sign is applied to S2 = y2 ZZZ1 (and to the rare
    // doubling's ZZZ3) instead of to y2: a select of y or -y as a multiply operand compiles to
    // 64 x 64-bit products (the sign extension is not seen through the select)
    VK_HD static Acc madd(const Acc& p, const Aff& q, bool neg) {
        if (p.inf) {
            Acc r;
            r.x = q.x;
            r.y = neg ? neg30<P>(q.y) : q.y;
            r.zz = one30<P>();
            r.zzz = one30<P>();
            r.inf = false;
            return r;
        }
        const f30<P> U2 = mul30<P>(q.x, p.zz);
        const f30<P> S2p = mul30<P>(q.y, p.zzz);
        const f30<P> S2 = neg ? neg30<P>(S2p) : S2p;
        const f30<P> Pd = sub30<P>(U2, p.x);
        const f30<P> R = sub30<P>(S2, p.y);
        const f30<P> PP = sqr30<P>(Pd);
        const f30<P> PPP = mul30<P>(Pd, PP);
        const f30<P> Q = mul30<P>(p.x, PP);
        Acc r;
        {
            const f30<P> RR = sqr30<P>(R);
            f30<P> x3;
#pragma unroll
            for (int j = 0; j < P::L; j++) x3.v[j] = RR.v[j] - PPP.v[j] - Q.v[j] - Q.v[j];
            r.x = norm30w<P>(x3);
        }
        // Y3 = R (Q - X3) - Y1 PPP with one reduction
        r.y = mul2sum30<P>(R, sub30<P>(Q, r.x), p.y, neg30<P>(PPP));
        r.zz = mul30<P>(p.zz, PP);
        r.zzz = mul30<P>(p.zzz, PPP);
        r.inf = false;
        // P == 0 mod p: q = +-acc (rare). r is overwritten inside the test, not returned from an
        // else: with `return r` on one side the compiler sinks Y3 and ZZZ3 past the test, and
        // their operands (product outputs, extended to i64 in the block before) become 64 x 64-bit
        // products (ff30.hpp opq30)
        if (is_zero_mo30<P>(r.zz)) {
            // R^2 = 0 iff R = 0 (a product by the constant one30 compiles to 64 x 64-bit multiplies)
            if (is_zero_mo30<P>(sqr30<P>(R))) {
                r = dbl_aff(q.x, q.y);  // 2 (x, -y) = (X3, Y3, ZZ3, -ZZZ3) of 2 (x, y)
                if (neg) r.zzz = neg30<P>(r.zzz);
            } else {
                r = zero();
            }
        }
        return r;
    }
    // dbl-2008-s-1
    VK_HD static Acc dbl(const Acc& p) {
        if (p.inf) return p;
        const f30<P> U = add30<P>(p.y, p.y);
        const f30<P> V = sqr30<P>(U);
        const f30<P> W = mul30<P>(U, V);
        const f30<P> S = mul30<P>(p.x, V);
        const f30<P> X2 = sqr30<P>(p.x);
        f30<P> M;
#pragma unroll
        for (int j = 0; j < P::L; j++) M.v[j] = 3 * X2.v[j];
        M = norm30w<P>(M);
        Acc r;
        const f30<P> MM = sqr30<P>(M);
        f30<P> x3;
#pragma unroll
        for (int j = 0; j < P::L; j++) x3.v[j] = MM.v[j] - 2 * S.v[j];
        r.x = norm30w<P>(x3);
        r.y = mul2sum30<P>(M, sub30<P>(S, r.x), W, neg30<P>(p.y));
        r.zz = mul30<P>(V, p.zz);
        r.zzz = mul30<P>(W, p.zzz);
        r.inf = is_zero_mo30<P>(r.zz);  // y == 0: 2P = O
        return r;
    }
    // add-2008-s (both operands general XYZZ accumulators)
    VK_HD static Acc add(const Acc& p, const Acc& q) {
        if (p.inf) return q;
        if (q.inf) return p;
        const f30<P> U1 = mul30<P>(p.x, q.zz);
        const f30<P> U2 = mul30<P>(q.x, p.zz);
        const f30<P> S1 = mul30<P>(p.y, q.zzz);
        const f30<P> S2 = mul30<P>(q.y, p.zzz);
        const f30<P> Pd = sub30<P>(U2, U1);
        const f30<P> R = sub30<P>(S2, S1);
        const f30<P> PP = sqr30<P>(Pd);
        const f30<P> PPP = mul30<P>(Pd, PP);
        const f30<P> Q = mul30<P>(U1, PP);
        Acc r;
        {
            const f30<P> RR = sqr30<P>(R);
            f30<P> x3;
#pragma unroll
            for (int j = 0; j < P::L; j++) x3.v[j] = RR.v[j] - PPP.v[j] - Q.v[j] - Q.v[j];
            r.x = norm30w<P>(x3);
        }
        r.y = mul2sum30<P>(R, sub30<P>(Q, r.x), S1, neg30<P>(PPP));
        r.zz = mul30<P>(mul30<P>(p.zz, q.zz), PP);
        r.zzz = mul30<P>(mul30<P>(p.zzz, q.zzz), PPP);
        r.inf = false;
        if (is_zero_mo30<P>(r.zz))  // P == 0 mod p: q = +-p (rare; r overwritten in place, as madd)
            r = is_zero_mo30<P>(sqr30<P>(R)) ? dbl(p) : zero();
        return r;
    }
#ifdef __HIPCC__
    // 4-lane cooperative add for the latency-bound tails (as SW29::add_quad): the lanes of a quad
    // hold the same operands, each computes one product of a round (operands by role = lane & 3),
    // products broadcast inside the quad with DPP quad_perm. Every lane of a quad must call it with
    // identical p, q.
    static constexpr bool quad = true;
    template <int K>
    __device__ static f30<P> qb(const f30<P>& x) {
        f30<P> r;
#pragma unroll
        for (int j = 0; j < P::L; j++) r.v[j] = __builtin_amdgcn_mov_dpp(x.v[j], K * 0x55, 0xf, 0xf, false);
        return r;
    }
    // by masks (a select of values becomes a load through a selected address: scratch)
    __device__ static f30<P> sel4(uint32_t role, const f30<P>& a0, const f30<P>& a1, const f30<P>& a2,
                                  const f30<P>& a3) {
        const int32_t m0 = -(int32_t)(role == 0), m1 = -(int32_t)(role == 1);
        const int32_t m2 = -(int32_t)(role == 2), m3 = -(int32_t)(role == 3);
        f30<P> r;
#pragma unroll
        for (int j = 0; j < P::L; j++) r.v[j] = (a0.v[j] & m0) | (a1.v[j] & m1) | (a2.v[j] & m2) | (a3.v[j] & m3);
        return r;
    }
    __device__ __forceinline__ static Acc add_quad(const Acc& p, const Acc& q, uint32_t role) {
        if (p.inf) return q;
        if (q.inf) return p;
        // round 1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
        const f30<P> m1 = mul30<P>(sel4(role, p.x, q.x, p.y, q.y), sel4(role, q.zz, p.zz, q.zzz, p.zzz));
        const f30<P> U1 = qb<0>(m1), U2 = qb<1>(m1), S1 = qb<2>(m1), S2 = qb<3>(m1);
        const f30<P> Pd = sub30<P>(U2, U1), R = sub30<P>(S2, S1);
        // round 2: PP = P^2, RR = R^2, ZZ1 ZZ2, ZZZ1 ZZZ2
        const f30<P> m2 = mul30<P>(sel4(role, Pd, R, p.zz, p.zzz), sel4(role, Pd, R, q.zz, q.zzz));
        const f30<P> PP = qb<0>(m2), RR = qb<1>(m2), ZZ12 = qb<2>(m2), ZZZ12 = qb<3>(m2);
        if (is_zero_mo30<P>(PP)) {  // P == 0 mod p: q = +-p (rare; uniform inside the quad)
            if (is_zero_mo30<P>(RR)) return dbl(p);
            return zero();
        }
        // round 3: PPP = P PP, Q = U1 PP, ZZ3 = ZZ1 ZZ2 PP (role 3 repeats role 2)
        const f30<P> m3 = mul30<P>(sel4(role, Pd, U1, ZZ12, ZZ12), PP);
        const f30<P> PPP = qb<0>(m3), Q = qb<1>(m3), ZZ3 = qb<2>(m3);
        Acc r;
        f30<P> x3;
#pragma unroll
        for (int j = 0; j < P::L; j++) x3.v[j] = RR.v[j] - PPP.v[j] - Q.v[j] - Q.v[j];
        r.x = norm30w<P>(x3);
        // round 4: Y3 = R (Q - X3) - S1 PPP (roles 0, 2); ZZZ3 = ZZZ1 ZZZ2 PPP + 0 (roles 1, 3)
        const f30<P> z = zero30<P>();
        const bool ev = (role & 1) == 0;
        const f30<P> QX = sub30<P>(Q, r.x), nP = neg30<P>(PPP);
        const f30<P> m4 = mul2sum30<P>(ev ? R : ZZZ12, ev ? QX : PPP, ev ? S1 : z, ev ? nP : z);
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
        r.x = to_mont32_30<P, F>(a.x);
        r.y = to_mont32_30<P, F>(a.y);
        r.zz = to_mont32_30<P, F>(a.zz);
        r.zzz = to_mont32_30<P, F>(a.zzz);
        return r;
    }
    // ec.hpp affine point (x R) -> packed 30 (x R')
    VK_HD static void pack_aff(const OAff& a, OAff* out) {
        OAff o;
        uint32_t u[P::L];
        canon30<P>(from_mont32_30<P, F>(a.x), u);
        pack30<P>(u, o.x.v);
        canon30<P>(from_mont32_30<P, F>(a.y), u);
        pack30<P>(u, o.y.v);
        *out = o;
    }
};

}  // namespace vk
