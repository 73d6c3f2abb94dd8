// Host check of the radix-2^29 point arithmetic (verkle-kzg_amd/csrc/ec29.hpp) against the
// 32-bit-limb formulas of ec.hpp: chains of mixed adds with random signs, full adds, doublings,
// and the exceptional cases (q = acc, q = -acc, zero operands), compared as affine points.
// Prints one JSON line per curve with the number of comparisons and mismatches.
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../verkle-kzg_amd/csrc/ec29.hpp"
using namespace vk;

static uint64_t rs = 0x243F6A8885A308D3ull;
static uint64_t rnd64() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}

template <class C>
struct G;
template <>
struct G<BN254G1> {
    static uint32_t x(int i) { return i == 0 ? 1u : 0u; }
    static uint32_t y(int i) { return i == 0 ? 2u : 0u; }
};
template <>
struct G<BLS381G1> {
    static uint32_t x(int i) {
        const uint32_t v[] = {0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu, 0x171bac58u, 0xa14e3a3fu,
                              0x9774b905u, 0xc3688c4fu, 0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u};
        return v[i];
    }
    static uint32_t y(int i) {
        const uint32_t v[] = {0x46c5e7e1u, 0x0caa2329u, 0xa2888ae4u, 0xd03cc744u, 0x2c04b3edu, 0x00db18cbu,
                              0xd5d00af6u, 0xfcf5e095u, 0x741d8ae4u, 0xa09e30edu, 0xe3aaa0f1u, 0x08b3f481u};
        return v[i];
    }
};
template <>
struct G<Bandersnatch> {
    static uint32_t x(int i) {
        const uint32_t v[] = {0xa252ae18u, 0xe1e71866u, 0xad998465u, 0x2b79c022u,
                              0x7bbe42f3u, 0x74371177u, 0x2c0b34c5u, 0x29c132ccu};
        return v[i];
    }
    static uint32_t y(int i) {
        const uint32_t v[] = {0xcc974166u, 0x5e3167b6u, 0xeee46460u, 0x358cad81u,
                              0xbadcd586u, 0x157d8b50u, 0xda123e0fu, 0x2a6c669eu};
        return v[i];
    }
};

template <class C>
static typename C::Aff to_aff_old(const typename C::Acc& a, bool* inf) {
    typename C::Aff r{};
    fe<typename C::F> x, y;
    *inf = !C::to_aff(a, x, y);
    r.x = x;
    r.y = y;
    if constexpr (C::is_te) r.kt = fe_mul<typename C::F>(fe_mul<typename C::F>(x, y), C::d());
    return r;
}

template <class C>
static bool same(const typename C::Acc& a, const typename C::Acc& b) {
    bool ia, ib;
    auto pa = to_aff_old<C>(a, &ia), pb = to_aff_old<C>(b, &ib);
    if (ia || ib) return ia == ib;
    for (int k = 0; k < C::F::N; k++)
        if (pa.x.v[k] != pb.x.v[k] || pa.y.v[k] != pb.y.v[k]) return false;
    return true;
}

template <class C>
static void run(const char* name) {
    using F = typename C::F;
    using FC = typename Fast29<C>::type;
    using Acc = typename C::Acc;
    using Aff = typename C::Aff;
    fe<F> gx, gy;
    for (int k = 0; k < F::N; k++) {
        gx.v[k] = G<C>::x(k);
        gy.v[k] = G<C>::y(k);
    }
    Aff g{};
    g.x = fe_to_mont<F>(gx);
    g.y = fe_to_mont<F>(gy);
    if constexpr (C::is_te) g.kt = fe_mul<F>(fe_mul<F>(g.x, g.y), C::d());
    // random multiples of the generator (old form, affine) and their packed-29 copies
    const int NP = 24;
    std::vector<Aff> pts(NP), fast(NP);
    for (int i = 0; i < NP; i++) {
        uint64_t s = rnd64() | 1;
        Acc acc = C::zero();
        for (int b = 63; b >= 0; b--) {
            acc = C::dbl(acc);
            if ((s >> b) & 1) acc = C::madd(acc, g, false);
        }
        bool inf;
        pts[i] = to_aff_old<C>(acc, &inf);
        FC::pack_aff(pts[i], &fast[i]);
    }
    int checks = 0, bad = 0;
    // mixed-add chains with random signs; every 7th step re-adds the previous point (doubling
    // case when the accumulator equals it) and every 11th subtracts the accumulator's last add
    for (int chain = 0; chain < 6; chain++) {
        Acc ao = C::zero();
        typename FC::Acc af = FC::zero();
        for (int step = 0; step < 40; step++) {
            const int i = (int)(rnd64() % NP);
            const bool neg = (rnd64() & 1) != 0;
            ao = C::madd(ao, pts[i], neg);
            af = FC::madd(af, FC::load(&fast[i]), neg);
            checks++;
            bad += !same<C>(ao, FC::store(af));
        }
    }
    // exceptional: acc = P, then + P (double), then - 2P ... via a fresh chain
    for (int i = 0; i < 4; i++) {
        Acc ao = C::zero();
        typename FC::Acc af = FC::zero();
        for (int r = 0; r < 3; r++) {  // P, 2P (doubling case), 3P
            ao = C::madd(ao, pts[i], false);
            af = FC::madd(af, FC::load(&fast[i]), false);
            checks++;
            bad += !same<C>(ao, FC::store(af));
        }
        Acc z = C::madd(C::madd(C::zero(), pts[i], false), pts[i], true);                     // P - P
        typename FC::Acc zf = FC::madd(FC::madd(FC::zero(), FC::load(&fast[i]), false), FC::load(&fast[i]), true);
        checks++;
        bad += !same<C>(z, FC::store(zf));
        // full adds: a + b, a + a, a + (-a), zero operands
        typename FC::Acc a = FC::madd(FC::madd(FC::zero(), FC::load(&fast[i]), false), FC::load(&fast[i + 1]), false);
        typename FC::Acc b = FC::madd(FC::zero(), FC::load(&fast[i + 2]), true);
        Acc ao2 = C::madd(C::madd(C::zero(), pts[i], false), pts[i + 1], false);
        Acc bo = C::madd(C::zero(), pts[i + 2], true);
        checks += 4;
        bad += !same<C>(C::add(ao2, bo), FC::store(FC::add(a, b)));
        bad += !same<C>(C::add(ao2, ao2), FC::store(FC::add(a, a)));
        bad += !same<C>(C::add(ao2, C::neg(ao2)), FC::store(FC::add(a, FC::madd(FC::madd(FC::zero(),
                                                 FC::load(&fast[i]), true), FC::load(&fast[i + 1]), true))));
        bad += !same<C>(C::add(C::zero(), bo), FC::store(FC::add(FC::zero(), b)));
        if constexpr (!C::is_te) {
            checks++;
            bad += !same<C>(C::dbl(ao2), FC::store(FC::dbl(a)));
        }
    }
    printf("{\"curve\":\"%s\",\"checks\":%d,\"mismatches\":%d}\n", name, checks, bad);
}

int main() {
    run<BLS381G1>("bls12_381");
    run<BN254G1>("bn254");
    run<Bandersnatch>("bandersnatch");
    return 0;
}
