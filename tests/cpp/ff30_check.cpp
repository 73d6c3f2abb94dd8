// Host check of the signed radix-2^30 field arithmetic (verkle-kzg_amd/csrc/ff30.hpp) and its
// mixed add (ec30.hpp): JSON lines with the integer values of operands and results for
// tests/test_ff30.py (congruences mod p, output bounds, limb states), and the mixed add compared
// word for word with the radix-2^29 one (ec29.hpp, the shipped accumulate's) on the same inputs.
#include <cstdio>
#include <cstdint>
#include "../../verkle-kzg_amd/csrc/ec29.hpp"
#include "../../verkle-kzg_amd/csrc/ec30.hpp"
using namespace vk;
using P = F30BLS381Fq;
using P29 = F29BLS381Fq;
using F = BLS381Fq;

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 16);
}

static void pr(const char* tag, const f30<P>& x) {
    printf("\"%s\":[", tag);
    for (int j = 0; j < P::L; j++) printf("%s%d", j ? "," : "", x.v[j]);
    printf("]");
}

// mode 0: exact limbs, small top; 1: every limb at -2^29 (stress); 2: every limb at 2^29 + 2
// (near stress); the top limb at +-(4 p's top limb)
static f30<P> rand30(int mode) {
    f30<P> x;
    for (int j = 0; j < P::L - 1; j++)
        x.v[j] = mode == 1 ? -(1 << 29) : mode == 2 ? (1 << 29) + 2 : sext30(rnd());
    const int32_t top = P::p(P::L - 1) * 4;
    x.v[P::L - 1] = mode == 1 ? -top : mode == 2 ? top : (int32_t)(rnd() % (2 * top + 1)) - top;
    return x;
}

static fe<F> rand_fe() {  // canonical: below p's top word
    fe<F> a;
    for (int k = 0; k < F::N; k++) a.v[k] = rnd();
    a.v[F::N - 1] %= 0x1a0111eau;
    return a;
}

static bool same(const fe<F>& a, const fe<F>& b) {
    for (int k = 0; k < F::N; k++)
        if (a.v[k] != b.v[k]) return false;
    return true;
}

int main() {
    for (int it = 0; it < 300; it++) {
        const int mode = it < 30 ? 1 : it < 60 ? 2 : 0;
        const f30<P> a = rand30(mode), b = rand30(mode);
        const f30<P> c = rand30(mode == 1 ? 2 : mode), d = rand30(mode == 2 ? 1 : mode);
        const f30<P> r = mul30<P>(a, b);
        printf("{\"op\":\"mul\","); pr("a", a); printf(","); pr("b", b); printf(","); pr("r", r); printf("}\n");
        const f30<P> q = sqr30<P>(a);
        printf("{\"op\":\"mul\","); pr("a", a); printf(","); pr("b", a); printf(","); pr("r", q); printf("}\n");
        const f30<P> m2 = mul2sum30<P>(a, b, c, d);
        printf("{\"op\":\"mul2\","); pr("a", a); printf(","); pr("b", b); printf(","); pr("c", c); printf(",");
        pr("d", d); printf(","); pr("r", m2); printf("}\n");
        const f30<P> s = add30<P>(a, b), t = sub30<P>(a, c);
        printf("{\"op\":\"add\","); pr("a", a); printf(","); pr("b", b); printf(","); pr("r", s); printf("}\n");
        printf("{\"op\":\"sub\","); pr("a", a); printf(","); pr("b", c); printf(","); pr("r", t); printf("}\n");
        uint32_t u[P::L];
        canon30<P>(r, u);
        printf("{\"op\":\"canon\","); pr("a", r); printf(",\"r\":[");
        for (int j = 0; j < P::L; j++) printf("%s%u", j ? "," : "", u[j]);
        printf("]}\n");
        // 32-bit Montgomery form (x R) -> x R' -> back
        const fe<F> m = rand_fe();
        const f30<P> x30 = from_mont32_30<P, F>(m);
        const fe<F> back = to_mont32_30<P, F>(x30);
        printf("{\"op\":\"mont\",\"a\":[");
        for (int k = 0; k < F::N; k++) printf("%s%u", k ? "," : "", m.v[k]);
        printf("],"); pr("r", x30); printf(",\"back\":[");
        for (int k = 0; k < F::N; k++) printf("%s%u", k ? "," : "", back.v[k]);
        printf("],\"zero_mo\":%d,\"rzero\":%d}\n", is_zero_mo30<P>(r) ? 1 : 0, 0);
    }
    // mixed adds: chains of 64 over random field elements, radix 2^30 against radix 2^29, plus
    // the doubling (q = acc) and cancelling (q = -acc) cases; compared in the 32-bit form
    using S29 = SW29<BLS381G1, P29>;
    using S30 = SW30<BLS381G1, P>;
    int bad = 0, checked = 0;
    for (int chain = 0; chain < 40; chain++) {
        fe<F> w[4];
        for (auto& x : w) x = rand_fe();
        S29::Acc a29;
        S30::Acc a30;
        a29.x = from_mont32<P29, F>(w[0]); a29.y = from_mont32<P29, F>(w[1]);
        a29.zz = from_mont32<P29, F>(w[2]); a29.zzz = from_mont32<P29, F>(w[3]);
        a30.x = from_mont32_30<P, F>(w[0]); a30.y = from_mont32_30<P, F>(w[1]);
        a30.zz = from_mont32_30<P, F>(w[2]); a30.zzz = from_mont32_30<P, F>(w[3]);
        a29.inf = a30.inf = chain == 0;
        for (int step = 0; step < 64; step++) {
            const fe<F> qx = rand_fe(), qy = rand_fe();
            S29::Aff q29{from_mont32<P29, F>(qx), from_mont32<P29, F>(qy)};
            S30::Aff q30{from_mont32_30<P, F>(qx), from_mont32_30<P, F>(qy)};
            const bool neg = (step & 3) == 1;
            if (chain >= 36 && step == 63) {  // q = (acc x / zz, acc y / zzz) via a fresh affine acc
                a29.x = q29.x; a29.y = neg ? neg29<P29, 2>(q29.y) : q29.y; a29.zz = a29.zzz = one29<P29>();
                a30.x = q30.x; a30.y = neg ? neg30<P>(q30.y) : q30.y; a30.zz = a30.zzz = one30<P>();
                if (chain >= 38) {  // cancelling: acc = -q
                    a29.y = neg29<P29, 2>(a29.y);
                    a30.y = neg30<P>(a30.y);
                }
            }
            a29 = S29::madd(a29, q29, neg);
            a30 = S30::madd(a30, q30, neg);
            checked++;
            if (a29.inf != a30.inf) {
                bad++;
                continue;
            }
            if (a29.inf) continue;
            const fe<F> o29[4] = {to_mont32<P29, F>(a29.x), to_mont32<P29, F>(a29.y), to_mont32<P29, F>(a29.zz),
                                  to_mont32<P29, F>(a29.zzz)};
            const fe<F> o30[4] = {to_mont32_30<P, F>(a30.x), to_mont32_30<P, F>(a30.y), to_mont32_30<P, F>(a30.zz),
                                  to_mont32_30<P, F>(a30.zzz)};
            for (int k = 0; k < 4; k++)
                if (!same(o29[k], o30[k])) bad++;
        }
        printf("{\"op\":\"madd_chain\",\"chain\":%d,\"inf\":%d}\n", chain, a30.inf ? 1 : 0);
    }
    printf("{\"op\":\"madd\",\"checked\":%d,\"bad\":%d}\n", checked, bad);
    // general adds (the fix-up / tail), doublings, equal and opposite operands, and the table
    // path: pack_aff -> load -> an affine accumulator -> store
    auto acc_pair = [&](S29::Acc& a29, S30::Acc& a30) {
        fe<F> w[4];
        for (auto& x : w) x = rand_fe();
        a29.x = from_mont32<P29, F>(w[0]); a29.y = from_mont32<P29, F>(w[1]);
        a29.zz = from_mont32<P29, F>(w[2]); a29.zzz = from_mont32<P29, F>(w[3]);
        a30.x = from_mont32_30<P, F>(w[0]); a30.y = from_mont32_30<P, F>(w[1]);
        a30.zz = from_mont32_30<P, F>(w[2]); a30.zzz = from_mont32_30<P, F>(w[3]);
        a29.inf = a30.inf = false;
    };
    auto differ = [&](const S29::Acc& a29, const S30::Acc& a30) {
        const BLS381G1::Acc o29 = S29::store(a29), o30 = S30::store(a30);
        if (a29.inf != a30.inf) return 1;
        return (!same(o29.x, o30.x) || !same(o29.y, o30.y) || !same(o29.zz, o30.zz) || !same(o29.zzz, o30.zzz)) ? 1 : 0;
    };
    int abad = 0, achecked = 0;
    for (int chain = 0; chain < 24; chain++) {
        S29::Acc a29, b29;
        S30::Acc a30, b30;
        acc_pair(a29, a30);
        for (int step = 0; step < 32; step++) {
            acc_pair(b29, b30);
            if (step == 31 && chain >= 20) {  // equal operands (doubling) / opposite (infinity)
                b29 = a29;
                b30 = a30;
                if (chain >= 22) {
                    b29.y = neg29<P29, 2>(b29.y);
                    b30.y = neg30<P>(b30.y);
                }
            }
            if (step % 8 == 7) {
                a29 = S29::dbl(a29);
                a30 = S30::dbl(a30);
                achecked++;
                abad += differ(a29, a30);
            }
            a29 = S29::add(a29, b29);
            a30 = S30::add(a30, b30);
            achecked++;
            abad += differ(a29, a30);
        }
    }
    int tbad = 0;
    for (int i = 0; i < 64; i++) {
        BLS381G1::Aff a, p29, p30;
        a.x = rand_fe();
        a.y = rand_fe();
        S29::pack_aff(a, &p29);
        S30::pack_aff(a, &p30);
        const S29::Aff l29 = S29::load(&p29);
        const S30::Aff l30 = S30::load(&p30);
        S29::Acc z29 = S29::zero();
        S30::Acc z30 = S30::zero();
        z29 = S29::madd(z29, l29, i & 1);
        z30 = S30::madd(z30, l30, i & 1);
        tbad += differ(z29, z30);
    }
    printf("{\"op\":\"add\",\"checked\":%d,\"bad\":%d,\"table_bad\":%d}\n", achecked, abad, tbad);
    return 0;
}
