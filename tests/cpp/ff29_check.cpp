// Host check of the radix-2^29 field arithmetic (verkle-kzg_amd/csrc/ff29.hpp): prints one JSON
// line per operation with the integer values of the operands and the result; the Python side
// (tests/test_ff29.py) checks congruences mod p and the bounds the kernels rely on.
#include <cstdio>
#include <cstdint>
#include "../../verkle-kzg_amd/csrc/ff29.hpp"
using namespace vk;

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 16);
}

template <class P>
static void pr(const char* tag, const f29<P>& x) {
    printf("\"%s\":[", tag);
    for (int j = 0; j < P::L; j++) printf("%s%u", j ? "," : "", x.v[j]);
    printf("]");
}

// random element: mode 0 canonical-ish (< 2^(bits of p) limb-normalised), 1 max-limb stress
template <class P>
static f29<P> rand29(int mode) {
    f29<P> x;
    for (int j = 0; j < P::L; j++) x.v[j] = mode == 1 ? (M29 + 8) : (rnd() & M29);
    x.v[P::L - 1] = mode == 1 ? (P::p(P::L - 1) * 4) : (rnd() % (P::p(P::L - 1) + 1));
    return x;
}

template <class P, class F>
static void run(const char* name) {
    for (int it = 0; it < 200; it++) {
        const int mode = it < 20 ? 1 : 0;
        f29<P> a = rand29<P>(mode), b = rand29<P>(mode);
        f29<P> r = mul29<P>(a, b);
        printf("{\"f\":\"%s\",\"op\":\"mul\",", name); pr("a", a); printf(","); pr("b", b); printf(","); pr("r", r); printf("}\n");
        f29<P> q = sqr29<P>(a);
        printf("{\"f\":\"%s\",\"op\":\"mul\",", name); pr("a", a); printf(","); pr("b", a); printf(","); pr("r", q); printf("}\n");
        // products of carry-less sums (add29_raw): one raw operand at every L, two at L <= 9 (the
        // Edwards mixed add's (X + Y)(x + y)); stress operands put every limb at 2^30 + 14
        {
            const f29<P> ra = add29_raw<P>(a, b), rb = add29_raw<P>(b, a);
            const f29<P> r1 = mul29<P>(ra, b);
            printf("{\"f\":\"%s\",\"op\":\"mul\",", name); pr("a", ra); printf(","); pr("b", b); printf(","); pr("r", r1); printf("}\n");
            if constexpr (P::L <= 9) {
                const f29<P> r2 = mul29<P>(ra, rb);
                printf("{\"f\":\"%s\",\"op\":\"mul\",", name); pr("a", ra); printf(","); pr("b", rb); printf(","); pr("r", r2); printf("}\n");
            }
        }
        f29<P> s = add29<P>(a, b);
        printf("{\"f\":\"%s\",\"op\":\"add\",", name); pr("a", a); printf(","); pr("b", b); printf(","); pr("r", s); printf("}\n");
        // subtrahend below p (a mul output): sub2 / sub4 / sub16
        f29<P> c = mul29<P>(b, b);
        f29<P> c2 = add29<P>(c, c);
        f29<P> d2 = sub29<P, 4>(a, c), d16 = sub29<P, 16>(r, c2);
        printf("{\"f\":\"%s\",\"op\":\"sub4\",", name); pr("a", a); printf(","); pr("b", c); printf(","); pr("r", d2); printf("}\n");
        printf("{\"f\":\"%s\",\"op\":\"sub16\",", name); pr("a", r); printf(","); pr("b", c2); printf(","); pr("r", d16); printf("}\n");
        // lazy sum of products (mul2sum29), as in the Y3 formulas (d = 4p - a product output),
        // and with four max-limb operands (column bound)
        f29<P> nc = neg29<P, 4>(c);
        f29<P> m2 = mul2sum29<P>(a, b, r, nc), m3 = mul2sum29<P>(a, b, b, a);
        printf("{\"f\":\"%s\",\"op\":\"mul2\",", name); pr("a", a); printf(","); pr("b", b); printf(",");
        pr("c", r); printf(","); pr("d", nc); printf(","); pr("r", m2); printf("}\n");
        printf("{\"f\":\"%s\",\"op\":\"mul2\",", name); pr("a", a); printf(","); pr("b", b); printf(",");
        pr("c", b); printf(","); pr("d", a); printf(","); pr("r", m3); printf("}\n");
        f29<P> cn = canon29<P>(r);
        printf("{\"f\":\"%s\",\"op\":\"canon\",", name); pr("a", r); printf(","); pr("r", cn); printf("}\n");
        uint32_t w[P::N];
        pack29<P>(cn, w);
        f29<P> u = unpack29<P>(w);
        printf("{\"f\":\"%s\",\"op\":\"unpack\",", name); pr("a", cn); printf(","); pr("r", u); printf("}\n");
        // 32-bit Montgomery (x R) -> x R' and back
        fe<F> m;
        for (int k = 0; k < P::N; k++) m.v[k] = w[k];  // canonical value < p
        f29<P> x29 = from_mont32<P, F>(m);
        fe<F> back = to_mont32<P, F>(x29);
        printf("{\"f\":\"%s\",\"op\":\"mont\",", name); pr("a", cn); printf(","); pr("r", x29);
        printf(",\"back\":[");
        for (int k = 0; k < P::N; k++) printf("%s%u", k ? "," : "", back.v[k]);
        printf("],\"zero_mo\":%d}\n", is_zero_mo29<P>(r) ? 1 : 0);
    }
}

int main() {
    run<F29BLS381Fq, BLS381Fq>("bls12_381_fq");
    run<F29BN254Fq, BN254Fq>("bn254_fq");
    run<F29BLS381Fr, BLS381Fr>("bls12_381_fr");
    return 0;
}
