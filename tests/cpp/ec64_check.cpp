// Host check of the 64-bit-limb XYZZ arithmetic (verkle-kzg_amd/csrc/host/ec64.hpp) used by the
// MSM's host Horner pass, against the ec.hpp formulas: random doubling / add chains and the
// exceptional cases (p + p, p + (-p), identity operands), compared word for word (same
// formulas, same canonical Montgomery form). Prints one JSON line per curve.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../verkle-kzg_amd/csrc/host/ec64.hpp"
using namespace vk;

static uint64_t rs = 0x6A09E667F3BCC909ull;
static uint64_t rnd64() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}

template <class C>
static bool same(const typename C::Acc& a, const h64::Acc<typename C::F>& b) {
    const typename C::Acc bb = h64::to<C>(b);
    return memcmp(&a, &bb, sizeof a) == 0;
}

// a random canonical field element in Montgomery form (x R mod p from a random x < p)
template <class F>
static fe<F> rnd_fe() {
    fe<F> x;
    for (int k = 0; k < F::N; k++) x.v[k] = (uint32_t)rnd64();
    x.v[F::N - 1] &= (F::p(F::N - 1) >> 1);  // below p
    return fe_to_mont<F>(x);
}

template <class C>
static void run(const char* name) {
    using F = typename C::F;
    int checks = 0, bad = 0;
    for (int chain = 0; chain < 8; chain++) {
        // arbitrary XYZZ tuples exercise the field formulas; the group law is checked by the
        // GPU MSM tests end to end
        typename C::Acc a, b;
        a.x = rnd_fe<F>(); a.y = rnd_fe<F>(); a.zz = rnd_fe<F>(); a.zzz = rnd_fe<F>();
        b.x = rnd_fe<F>(); b.y = rnd_fe<F>(); b.zz = rnd_fe<F>(); b.zzz = rnd_fe<F>();
        h64::Acc<F> ha = h64::from<C>(a), hb = h64::from<C>(b);
        for (int step = 0; step < 40; step++) {
            if (rnd64() & 1) {
                a = C::dbl(a);
                ha = h64::dbl<F>(ha);
            } else {
                a = C::add(a, b);
                ha = h64::add_pt<F>(ha, hb);
            }
            checks++;
            bad += !same<C>(a, ha);
        }
        // exceptional cases: p + p (doubling), p + (-p) (identity), identity operands
        typename C::Acc na = C::neg(a);
        h64::Acc<F> hna = h64::from<C>(na);
        checks += 5;
        bad += !same<C>(C::add(a, a), h64::add_pt<F>(ha, ha));
        bad += !same<C>(C::add(a, na), h64::add_pt<F>(ha, hna));
        bad += !same<C>(C::add(C::zero(), a), h64::add_pt<F>(h64::zero<F>(), ha));
        bad += !same<C>(C::add(a, C::zero()), h64::add_pt<F>(ha, h64::zero<F>()));
        bad += !same<C>(C::dbl(C::zero()), h64::dbl<F>(h64::zero<F>()));
    }
    printf("{\"curve\":\"%s\",\"checks\":%d,\"mismatches\":%d}\n", name, checks, bad);
}

int main() {
    run<BLS381G1>("bls12_381");
    run<BN254G1>("bn254");
    return 0;
}
