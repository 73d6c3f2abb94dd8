// Host check of the divstep field inversion (verkle-kzg_amd/csrc/ff.hpp fe_inv_host, used by
// fe_inv_bin on the host) against Fermat's a^(p-2) (fe_inv) on every field of the library:
// random Montgomery values, the edges 1, 2, p - 1, p - 2 and values with long runs of zero /
// one bits, and a * a^-1 == 1. Prints one JSON line per field: checks, mismatches, and the mean
// time per inversion (us) of the divstep and Fermat versions.
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../verkle-kzg_amd/csrc/ff.hpp"
using namespace vk;

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd64() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}

template <class F>
static fe<F> reduce(fe<F> a) {  // into [0, p) by repeated subtraction (inputs < 2^(32N))
    for (int k = 0; k < 64; k++) {
        fe<F> p;
        for (int i = 0; i < F::N; i++) p.v[i] = F::p(i);
        if (!fe_geq_raw<F>(a, p)) break;
        fe_sub_raw<F>(a, p);
    }
    return a;
}

template <class F>
static void run(const char* name) {
    std::vector<fe<F>> xs;
    auto from_u64 = [](uint64_t x) {
        fe<F> a = fe_zero<F>();
        a.v[0] = (uint32_t)x;
        a.v[1] = (uint32_t)(x >> 32);
        return a;
    };
    fe<F> pm1, pm2;
    for (int i = 0; i < F::N; i++) pm1.v[i] = pm2.v[i] = F::p(i);
    pm1.v[0] -= 1;
    pm2.v[0] -= 2;
    xs.push_back(from_u64(1));
    xs.push_back(from_u64(2));
    xs.push_back(from_u64(3));
    xs.push_back(pm1);
    xs.push_back(pm2);
    for (int k = 0; k < 32 * F::N; k += 7) {  // single bits, and runs of ones below them
        fe<F> a = fe_zero<F>(), b = fe_zero<F>();
        a.v[k / 32] = 1u << (k % 32);
        for (int j = 0; j <= k; j++) b.v[j / 32] |= 1u << (j % 32);
        xs.push_back(reduce<F>(a));
        xs.push_back(reduce<F>(b));
    }
    for (int k = 0; k < 2000; k++) {
        fe<F> a;
        for (int i = 0; i < F::N; i += 2) {
            const uint64_t r = rnd64();
            a.v[i] = (uint32_t)r;
            a.v[i + 1] = (uint32_t)(r >> 32);
        }
        a.v[F::N - 1] &= 0x7fffffffu;
        a = reduce<F>(a);
        if (!fe_is_zero<F>(a)) xs.push_back(a);
    }
    int mism = 0;
    const fe<F> one = fe_one<F>();
    for (const auto& a : xs) {
        if (fe_is_zero<F>(a)) continue;
        const fe<F> x = fe_inv_bin<F>(a), y = fe_inv<F>(a);
        if (!fe_eq<F>(x, y) || !fe_eq<F>(fe_mul<F>(a, x), one)) mism++;
    }
    const int T = 400;
    auto t0 = std::chrono::steady_clock::now();
    fe<F> acc = xs[7];
    for (int k = 0; k < T; k++) {
        acc = fe_inv_bin<F>(acc);
        acc.v[0] ^= (uint32_t)k | 1u;
        acc = reduce<F>(acc);
        if (fe_is_zero<F>(acc)) acc = one;
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int k = 0; k < T / 8; k++) {
        acc = fe_inv<F>(acc);
        acc.v[0] ^= (uint32_t)k | 1u;
        acc = reduce<F>(acc);
        if (fe_is_zero<F>(acc)) acc = one;
    }
    auto t2 = std::chrono::steady_clock::now();
    printf("{\"field\": \"%s\", \"checks\": %zu, \"mismatches\": %d, \"divstep_us\": %.2f, \"fermat_us\": %.2f, \"x\": %u}\n",
           name, xs.size(), mism, std::chrono::duration<double, std::micro>(t1 - t0).count() / T,
           std::chrono::duration<double, std::micro>(t2 - t1).count() / (T / 8), acc.v[0] & 1u);
}

int main() {
    run<BN254Fq>("bn254_fq");
    run<BN254Fr>("bn254_fr");
    run<BLS381Fq>("bls12_381_fq");
    run<BLS381Fr>("bls12_381_fr");
    run<BandFr>("bandersnatch_fr");
    return 0;
}
