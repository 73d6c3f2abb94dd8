// Host EC / field operation timings (the MSM's host fold and affine step, the IPA rounds' partial
// sums): BLS12-381 Fq and BN254 Fq multiply, BLS12-381 / BN254 XYZZ add and doubling, field
// inversion. Build flags are the A/B (e.g. with and without -mbmi2 -madx):
//   hipcc -O3 -std=c++17 -x hip --offload-arch=gfx950 [-Xarch_host -mbmi2 -Xarch_host -madx] hostops.cpp
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include "../csrc/ec.hpp"
using namespace vk;

template <class C>
static void run(const char* name, const uint32_t* gx, const uint32_t* gy) {
    using F = typename C::F;
    using Acc = typename C::Acc;
    fe<F> x, y;
    for (int i = 0; i < F::N; i++) {
        x.v[i] = gx[i];
        y.v[i] = gy[i];
    }
    Acc g = C::zero();
    g.x = fe_to_mont<F>(x);
    g.y = fe_to_mont<F>(y);
    g.zz = fe_one<F>();
    g.zzz = fe_one<F>();
    Acc a = C::dbl(g);
    double b_mul = 1e9, b_add = 1e9, b_dbl = 1e9, b_inv = 1e9;
    for (int rep = 0; rep < 7; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        fe<F> m = a.x;
        for (int i = 0; i < 200000; i++) m = fe_mul<F>(m, a.y);
        auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < 5000; i++) a = C::add(a, g);
        auto t2 = std::chrono::steady_clock::now();
        for (int i = 0; i < 5000; i++) a = C::dbl(a);
        auto t3 = std::chrono::steady_clock::now();
        fe<F> v = a.x;
        for (int i = 0; i < 1000; i++) {
            v = fe_inv_bin<F>(v);
            v.v[0] ^= 2;
        }
        auto t4 = std::chrono::steady_clock::now();
        b_mul = std::min(b_mul, std::chrono::duration<double, std::nano>(t1 - t0).count() / 200000);
        b_add = std::min(b_add, std::chrono::duration<double, std::nano>(t2 - t1).count() / 5000);
        b_dbl = std::min(b_dbl, std::chrono::duration<double, std::nano>(t3 - t2).count() / 5000);
        b_inv = std::min(b_inv, std::chrono::duration<double, std::nano>(t4 - t3).count() / 1000);
        if (m.v[0] == 7 && v.v[1] == 9) printf(" ");
    }
    printf("%s: mul %.1f ns, add %.0f ns, dbl %.0f ns, inv %.0f ns\n", name, b_mul, b_add, b_dbl, b_inv);
}

int main() {
    const uint32_t bx[] = {0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu, 0x171bac58u, 0xa14e3a3fu,
                           0x9774b905u, 0xc3688c4fu, 0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u};
    const uint32_t by[] = {0x46c5e7e1u, 0x0caa2329u, 0xa2888ae4u, 0xd03cc744u, 0x2c04b3edu, 0x00db18cbu,
                           0xd5d00af6u, 0xfcf5e095u, 0x741d8ae4u, 0xa09e30edu, 0xe3aaa0f1u, 0x08b3f481u};
    const uint32_t nx[] = {1, 0, 0, 0, 0, 0, 0, 0}, ny[] = {2, 0, 0, 0, 0, 0, 0, 0};
    run<BLS381G1>("bls12_381", bx, by);
    run<BN254G1>("bn254", nx, ny);
    return 0;
}
