// Host-side EC op timing (the MSM's final Horner pass runs on the host).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include "../csrc/ec.hpp"
using namespace vk;
int main() {
    using C = BLS381G1;
    C::Acc a = C::zero(), b;
    for (int i = 0; i < C::ACC_WORDS; i++) reinterpret_cast<uint32_t*>(&b)[i] = 0x12345 * (i + 1);
    reinterpret_cast<uint32_t*>(&b)[11] &= 0xfff; reinterpret_cast<uint32_t*>(&b)[23] &= 0xfff;
    reinterpret_cast<uint32_t*>(&b)[35] &= 0xfff; reinterpret_cast<uint32_t*>(&b)[47] &= 0xfff;
    a = b;
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int k = 0; k < 10000; k++) a = C::dbl(a);
    auto t1 = std::chrono::high_resolution_clock::now();
    for (int k = 0; k < 10000; k++) a = C::add(a, b);
    auto t2 = std::chrono::high_resolution_clock::now();
    fe<BLS381Fq> x = b.x, y = b.y;
    for (int k = 0; k < 100000; k++) x = fe_mul<BLS381Fq>(x, y);
    auto t3 = std::chrono::high_resolution_clock::now();
    fe<BLS381Fq> z = x;
    for (int k = 0; k < 2000; k++) z = fe_add<BLS381Fq>(fe_inv_bin<BLS381Fq>(z), y);
    auto t4 = std::chrono::high_resolution_clock::now();
    fe<BN254Fr> zr;
    for (int i = 0; i < 8; i++) zr.v[i] = 0x9876543u * (i + 3);
    zr.v[7] &= 0xfffffff;
    for (int k = 0; k < 2000; k++) zr = fe_add<BN254Fr>(fe_inv_bin<BN254Fr>(zr), zr);
    auto t5 = std::chrono::high_resolution_clock::now();
    printf("inv_bin bls_fq %.2f us, bn254_fr %.2f us (%u %u)\n", std::chrono::duration<double, std::micro>(t4 - t3).count() / 2000,
           std::chrono::duration<double, std::micro>(t5 - t4).count() / 2000, z.v[0], zr.v[0]);
    printf("dbl %.1f ns, add %.1f ns, mul %.1f ns  (%u)\n", std::chrono::duration<double, std::nano>(t1 - t0).count() / 1e4,
           std::chrono::duration<double, std::nano>(t2 - t1).count() / 1e4,
           std::chrono::duration<double, std::nano>(t3 - t2).count() / 1e5, a.x.v[0] ^ x.v[0]);
}
