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
    printf("dbl %.1f ns, add %.1f ns, mul %.1f ns  (%u)\n", std::chrono::duration<double, std::nano>(t1 - t0).count() / 1e4,
           std::chrono::duration<double, std::nano>(t2 - t1).count() / 1e4,
           std::chrono::duration<double, std::nano>(t3 - t2).count() / 1e5, a.x.v[0] ^ x.v[0]);
}
