// Latency of one XYZZ full add (SW29::add, one lane per add) against the 4-lane cooperative add
// (SW29::add_quad) in a dependent chain, BLS12-381 G1 radix-2^29, at one wave on the chip and at
// one wave per SIMD (the occupancy of the MSM tail kernels). Prints JSON lines: cycles per add
// (clock64 of wave 0) and ms per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../csrc/ec29.hpp"
using namespace vk;
using A = Fast29<BLS381G1>::type;
using Acc = A::Acc;

__device__ void seed_acc(Acc& a, uint32_t s) {
    using P = decltype(a.x);
    auto fill = [&](P& f, uint32_t k) {
        for (int i = 0; i < (int)(sizeof(f.v) / 4); i++) f.v[i] = ((s + k) * 2654435761u + i * 40503u) & 0x1fffffffu;
        f.v[sizeof(f.v) / 4 - 1] &= 0x7u;
    };
    fill(a.x, 1);
    fill(a.y, 2);
    fill(a.zz, 3);
    fill(a.zzz, 4);
    a.inf = false;
}

template <int MODE>  // 0: full add per lane, 1: quad add (4 lanes per add)
__global__ void __launch_bounds__(64) k_chain(uint32_t* out, long long* cyc, int iters) {
    Acc v, w;
    const uint32_t lane = threadIdx.x, g = MODE == 1 ? lane >> 2 : lane;
    seed_acc(v, g + 17 * blockIdx.x);
    seed_acc(w, g + 1000 + 17 * blockIdx.x);
    const long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        if constexpr (MODE == 0) v = A::add(v, w);
        else v = A::add_quad(v, w, lane & 3);
    }
    const long long t1 = clock64();
    uint32_t acc = 0;
    for (int i = 0; i < (int)(sizeof(v.x.v) / 4); i++) acc ^= v.x.v[i] ^ v.zzz.v[i];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE>
void run(const char* name, int blocks, int iters) {
    uint32_t* out;
    long long* cyc;
    (void)hipMalloc(&out, (size_t)blocks * 64 * 4);
    (void)hipMalloc(&cyc, 8);
    k_chain<MODE><<<blocks, 64>>>(out, cyc, 2);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_chain<MODE><<<blocks, 64>>>(out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"%s\", \"waves\": %d, \"iters\": %d, \"cycles_per_add\": %.0f, \"us_per_add\": %.2f}\n", name,
           blocks, iters, (double)c / iters, ms * 1000.0 / iters);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    for (int blocks : {1, 1024}) {
        run<0>("full_add", blocks, 64);
        run<1>("quad_add", blocks, 64);
    }
    return 0;
}
