// Latency vs throughput of the asm field multiply on gfx950: a single wave's dependent chain
// (cycles per multiply) and two independent chains issued as two asm blocks, at one wave on
// the chip and at 1-2 waves per SIMD. Prints JSON lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../csrc/ec.hpp"
#include "../csrc/ff29.hpp"
using namespace vk;

template <class F>
__device__ void seed_fe(fe<F>& a, uint32_t s) {
    for (int i = 0; i < F::N; i++) a.v[i] = s * 2654435761u + i * 40503u;
    a.v[F::N - 1] &= 0xffffu;
}

template <class P>
__device__ void seed29(f29<P>& a, uint32_t s) {
    for (int i = 0; i < P::L; i++) a.v[i] = (s * 2654435761u + i * 40503u) & 0x1fffffffu;
    a.v[P::L - 1] &= 0x7u;
}
template <class P>
__global__ void k_chain29(uint32_t* out, long long* cyc, int iters) {
    f29<P> x, y;
    seed29(x, threadIdx.x + 1);
    seed29(y, blockIdx.x + 7);
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) x = mul29<P>(x, y);
    long long t1 = clock64();
    uint32_t acc = 0;
    for (int i = 0; i < P::L; i++) acc ^= x.v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
template <class P>
void run29(const char* name, int blocks, int threads, int iters) {
    uint32_t* out;
    long long* cyc;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    (void)hipMalloc(&cyc, 8);
    k_chain29<P><<<blocks, threads>>>(out, cyc, 4);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_chain29<P><<<blocks, threads>>>(out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"probe\":\"%s\",\"blocks\":%d,\"cycles_per_mul\":%.1f,\"ms\":%.3f,\"Gmul_per_s\":%.2f}\n", name, blocks,
           (double)c / iters, ms, (double)iters * blocks * threads / ms / 1e6);
}

// mode 0: one chain; 1: two chains, separate asm blocks
template <class F, int MODE>
__global__ void k_chain(uint32_t* out, long long* cyc, int iters) {
    fe<F> x, y, z, w;
    seed_fe(x, threadIdx.x + 1);
    seed_fe(y, blockIdx.x + 7);
    seed_fe(z, threadIdx.x + 99);
    seed_fe(w, blockIdx.x + 13);
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        if constexpr (MODE == 0) {
            x = fe_mul<F>(x, y);
        } else if constexpr (MODE == 1) {
            x = fe_mul<F>(x, y);
            z = fe_mul<F>(z, w);
        }
    }
    long long t1 = clock64();
    uint32_t acc = 0;
    for (int i = 0; i < F::N; i++) acc ^= x.v[i] ^ z.v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <class F, int MODE>
void run(const char* name, int blocks, int threads, int iters) {
    uint32_t* out;
    long long* cyc;
    hipMalloc(&out, (size_t)blocks * threads * 4);
    hipMalloc(&cyc, 8);
    k_chain<F, MODE><<<blocks, threads>>>(out, cyc, 4);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_chain<F, MODE><<<blocks, threads>>>(out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double muls = (double)iters * (MODE == 0 ? 1 : 2);
    printf("{\"probe\":\"%s\",\"blocks\":%d,\"threads\":%d,\"cycles_per_mul\":%.1f,\"ms\":%.3f,\"Gmul_per_s\":%.2f}\n",
           name, blocks, threads, c / muls, ms, muls * blocks * threads / ms / 1e6);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    // latency: one wave on the whole chip
    run<BLS381Fq, 0>("fq12 single chain, 1 wave", 1, 64, 2000);
    run<BLS381Fq, 1>("fq12 two chains (2 asm blocks), 1 wave", 1, 64, 1000);
    run<BLS381Fr, 0>("fr8 single chain, 1 wave", 1, 64, 2000);
    run<BLS381Fr, 1>("fr8 two chains (2 asm blocks), 1 wave", 1, 64, 1000);
    run29<Q29>("q29 (14x29-bit) single chain, 1 wave", 1, 64, 2000);
    run29<R29>("r29 (9x29-bit) single chain, 1 wave", 1, 64, 2000);
    for (int wps = 1; wps <= 4; wps *= 2) {
        run29<Q29>("q29 full chip", 256 * wps, 256, 2000);
        run29<R29>("r29 full chip", 256 * wps, 256, 2000);
    }
    // throughput: 1 and 2 waves per SIMD over 256 CUs
    for (int wps = 1; wps <= 2; wps++) {
        run<BLS381Fq, 0>("fq12 single chain, full chip", 256 * wps, 256, 2000);
        run<BLS381Fq, 1>("fq12 two chains (2 asm blocks), full chip", 256 * wps, 256, 1000);
    }
    return 0;
}
