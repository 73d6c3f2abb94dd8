// A/B of the mixed add in the bucket-accumulate shape: radix 2^29 (ec29.hpp, 14 limbs, the
// shipped k_msm_accumulate) against signed radix 2^30 (ec30.hpp, 13 limbs) for BLS12-381.
// Each thread runs ITERS mixed adds onto one accumulator, the bases gathered at pseudo-random
// rows of a 2^20-point table in HBM (next base loaded before the add, as the accumulate does);
// both kernels start from the same 32-bit Montgomery inputs and their final accumulators are
// compared word for word on the device. Prints JSON lines.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 s30probe.hip -o s30probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "../csrc/ec29.hpp"
#include "../csrc/ec30.hpp"
using namespace vk;
using F = BLS381Fq;
using P29 = F29BLS381Fq;
using P30 = F30BLS381Fq;
using S29 = SW29<BLS381G1, P29>;
using S30 = SW30<BLS381G1, P30>;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ fe<F> rand_fe(uint32_t s) {
    fe<F> a;
    for (int k = 0; k < F::N; k++) a.v[k] = mix(s * 16u + k + 1u);
    a.v[F::N - 1] %= 0x1a0111eau;
    return a;
}

__global__ void k_init(S29::Aff* t29, S30::Aff* t30, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fe<F> x = rand_fe(2 * i), y = rand_fe(2 * i + 1);
    t29[i].x = from_mont32<P29, F>(x);
    t29[i].y = from_mont32<P29, F>(y);
    t30[i].x = from_mont32_30<P30, F>(x);
    t30[i].y = from_mont32_30<P30, F>(y);
}

template <class S, class T>
__global__ void __launch_bounds__(256) k_loop(const T* __restrict__ tab, uint32_t mask, int iters,
                                              fe<F>* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    typename S::Acc acc = S::zero();
    uint32_t idx = mix(t + 0x1234567u);
    typename S::Aff nxt = tab[idx & mask];
    for (int i = 0; i < iters; i++) {
        const typename S::Aff q = nxt;
        idx = mix(idx);
        nxt = tab[idx & mask];
        acc = S::madd(acc, q, (idx >> 31) != 0);
    }
    fe<F> o[4];
    if constexpr (std::is_same<S, S29>::value) {
        o[0] = to_mont32<P29, F>(acc.x); o[1] = to_mont32<P29, F>(acc.y);
        o[2] = to_mont32<P29, F>(acc.zz); o[3] = to_mont32<P29, F>(acc.zzz);
    } else {
        o[0] = to_mont32_30<P30, F>(acc.x); o[1] = to_mont32_30<P30, F>(acc.y);
        o[2] = to_mont32_30<P30, F>(acc.zz); o[3] = to_mont32_30<P30, F>(acc.zzz);
    }
    for (int k = 0; k < 4; k++) out[4 * (size_t)t + k] = o[k];
}

__global__ void k_cmp(const fe<F>* a, const fe<F>* b, size_t n, uint32_t* bad) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < F::N; k++)
        if (a[i].v[k] != b[i].v[k]) {
            atomicAdd(bad, 1u);
            return;
        }
}

template <class S, class T>
static float run(const T* tab, int blocks, int iters, fe<F>* out) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_loop<S, T>), dim3(blocks), dim3(256), 0, 0, tab, (1u << 20) - 1, iters, out);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint32_t n = 1u << 20;
    const int blocks = 2048;
    const size_t threads = (size_t)blocks * 256;
    S29::Aff* t29;
    S30::Aff* t30;
    fe<F>*o29, *o30;
    uint32_t* bad;
    CK(hipMalloc(&t29, n * sizeof(S29::Aff)));
    CK(hipMalloc(&t30, n * sizeof(S30::Aff)));
    CK(hipMalloc(&o29, threads * 4 * sizeof(fe<F>)));
    CK(hipMalloc(&o30, threads * 4 * sizeof(fe<F>)));
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_init, dim3(n / 256), dim3(256), 0, 0, t29, t30, n);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    hipFuncAttributes a29, a30;
    CK(hipFuncGetAttributes(&a29, reinterpret_cast<const void*>(&k_loop<S29, S29::Aff>)));
    CK(hipFuncGetAttributes(&a30, reinterpret_cast<const void*>(&k_loop<S30, S30::Aff>)));
    printf("{\"vgprs29\":%d,\"vgprs30\":%d,\"threads\":%zu,\"iters\":%d}\n", a29.numRegs, a30.numRegs, threads, iters);
    run<S29>(t29, blocks, iters, o29);  // warm-up
    run<S30>(t30, blocks, iters, o30);
    const double madds = (double)threads * iters;
    for (int r = 0; r < reps; r++) {
        const float m29 = run<S29>(t29, blocks, iters, o29);
        const float m30 = run<S30>(t30, blocks, iters, o30);
        printf("{\"rep\":%d,\"ms29\":%.3f,\"ms30\":%.3f,\"Gmadd29\":%.3f,\"Gmadd30\":%.3f,\"ratio\":%.4f}\n", r, m29, m30,
               madds / m29 / 1e6, madds / m30 / 1e6, m30 / m29);
        fflush(stdout);
    }
    hipLaunchKernelGGL(k_cmp, dim3((unsigned)((threads * 4 + 255) / 256)), dim3(256), 0, 0, o29, o30, threads * 4, bad);
    CK(hipGetLastError());
    uint32_t hb = 0;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("{\"compared\":%zu,\"mismatches\":%u}\n", threads * 4, hb);
    return hb != 0;
}
