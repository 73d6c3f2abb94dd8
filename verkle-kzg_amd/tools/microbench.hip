// Field-multiply and v_mad_u64_u32 throughput microbenchmark (gfx950). Prints JSON lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../csrc/ec.hpp"
using namespace vk;

__global__ void k_mad(uint32_t* out, uint32_t seed, int iters) {
    uint32_t x = seed + threadIdx.x, y = seed * 3 + blockIdx.x;
    uint64_t a0 = x, a1 = y, a2 = x ^ y, a3 = x + y, a4 = 5, a5 = 7, a6 = 9, a7 = 11;
    for (int i = 0; i < iters; i++) {
#define M(a) a = (uint64_t)(uint32_t)a * x + (a >> 32);
        M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

__global__ void k_fma64(uint32_t* out, uint32_t seed, int iters) {
    double x = 1.0 + threadIdx.x * 1e-9, y = 1e-3 * seed;
    double a0 = x, a1 = y, a2 = x * y, a3 = x + y, a4 = 5, a5 = 7, a6 = 9, a7 = 11;
    for (int i = 0; i < iters; i++) {
#define F(a) a = __builtin_fma(a, x, y);
        F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ void k_mul24(uint32_t* out, uint32_t seed, int iters) {
    uint32_t x = (seed + threadIdx.x) & 0xffffff, y = seed * 3 + blockIdx.x;
    uint32_t a0 = x, a1 = y, a2 = x ^ y, a3 = x + y, a4 = 5, a5 = 7, a6 = 9, a7 = 11;
    for (int i = 0; i < iters; i++) {
#define U(a) a = __umul24(a, x) + y;
        U(a0) U(a1) U(a2) U(a3) U(a4) U(a5) U(a6) U(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed, int iters) {
    uint32_t x = seed + threadIdx.x, y = seed * 3 + blockIdx.x;
    uint32_t a0 = x, a1 = y, a2 = x ^ y, a3 = x + y, a4 = 5, a5 = 7, a6 = 9, a7 = 11;
    for (int i = 0; i < iters; i++) {
#define L(a) a = a * x + y;
        L(a0) L(a1) L(a2) L(a3) L(a4) L(a5) L(a6) L(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <class F>
__global__ void k_fmul(uint32_t* out, uint32_t seed, int iters) {
    fe<F> a, b, c, d;
    for (int i = 0; i < F::N; i++) {
        a.v[i] = seed * (i + 1) + threadIdx.x;
        b.v[i] = seed ^ (i * 77);
        c.v[i] = i + blockIdx.x;
        d.v[i] = seed + i;
    }
    a.v[F::N - 1] &= 0xfffff; b.v[F::N - 1] &= 0xfffff; c.v[F::N - 1] &= 0xfffff; d.v[F::N - 1] &= 0xfffff;
    for (int i = 0; i < iters; i++) {
        a = fe_mul<F>(a, b);
        c = fe_mul<F>(c, d);
        b = fe_mul<F>(b, c);
        d = fe_mul<F>(d, a);
    }
    uint32_t r = 0;
    for (int i = 0; i < F::N; i++) r ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// EC mixed-add chain with the operand in registers (no memory): compute ceiling of the
// accumulate / fixed-base commit inner loops
template <class C>
__global__ void k_madd(uint32_t* out, uint32_t seed, int iters) {
    typename C::Aff P;
    uint32_t* pw = reinterpret_cast<uint32_t*>(&P);
    for (int k = 0; k < (int)(sizeof(P) / 4); k++) pw[k] = (seed * 2654435761u + k * 77 + threadIdx.x) & 0x0fffffff;
    typename C::Acc acc = C::from_aff(P, false);
    for (int i = 0; i < iters; i++) {
        acc = C::madd(acc, P, (i & 1) != 0);
        pw[0] ^= i;
    }
    const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
    uint32_t r = 0;
    for (int k = 0; k < C::ACC_WORDS; k++) r ^= aw[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <class K>
static double timeit(K kern, int blocks, int iters, uint32_t* out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* out;
    int blocks = 256 * 16;
    hipMalloc(&out, blocks * 256 * 4);
    double ms = timeit(k_mad, blocks, 4096, out);
    double mads = (double)blocks * 256 * 4096 * 8;
    printf("{\"bench\":\"v_mad_u64_u32\",\"ms\":%.3f,\"Gop_per_s\":%.1f}\n", ms, mads / ms / 1e6);
    ms = timeit(k_fma64, blocks, 4096, out);
    printf("{\"bench\":\"v_fma_f64\",\"ms\":%.3f,\"Gop_per_s\":%.1f}\n", ms, mads / ms / 1e6);
    ms = timeit(k_mul24, blocks, 4096, out);
    printf("{\"bench\":\"v_mad_u32_u24\",\"ms\":%.3f,\"Gop_per_s\":%.1f}\n", ms, mads / ms / 1e6);
    ms = timeit(k_mullo, blocks, 4096, out);
    printf("{\"bench\":\"v_mad_u32 (mul_lo+add)\",\"ms\":%.3f,\"Gop_per_s\":%.1f}\n", ms, mads / ms / 1e6);
    ms = timeit(k_fmul<BLS381Fq>, blocks, 256, out);
    double muls = (double)blocks * 256 * 256 * 4;
    printf("{\"bench\":\"fe_mul_bls381_fq_12limb\",\"ms\":%.3f,\"Gmul_per_s\":%.2f}\n", ms, muls / ms / 1e6);
    ms = timeit(k_fmul<BLS381Fr>, blocks, 256, out);
    printf("{\"bench\":\"fe_mul_bls381_fr_8limb\",\"ms\":%.3f,\"Gmul_per_s\":%.2f}\n", ms, muls / ms / 1e6);
    ms = timeit(k_fmul<BN254Fq>, blocks, 256, out);
    printf("{\"bench\":\"fe_mul_bn254_fq_8limb\",\"ms\":%.3f,\"Gmul_per_s\":%.2f}\n", ms, muls / ms / 1e6);
    // occupancy sweep of the 12-limb multiply: 1 / 2 waves per SIMD (256 / 512 blocks of 256)
    for (int bl : {256, 512, 1024}) {
        double t = timeit(k_fmul<BLS381Fq>, bl, 1024, out);
        double m = (double)bl * 256 * 1024 * 4;
        printf("{\"bench\":\"fe_mul_bls381_fq_blocks_%d\",\"ms\":%.3f,\"Gmul_per_s\":%.2f,\"us_per_mul_per_wave\":%.3f}\n",
               bl, t, m / t / 1e6, t * 1e3 / (1024.0 * 4));
    }
    ms = timeit(k_madd<BLS381G1>, blocks, 64, out);
    double madds = (double)blocks * 256 * 64;
    printf("{\"bench\":\"madd_bls381_xyzz_chain\",\"ms\":%.3f,\"Gmadd_per_s\":%.2f}\n", ms, madds / ms / 1e6);
    ms = timeit(k_madd<Bandersnatch>, blocks, 64, out);
    printf("{\"bench\":\"madd_bandersnatch_ext_chain\",\"ms\":%.3f,\"Gmadd_per_s\":%.2f}\n", ms, madds / ms / 1e6);
    ms = timeit(k_madd<BN254G1>, blocks, 64, out);
    printf("{\"bench\":\"madd_bn254_xyzz_chain\",\"ms\":%.3f,\"Gmadd_per_s\":%.2f}\n", ms, madds / ms / 1e6);
    return 0;
}
