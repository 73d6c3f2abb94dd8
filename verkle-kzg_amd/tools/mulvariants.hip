// Experiment: field-mul code shapes inside an XYZZ mixed-add loop (BLS12-381). Prints JSON.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../csrc/ec.hpp"
#include "../csrc/mul_asm.hpp"
using namespace vk;
using F = BLS381Fq;

// V2: inline CIOS with the outer loop rolled (b shifted down each row): small code, no calls
template <class F>
__device__ __forceinline__ fe<F> mul_rolled(const fe<F>& a, fe<F> b) {
    constexpr int N = F::N;
    uint32_t t[N];
#pragma unroll
    for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        uint32_t bi = b.v[0];
#pragma unroll
        for (int k = 0; k < N - 1; k++) b.v[k] = b.v[k + 1];
        uint64_t A = (uint64_t)a.v[0] * bi + t[0];
        t[0] = (uint32_t)A;
        uint32_t m = t[0] * F::inv;
        uint64_t C = (uint64_t)m * F::p(0) + t[0];
#pragma unroll
        for (int j = 1; j < N; j++) {
            A = (uint64_t)a.v[j] * bi + t[j] + (A >> 32);
            C = (uint64_t)m * F::p(j) + (uint32_t)A + (C >> 32);
            t[j - 1] = (uint32_t)C;
        }
        t[N - 1] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
    }
    fe<F> r;
#pragma unroll
    for (int j = 0; j < N; j++) r.v[j] = t[j];
    return fe_reduce_once<F>(r);
}


// V4: product-scanning (Comba) Montgomery with the carry-out of v_mad_u64_u32 counted by
// v_addc (inline asm): 2 instructions per 32x32 product, no zero-extension moves.
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& ovf, uint32_t x, uint32_t y) {
    uint64_t c;
    asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
                 : "+v"(acc), "=&s"(c), "+v"(ovf) : "v"(x), "v"(y));
}
template <class F>
__device__ __forceinline__ fe<F> mul_ps(const fe<F>& a, const fe<F>& b) {
    constexpr int N = F::N;
    uint32_t m[N];
    fe<F> r;
    uint64_t acc = 0;
    uint32_t ovf = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) mac(acc, ovf, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) mac(acc, ovf, m[i], F::p(k - i));
        if (k < N) {
            m[k] = (uint32_t)acc * F::inv;
            mac(acc, ovf, m[k], F::p(0));
        } else {
            r.v[k - N] = (uint32_t)acc;
        }
        acc = (acc >> 32) | ((uint64_t)ovf << 32);
        ovf = 0;
    }
    r.v[N - 1] = (uint32_t)acc;
    return fe_reduce_once<F>(r);
}
struct MulPS { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_ps<G>(a, b); } };


// V6: CIOS where each mad addend is produced as a register pair by add-with-carry
__device__ __forceinline__ uint64_t add32x2(uint32_t x, uint32_t y) {
    uint32_t c;
    uint32_t lo = __builtin_addc(x, y, 0u, &c);
    return ((uint64_t)c << 32) | lo;
}
template <class F>
__device__ __forceinline__ fe<F> mul_v6(const fe<F>& a, fe<F> b) {
    constexpr int N = F::N;
    uint32_t t[N];
#pragma unroll
    for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        uint32_t bi = b.v[0];
#pragma unroll
        for (int k = 0; k < N - 1; k++) b.v[k] = b.v[k + 1];
        uint64_t A = (uint64_t)a.v[0] * bi + t[0];
        uint32_t m = (uint32_t)A * F::inv;
        uint64_t C = (uint64_t)m * F::p(0) + (uint32_t)A;
#pragma unroll
        for (int j = 1; j < N; j++) {
            A = (uint64_t)a.v[j] * bi + add32x2(t[j], (uint32_t)(A >> 32));
            C = (uint64_t)m * F::p(j) + add32x2((uint32_t)A, (uint32_t)(C >> 32));
            t[j - 1] = (uint32_t)C;
        }
        t[N - 1] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
    }
    fe<F> r;
#pragma unroll
    for (int j = 0; j < N; j++) r.v[j] = t[j];
    return fe_reduce_once<F>(r);
}
struct MulV6 { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_v6<G>(a, b); } };


// V8: row-parallel CIOS: all N products of a row are independent mads onto {t_j, 0} pairs,
// followed by one add-with-carry chain (VCC) per half-row; no 64-bit carry arithmetic.
template <class F>
__device__ __forceinline__ fe<F> mul_v8(const fe<F>& a, const fe<F>& b) {
    constexpr int N = F::N;
    uint64_t X[N + 1];
#pragma unroll
    for (int j = 0; j <= N; j++) X[j] = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint64_t P[N];
#pragma unroll
        for (int j = 0; j < N; j++) P[j] = (uint64_t)a.v[j] * b.v[i] + X[j];
        // t_j = lo(P_j) + hi(P_{j-1}) + carry ; top word t_N = X[N] + hi(P_{N-1}) + carry
        uint32_t c = 0;
        uint32_t t[N + 1];
        t[0] = (uint32_t)P[0];
#pragma unroll
        for (int j = 1; j < N; j++) t[j] = __builtin_addc((uint32_t)P[j], (uint32_t)(P[j - 1] >> 32), c, &c);
        t[N] = __builtin_addc((uint32_t)X[N], (uint32_t)(P[N - 1] >> 32), c, &c);
        uint32_t m = t[0] * F::inv;
#pragma unroll
        for (int j = 0; j < N; j++) P[j] = (uint64_t)m * F::p(j) + t[j];
        // shift down one limb: X_{j-1} = lo(P_j) + hi(P_{j-1}) + carry
        c = 0;
#pragma unroll
        for (int j = 1; j < N; j++) X[j - 1] = __builtin_addc((uint32_t)P[j], (uint32_t)(P[j - 1] >> 32), c, &c);
        X[N - 1] = __builtin_addc(t[N], (uint32_t)(P[N - 1] >> 32), c, &c);
        X[N] = 0;  // no-carry bound: t < 2p < 2^(32N)
    }
    fe<F> r;
#pragma unroll
    for (int j = 0; j < N; j++) r.v[j] = (uint32_t)X[j];
    return fe_reduce_once<F>(r);
}
struct MulV8 { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_v8<G>(a, b); } };
template <class G>
__device__ __noinline__ fe<G> mul_v8_noinline(const fe<G> a, const fe<G> b) { return mul_v8<G>(a, b); }
struct MulV8N { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_v8_noinline<G>(a, b); } };

struct MulAsm { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return fe_mul_asm12<G>(a, b); } };
template <class G>
__device__ __noinline__ fe<G> mul_asm_noinline(const fe<G> a, const fe<G> b) { return fe_mul_asm12<G>(a, b); }
struct MulAsmN { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_asm_noinline<G>(a, b); } };
struct MulNoinline { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return fe_mul<G>(a, b); } };
struct MulRolled { template <class G> __device__ static fe<G> mul(const fe<G>& a, const fe<G>& b) { return mul_rolled<G>(a, b); } };

template <class M>
struct XYZZ {
    using Acc = BLS381G1::Acc; using Aff = BLS381G1::Aff;
    __device__ static Acc madd(const Acc& p, const Aff& q) {
        fe<F> U2 = M::mul(q.x, p.zz);
        fe<F> S2 = M::mul(q.y, p.zzz);
        fe<F> P = fe_sub<F>(U2, p.x);
        fe<F> R = fe_sub<F>(S2, p.y);
        fe<F> PP = M::mul(P, P);
        fe<F> PPP = M::mul(P, PP);
        fe<F> Q = M::mul(p.x, PP);
        Acc r;
        r.x = fe_sub<F>(fe_sub<F>(M::mul(R, R), PPP), fe_dbl<F>(Q));
        r.y = fe_sub<F>(M::mul(R, fe_sub<F>(Q, r.x)), M::mul(p.y, PPP));
        r.zz = M::mul(p.zz, PP);
        r.zzz = M::mul(p.zzz, PPP);
        return r;
    }
};

template <class M>
__device__ __noinline__ BLS381G1::Acc madd_call(const BLS381G1::Acc& p, const BLS381G1::Aff& q) { return XYZZ<M>::madd(p, q); }
template <class M> struct Called { __device__ static BLS381G1::Acc madd(const BLS381G1::Acc& p, const BLS381G1::Aff& q) { return madd_call<M>(p, q); } };
template <class M> struct Inl { __device__ static BLS381G1::Acc madd(const BLS381G1::Acc& p, const BLS381G1::Aff& q) { return XYZZ<M>::madd(p, q); } };

__global__ void k_check(uint32_t* bad, uint32_t seed) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    fe<F> a, b;
    uint32_t x = seed ^ (t * 2654435761u);
    for (int i = 0; i < F::N; i++) { x = x * 1664525u + 1013904223u; a.v[i] = x; x = x * 1664525u + 1013904223u; b.v[i] = x; }
    a.v[F::N - 1] &= 0x0fffffff; b.v[F::N - 1] &= 0x0fffffff;
    for (int it = 0; it < 8; it++) {
        fe<F> r1 = fe_mul<F>(a, b), r2 = mul_ps<F>(a, b), r3 = mul_v6<F>(a, b), r4 = mul_v8<F>(a, b), r5 = fe_mul_asm12<F>(a, b);
        if (!fe_eq<F>(r1, r5)) atomicAdd(bad + 1, 1u);
        if (!fe_eq<F>(r1, r4)) atomicAdd(bad, 1u);
        if (!fe_eq<F>(r1, r3)) atomicAdd(bad, 1u);
        if (!fe_eq<F>(r1, r2)) atomicAdd(bad, 1u);
        a = r1; b = fe_add<F>(b, r1);
    }
}

template <class M>
__global__ void __launch_bounds__(256) k_loop(const BLS381G1::Aff* bases, uint32_t nb, int iters, BLS381G1::Acc* out) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    BLS381G1::Acc acc;
    acc.x = bases[t % nb].x; acc.y = bases[t % nb].y; acc.zz = fe_one<F>(); acc.zzz = fe_one<F>();
    uint32_t idx = t * 2654435761u;
    for (int i = 0; i < iters; i++) {
        idx = idx * 1664525u + 1013904223u;
        acc = M::madd(acc, bases[idx % nb]);
    }
    out[t] = acc;
}

template <class M>
static void run(const char* name, BLS381G1::Aff* b, BLS381G1::Acc* o) {
    int blocks = 256 * 8, iters = 64;
    hipLaunchKernelGGL(k_loop<M>, dim3(blocks), dim3(256), 0, 0, b, 1u << 20, iters, o);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_loop<M>, dim3(blocks), dim3(256), 0, 0, b, 1u << 20, iters, o);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double madds = (double)blocks * 256 * iters;
    printf("{\"variant\":\"%s\",\"ms\":%.3f,\"Gmadd_per_s\":%.3f,\"Gmul_per_s\":%.2f}\n", name, ms, madds / ms / 1e6, madds * 10 / ms / 1e6);
}

int main() {
    BLS381G1::Aff* b; BLS381G1::Acc* o;
    hipMalloc(&b, (1u << 20) * sizeof(BLS381G1::Aff));
    hipMemset(b, 0x11, (1u << 20) * sizeof(BLS381G1::Aff));
    hipMalloc(&o, 256 * 8 * 256 * sizeof(BLS381G1::Acc));
    uint32_t* bad; hipMalloc(&bad, 8); hipMemset(bad, 0, 8);
    for (int s = 0; s < 16; s++) hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, bad, (uint32_t)s * 7919u);
    uint32_t hb[2] = {0, 0}; hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost);
    printf("{\"check_mismatches_ps_v6_v8\":%u, \"check_mismatches_asm\":%u}\n", hb[0], hb[1]);
    for (int rep = 0; rep < 2; rep++) {
    run<Inl<MulNoinline>>("noinline_mul", b, o);

    run<Inl<MulAsm>>("asm_inline", b, o);
    run<Inl<MulAsmN>>("asm_noinline", b, o);
    }
    return 0;
}
