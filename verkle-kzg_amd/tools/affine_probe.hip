// Batched-affine accumulation probe, BLS12-381 G1 on the shipped signed
// radix-2^30 engine (ff30.hpp / ec30.hpp), in the bucket-accumulate shape of tools/s30probe.hip:
// every lane folds ITERS points gathered at pseudo-random rows of a 2^20-point table into one
// accumulator (the next point loaded before the add, as k_msm_accumulate does).
//   xyzz    : the shipped XYZZ mixed add (SW30::madd, 8M + 2S) -- the baseline
//   aff_w   : affine accumulators, Montgomery's trick across the 64 lanes of a wave: the lanes'
//             (x2 - x1) in a prefix / suffix product scan over the wave (shuffles), ONE Fermat
//             inversion of the wave's product per step (4-bit windows, table in LDS), then each
//             lane's inverse = prefix(l - 1) suffix(l + 1) / total and the affine add (2M + 1S)
//   aff_b<W>: the same, one inversion per BLOCK of W waves per step: wave totals in LDS, wave 0
//             inverts the block's product while the others wait at the barrier
// All kernels add the same point sequence per lane; the affine results are checked against the
// XYZZ accumulators on the device (x ZZ == X, y ZZZ == Y mod p). Prints JSON lines (ms per kernel,
// adds/s). VALU instructions per add: run under rocprofv3 --pmc SQ_INSTS_VALU (scripts in
// profiles/r06/affine_probe/). A pow-only kernel gives the instructions of one inversion.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 affine_probe.hip -o affine_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../csrc/ec30.hpp"
using namespace vk;
using F = BLS381Fq;
using P30 = F30BLS381Fq;
using S30 = SW30<BLS381G1, P30>;
using E = f30<P30>;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// p - 2 in 4-bit digits, most significant first (BLS12-381 Fq)
__constant__ uint8_t EXP_NIB[96] = {
    1, 10, 0, 1, 1, 1, 14, 10, 3, 9, 7, 15, 14, 6, 9, 10, 4, 11, 1, 11, 10, 7, 11, 6, 4, 3, 4, 11, 10, 12, 13, 7,
    6, 4, 7, 7, 4, 11, 8, 4, 15, 3, 8, 5, 1, 2, 11, 15, 6, 7, 3, 0, 13, 2, 10, 0, 15, 6, 11, 0, 15, 6, 2, 4,
    1, 14, 10, 11, 15, 15, 15, 14, 11, 1, 5, 3, 15, 15, 15, 15, 11, 9, 15, 14, 15, 15, 15, 15, 15, 15, 15, 15, 10, 10, 10, 9};

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
__global__ void k_init(S30::Aff* t30, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    t30[i].x = from_mont32_30<P30, F>(rand_fe(2 * i));
    t30[i].y = from_mont32_30<P30, F>(rand_fe(2 * i + 1));
}

__device__ __forceinline__ E shfl_up_e(const E& v, int d) {
    E o;
#pragma unroll
    for (int j = 0; j < P30::L; j++) o.v[j] = __shfl_up(v.v[j], d, 64);
    return o;
}
__device__ __forceinline__ E shfl_down_e(const E& v, int d) {
    E o;
#pragma unroll
    for (int j = 0; j < P30::L; j++) o.v[j] = __shfl_down(v.v[j], d, 64);
    return o;
}
__device__ __forceinline__ E shfl_e(const E& v, int src) {
    E o;
#pragma unroll
    for (int j = 0; j < P30::L; j++) o.v[j] = __shfl(v.v[j], src, 64);
    return o;
}
__device__ __forceinline__ E sel(bool c, const E& a, const E& b) {
    E r;
#pragma unroll
    for (int j = 0; j < P30::L; j++) r.v[j] = c ? a.v[j] : b.v[j];
    return r;
}

// a^(p - 2) (Montgomery form in and out): 4-bit windows, the 16 powers in this wave's LDS slot
// (the argument is uniform over the wave in every caller, so one copy serves all lanes)
// (opq30: the value is wave-uniform, and without the opaque copy the compiler moves much of the
// chain to the scalar unit -- s_mul_i32 / s_mul_hi_i32 pairs at ~2 ms per inversion on a lone wave)
__device__ E pow_inv(const E& a_in, E* tab) {
    const int lane = threadIdx.x & 63;
    const E a = opq30<P30>(a_in);
    E x = opq30<P30>(one30<P30>());
    if (lane == 0) tab[0] = x;
    E pw = a;
    for (int k = 1; k < 16; k++) {  // a^k
        if (lane == 0) tab[k] = pw;
        pw = mul30<P30>(pw, a);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    for (int i = 0; i < 96; i++) {
        if (i) {
            for (int s = 0; s < 4; s++) x = sqr30<P30>(x);
        }
        x = mul30<P30>(x, opq30<P30>(tab[EXP_NIB[i]]));
    }
    return x;
}

__global__ void __launch_bounds__(256) k_xyzz(const S30::Aff* __restrict__ tab, uint32_t mask, int iters,
                                              S30::Acc* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    S30::Acc acc = S30::zero();
    uint32_t idx = mix(t + 0x1234567u);
    S30::Aff nxt = tab[idx & mask];
    for (int i = 0; i < iters; i++) {
        const S30::Aff q = nxt;
        idx = mix(idx);
        nxt = tab[idx & mask];
        acc = S30::madd(acc, q, false);
    }
    out[t] = acc;
}

// W waves per block; W = 1: one inversion per wave step, W > 1: one per block step
template <int W>
__global__ void __launch_bounds__(64 * W) k_affine(const S30::Aff* __restrict__ tab, uint32_t mask, int iters,
                                                   S30::Aff* __restrict__ out) {
    __shared__ E ptab[W][16];
    __shared__ E wtot[W], winv[W];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t idx = mix(t + 0x1234567u);
    S30::Aff a = tab[idx & mask];
    idx = mix(idx);
    S30::Aff nxt = tab[idx & mask];
    const E one = one30<P30>();
    for (int i = 1; i < iters; i++) {
        const S30::Aff q = nxt;
        idx = mix(idx);
        nxt = tab[idx & mask];
        const E d = sub30<P30>(q.x, a.x);
        // inclusive prefix (S) and suffix (U) products of d over the wave's lanes
        E S = d, U = d;
        for (int k = 1; k < 64; k <<= 1) {
            const E so = shfl_up_e(S, k), uo = shfl_down_e(U, k);
            S = mul30<P30>(S, sel(lane >= k, so, one));
            U = mul30<P30>(U, sel(lane + k < 64, uo, one));
        }
        const E Sx = sel(lane > 0, shfl_up_e(S, 1), one);     // prefix of lanes < l
        const E Ux = sel(lane < 63, shfl_down_e(U, 1), one);  // suffix of lanes > l
        E tot = shfl_e(S, 63);                                // the wave's product (uniform)
        E itot;
        if constexpr (W == 1) {
            itot = pow_inv(tot, ptab[0]);
        } else {
            if (lane == 0) wtot[wv] = tot;
            __syncthreads();
            if (wv == 0) {
                E all = opq30<P30>(wtot[0]);
                for (int v = 1; v < W; v++) all = mul30<P30>(all, opq30<P30>(wtot[v]));
                const E inv = pow_inv(all, ptab[0]);
                // lane v < W: the inverse of wave v's total = inv * product of the other totals
                E oth = opq30<P30>(one);
                for (int v = 0; v < W; v++) oth = mul30<P30>(oth, sel(v == lane, one, opq30<P30>(wtot[v])));
                if (lane < W) winv[lane] = mul30<P30>(inv, oth);
            }
            __syncthreads();
            itot = winv[wv];
        }
        const E inv_d = mul30<P30>(mul30<P30>(Sx, Ux), itot);
        const E lam = mul30<P30>(sub30<P30>(q.y, a.y), inv_d);
        const E x3 = sub30<P30>(sub30<P30>(sqr30<P30>(lam), a.x), q.x);
        const E y3 = sub30<P30>(mul30<P30>(lam, sub30<P30>(a.x, x3)), a.y);
        a.x = x3;
        a.y = y3;
        if constexpr (W > 1) __syncthreads();  // wtot / winv reused next step
    }
    out[t] = a;
}

// instructions of one inversion: every lane inverts its own value (POWS times)
__global__ void __launch_bounds__(64) k_pow(const S30::Aff* __restrict__ tab, int pows, S30::Aff* __restrict__ out) {
    __shared__ E ptab[16];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    E x = tab[t].x;
    const E x0 = shfl_e(x, 0);
    E r = x0;
    for (int i = 0; i < pows; i++) r = pow_inv(r, ptab);
    out[t].x = r;
}

// x ZZ == X and y ZZZ == Y (mod p) per lane
__global__ void k_check(const S30::Acc* __restrict__ xy, const S30::Aff* __restrict__ af, size_t n,
                        uint32_t* __restrict__ bad) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t u0[P30::L], u1[P30::L], u2[P30::L], u3[P30::L];
    canon30<P30>(mul30<P30>(af[i].x, xy[i].zz), u0);
    canon30<P30>(xy[i].x, u1);
    canon30<P30>(mul30<P30>(af[i].y, xy[i].zzz), u2);
    canon30<P30>(xy[i].y, u3);
    for (int j = 0; j < P30::L; j++)
        if (u0[j] != u1[j] || u2[j] != u3[j]) {
            atomicAdd(bad, 1u);
            return;
        }
}

template <class K>
static float timed(K launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    launch();
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
    const int iters = argc > 1 ? atoi(argv[1]) : 32;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const uint32_t n = 1u << 20;
    const int blocks = 512;  // 131,072 lanes: the accumulate's 2 waves per SIMD
    const size_t threads = (size_t)blocks * 256;
    S30::Aff *tab, *oa;
    S30::Acc* ox;
    uint32_t* bad;
    CK(hipMalloc(&tab, n * sizeof(S30::Aff)));
    CK(hipMalloc(&oa, threads * sizeof(S30::Aff)));
    CK(hipMalloc(&ox, threads * sizeof(S30::Acc)));
    CK(hipMalloc(&bad, 4));
    hipLaunchKernelGGL(k_init, dim3(n / 256), dim3(256), 0, 0, tab, n);
    CK(hipDeviceSynchronize());
    hipFuncAttributes ax, a1, a4, a8;
    CK(hipFuncGetAttributes(&ax, reinterpret_cast<const void*>(&k_xyzz)));
    CK(hipFuncGetAttributes(&a1, reinterpret_cast<const void*>(&k_affine<1>)));
    CK(hipFuncGetAttributes(&a4, reinterpret_cast<const void*>(&k_affine<4>)));
    CK(hipFuncGetAttributes(&a8, reinterpret_cast<const void*>(&k_affine<8>)));
    printf("{\"vgprs_xyzz\":%d,\"vgprs_aff_w\":%d,\"vgprs_aff_b4\":%d,\"vgprs_aff_b8\":%d,\"lanes\":%zu,\"iters\":%d}\n",
           ax.numRegs, a1.numRegs, a4.numRegs, a8.numRegs, threads, iters);
    const uint32_t mask = n - 1;
    auto run_x = [&] { hipLaunchKernelGGL(k_xyzz, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, ox); };
    auto run_w = [&] { hipLaunchKernelGGL((k_affine<1>), dim3(blocks * 4), dim3(64), 0, 0, tab, mask, iters, oa); };
    auto run_b4 = [&] { hipLaunchKernelGGL((k_affine<4>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, oa); };
    auto run_b8 = [&] { hipLaunchKernelGGL((k_affine<8>), dim3(blocks / 2), dim3(512), 0, 0, tab, mask, iters, oa); };
    auto check = [&](const char* what) {
        CK(hipMemset(bad, 0, 4));
        hipLaunchKernelGGL(k_check, dim3((unsigned)(threads / 256)), dim3(256), 0, 0, ox, oa, threads, bad);
        CK(hipGetLastError());
        uint32_t hb = 0;
        CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("{\"check\":\"%s\",\"lanes\":%zu,\"mismatches\":%u}\n", what, threads, hb);
        fflush(stdout);
        return hb;
    };
    uint32_t nbad = 0;
    run_x();
    run_w();
    CK(hipDeviceSynchronize());
    nbad += check("aff_w");
    run_b4();
    CK(hipDeviceSynchronize());
    nbad += check("aff_b4");
    run_b8();
    CK(hipDeviceSynchronize());
    nbad += check("aff_b8");
    const double adds = (double)threads * (iters - 1);  // the affine kernels start from the first point
    for (int r = 0; r < reps; r++) {
        const float mx = timed(run_x), mw = timed(run_w), m4 = timed(run_b4), m8 = timed(run_b8);
        printf("{\"rep\":%d,\"ms_xyzz\":%.3f,\"ms_aff_w\":%.3f,\"ms_aff_b4\":%.3f,\"ms_aff_b8\":%.3f,"
               "\"Gadd_xyzz\":%.4f,\"Gadd_aff_w\":%.4f,\"Gadd_aff_b4\":%.4f,\"Gadd_aff_b8\":%.4f}\n",
               r, mx, mw, m4, m8, (double)threads * iters / mx / 1e6, adds / mw / 1e6, adds / m4 / 1e6, adds / m8 / 1e6);
        fflush(stdout);
    }
    // one inversion's cost: 64 lanes x `pows` inversions per wave, 1024 waves
    const int pows = 4;
    const float mp = timed([&] { hipLaunchKernelGGL(k_pow, dim3(1024), dim3(64), 0, 0, tab, pows, oa); });
    printf("{\"pow_kernel_ms\":%.3f,\"waves\":1024,\"inversions_per_wave\":%d}\n", mp, pows);
    return nbad != 0;
}
