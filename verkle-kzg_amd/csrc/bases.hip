// Base tables: upload (canonical -> Montgomery, on-curve validation), synthetic generation
// (s_i * G on the device), download. Replaces the reference's CRS storage
// (IPAUniversalParams::g, ipa/mod.rs:22-28; KZGKey::lagrange_commitments, kzg/mod.rs:28-40),
// which arkworks keeps as projective Montgomery points; the engine keeps affine
// Montgomery (64 B BN254, 96 B BLS12-381, 96 B Bandersnatch (x, y, d*x*y)).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "ec.hpp"

namespace vk {

template <class C>
struct Gen;
template <>
struct Gen<BN254G1> {
    VK_HD static uint32_t x(int i) { return i == 0 ? 1u : 0u; }
    VK_HD static uint32_t y(int i) { return i == 0 ? 2u : 0u; }
};
template <>
struct Gen<BLS381G1> {
    VK_HD static uint32_t x(int i) {
        constexpr uint32_t v[] = {0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu, 0x171bac58u, 0xa14e3a3fu,
                                  0x9774b905u, 0xc3688c4fu, 0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u};
        return v[i];
    }
    VK_HD static uint32_t y(int i) {
        constexpr uint32_t v[] = {0x46c5e7e1u, 0x0caa2329u, 0xa2888ae4u, 0xd03cc744u, 0x2c04b3edu, 0x00db18cbu,
                                  0xd5d00af6u, 0xfcf5e095u, 0x741d8ae4u, 0xa09e30edu, 0xe3aaa0f1u, 0x08b3f481u};
        return v[i];
    }
};
template <>
struct Gen<Bandersnatch> {
    VK_HD static uint32_t x(int i) {
        constexpr uint32_t v[] = {0xa252ae18u, 0xe1e71866u, 0xad998465u, 0x2b79c022u,
                                  0x7bbe42f3u, 0x74371177u, 0x2c0b34c5u, 0x29c132ccu};
        return v[i];
    }
    VK_HD static uint32_t y(int i) {
        constexpr uint32_t v[] = {0xcc974166u, 0x5e3167b6u, 0xeee46460u, 0x358cad81u,
                                  0xbadcd586u, 0x157d8b50u, 0xda123e0fu, 0x2a6c669eu};
        return v[i];
    }
};

// ------------------------------------------------------------------ on-curve + conversions
template <class C>
__device__ __forceinline__ bool on_curve(const fe<typename C::F>& x, const fe<typename C::F>& y) {
    using F = typename C::F;
    fe<F> x2 = fe_sqr<F>(x), y2 = fe_sqr<F>(y);
    if constexpr (!C::is_te) {
        fe<F> b = fe_zero<F>();
        b.v[0] = (uint32_t)C::COEFF_B;
        b = fe_to_mont<F>(b);
        return fe_eq<F>(fe_add<F>(fe_mul<F>(x2, x), b), y2);
    } else {
        fe<F> lhs = fe_sub<F>(y2, fe_mul_small<F, 5>(x2));
        fe<F> rhs = fe_add<F>(fe_one<F>(), fe_mul<F>(fe_mul<F>(x2, y2), C::d()));
        return fe_eq<F>(lhs, rhs);
    }
}

template <class C>
__device__ __forceinline__ typename C::Aff make_aff(const fe<typename C::F>& x, const fe<typename C::F>& y) {
    typename C::Aff a;
    a.x = x;
    a.y = y;
    if constexpr (C::is_te) a.kt = fe_mul<typename C::F>(fe_mul<typename C::F>(x, y), C::d());
    return a;
}

template <class C>
__global__ void k_upload(const uint32_t* __restrict__ xy, const uint8_t* __restrict__ inf, uint32_t n,
                         typename C::Aff* __restrict__ out, uint8_t* __restrict__ out_inf,
                         uint32_t* __restrict__ bad) {
    using F = typename C::F;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe<F> x, y;
#pragma unroll
    for (int k = 0; k < F::N; k++) {
        x.v[k] = xy[(size_t)i * 2 * F::N + k];
        y.v[k] = xy[(size_t)i * 2 * F::N + F::N + k];
    }
    uint8_t isinf = inf ? inf[i] : 0;
    if (isinf) {
        x = fe_zero<F>();
        y = C::is_te ? fe_one<F>() : fe_zero<F>();
    } else {
        // canonical range check (x, y < p): reduce_once leaves values >= p changed
        if (!fe_eq<F>(fe_reduce_once<F>(x), x) || !fe_eq<F>(fe_reduce_once<F>(y), y)) {
            atomicOr(bad, 1u);
            return;
        }
        x = fe_to_mont<F>(x);
        y = fe_to_mont<F>(y);
        if (!on_curve<C>(x, y)) atomicOr(bad, 1u);
    }
    out[i] = make_aff<C>(x, y);
    out_inf[i] = isinf;
}

template <class C>
__global__ void k_download(const typename C::Aff* __restrict__ in, const uint8_t* __restrict__ inf,
                           uint32_t n, uint32_t* __restrict__ xy) {
    using F = typename C::F;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe<F> x = fe_from_mont<F>(in[i].x), y = fe_from_mont<F>(in[i].y);
    if (inf[i]) {
        x = fe_zero<F>();
        y = fe_zero<F>();
    }
#pragma unroll
    for (int k = 0; k < F::N; k++) {
        xy[(size_t)i * 2 * F::N + k] = x.v[k];
        xy[(size_t)i * 2 * F::N + F::N + k] = y.v[k];
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// P_i = s_i * G with s_i from splitmix64(seed, i), s_i < 2^(bits-2); affine via one inversion
template <class C>
__global__ void k_random(uint64_t seed, uint32_t n, int sbits, typename C::Aff* __restrict__ out,
                         uint8_t* __restrict__ out_inf) {
    using F = typename C::F;
    using Acc = typename C::Acc;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st = seed * 0x100000001b3ull + i;
    uint64_t s[4];
    for (int k = 0; k < 4; k++) s[k] = splitmix64(st);
    int topbits = sbits - 2 - 192;  // bits used in the top limb
    s[3] &= (topbits >= 64) ? ~0ull : ((1ull << topbits) - 1);
    s[0] |= 1;  // never zero
    typename C::Aff g;
    fe<F> gx, gy;
#pragma unroll
    for (int k = 0; k < F::N; k++) {
        gx.v[k] = Gen<C>::x(k);
        gy.v[k] = Gen<C>::y(k);
    }
    gx = fe_to_mont<F>(gx);
    gy = fe_to_mont<F>(gy);
    g = make_aff<C>(gx, gy);
    Acc acc = C::zero();
    for (int b = 255; b >= 0; b--) {
        acc = C::dbl(acc);
        if ((s[b >> 6] >> (b & 63)) & 1) acc = C::madd(acc, g, false);
    }
    fe<F> x, y;
    C::to_aff(acc, x, y);
    out[i] = make_aff<C>(x, y);
    out_inf[i] = 0;
}

// ------------------------------------------------------------------ host entry points
template <class C>
static int fill_t(vc_ctx* ctx, Table* t, const uint64_t* xy, const uint8_t* inf, size_t n) {
    using Aff = typename C::Aff;
    using F = typename C::F;
    t->curve = ctx->curve;
    t->n = n;
    t->fb_c = t->fb_W = 0;  // any fixed-base tables are stale now: give their memory back
    t->fb_auto = false;
    t->fb.release();
    delete t->lead;  // (its bases are this table's first ones)
    t->lead = nullptr;
    t->lead_k = t->lead_c = 0;
    t->subgroup = -1;
    t->fast_ok = t->phi_ok = t->win_ok = 0;
    VK_TRY(t->bases.ensure(std::max<size_t>(n, 1) * sizeof(Aff)));
    VK_TRY(t->inf.ensure(std::max<size_t>(n, 1)));
    if (n == 0) return VC_OK;
    DevBuf dxy(ctx), dinf(ctx), dbad(ctx);
    VK_TRY(dxy.ensure(n * 2 * F::N * 4));
    VK_TRY(dinf.ensure(n));
    VK_TRY(dbad.ensure(4));
    VK_CHECK_HIP(hipMemcpyAsync(dxy.p, xy, n * 2 * F::N * 4, hipMemcpyHostToDevice, ctx->stream));
    if (inf) VK_CHECK_HIP(hipMemcpyAsync(dinf.p, inf, n, hipMemcpyHostToDevice, ctx->stream));
    VK_CHECK_HIP(hipMemsetAsync(dbad.p, 0, 4, ctx->stream));
    hipLaunchKernelGGL(k_upload<C>, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, dxy.as<uint32_t>(),
                       inf ? dinf.as<uint8_t>() : nullptr, (uint32_t)n, t->bases.as<Aff>(), t->inf.as<uint8_t>(),
                       dbad.as<uint32_t>());
    VK_CHECK_HIP(hipGetLastError());
    uint32_t bad = 0;
    VK_CHECK_HIP(hipMemcpyAsync(&bad, dbad.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return bad ? VC_E_NOT_ON_CURVE : VC_OK;
}

template <class C>
static int upload_t(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, int* id) {
    Table* t = new Table();
    int st = fill_t<C>(ctx, t, xy, inf, n);
    if (st != VC_OK) {
        delete t;
        return st;
    }
    ctx->tables.push_back(t);
    *id = (int)ctx->tables.size() - 1;
    return VC_OK;
}

int bases_fill(vc_ctx* ctx, Table* t, const uint64_t* xy, const uint8_t* inf, size_t n) {
    switch (ctx->curve) {
        case VC_CURVE_BN254: return fill_t<BN254G1>(ctx, t, xy, inf, n);
        case VC_CURVE_BLS12_381: return fill_t<BLS381G1>(ctx, t, xy, inf, n);
        case VC_CURVE_BANDERSNATCH: return fill_t<Bandersnatch>(ctx, t, xy, inf, n);
    }
    return VC_E_INVALID;
}

template <class C, class Fr>
static int random_t(vc_ctx* ctx, uint64_t seed, size_t n, int* id) {
    using Aff = typename C::Aff;
    Table* t = new Table();
    t->curve = ctx->curve;
    t->n = n;
    t->subgroup = 1;  // multiples of the generator
    int st = t->bases.ensure(std::max<size_t>(n, 1) * sizeof(Aff));
    if (st == VC_OK) st = t->inf.ensure(std::max<size_t>(n, 1));
    if (st != VC_OK) {
        delete t;
        return st;
    }
    if (n > 0) {
        hipLaunchKernelGGL(k_random<C>, dim3((n + 127) / 128), dim3(128), 0, ctx->stream, seed,
                           (uint32_t)n, Fr::BITS, t->bases.as<Aff>(), t->inf.as<uint8_t>());
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess) {
            delete t;
            return VC_E_HIP;
        }
    }
    ctx->tables.push_back(t);
    *id = (int)ctx->tables.size() - 1;
    return VC_OK;
}

template <class C>
static int download_t(vc_ctx* ctx, Table* t, uint64_t* xy, uint8_t* inf) {
    using F = typename C::F;
    if (t->n == 0) return VC_OK;
    DevBuf d;
    VK_TRY(d.ensure(t->n * 2 * F::N * 4));
    hipLaunchKernelGGL(k_download<C>, dim3((t->n + 255) / 256), dim3(256), 0, ctx->stream,
                       t->bases.as<typename C::Aff>(), t->inf.as<uint8_t>(), (uint32_t)t->n,
                       d.as<uint32_t>());
    VK_CHECK_HIP(hipGetLastError());
    VK_CHECK_HIP(hipMemcpyAsync(xy, d.p, t->n * 2 * F::N * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (inf) VK_CHECK_HIP(hipMemcpyAsync(inf, t->inf.p, t->n, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

int bases_upload(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, int* id) {
    switch (ctx->curve) {
        case VC_CURVE_BN254: return upload_t<BN254G1>(ctx, xy, inf, n, id);
        case VC_CURVE_BLS12_381: return upload_t<BLS381G1>(ctx, xy, inf, n, id);
        case VC_CURVE_BANDERSNATCH: return upload_t<Bandersnatch>(ctx, xy, inf, n, id);
    }
    return VC_E_INVALID;
}
int bases_random(vc_ctx* ctx, uint64_t seed, size_t n, int* id) {
    switch (ctx->curve) {
        case VC_CURVE_BN254: return random_t<BN254G1, BN254Fr>(ctx, seed, n, id);
        case VC_CURVE_BLS12_381: return random_t<BLS381G1, BLS381Fr>(ctx, seed, n, id);
        case VC_CURVE_BANDERSNATCH: return random_t<Bandersnatch, BandFr>(ctx, seed, n, id);
    }
    return VC_E_INVALID;
}
int bases_download(vc_ctx* ctx, Table* t, uint64_t* xy, uint8_t* inf) {
    switch (t->curve) {
        case VC_CURVE_BN254: return download_t<BN254G1>(ctx, t, xy, inf);
        case VC_CURVE_BLS12_381: return download_t<BLS381G1>(ctx, t, xy, inf);
        case VC_CURVE_BANDERSNATCH: return download_t<Bandersnatch>(ctx, t, xy, inf);
    }
    return VC_E_INVALID;
}

// ------------------------------------------------------------------ host point helpers
template <class C>
static int acc_to_affine_t(const uint32_t* accw, uint64_t* out_xy, uint8_t* out_inf) {
    using F = typename C::F;
    typename C::Acc a;
    memcpy(&a, accw, sizeof a);
    fe<F> x, y;
    bool fin = C::template to_aff<true>(a, x, y);
    if (!fin) {
        memset(out_xy, 0, 2 * F::N * 4);
        if (C::is_te) out_xy[0 + F::N / 2] = 1;  // y = 1
        *out_inf = 1;
        return VC_OK;
    }
    x = fe_from_mont<F>(x);
    y = fe_from_mont<F>(y);
    memcpy(out_xy, x.v, F::N * 4);
    memcpy(reinterpret_cast<uint32_t*>(out_xy) + F::N, y.v, F::N * 4);
    *out_inf = 0;
    return VC_OK;
}
// n accumulators -> canonical affine with ONE field inversion (Montgomery's trick over the
// denominators: ZZZ for XYZZ, Z for extended Edwards); the same outputs as acc_to_affine_t
template <class C>
static int acc_to_affine_batch_t(const uint32_t* accw, size_t n, uint64_t* out_xy, uint8_t* out_inf) {
    using F = typename C::F;
    using Acc = typename C::Acc;
    constexpr size_t AW = sizeof(Acc) / 4;
    auto den = [](const Acc& a) {
        if constexpr (C::is_te) return a.Z;
        else return a.zzz;
    };
    std::vector<Acc> a(n);
    std::vector<fe<F>> pre(n);
    std::vector<uint8_t> live(n);
    fe<F> run = fe_one<F>();
    for (size_t i = 0; i < n; i++) {
        memcpy(&a[i], accw + i * AW, sizeof(Acc));
        bool z;
        if constexpr (C::is_te) z = fe_is_zero<F>(a[i].Z);
        else z = C::is_zero(a[i]);
        live[i] = !z;
        pre[i] = run;
        if (live[i]) run = fe_mul<F>(run, den(a[i]));
    }
    fe<F> inv = fe_inv_bin<F>(run);
    for (size_t i = n; i-- > 0;) {
        uint64_t* xy = out_xy + i * F::N;  // 2 N 32-bit words = N u64 words per point
        fe<F> x, y;
        bool fin = false;
        if (live[i]) {
            const fe<F> id = fe_mul<F>(inv, pre[i]);  // 1 / den(a_i)
            inv = fe_mul<F>(inv, den(a[i]));
            if constexpr (C::is_te) {
                x = fe_mul<F>(a[i].X, id);
                y = fe_mul<F>(a[i].Y, id);
                fin = !(fe_is_zero<F>(x) && fe_eq<F>(y, fe_one<F>()));
            } else {
                const fe<F> t = fe_mul<F>(id, a[i].zz);  // 1 / Z
                x = fe_mul<F>(a[i].x, fe_sqr<F>(t));
                y = fe_mul<F>(a[i].y, id);
                fin = true;
            }
        }
        if (!fin) {
            memset(xy, 0, 2 * F::N * 4);
            if (C::is_te) xy[0 + F::N / 2] = 1;  // y = 1
            out_inf[i] = 1;
            continue;
        }
        x = fe_from_mont<F>(x);
        y = fe_from_mont<F>(y);
        memcpy(xy, x.v, F::N * 4);
        memcpy(reinterpret_cast<uint32_t*>(xy) + F::N, y.v, F::N * 4);
        out_inf[i] = 0;
    }
    return VC_OK;
}
template <class C>
static int acc_sum_t(const uint32_t* accs, size_t k, uint32_t* out) {
    typename C::Acc r = C::zero();
    for (size_t i = 0; i < k; i++) {
        typename C::Acc a;
        memcpy(&a, accs + i * (sizeof(a) / 4), sizeof a);
        r = C::add(r, a);
    }
    memcpy(out, &r, sizeof r);
    return VC_OK;
}
int acc_to_affine(int curve, const uint32_t* acc, uint64_t* out_xy, uint8_t* out_inf) {
    switch (curve) {
        case VC_CURVE_BN254: return acc_to_affine_t<BN254G1>(acc, out_xy, out_inf);
        case VC_CURVE_BLS12_381: return acc_to_affine_t<BLS381G1>(acc, out_xy, out_inf);
        case VC_CURVE_BANDERSNATCH: return acc_to_affine_t<Bandersnatch>(acc, out_xy, out_inf);
    }
    return VC_E_INVALID;
}
int acc_to_affine_batch(int curve, const uint32_t* accs, size_t n, uint64_t* out_xy, uint8_t* out_inf) {
    switch (curve) {
        case VC_CURVE_BN254: return acc_to_affine_batch_t<BN254G1>(accs, n, out_xy, out_inf);
        case VC_CURVE_BLS12_381: return acc_to_affine_batch_t<BLS381G1>(accs, n, out_xy, out_inf);
        case VC_CURVE_BANDERSNATCH: return acc_to_affine_batch_t<Bandersnatch>(accs, n, out_xy, out_inf);
    }
    return VC_E_INVALID;
}
int acc_sum(int curve, const uint32_t* accs, size_t k, uint32_t* out) {
    switch (curve) {
        case VC_CURVE_BN254: return acc_sum_t<BN254G1>(accs, k, out);
        case VC_CURVE_BLS12_381: return acc_sum_t<BLS381G1>(accs, k, out);
        case VC_CURVE_BANDERSNATCH: return acc_sum_t<Bandersnatch>(accs, k, out);
    }
    return VC_E_INVALID;
}
int point_words(int curve) {
    switch (curve) {
        case VC_CURVE_BN254: return BN254G1::ACC_WORDS;
        case VC_CURVE_BLS12_381: return BLS381G1::ACC_WORDS;
        case VC_CURVE_BANDERSNATCH: return Bandersnatch::ACC_WORDS;
    }
    return 0;
}
int aff_limbs64(int curve) { return curve == VC_CURVE_BLS12_381 ? 6 : 4; }

// ------------------------------------------------------------------ VALU peak probe
// Issue rate of v_mad_u64_u32 (64 independent mads per iteration in asm, 8 waves per SIMD): a
// wave64 64-bit mad issues in 4 cycles per SIMD on gfx950 (tools/issueprobe.hip), like the VCC
// carry adds; plain 32-bit adds issue in 2. The MSM kernels' VALU roofline is priced against
// this rate (lane-operations per second).
#define VK_MADS8_                                              \
    "v_mad_u64_u32 v[10:11], s[98:99], %0, %1, v[20:21]\n\t" \
    "v_mad_u64_u32 v[12:13], s[98:99], %0, %1, v[22:23]\n\t" \
    "v_mad_u64_u32 v[14:15], s[98:99], %0, %1, v[24:25]\n\t" \
    "v_mad_u64_u32 v[16:17], s[98:99], %0, %1, v[26:27]\n\t" \
    "v_mad_u64_u32 v[18:19], s[98:99], %0, %1, v[28:29]\n\t" \
    "v_mad_u64_u32 v[30:31], s[98:99], %0, %1, v[20:21]\n\t" \
    "v_mad_u64_u32 v[32:33], s[98:99], %0, %1, v[22:23]\n\t" \
    "v_mad_u64_u32 v[34:35], s[98:99], %0, %1, v[24:25]\n\t"
__global__ void __launch_bounds__(256) k_mad_probe(uint32_t* out, uint32_t seed, int iters) {
    uint32_t x = seed + threadIdx.x, y = seed * 3 + blockIdx.x;
    for (int i = 0; i < iters; i++) {
        asm volatile(VK_MADS8_ VK_MADS8_ VK_MADS8_ VK_MADS8_ VK_MADS8_ VK_MADS8_ VK_MADS8_ VK_MADS8_
                     :: "v"(x), "v"(y)
                     : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v30", "v31", "v32",
                       "v33", "v34", "v35", "s98", "s99");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y;
}
#undef VK_MADS8_

int device_mad_rate(vc_ctx* ctx, double* tera_per_s) {
    const int blocks = 8192, iters = 512;
    DevBuf out;
    VK_TRY(out.ensure((size_t)blocks * 256 * 4));
    hipEvent_t a, b;
    VK_CHECK_HIP(hipEventCreate(&a));
    VK_CHECK_HIP(hipEventCreate(&b));
    hipLaunchKernelGGL(k_mad_probe, dim3(blocks), dim3(256), 0, ctx->stream, out.as<uint32_t>(), 1u, iters);
    VK_CHECK_HIP(hipEventRecord(a, ctx->stream));
    hipLaunchKernelGGL(k_mad_probe, dim3(blocks), dim3(256), 0, ctx->stream, out.as<uint32_t>(), 2u, iters);
    VK_CHECK_HIP(hipEventRecord(b, ctx->stream));
    VK_CHECK_HIP(hipEventSynchronize(b));
    float ms = 0;
    VK_CHECK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *tera_per_s = (double)blocks * 256 * iters * 64 / (ms * 1e-3) / 1e12;
    return VC_OK;
}

}  // namespace vk
