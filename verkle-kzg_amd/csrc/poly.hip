// Scalar-field kernels of the protocol layer (gfx950): domain powers, batched inversion,
// the KZG quotients (reference lagrange_basis.rs:91-142 + precompute.rs:72-90) and the
// KZG Lagrange SRS (kzg/mod.rs:115-124 via SURVEY Appendix A.7).
//
// The reference divides per element (two Fr inversions per i in divide_by_vanishing); here
// every denominator goes through one chunked Montgomery batch inversion whose per-chunk
// inverse is the binary extended Euclid (latency ~1/50 of a Fermat chain), and the two
// sums the formulas need (barycentric y, q_m) are block reductions.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "ec.hpp"
#include "poly.hpp"

namespace vk {

template <class F>
__global__ void k_canon_to_mont(const fe<F>* __restrict__ in, size_t n, size_t n_valid, fe<F>* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = i < n_valid ? fe_to_mont<F>(in[i]) : fe_zero<F>();
}
template <class F>
__global__ void k_mont_to_canon(const fe<F>* __restrict__ in, size_t n, fe<F>* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = fe_from_mont<F>(in[i]);
}

// out[i] = w^i
template <class F>
__global__ void k_powers(fe<F> w, size_t n, fe<F>* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe<F> r = fe_one<F>(), b = w;
    size_t e = i;
    while (e) {
        if (e & 1) r = fe_mul<F>(r, b);
        e >>= 1;
        if (e) b = fe_sqr<F>(b);
    }
    out[i] = r;
}

// out[k] = 1 / in[k] for k < n (zeros map to zero). Montgomery's trick at two levels: each
// thread multiplies a chunk of CH, a workgroup scans its 256 chunk products (prefix and suffix,
// LDS) and inverts their product, then every chunk's inverse is
// inv(total) * prefix * suffix and the chunk is substituted backwards. One inversion per 256 CH
// elements (per chunk before: 65,536 inversions for a 2^20 KZG quotient, 0.46 ms).
// The workgroup products are inverted on the host (as commit.hip's split normalisation): a
// per-workgroup lane inversion was ~130 us of serial binary Euclid on one GPU lane, the host
// inverts all workgroup products with one inversion in a few us. k_binv_prep leaves the chunk
// prefix products in out[], each chunk the product of its workgroup's OTHER chunk products, and
// the workgroup product; k_binv_finish substitutes backwards.
template <class F>
__global__ void __launch_bounds__(256) k_binv_prep(const fe<F>* __restrict__ in, fe<F>* __restrict__ out, size_t n,
                                                  int CH, fe<F>* __restrict__ others, fe<F>* __restrict__ tot) {
    __shared__ fe<F> pre[256], suf[256];
    const uint32_t t = threadIdx.x;
    const size_t c = (size_t)blockIdx.x * 256 + t;
    const size_t lo = c * CH;
    const size_t hi = lo + CH < n ? lo + CH : n;
    fe<F> acc = fe_one<F>();
    for (size_t k = lo; k < hi; k++) {
        fe<F> v = in[k];
        if (!fe_is_zero<F>(v)) acc = fe_mul<F>(acc, v);
        out[k] = acc;  // chunk prefix products
    }
    pre[t] = acc;
    suf[t] = acc;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
        fe<F> p = pre[t], q = suf[t];
        if (t >= off) p = fe_mul<F>(pre[t - off], p);
        if (t + off < 256) q = fe_mul<F>(q, suf[t + off]);
        __syncthreads();
        pre[t] = p;
        suf[t] = q;
        __syncthreads();
    }
    fe<F> o = fe_one<F>();
    if (t > 0) o = pre[t - 1];
    if (t < 255) o = t > 0 ? fe_mul<F>(o, suf[t + 1]) : suf[t + 1];
    others[c] = o;
    if (t == 0) tot[blockIdx.x] = pre[255];
}

template <class F>
__global__ void __launch_bounds__(256) k_binv_finish(const fe<F>* __restrict__ in, fe<F>* __restrict__ out, size_t n,
                                                    int CH, const fe<F>* __restrict__ others,
                                                    const fe<F>* __restrict__ binv) {
    const size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t lo = c * CH;
    if (lo >= n) return;
    const size_t hi = lo + CH < n ? lo + CH : n;
    fe<F> inv = fe_mul<F>(binv[blockIdx.x], others[c]);  // 1 / (this chunk's product)
    for (size_t k = hi; k-- > lo;) {
        fe<F> v = in[k];
        if (fe_is_zero<F>(v)) {
            out[k] = fe_zero<F>();
            continue;
        }
        fe<F> prev = k > lo ? out[k - 1] : fe_one<F>();
        out[k] = fe_mul<F>(inv, prev);
        inv = fe_mul<F>(inv, v);
    }
}

// den[i] = w^i - z   (out of domain)   or   w^i - w^m with den[m] = 1 (in domain)
template <class F>
__global__ void k_den(const fe<F>* __restrict__ pw, size_t n, fe<F> z, long long m, fe<F>* __restrict__ den) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    den[i] = ((long long)i == m) ? fe_one<F>() : fe_sub<F>(pw[i], z);
}

// partial[b] = sum over the block's i of f_i * w^i * inv_i  (f_i = 0 beyond max)
template <class F>
__global__ void __launch_bounds__(256) k_bary_partial(const fe<F>* __restrict__ f, size_t max,
                                                     const fe<F>* __restrict__ pw, const fe<F>* __restrict__ inv,
                                                     size_t n, fe<F>* __restrict__ partial) {
    __shared__ fe<F> sh[256];
    size_t i0 = (size_t)blockIdx.x * 256 * 8 + threadIdx.x;
    fe<F> acc = fe_zero<F>();
    for (int k = 0; k < 8; k++) {
        size_t i = i0 + (size_t)k * 256;
        if (i < n && i < max) acc = fe_add<F>(acc, fe_mul<F>(fe_mul<F>(f[i], pw[i]), inv[i]));
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) sh[threadIdx.x] = fe_add<F>(sh[threadIdx.x], sh[threadIdx.x + h]);
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

// in domain at m: q_i = (f_i - f_m) * inv_i (i != m); partial sums of q_i * w^i for q_m
// (f_m read here: the host needs no round trip before the launch)
template <class F>
__global__ void __launch_bounds__(256) k_q_in(const fe<F>* __restrict__ f, size_t max, const fe<F>* __restrict__ inv,
                                             const fe<F>* __restrict__ pw, size_t n, size_t m,
                                             fe<F>* __restrict__ q, fe<F>* __restrict__ partial) {
    __shared__ fe<F> sh[256];
    const fe<F> fm = m < max ? f[m] : fe_zero<F>();
    size_t i0 = (size_t)blockIdx.x * 256 * 8 + threadIdx.x;
    fe<F> acc = fe_zero<F>();
    for (int k = 0; k < 8; k++) {
        size_t i = i0 + (size_t)k * 256;
        if (i >= n) break;
        if (i == m) {
            q[i] = fe_zero<F>();
            continue;
        }
        fe<F> fi = i < max ? f[i] : fe_zero<F>();
        fe<F> qi = fe_mul<F>(fe_sub<F>(fi, fm), inv[i]);
        q[i] = qi;
        acc = fe_add<F>(acc, fe_mul<F>(qi, pw[i]));
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) sh[threadIdx.x] = fe_add<F>(sh[threadIdx.x], sh[threadIdx.x + h]);
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

template <class F>
__global__ void k_set(fe<F>* __restrict__ a, size_t i, fe<F> v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a[i] = v;
}

// one block: s = sum of the nb block partials; in domain a[m] = k s (q_m = -w^-m sum q_i w^i),
// outside *y = k s (y = -t sum f_i w^i inv_i) -- on the device, so the open has no host round
// trip between the quotient and the MSM
template <class F>
__global__ void __launch_bounds__(256) k_fold_partials(const fe<F>* __restrict__ partial, size_t nb, fe<F> k,
                                                      fe<F>* __restrict__ dst) {
    __shared__ fe<F> sh[256];
    fe<F> acc = fe_zero<F>();
    for (size_t b = threadIdx.x; b < nb; b += 256) acc = fe_add<F>(acc, partial[b]);
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) sh[threadIdx.x] = fe_add<F>(sh[threadIdx.x], sh[threadIdx.x + h]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *dst = fe_mul<F>(k, sh[0]);
}

// q_i = (f_i - y) * inv_i (outside domain), y on the device
template <class F>
__global__ void k_q_out(const fe<F>* __restrict__ f, size_t max, const fe<F>* __restrict__ inv, size_t n,
                          const fe<F>* __restrict__ yp, fe<F>* __restrict__ q) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fe<F> y = *yp;
    fe<F> fi = i < max ? f[i] : fe_zero<F>();
    q[i] = fe_mul<F>(fe_sub<F>(fi, y), inv[i]);
}

// ---------------------------------------------------------------- Lagrange SRS (A.7)
// c_j = n^-1 * ((s w^-j)^m - 1) / (s w^-j - 1); the numerator/denominator pass, then one
// batch inversion, then the fixed-base scalar multiplications c_j * G.
template <class F>
__global__ void k_srs_num_den(const fe<F>* __restrict__ pw_inv, size_t n, fe<F> s, uint64_t m, fe<F> ninv,
                              fe<F>* __restrict__ num, fe<F>* __restrict__ den) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    fe<F> b = fe_mul<F>(s, pw_inv[j]);
    fe<F> r = fe_one<F>(), x = b;
    uint64_t e = m;
    while (e) {
        if (e & 1) r = fe_mul<F>(r, x);
        e >>= 1;
        if (e) x = fe_sqr<F>(x);
    }
    num[j] = fe_mul<F>(fe_sub<F>(r, fe_one<F>()), ninv);
    den[j] = fe_sub<F>(b, fe_one<F>());
}
template <class F>
__global__ void k_mul_elem(fe<F>* __restrict__ a, const fe<F>* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    a[i] = fe_mul<F>(a[i], b[i]);
}

template <class C, class Fr>
__global__ void k_fixed_mul_gen(const fe<Fr>* __restrict__ sc_mont, size_t n, typename C::Aff g,
                                typename C::Acc* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe<Fr> s = fe_from_mont<Fr>(sc_mont[i]);
    typename C::Acc acc = C::zero();
    for (int b = Fr::N * 32 - 1; b >= 0; b--) {
        acc = C::dbl(acc);
        if ((s.v[b >> 5] >> (b & 31)) & 1) acc = C::madd(acc, g, false);
    }
    out[i] = acc;
}

// ---------------------------------------------------------------- host drivers
template <class F>
static fe<F> host_pow(fe<F> a, uint64_t e) {
    fe<F> r = fe_one<F>();
    for (; e; e >>= 1) {
        if (e & 1) r = fe_mul<F>(r, a);
        a = fe_sqr<F>(a);
    }
    return r;
}

template <class F>
int domain_powers(vc_ctx* ctx, const fe<F>& w, size_t n, fe<F>* d_out) {
    VK_LAUNCH(ctx, "powers", (k_powers<F>), (n + 255) / 256, 256, 0, w, n, d_out);
    return VC_OK;
}

// synchronises the stream once (the host inversion between the two kernels)
template <class F>
int batch_inverse(vc_ctx* ctx, const fe<F>* d_in, fe<F>* d_out, size_t n) {
    if (n == 0) return VC_OK;
    const int CH = n >= (1u << 18) ? 16 : 4;
    const size_t chunks = (n + CH - 1) / CH;
    const size_t nblk = (chunks + 255) / 256;
    DevBuf others(ctx), tot(ctx);
    VK_TRY(others.ensure(nblk * 256 * sizeof(fe<F>)));
    VK_TRY(tot.ensure(nblk * sizeof(fe<F>)));
    VK_TRY(ctx->pin_norm.ensure(2 * nblk * sizeof(fe<F>)));
    fe<F>* h = ctx->pin_norm.as<fe<F>>();
    VK_LAUNCH(ctx, "binv_prep", (k_binv_prep<F>), nblk, 256, 0, d_in, d_out, n, CH, others.as<fe<F>>(),
              tot.as<fe<F>>());
    VK_CHECK_HIP(hipMemcpyAsync(h, tot.p, nblk * sizeof(fe<F>), hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    fe<F>* inv = h + nblk;  // Montgomery's trick over the workgroup products (never zero)
    inv[0] = h[0];
    for (size_t b = 1; b < nblk; b++) inv[b] = fe_mul<F>(inv[b - 1], h[b]);
    fe<F> run = fe_inv_bin<F>(inv[nblk - 1]);
    for (size_t b = nblk - 1; b > 0; b--) {
        const fe<F> ib = fe_mul<F>(run, inv[b - 1]);
        run = fe_mul<F>(run, h[b]);
        inv[b] = ib;
    }
    inv[0] = run;
    VK_CHECK_HIP(hipMemcpyAsync(tot.p, inv, nblk * sizeof(fe<F>), hipMemcpyHostToDevice, ctx->stream));
    VK_LAUNCH(ctx, "binv_finish", (k_binv_finish<F>), nblk, 256, 0, d_in, d_out, n, CH, others.as<fe<F>>(),
              tot.as<fe<F>>());
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // the pinned inverses are reused by the next call
    return VC_OK;
}

// inv[i] = w^-m / (w^((i - m) mod n) - 1) = 1 / (w^i - w^m)  (i != m), from the per-domain
// table inv1[k] = 1/(w^k - 1): the in-domain quotient needs no inversion per open
template <class F>
__global__ void k_inv_shift(const fe<F>* __restrict__ inv1, size_t n, size_t m, fe<F> wminv, fe<F>* __restrict__ inv) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    inv[i] = i == m ? fe_zero<F>() : fe_mul<F>(wminv, inv1[(i + n - m) & (n - 1)]);
}

template <class F>
static std::string dkey(const char* tag, size_t n) {
    return std::string(tag) + ":" + std::to_string(F::BITS) + ":" + std::to_string(F::N) + ":" + std::to_string(n);
}

// domain powers w^i, i < n (cached per ctx: PrecomputedLagrange keeps them too, precompute.rs:25-58)
template <class F>
static int cached_powers(vc_ctx* ctx, const fe<F>& omega, size_t n, fe<F>** out) {
    auto& slot = ctx->dcache[dkey<F>("pw", n)];
    if (!slot) {
        auto b = std::make_unique<DevBuf>();
        VK_TRY(b->ensure(n * sizeof(fe<F>)));
        VK_TRY(domain_powers<F>(ctx, omega, n, b->as<fe<F>>()));
        slot = std::move(b);
    }
    *out = reinterpret_cast<fe<F>*>(slot->p);
    return VC_OK;
}

// inv1[k] = 1/(w^k - 1) for 0 < k < n (inv1[0] unused), cached per ctx
template <class F>
static int cached_inv1(vc_ctx* ctx, const fe<F>* pw, size_t n, fe<F>** out) {
    auto& slot = ctx->dcache[dkey<F>("inv1", n)];
    if (!slot) {
        auto b = std::make_unique<DevBuf>();
        DevBuf den;
        VK_TRY(b->ensure(n * sizeof(fe<F>)));
        VK_TRY(den.ensure(n * sizeof(fe<F>)));
        VK_LAUNCH(ctx, "kzg_den", (k_den<F>), (n + 255) / 256, 256, 0, pw, n, fe_one<F>(), 0LL, den.as<fe<F>>());
        VK_TRY(batch_inverse<F>(ctx, den.as<fe<F>>(), b->as<fe<F>>(), n));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // den is freed on return
        slot = std::move(b);
    }
    *out = reinterpret_cast<fe<F>*>(slot->p);
    return VC_OK;
}

template <class F>
int domain_tables(vc_ctx* ctx, const fe<F>& w, size_t n, const fe<F>** pw, const fe<F>** pwi, const fe<F>** inv1) {
    fe<F>* a = nullptr;
    VK_TRY(cached_powers<F>(ctx, w, n, &a));
    *pw = a;
    if (inv1) {
        fe<F>* b = nullptr;
        VK_TRY(cached_inv1<F>(ctx, a, n, &b));
        *inv1 = b;
    }
    if (pwi) {
        auto& slot = ctx->dcache[dkey<F>("pwi", n)];
        if (!slot) {
            auto b = std::make_unique<DevBuf>();
            VK_TRY(b->ensure(n * sizeof(fe<F>)));
            VK_TRY(domain_powers<F>(ctx, fe_inv_bin<F>(w), n, b->as<fe<F>>()));
            slot = std::move(b);
        }
        *pwi = reinterpret_cast<const fe<F>*>(slot->p);
    }
    return VC_OK;
}

// q and y for KZG prove_point (device, Montgomery). point given in Montgomery form. The stream is
// not synchronised in the domain and once (the batch inversion's host step) outside it: y (a
// device value) is copied into *y_out (page-locked host memory) asynchronously, so the caller
// reads *y_out only after synchronising ctx->stream (its MSM does).
template <class F>
int kzg_quotient_dev(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t max, const fe<F>& point, const fe<F>& omega,
                     fe<F>* d_q, fe<F>* y_out, DevBuf& pw, DevBuf& tmp, DevBuf& part) {
    hipStream_t st = ctx->stream;
    (void)pw;
    VK_TRY(tmp.ensure(n * sizeof(fe<F>)));
    fe<F>* den = d_q;  // denominators staged in the output buffer, inverses in tmp
    size_t nblk = (n + 2047) / 2048;
    VK_TRY(part.ensure((nblk + 1) * sizeof(fe<F>)));
    fe<F>* d_y = part.as<fe<F>>() + nblk;  // the device y, after the block partials
    fe<F>* pwp = nullptr;
    VK_TRY(cached_powers<F>(ctx, omega, n, &pwp));
    fe<F>* inv = tmp.as<fe<F>>();
    // prove_point: `point <= size` -> in-domain branch with index to_usize(point)
    fe<F> pc = fe_from_mont<F>(point);
    bool small = true;
    for (int i = 2; i < F::N; i++) small &= pc.v[i] == 0;
    uint64_t pv = (uint64_t)pc.v[0] | ((uint64_t)pc.v[1] << 32);
    if (small && pv <= n) {
        if (pv == n) return VC_E_DOMAIN;  // reference: vanishing_at(size) out of bounds
        size_t m = (size_t)pv;
        // w^-m = w^(n - m) on the host (the powers table holds the same values)
        const fe<F> wminv = host_pow<F>(omega, (n - m) & (n - 1));
        fe<F>* inv1 = nullptr;
        VK_TRY(cached_inv1<F>(ctx, pwp, n, &inv1));
        VK_LAUNCH(ctx, "kzg_inv_shift", (k_inv_shift<F>), (n + 255) / 256, 256, 0, inv1, n, m, wminv, inv);
        VK_LAUNCH(ctx, "kzg_q_in", (k_q_in<F>), nblk, 256, 0, d_f, max, inv, pwp, n, m, d_q, part.as<fe<F>>());
        // q_m = -w^-m * sum_{i != m} q_i w^i
        VK_LAUNCH(ctx, "kzg_fold", (k_fold_partials<F>), 1, 256, 0, part.as<fe<F>>(), nblk, fe_neg<F>(wminv), d_q + m);
        // y = evaluate(point): the stored value, or 0 inside [max, size]
        if (m < max) {
            VK_CHECK_HIP(hipMemcpyAsync(y_out, d_f + m, sizeof(fe<F>), hipMemcpyDeviceToHost, st));
        } else {
            *y_out = fe_zero<F>();
        }
        return VC_OK;
    }
    // outside: inv_i = 1/(w^i - z); y = -t * sum f_i w^i inv_i, t = (z^n - 1)/n
    VK_LAUNCH(ctx, "kzg_den", (k_den<F>), (n + 255) / 256, 256, 0, pwp, n, point, (long long)-1, den);
    VK_TRY(batch_inverse<F>(ctx, den, inv, n));
    fe<F> nn = fe_zero<F>();
    nn.v[0] = (uint32_t)n;
    nn.v[1] = (uint32_t)((uint64_t)n >> 32);
    const fe<F> t = fe_mul<F>(fe_sub<F>(host_pow<F>(point, n), fe_one<F>()), fe_inv_bin<F>(fe_to_mont<F>(nn)));
    VK_LAUNCH(ctx, "kzg_bary", (k_bary_partial<F>), nblk, 256, 0, d_f, max, pwp, inv, n, part.as<fe<F>>());
    VK_LAUNCH(ctx, "kzg_fold", (k_fold_partials<F>), 1, 256, 0, part.as<fe<F>>(), nblk, fe_neg<F>(t), d_y);
    VK_LAUNCH(ctx, "kzg_q_out", (k_q_out<F>), (n + 255) / 256, 256, 0, d_f, max, inv, n, d_y, d_q);
    VK_CHECK_HIP(hipMemcpyAsync(y_out, d_y, sizeof(fe<F>), hipMemcpyDeviceToHost, st));
    return VC_OK;
}

// ---- index-range shards of the quotient (vc_group_kzg_prove): a member holds f
// and q on [lo, lo + L) of the domain; the one global sum each case needs (in the domain q_m's
// sum of q_i w^i, outside the barycentric sum of f_i w^i inv_i) leaves as one field partial per
// member, and the finish gets the members' total back.
// in domain at m (lagrange_basis.rs:91-119): q_i = (f_i - f_m) / (w^i - w^m), block partials of
// q_i w^i; f_m by value (it may lie in another member's slice)
template <class F>
__global__ void __launch_bounds__(256) k_q_in_range(const fe<F>* __restrict__ f, size_t nvalid,
                                                   const fe<F>* __restrict__ inv1, const fe<F>* __restrict__ pw,
                                                   size_t n, size_t lo, size_t L, size_t m, fe<F> wminv, fe<F> fm,
                                                   fe<F>* __restrict__ q, fe<F>* __restrict__ partial) {
    __shared__ fe<F> sh[256];
    size_t i0 = (size_t)blockIdx.x * 256 * 8 + threadIdx.x;
    fe<F> acc = fe_zero<F>();
    for (int k = 0; k < 8; k++) {
        const size_t i = i0 + (size_t)k * 256;  // local index; global lo + i
        if (i >= L) break;
        const size_t gi = lo + i;
        if (gi == m) {
            q[i] = fe_zero<F>();
            continue;
        }
        const fe<F> fi = i < nvalid ? f[i] : fe_zero<F>();
        const fe<F> inv = fe_mul<F>(wminv, inv1[(gi + n - m) & (n - 1)]);  // 1 / (w^gi - w^m)
        const fe<F> qi = fe_mul<F>(fe_sub<F>(fi, fm), inv);
        q[i] = qi;
        acc = fe_add<F>(acc, fe_mul<F>(qi, pw[gi]));
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) sh[threadIdx.x] = fe_add<F>(sh[threadIdx.x], sh[threadIdx.x + h]);
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}
// outside: q_i = (f_i - y) inv_i with y by value
template <class F>
__global__ void k_q_out_v(const fe<F>* __restrict__ f, size_t nvalid, const fe<F>* __restrict__ inv, size_t L, fe<F> y,
                          fe<F>* __restrict__ q) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L) return;
    const fe<F> fi = i < nvalid ? f[i] : fe_zero<F>();
    q[i] = fe_mul<F>(fe_sub<F>(fi, y), inv[i]);
}

// phase 1 of a range share: d_f = f on [lo, lo + L) (Montgomery; entries >= nvalid are zero), q
// on the slice (in domain) or the inverses inv_i = 1 / (w^(lo+i) - z) (outside) into d_inv, and
// this share's partial of the global sum into *partial (host; the stream is synchronised)
template <class F>
int kzg_range_part(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t nvalid, size_t lo, size_t L, const fe<F>& point,
                   const fe<F>& omega, bool in_domain, size_t m, const fe<F>& fm, fe<F>* d_q, fe<F>* d_inv,
                   DevBuf& part, fe<F>* partial) {
    hipStream_t st = ctx->stream;
    const size_t nblk = std::max<size_t>(1, (L + 2047) / 2048);
    VK_TRY(part.ensure((nblk + 1) * sizeof(fe<F>)));
    fe<F>* d_sum = part.as<fe<F>>() + nblk;
    fe<F>* pwp = nullptr;
    VK_TRY(cached_powers<F>(ctx, omega, n, &pwp));
    if (in_domain) {
        const fe<F> wminv = host_pow<F>(omega, (n - m) & (n - 1));
        fe<F>* inv1 = nullptr;
        VK_TRY(cached_inv1<F>(ctx, pwp, n, &inv1));
        VK_LAUNCH(ctx, "kzg_q_in", (k_q_in_range<F>), nblk, 256, 0, d_f, nvalid, inv1, pwp, n, lo, L, m, wminv, fm,
                  d_q, part.as<fe<F>>());
    } else {
        VK_LAUNCH(ctx, "kzg_den", (k_den<F>), (L + 255) / 256, 256, 0, pwp + lo, L, point, (long long)-1, d_q);
        VK_TRY(batch_inverse<F>(ctx, d_q, d_inv, L));
        VK_LAUNCH(ctx, "kzg_bary", (k_bary_partial<F>), nblk, 256, 0, d_f, nvalid, pwp + lo, d_inv, L, part.as<fe<F>>());
    }
    VK_LAUNCH(ctx, "kzg_fold", (k_fold_partials<F>), 1, 256, 0, part.as<fe<F>>(), nblk, fe_one<F>(), d_sum);
    VK_TRY(ctx->pin_y.ensure(sizeof(fe<F>)));
    VK_CHECK_HIP(hipMemcpyAsync(ctx->pin_y.p, d_sum, sizeof(fe<F>), hipMemcpyDeviceToHost, st));
    VK_CHECK_HIP(hipStreamSynchronize(st));
    *partial = *ctx->pin_y.as<fe<F>>();
    return VC_OK;
}
// phase 2: with the members' total, in domain q_m = -w^-m total (written by the share holding
// m), outside y = -t total ((z^n - 1) / n) and q_i = (f_i - y) inv_i; *y_mont = y outside
template <class F>
int kzg_range_finish(vc_ctx* ctx, size_t n, const fe<F>* d_f, size_t nvalid, size_t lo, size_t L, const fe<F>& point,
                     const fe<F>& omega, bool in_domain, size_t m, const fe<F>& total, fe<F>* d_q, const fe<F>* d_inv,
                     fe<F>* y_mont) {
    if (in_domain) {
        const fe<F> wminv = host_pow<F>(omega, (n - m) & (n - 1));
        if (m >= lo && m < lo + L)
            VK_LAUNCH(ctx, "kzg_set", (k_set<F>), 1, 64, 0, d_q, m - lo, fe_mul<F>(fe_neg<F>(wminv), total));
        return VC_OK;
    }
    fe<F> nn = fe_zero<F>();
    nn.v[0] = (uint32_t)n;
    nn.v[1] = (uint32_t)((uint64_t)n >> 32);
    const fe<F> t = fe_mul<F>(fe_sub<F>(host_pow<F>(point, n), fe_one<F>()), fe_inv_bin<F>(fe_to_mont<F>(nn)));
    const fe<F> y = fe_mul<F>(fe_neg<F>(t), total);
    *y_mont = y;
    if (L) VK_LAUNCH(ctx, "kzg_q_out", (k_q_out_v<F>), (L + 255) / 256, 256, 0, d_f, nvalid, d_inv, L, y, d_q);
    return VC_OK;
}

template <class F>
int canon_to_mont_dev(vc_ctx* ctx, const void* d_in, size_t n, size_t n_valid, fe<F>* d_out) {
    VK_LAUNCH(ctx, "to_mont", (k_canon_to_mont<F>), (n + 255) / 256, 256, 0, reinterpret_cast<const fe<F>*>(d_in), n,
              n_valid, d_out);
    return VC_OK;
}
template <class F>
int mont_to_canon_dev(vc_ctx* ctx, const fe<F>* d_in, size_t n, void* d_out) {
    VK_LAUNCH(ctx, "to_canon", (k_mont_to_canon<F>), (n + 255) / 256, 256, 0, d_in, n, reinterpret_cast<fe<F>*>(d_out));
    return VC_OK;
}

// Lagrange SRS points (projective accumulators) for max_items over a domain of size n
template <class C, class Fr>
int kzg_srs_dev(vc_ctx* ctx, size_t max_items, size_t n, const fe<Fr>& s_mont, const fe<Fr>& omega,
                const typename C::Aff& g, typename C::Acc* d_out) {
    DevBuf pwi, num, den;
    VK_TRY(pwi.ensure(n * sizeof(fe<Fr>)));
    VK_TRY(num.ensure(n * sizeof(fe<Fr>)));
    VK_TRY(den.ensure(n * sizeof(fe<Fr>)));
    fe<Fr> winv = fe_inv_bin<Fr>(omega);
    VK_TRY(domain_powers<Fr>(ctx, winv, n, pwi.as<fe<Fr>>()));
    fe<Fr> nn = fe_zero<Fr>();
    nn.v[0] = (uint32_t)n;
    nn.v[1] = (uint32_t)((uint64_t)n >> 32);
    fe<Fr> ninv = fe_inv_bin<Fr>(fe_to_mont<Fr>(nn));
    VK_LAUNCH(ctx, "srs_num_den", (k_srs_num_den<Fr>), (n + 255) / 256, 256, 0, pwi.as<fe<Fr>>(), n, s_mont,
              (uint64_t)max_items, ninv, num.as<fe<Fr>>(), den.as<fe<Fr>>());
    VK_TRY(batch_inverse<Fr>(ctx, den.as<fe<Fr>>(), pwi.as<fe<Fr>>(), n));  // pwi no longer needed
    VK_LAUNCH(ctx, "srs_mul", (k_mul_elem<Fr>), (n + 255) / 256, 256, 0, num.as<fe<Fr>>(), pwi.as<fe<Fr>>(), n);
    VK_LAUNCH(ctx, "srs_points", (k_fixed_mul_gen<C, Fr>), (n + 127) / 128, 128, 0, num.as<fe<Fr>>(), n, g, d_out);
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

// explicit instantiations
#define VK_INST_F(F)                                                                                   \
    template int domain_powers<F>(vc_ctx*, const fe<F>&, size_t, fe<F>*);                             \
    template int batch_inverse<F>(vc_ctx*, const fe<F>*, fe<F>*, size_t);                                           \
    template int domain_tables<F>(vc_ctx*, const fe<F>&, size_t, const fe<F>**, const fe<F>**, const fe<F>**); \
    template int kzg_quotient_dev<F>(vc_ctx*, size_t, const fe<F>*, size_t, const fe<F>&, const fe<F>&, \
                                     fe<F>*, fe<F>*, DevBuf&, DevBuf&, DevBuf&);                       \
    template int canon_to_mont_dev<F>(vc_ctx*, const void*, size_t, size_t, fe<F>*);                  \
    template int mont_to_canon_dev<F>(vc_ctx*, const fe<F>*, size_t, void*);                           \
    template int kzg_range_part<F>(vc_ctx*, size_t, const fe<F>*, size_t, size_t, size_t, const fe<F>&, \
                                   const fe<F>&, bool, size_t, const fe<F>&, fe<F>*, fe<F>*, DevBuf&, fe<F>*); \
    template int kzg_range_finish<F>(vc_ctx*, size_t, const fe<F>*, size_t, size_t, size_t, const fe<F>&, \
                                     const fe<F>&, bool, size_t, const fe<F>&, fe<F>*, const fe<F>*, fe<F>*);
VK_INST_F(BN254Fr)
VK_INST_F(BLS381Fr)
template int kzg_srs_dev<BN254G1, BN254Fr>(vc_ctx*, size_t, size_t, const fe<BN254Fr>&, const fe<BN254Fr>&,
                                           const BN254G1::Aff&, BN254G1::Acc*);
template int kzg_srs_dev<BLS381G1, BLS381Fr>(vc_ctx*, size_t, size_t, const fe<BLS381Fr>&, const fe<BLS381Fr>&,
                                             const BLS381G1::Aff&, BLS381G1::Acc*);

}  // namespace vk
