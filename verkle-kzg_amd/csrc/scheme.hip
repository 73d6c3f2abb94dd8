// Protocol layer on the GPU engine (reference: vector-commit/src/{ipa,kzg}/mod.rs,
// multiproof.rs, lagrange_basis.rs, precompute.rs). Serial Fiat-Shamir stays on the host
// (scheme_host.cpp); every MSM, batch of commitments, quotient and big field pass runs on
// the device.
//
// IPA prover without point folding: the reference folds the generators every round
// (vec_add_and_distribute on points, utils.rs:31-38 -- m full scalar multiplications per
// round). Here the folded generator g^(k)_j is kept as scalar coefficients over the ORIGINAL
// CRS (coeff_i, the prover-side twin of the verifier's points_coeffs), so each round's
// L and R are two width-(N+1) fixed-base commitments (q is base N) served by the
// precomputed window tables of commit.hip. Same group elements, no point folding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "ec.hpp"
#include "ff29.hpp"
#include "poly.hpp"
#include "scheme_internal.hpp"
#include "host/pool.hpp"

namespace vk {

using F = BN254Fr;
using C = BN254G1;
using Acc = C::Acc;

// ---------------------------------------------------------------- host point helpers
static Acc acc_of(const uint64_t* xy, bool inf) {
    if (inf) return C::zero();
    Acc a;
    a.x = canon_to_mont<BN254Fq>(xy);
    a.y = canon_to_mont<BN254Fq>(xy + 4);
    a.zz = fe_one<BN254Fq>();
    a.zzz = fe_one<BN254Fq>();
    return a;
}
static void aff_of(const Acc& a, uint64_t* xy, uint8_t* inf) {
    acc_to_affine(VC_CURVE_BN254, reinterpret_cast<const uint32_t*>(&a), xy, inf);
}
static Fr fr_of(const uint64_t* w) { return canon_to_mont<F>(w); }
static void canon_of(const Fr& a, uint64_t* w) { mont_to_canon<F>(a, w); }

static std::vector<Fr> host_batch_inv(const std::vector<Fr>& v) {
    std::vector<Fr> pre(v.size());
    Fr acc = fe_one<F>();
    for (size_t i = 0; i < v.size(); i++) {
        pre[i] = acc;
        if (!fe_is_zero<F>(v[i])) acc = fe_mul<F>(acc, v[i]);
    }
    Fr inv = fe_inv_bin<F>(acc);
    std::vector<Fr> out(v.size());
    for (size_t i = v.size(); i-- > 0;) {
        if (fe_is_zero<F>(v[i])) {
            out[i] = fe_zero<F>();
            continue;
        }
        out[i] = fe_mul<F>(inv, pre[i]);
        inv = fe_mul<F>(inv, v[i]);
    }
    return out;
}

static Fr fr_u64(uint64_t v) { return mont_from_u64<F>(v); }

// PrecomputedLagrange::compute_barycentric_coefficients (precompute.rs:72-90)
static std::vector<Fr> barycentric(size_t size, const Fr& point, const Fr& omega) {
    std::vector<Fr> res(size, fe_zero<F>());
    Fr pc = fe_from_mont<F>(point);
    bool small = true;
    for (int i = 2; i < 8; i++) small &= pc.v[i] == 0;
    uint64_t pv = (uint64_t)pc.v[0] | ((uint64_t)pc.v[1] << 32);
    if (small && pv < size) {
        res[pv] = fe_one<F>();
        return res;
    }
    Fr t = fe_mul<F>(fe_sub<F>(fe_pow_u64<F>(point, size), fe_one<F>()), fe_inv_bin<F>(fr_u64(size)));
    std::vector<Fr> pw(size), den(size);
    Fr w = fe_one<F>();
    for (size_t i = 0; i < size; i++) {
        pw[i] = w;
        den[i] = fe_sub<F>(point, w);
        w = fe_mul<F>(w, omega);
    }
    std::vector<Fr> inv = host_batch_inv(den);
    for (size_t i = 0; i < size; i++) res[i] = fe_mul<F>(fe_mul<F>(t, pw[i]), inv[i]);
    return res;
}

// compute_barycentric_coefficients divides by (point - w^i) for every i (precompute.rs:85,
// ark-ff Div = inverse().unwrap()): a point that is a domain element w^i but not below `size`
// as an integer (the one-hot branch, :75-79) makes the reference panic. host_batch_inv maps 1/0
// to 0, which would give all-zero weights and let verify accept y = 0 for any commitment, so
// the callers map this case to VC_E_DOMAIN instead (as the KZG B.4 panic).
static bool barycentric_panics(size_t size, const Fr& point) {
    Fr pc = fe_from_mont<F>(point);
    bool small = true;
    for (int i = 2; i < 8; i++) small &= pc.v[i] == 0;
    uint64_t pv = (uint64_t)pc.v[0] | ((uint64_t)pc.v[1] << 32);
    if (small && pv < size) return false;
    // point^size == 1  <=>  point is one of the size-th roots of unity w^i
    return fe_eq<F>(fe_pow_u64<F>(point, size), fe_one<F>());
}

// (zero b entries skipped: the in-domain barycentric weights are one-hot, so the IPA prover's
// evaluation and its first round's inner products are one product instead of N and N / 2)
static Fr inner(const Fr* a, const Fr* b, size_t n) {
    Fr s = fe_zero<F>();
    for (size_t i = 0; i < n; i++)
        if (!fe_is_zero<F>(b[i])) s = fe_add<F>(s, fe_mul<F>(a[i], b[i]));
    return s;
}

static bool is_pow2(size_t n) { return n && !(n & (n - 1)); }

// VKZG_HOST_TIMING=1: the IPA prover's / verifier's and the multiproof verifier's host and GPU phases on stderr (probe)
static double verify_clock_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool verify_timing() {
    static const bool on = getenv("VKZG_HOST_TIMING") && atoi(getenv("VKZG_HOST_TIMING")) != 0;
    return on;
}

// width-w fixed-base commitments of Montgomery scalars (host) -> canonical affine (host)
// overlap: host work run while the commit kernel runs (fb_commit_t)
// cols (optional, latency path only -- fb_small_path): compacted rows (ctx.hpp StrideCols)
static int commit_batch(vc_ctx* ctx, Table* t, size_t width, const Fr* sc, size_t batch, uint64_t* out_xy,
                        uint8_t* out_inf, const std::function<void()>* overlap = nullptr,
                        const StrideCols* cols = nullptr) {
    const size_t in_bytes = batch * width * 32, out_bytes = batch * 65;
    VK_TRY(ctx->ws[WS_MISC].ensure(out_bytes));
    uint8_t* dxy = ctx->ws[WS_MISC].as<uint8_t>();
    uint8_t* dinf = dxy + batch * 64;
    // pinned staging both ways (the IPA rounds call this 8 times per proof: pageable copies went
    // through bounce buffers), points and flags read back in one copy; the scalars are uploaded by
    // msm_batch_run, or read in place by its latency path
    VK_TRY(ctx->pin_io.ensure(std::max(in_bytes, out_bytes)));
    memcpy(ctx->pin_io.p, sc, in_bytes);
    bool on_host = false;
    VK_TRY(msm_batch_run(ctx, t, width, nullptr, batch, 1, dxy, dinf, out_xy, out_inf, &on_host, &ctx->pin_io,
                         overlap, cols));
    if (on_host) return VC_OK;
    VK_CHECK_HIP(hipMemcpyAsync(ctx->pin_io.p, dxy, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    memcpy(out_xy, ctx->pin_io.p, batch * 64);
    memcpy(out_inf, static_cast<const uint8_t*>(ctx->pin_io.p) + batch * 64, batch);
    return VC_OK;
}

// Straus on the host pool for the verifiers' few-point MSMs (IPA verify: C and the 2K proof
// points L_k / R_k, 17 at N = 256): on the GPU every term pays the Pippenger pipeline's fixed
// latency (upload, sort, accumulate, fix-up, reductions: ~0.25 ms for 17 points); here each pool
// thread takes a slice of the points -- 4-bit windows over 15 precomputed multiples, 252 shared
// doublings -- and the slices are added (~0.1 ms). The points are checked as bases_fill checks
// them (canonical coordinates, on the curve: VC_E_NOT_ON_CURVE).
constexpr size_t HOST_MSM_MAX = 64;
static int host_msm(const uint64_t* xy, const uint8_t* inf, const Fr* sc, size_t n, Acc* out) {
    using Fq = BN254Fq;
    std::vector<Acc> base(n, C::zero());
    for (size_t i = 0; i < n; i++) {
        if (inf[i]) continue;
        fe<Fq> x, y;
        memcpy(x.v, xy + 8 * i, 32);
        memcpy(y.v, xy + 8 * i + 4, 32);
        if (!fe_eq<Fq>(fe_reduce_once<Fq>(x), x) || !fe_eq<Fq>(fe_reduce_once<Fq>(y), y)) return VC_E_NOT_ON_CURVE;
        x = fe_to_mont<Fq>(x);
        y = fe_to_mont<Fq>(y);
        fe<Fq> b = fe_zero<Fq>();
        b.v[0] = (uint32_t)C::COEFF_B;
        if (!fe_eq<Fq>(fe_add<Fq>(fe_mul<Fq>(fe_sqr<Fq>(x), x), fe_to_mont<Fq>(b)), fe_sqr<Fq>(y)))
            return VC_E_NOT_ON_CURVE;
        base[i].x = x;
        base[i].y = y;
        base[i].zz = fe_one<Fq>();
        base[i].zzz = fe_one<Fq>();
    }
    HostPool& pool = host_pool();
    const unsigned T = (unsigned)std::max<size_t>(1, std::min<size_t>(pool.size(), n));
    std::vector<Acc> part(T, C::zero());
    pool.run([&](unsigned k) {
        if (k >= T) return;
        const size_t lo = n * k / T, hi = n * (k + 1) / T;
        std::vector<Acc> mult((hi - lo) * 16);
        std::vector<Fr> can(hi - lo);
        for (size_t i = lo; i < hi; i++) {
            Acc* m = &mult[(i - lo) * 16];
            m[1] = base[i];
            m[2] = C::dbl(base[i]);
            for (int j = 3; j < 16; j++) m[j] = C::add(m[j - 1], base[i]);
            can[i - lo] = fe_from_mont<F>(sc[i]);
        }
        Acc acc = C::zero();
        for (int w = 63; w >= 0; w--) {  // nibbles of the 256-bit canonical scalars, top first
            if (!C::is_zero(acc))
                for (int d = 0; d < 4; d++) acc = C::dbl(acc);
            for (size_t i = lo; i < hi; i++) {
                const uint32_t nib = (can[i - lo].v[w >> 3] >> (4 * (w & 7))) & 15u;
                if (nib) acc = C::add(acc, mult[(i - lo) * 16 + nib]);
            }
        }
        part[k] = acc;
    });
    Acc r = C::zero();
    for (const Acc& p : part) r = C::add(r, p);
    *out = r;
    return VC_OK;
}

// variable-base MSM over host points (ctx scratch table) with Montgomery scalars -> Acc
// filled: the points are in ctx->scratch already (bases_fill run by the caller)
static int msm_points(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, const std::vector<Fr>& sc, Acc* out,
                      bool filled = false) {
    size_t n = sc.size();
    if (n <= HOST_MSM_MAX) return host_msm(xy, inf, sc.data(), n, out);
    const double c0 = verify_timing() ? verify_clock_us() : 0.0;
    if (!filled) VK_TRY(bases_fill(ctx, &ctx->scratch, xy, inf, n));
    if (verify_timing()) {
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        fprintf(stderr, "msm_points n=%zu bases_fill_us=%.1f\n", n, verify_clock_us() - c0);
    }
    DevBuf d(ctx);
    VK_TRY(d.ensure(std::max<size_t>(n, 1) * 32));
    VK_CHECK_HIP(hipMemcpyAsync(d.p, sc.data(), n * 32, hipMemcpyHostToDevice, ctx->stream));
    VK_TRY(msm_run(ctx, &ctx->scratch, 0, d.p, n, 1, reinterpret_cast<uint32_t*>(out)));
    return VC_OK;
}

// ---------------------------------------------------------------- IPA prove (a8/a9)
struct IpaState {
    std::vector<Fr> a, b, coeff;
    Fr eval, w;
    vc_transcript* tr;
    bool own;
};

int ipa_prove_impl(vc_ctx* ctx, Table* t, size_t N, const std::vector<std::vector<Fr>>& data,
                   const std::vector<Acc>& coms, const std::vector<Fr>& points, vc_transcript** trs,
                   vc_ipa_proof* proofs) {
    const size_t B = data.size();
    if (!is_pow2(N) || t->n < N + 1) return VC_E_INVALID;
    size_t K = 0;
    while ((1ull << K) < N) K++;
    Fr omega = bn254_group_gen(N);
    std::vector<IpaState> st(B);
    for (size_t p = 0; p < B; p++) {
        if (proofs[p].rounds < K || !proofs[p].l_xy || !proofs[p].r_xy || !proofs[p].l_inf || !proofs[p].r_inf)
            return VC_E_INVALID;
        if (barycentric_panics(N, points[p])) return VC_E_DOMAIN;
    }
    // the per-proof host work (barycentric weights, transcripts, scalar rows, folds: ~600 field
    // multiplies per proof per round) is independent across proofs: up to 16 host threads
    auto par_for = [&](auto fn) { pool_for(0, B, 16, fn); };  // the persistent host pool (host/pool.hpp)
    par_for([&](size_t p) {
        IpaState& s = st[p];
        s.a = data[p];
        s.b = barycentric(N, points[p], omega);
        s.eval = inner(s.a.data(), s.b.data(), N);
        s.own = !(trs && trs[p]);
        s.tr = s.own ? vc_transcript_new("ipa") : trs[p];
        uint64_t cxy[8];
        uint8_t cinf;
        aff_of(coms[p], cxy, &cinf);
        transcript_append_point(s.tr, cxy, cinf, "C");
        transcript_append_fr(s.tr, points[p], "input point");
        transcript_append_fr(s.tr, s.eval, "output point");
        s.w = transcript_digest(s.tr, "w");
        s.coeff.assign(N, fe_one<F>());
    });
    // L (R) of a round has non-zeros only at the N / 2 bases i with i mod m >= m / 2 (< m / 2) and
    // at q. VKZG_IPA_COMPACT=1 (A/B probe) compacts the rows to those N / 2 + 1 bases on the latency
    // path: half the threads and half the block partials the host adds, but measured slower (prove
    // 0.80 vs 0.77 ms, kernel 62 vs 56 us per round: profiles/r05/ipa_compact/) -- the zero lanes of
    // the full rows make the first adds of the block tree identity adds, which the compacted rows
    // replace by real ones. Off by default.
    static const bool compact_env = getenv("VKZG_IPA_COMPACT") && atoi(getenv("VKZG_IPA_COMPACT")) == 1;
    const bool compact = compact_env && fb_small_path(ctx, t, N / 2 + 1, 2 * B);
    const size_t W = compact ? N / 2 + 1 : N + 1;
    // the rows on the device (IpaRows, the latency path's commit kernel): the host keeps a, b and
    // the q' <a, b> terms; the coefficient rows live in device memory and are folded there.
    // VKZG_IPA_DEV_ROWS=0 (read once; A/B probe): the host builds every row.
    static const bool dev_rows_env = !(getenv("VKZG_IPA_DEV_ROWS") && atoi(getenv("VKZG_IPA_DEV_ROWS")) == 0);
    const bool dev_rows = dev_rows_env && !compact && fb_small_path(ctx, t, N + 1, 2 * B);
    DevBuf d_coeff(ctx);
    std::vector<Fr> ones;  // round 0's coefficients (the upload reads it until the first round ends)
    Fr *pa = nullptr, *px = nullptr, *pq = nullptr;
    const uint8_t* dbase = nullptr;
    if (dev_rows) {
        VK_TRY(d_coeff.ensure(2 * B * N * 32));
        ones.assign(B * N, fe_one<F>());
        VK_CHECK_HIP(hipMemcpyAsync(d_coeff.p, ones.data(), B * N * 32, hipMemcpyHostToDevice, ctx->stream));
        VK_TRY(ctx->pin_ipa.ensure((B * N + 3 * B) * 32));
        pa = ctx->pin_ipa.as<Fr>();
        px = pa + B * N;
        pq = px + B;
        dbase = static_cast<const uint8_t*>(ctx->pin_ipa.dp);
    }
    std::vector<Fr> sc(dev_rows ? 0 : 2 * B * W);
    std::vector<uint64_t> oxy(2 * B * 8);
    std::vector<uint8_t> oinf(2 * B);
    double lap_fill = 0, lap_commit = 0, lap_fold = 0;
    for (size_t r = 0; r < K; r++) {
        const size_t m = N >> r, half = m / 2;
        const double c0 = verify_timing() ? verify_clock_us() : 0.0;
        if (dev_rows) {
            par_for([&](size_t p) {
                IpaState& s = st[p];
                memcpy(pa + p * N, s.a.data(), m * 32);
                pq[2 * p] = fe_mul<F>(s.w, inner(&s.a[0], &s.b[half], half));
                pq[2 * p + 1] = fe_mul<F>(s.w, inner(&s.a[half], &s.b[0], half));
            });
            IpaRows ir;
            ir.a = reinterpret_cast<const uint32_t*>(dbase);
            ir.x = reinterpret_cast<const uint32_t*>(dbase + (size_t)B * N * 32);
            ir.q = reinterpret_cast<const uint32_t*>(dbase + (size_t)(B * N + B) * 32);
            ir.coeff_in = reinterpret_cast<const uint32_t*>(d_coeff.as<uint8_t>() + (r & 1) * B * N * 32);
            ir.coeff_out = reinterpret_cast<uint32_t*>(d_coeff.as<uint8_t>() + ((r + 1) & 1) * B * N * 32);
            ir.N = (uint32_t)N;
            ir.m = (uint32_t)m;
            ir.h = (uint32_t)half;
            ir.fold = r > 0 ? 1u : 0u;
            ir.m_prev = (uint32_t)(2 * m);
            ir.h_prev = (uint32_t)m;
            const double c1 = verify_timing() ? verify_clock_us() : 0.0;
            VK_TRY(ctx->ws[WS_MISC].ensure(2 * B * 65));
            uint8_t* dxy = ctx->ws[WS_MISC].as<uint8_t>();
            bool on_host = false;
            VK_TRY(msm_batch_run(ctx, t, N + 1, nullptr, 2 * B, 1, dxy, dxy + 2 * B * 64, oxy.data(), oinf.data(),
                                 &on_host, nullptr, nullptr, nullptr, &ir));
            if (!on_host) {  // (the latency path returns host results: not expected)
                VK_CHECK_HIP(hipMemcpyAsync(oxy.data(), dxy, 2 * B * 64, hipMemcpyDeviceToHost, ctx->stream));
                VK_CHECK_HIP(hipMemcpyAsync(oinf.data(), dxy + 2 * B * 64, 2 * B, hipMemcpyDeviceToHost, ctx->stream));
                VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
            }
            const double c2 = verify_timing() ? verify_clock_us() : 0.0;
            par_for([&](size_t p) {
                IpaState& s = st[p];
                const uint64_t* Lxy = &oxy[(2 * p) * 8];
                const uint64_t* Rxy = &oxy[(2 * p + 1) * 8];
                memcpy(proofs[p].l_xy + r * 8, Lxy, 64);
                memcpy(proofs[p].r_xy + r * 8, Rxy, 64);
                proofs[p].l_inf[r] = oinf[2 * p];
                proofs[p].r_inf[r] = oinf[2 * p + 1];
                transcript_append_point(s.tr, Lxy, oinf[2 * p], "L");
                transcript_append_point(s.tr, Rxy, oinf[2 * p + 1], "R");
                Fr x = transcript_digest(s.tr, "x");
                // a <- a_L + x a_R ; b <- b_R + x b_L (the coefficients fold on the device)
                for (size_t j = 0; j < half; j++) {
                    s.a[j] = fe_add<F>(s.a[j], fe_mul<F>(x, s.a[j + half]));
                    s.b[j] = fe_add<F>(s.b[j + half], fe_mul<F>(x, s.b[j]));
                }
                s.a.resize(half);
                s.b.resize(half);
                px[p] = x;  // the next round's kernel folds the coefficients by it
            });
            if (verify_timing()) {
                const double c3 = verify_clock_us();
                lap_fill += c1 - c0, lap_commit += c2 - c1, lap_fold += c3 - c2;
            }
            continue;
        }
        // L (even commits): bases i with i mod m >= half, R (odd): i mod m < half, in index order
        // -- the k-th is (k / half) m + k mod half (+ half for L) --, then q
        StrideCols cols;
        if (compact) {
            cols.half = (uint32_t)half;
            cols.m = (uint32_t)m;
            cols.off_even = (uint32_t)half;
            cols.off_odd = 0;
            cols.n_main = (uint32_t)(N / 2);
            cols.extra = (uint32_t)N;
        }
        par_for([&](size_t p) {
            IpaState& s = st[p];
            Fr* sL = &sc[(2 * p) * W];
            Fr* sR = &sc[(2 * p + 1) * W];
            if (compact) {
                size_t kl = 0, kr = 0;
                for (size_t i = 0; i < N; i++) {
                    size_t j = i % m;
                    if (j >= half) sL[kl++] = fe_mul<F>(s.a[j - half], s.coeff[i]);
                    else sR[kr++] = fe_mul<F>(s.a[j + half], s.coeff[i]);
                }
            } else {
                // (round 0: every coefficient is one -- the rows are a's halves as they are)
                for (size_t i = 0; i < N; i++) {
                    size_t j = i % m;
                    if (j >= half) {
                        sL[i] = r == 0 ? s.a[j - half] : fe_mul<F>(s.a[j - half], s.coeff[i]);
                        sR[i] = fe_zero<F>();
                    } else {
                        sR[i] = r == 0 ? s.a[j + half] : fe_mul<F>(s.a[j + half], s.coeff[i]);
                        sL[i] = fe_zero<F>();
                    }
                }
            }
            // q' * <a_L, b_R> = q * (w <a_L, b_R>)
            sL[W - 1] = fe_mul<F>(s.w, inner(&s.a[0], &s.b[half], half));
            sR[W - 1] = fe_mul<F>(s.w, inner(&s.a[half], &s.b[0], half));
        });
        const double c1 = verify_timing() ? verify_clock_us() : 0.0;
        VK_TRY(commit_batch(ctx, t, W, sc.data(), 2 * B, oxy.data(), oinf.data(), nullptr,
                            compact ? &cols : nullptr));
        const double c2 = verify_timing() ? verify_clock_us() : 0.0;
        par_for([&](size_t p) {
            IpaState& s = st[p];
            const uint64_t* Lxy = &oxy[(2 * p) * 8];
            const uint64_t* Rxy = &oxy[(2 * p + 1) * 8];
            memcpy(proofs[p].l_xy + r * 8, Lxy, 64);
            memcpy(proofs[p].r_xy + r * 8, Rxy, 64);
            proofs[p].l_inf[r] = oinf[2 * p];
            proofs[p].r_inf[r] = oinf[2 * p + 1];
            transcript_append_point(s.tr, Lxy, oinf[2 * p], "L");
            transcript_append_point(s.tr, Rxy, oinf[2 * p + 1], "R");
            Fr x = transcript_digest(s.tr, "x");
            // a <- a_L + x a_R ; b <- b_R + x b_L ; g <- g_R + x g_L (coefficients)
            for (size_t j = 0; j < half; j++) {
                s.a[j] = fe_add<F>(s.a[j], fe_mul<F>(x, s.a[j + half]));
                s.b[j] = fe_add<F>(s.b[j + half], fe_mul<F>(x, s.b[j]));
            }
            s.a.resize(half);
            s.b.resize(half);
            for (size_t i = 0; i < N; i++)
                if ((i % m) < half) s.coeff[i] = fe_mul<F>(s.coeff[i], x);
        });
        if (verify_timing()) {
            const double c3 = verify_clock_us();
            lap_fill += c1 - c0, lap_commit += c2 - c1, lap_fold += c3 - c2;
        }
    }
    if (verify_timing())
        fprintf(stderr, "[ipa_prove] %zu proofs x %zu rounds: rows %.1f us, L/R commits %.1f us, transcript + folds %.1f us\n",
                B, K, lap_fill, lap_commit, lap_fold);
    for (size_t p = 0; p < B; p++) {
        proofs[p].rounds = K;
        canon_of(st[p].a[0], proofs[p].tip);
        canon_of(st[p].eval, proofs[p].y);
        if (st[p].own) vc_transcript_free(st[p].tr);
    }
    return VC_OK;
}

// ---------------------------------------------------------------- IPA verify (a10)
int ipa_verify_impl(vc_ctx* ctx, Table* t, size_t N, const Acc& com, const Fr& point, const vc_ipa_proof* pr,
                    vc_transcript* tr_in, int* result) {
    if (!is_pow2(N) || t->n < N + 1) return VC_E_INVALID;
    size_t K = pr->rounds;
    if ((1ull << K) != N) return VC_E_INVALID;  // gens = g[0..2^rounds], zip with points_coeffs
    const double t0 = verify_timing() ? verify_clock_us() : 0.0;
    Fr omega = bn254_group_gen(N);
    if (barycentric_panics(N, point)) return VC_E_DOMAIN;
    std::vector<Fr> b = barycentric(N, point, omega);
    bool own = tr_in == nullptr;
    vc_transcript* tr = own ? vc_transcript_new("ipa") : tr_in;
    uint64_t cxy[8];
    uint8_t cinf;
    aff_of(com, cxy, &cinf);
    Fr y = fr_of(pr->y), tip = fr_of(pr->tip);
    transcript_append_point(tr, cxy, cinf, "C");
    transcript_append_fr(tr, point, "input point");
    transcript_append_fr(tr, y, "output point");
    Fr w = transcript_digest(tr, "w");
    std::vector<Fr> xs(K);
    for (size_t k = 0; k < K; k++) {
        transcript_append_point(tr, pr->l_xy + 8 * k, pr->l_inf[k], "L");
        transcript_append_point(tr, pr->r_xy + 8 * k, pr->r_inf[k], "R");
        xs[k] = transcript_digest(tr, "x");
    }
    if (own) vc_transcript_free(tr);
    // points_coeffs: [1] -> each round c -> [c x, c]
    std::vector<Fr> s(1, fe_one<F>());
    for (size_t k = 0; k < K; k++) {
        std::vector<Fr> ns(2 * s.size());
        for (size_t i = 0; i < s.size(); i++) {
            ns[2 * i] = fe_mul<F>(s[i], xs[k]);
            ns[2 * i + 1] = s[i];
        }
        s.swap(ns);
    }
    Fr cb = inner(b.data(), s.data(), N);
    Fr prodx = fe_one<F>();
    for (auto& x : xs) prodx = fe_mul<F>(prodx, x);
    // fixed part over (g, q): -tip*s_i, (prodx*w*y - w*tip*<b,s>)
    std::vector<Fr> fs(N + 1);
    for (size_t i = 0; i < N; i++) fs[i] = fe_neg<F>(fe_mul<F>(tip, s[i]));
    fs[N] = fe_sub<F>(fe_mul<F>(fe_mul<F>(prodx, w), y), fe_mul<F>(fe_mul<F>(w, tip), cb));
    // variable part: prodx*C + sum_k P_k L_k + P_k x_k^2 R_k,  P_k = prod_{j>k} x_j
    std::vector<uint64_t> vxy(8 * (1 + 2 * K));
    std::vector<uint8_t> vinf(1 + 2 * K);
    std::vector<Fr> vs(1 + 2 * K);
    memcpy(&vxy[0], cxy, 64);
    vinf[0] = cinf;
    vs[0] = prodx;
    Fr P = fe_one<F>();
    for (size_t k = K; k-- > 0;) {
        memcpy(&vxy[8 * (1 + 2 * k)], pr->l_xy + 8 * k, 64);
        memcpy(&vxy[8 * (2 + 2 * k)], pr->r_xy + 8 * k, 64);
        vinf[1 + 2 * k] = pr->l_inf[k];
        vinf[2 + 2 * k] = pr->r_inf[k];
        vs[1 + 2 * k] = P;
        vs[2 + 2 * k] = fe_mul<F>(P, fe_sqr<F>(xs[k]));
        P = fe_mul<F>(P, xs[k]);
    }
    // the fixed part on the GPU, the variable part's Straus (<= HOST_MSM_MAX points: host pool)
    // while its kernel runs
    uint64_t axy[8];
    uint8_t ainf;
    Acc vb;
    int vst = VC_OK;
    double t_straus = 0.0;
    bool ran = false;
    const bool on_host = vs.size() <= HOST_MSM_MAX;
    const std::function<void()> straus = [&] {
        ran = true;
        const double s0 = verify_timing() ? verify_clock_us() : 0.0;
        vst = msm_points(ctx, vxy.data(), vinf.data(), vs, &vb);
        if (verify_timing()) t_straus = verify_clock_us() - s0;
    };
    const double t1 = verify_timing() ? verify_clock_us() : 0.0;
    VK_TRY(commit_batch(ctx, t, N + 1, fs.data(), 1, axy, &ainf, on_host ? &straus : nullptr));
    if (!ran) straus();
    VK_TRY(vst);
    if (verify_timing())
        fprintf(stderr, "ipa_verify host_prep_us=%.1f commit_and_straus_us=%.1f (straus %.1f)\n", t1 - t0,
                verify_clock_us() - t1, t_straus);
    Acc tot = C::add(acc_of(axy, ainf), vb);
    *result = C::is_zero(tot) ? 1 : 0;
    return VC_OK;
}

// ---------------------------------------------------------------- KZG (a3/a4/a5/a6/a7)
template <class Fr_>
static fe<Fr_> group_gen_t(uint64_t n, uint32_t gen) {
    fe<Fr_> e;
    for (int i = 0; i < Fr_::N; i++) e.v[i] = Fr_::p(i);
    e.v[0] -= 1;
    int lg = 0;
    while ((1ull << lg) < n) lg++;
    for (int s = 0; s < lg; s++) {
        for (int i = 0; i < Fr_::N - 1; i++) e.v[i] = (e.v[i] >> 1) | (e.v[i + 1] << 31);
        e.v[Fr_::N - 1] >>= 1;
    }
    return fe_pow_fe<Fr_, Fr_>(mont_from_u64<Fr_>(gen), e);
}
template <class Fr_>
static uint32_t fr_generator();
template <>
uint32_t fr_generator<BN254Fr>() { return 5; }
template <>
uint32_t fr_generator<BLS381Fr>() { return 7; }

// evals: host (d_evals == false) or device canonical scalars; out_acc != nullptr returns the
// un-normalised proof accumulator of window slice `part` of `parts` (multi-GPU) instead of
// the affine proof
template <class C_, class Fr_>
static int kzg_prove_t(vc_ctx* ctx, Table* t, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                       uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y_out, uint64_t* q_out, bool d_evals = false,
                       int part = 0, int parts = 1, uint32_t* out_acc = nullptr, uint64_t* com_xy = nullptr,
                       uint8_t* com_inf = nullptr) {
    if (!is_pow2(size) || max > size) return VC_E_INVALID;
    if (t && t->n < size) return VC_E_RANGE;
    DevBuf d_f(ctx), d_q(ctx), pw(ctx), tmp(ctx), part_buf(ctx);
    VK_TRY(d_f.ensure(size * 32));
    VK_TRY(d_q.ensure(size * 32));
    VK_TRY(tmp.ensure(size * 32));
    const void* ev_dev = tmp.p;
    if (d_evals) ev_dev = evals;
    else if (max > 0) VK_CHECK_HIP(hipMemcpyAsync(tmp.p, evals, max * 32, hipMemcpyHostToDevice, ctx->stream));
    VK_TRY(canon_to_mont_dev<Fr_>(ctx, ev_dev, size, max, d_f.as<fe<Fr_>>()));
    fe<Fr_> pm = canon_to_mont<Fr_>(point);
    fe<Fr_> omega = group_gen_t<Fr_>(size, fr_generator<Fr_>());
    // y arrives in page-locked memory once the stream has passed the quotient (read after a sync)
    VK_TRY(ctx->pin_y.ensure(sizeof(fe<Fr_>)));
    fe<Fr_>* yp = ctx->pin_y.as<fe<Fr_>>();
    VK_TRY(kzg_quotient_dev<Fr_>(ctx, size, d_f.as<fe<Fr_>>(), max, pm, omega, d_q.as<fe<Fr_>>(), yp, pw, tmp,
                                 part_buf));
    struct YOut {  // every return path below has synchronised the stream (or fails)
        vc_ctx* c;
        const fe<Fr_>* yp;
        uint64_t* out;
        ~YOut() {
            if (hipStreamSynchronize(c->stream) == hipSuccess) mont_to_canon<Fr_>(*yp, out);
        }
    } y_fin{ctx, yp, y_out};
    if (q_out) {
        VK_TRY(mont_to_canon_dev<Fr_>(ctx, d_q.as<fe<Fr_>>(), size, tmp.p));
        VK_CHECK_HIP(hipMemcpyAsync(q_out, tmp.p, size * 32, hipMemcpyDeviceToHost, ctx->stream));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    }
    if (t && com_xy) {  // commitment + proof: the two MSMs over the SRS as one batched pipeline
        const void* sc[2] = {d_f.p, d_q.p};
        const int mt[2] = {1, 1};
        const int words = point_words(ctx->curve);
        std::vector<uint32_t> acc(2 * (size_t)words);
        VK_TRY(msm_run_many(ctx, t, sc, mt, size, 2, acc.data()));
        VK_TRY(acc_to_affine(ctx->curve, acc.data(), com_xy, com_inf));
        VK_TRY(acc_to_affine(ctx->curve, acc.data() + words, proof_xy, proof_inf));
    } else if (t && out_acc) {
        VK_TRY(msm_run(ctx, t, 0, d_q.p, size, 1, out_acc, part, parts));
    } else if (t && t->fb_c != 0 && size <= 1024) {
        // a small proof MSM over a table that has fixed-base window tables (vc_fixed_base_precompute):
        // the batched commit's latency path -- one launch, the block partials added on the host --
        // instead of a Pippenger pipeline of ~12 latency-bound launches (benches/kzg.rs: 32 terms)
        const size_t xyb = (size_t)C_::F::N * 8;  // canonical affine x, y
        VK_TRY(ctx->ws[WS_MISC].ensure(xyb + 1));
        uint8_t* dxy = ctx->ws[WS_MISC].as<uint8_t>();
        bool on_host = false;
        VK_TRY(msm_batch_run(ctx, t, size, d_q.p, 1, 1, dxy, dxy + xyb, proof_xy, proof_inf, &on_host));
        if (!on_host) {
            VK_CHECK_HIP(hipMemcpyAsync(proof_xy, dxy, xyb, hipMemcpyDeviceToHost, ctx->stream));
            VK_CHECK_HIP(hipMemcpyAsync(proof_inf, dxy + xyb, 1, hipMemcpyDeviceToHost, ctx->stream));
            VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        }
    } else if (t) {
        std::vector<uint32_t> acc(point_words(ctx->curve));
        VK_TRY(msm_run(ctx, t, 0, d_q.p, size, 1, acc.data()));
        VK_TRY(acc_to_affine(ctx->curve, acc.data(), proof_xy, proof_inf));
    }
    return VC_OK;
}

// ---------------------------------------------------------------- FK all-point openings (f4)
// KZG::prove_all_points (kzg/mod.rs:200-235): radix-2 FFTs over G1 (a butterfly multiplies a
// point by a twiddle: one double-and-add scalar multiplication) and over Fr, natural-order in and
// out (bit reversal, then iterative Cooley-Tukey), as ark-poly's Radix2EvaluationDomain computes
// them (fft: y_i = sum_j a_j w^(ij); ifft: a_j = n^-1 sum_i y_i w^(-ij)). Dead code in the
// reference (no caller; its test at :299 has no #[test]); see DESIGN.md for both modes.
template <class C, class Fr_>
__device__ typename C::Acc pt_mul_fe(const typename C::Acc& p, const fe<Fr_>& k_mont) {
    const fe<Fr_> k = fe_from_mont<Fr_>(k_mont);
    typename C::Acc r = C::zero();
    bool started = false;
    for (int i = Fr_::N * 32 - 1; i >= 0; i--) {
        const bool bit = (k.v[i >> 5] >> (i & 31)) & 1u;
        if (started) r = C::dbl(r);
        if (bit) {
            r = started ? C::add(r, p) : p;
            started = true;
        }
    }
    return r;
}
__device__ __forceinline__ uint32_t bitrev32(uint32_t i, int lg) { return lg ? (__brev(i) >> (32 - lg)) : 0u; }

template <class T>
__global__ void k_bitrev(const T* __restrict__ in, T* __restrict__ out, uint32_t n, int lg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[bitrev32(i, lg)] = in[i];
}
// one stage (blocks of 2 half): a[i0], a[i1] <- u + w v, u - w v with w = tw[j * step]
template <class C, class Fr_>
__global__ void k_pt_stage(typename C::Acc* __restrict__ a, uint32_t n, uint32_t half, const fe<Fr_>* __restrict__ tw,
                           uint32_t step) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n / 2) return;
    const uint32_t blk = g / half, j = g % half;
    const uint32_t i0 = blk * 2 * half + j, i1 = i0 + half;
    const typename C::Acc u = a[i0];
    const typename C::Acc v = j == 0 ? a[i1] : pt_mul_fe<C, Fr_>(a[i1], tw[j * step]);
    a[i0] = C::add(u, v);
    a[i1] = C::add(u, C::neg(v));
}
template <class Fr_>
__global__ void k_fr_stage(fe<Fr_>* __restrict__ a, uint32_t n, uint32_t half, const fe<Fr_>* __restrict__ tw,
                           uint32_t step) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n / 2) return;
    const uint32_t blk = g / half, j = g % half;
    const uint32_t i0 = blk * 2 * half + j, i1 = i0 + half;
    const fe<Fr_> u = a[i0], v = fe_mul<Fr_>(a[i1], tw[j * step]);
    a[i0] = fe_add<Fr_>(u, v);
    a[i1] = fe_sub<Fr_>(u, v);
}
// a[i] <- a[i] * (s ? s[i] : k)
template <class C, class Fr_>
__global__ void k_pt_scale(typename C::Acc* __restrict__ a, uint32_t n, const fe<Fr_>* __restrict__ s, fe<Fr_> k) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = pt_mul_fe<C, Fr_>(a[i], s ? s[i] : k);
}
template <class Fr_>
__global__ void k_fr_scale(fe<Fr_>* __restrict__ a, uint32_t n, fe<Fr_> k) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = fe_mul<Fr_>(a[i], k);
}
template <class C>
__global__ void k_aff_to_acc(const typename C::Aff* __restrict__ in, const uint8_t* __restrict__ inf, uint32_t n,
                             typename C::Acc* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = inf[i] ? C::zero() : C::from_aff(in[i], false);
}
// out[i] = src[map(i)] or the identity: reversed prefix (mode 0's s_hat) / reversed shifted
// prefix (mode 1's S') / a window (mode 1's h)
template <class C>
__global__ void k_pt_gather(const typename C::Acc* __restrict__ src, uint32_t n, int64_t base, int64_t dir,
                            uint32_t valid, typename C::Acc* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i < valid ? src[base + dir * (int64_t)i] : C::zero();
}

static int lg2_of(size_t n) {
    int lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    return lg;
}
// in-place FFT (inverse: iFFT incl. the 1/n) of n = 2^k points / field elements in a DevBuf
template <class C, class Fr_>
static int pt_fft(vc_ctx* ctx, DevBuf& a, size_t n, bool inverse) {
    using Acc = typename C::Acc;
    if (n <= 1) return VC_OK;
    const int lg = lg2_of(n);
    const fe<Fr_> w = group_gen_t<Fr_>(n, fr_generator<Fr_>());
    DevBuf tw(ctx), tmp(ctx);
    VK_TRY(tw.ensure(n / 2 * sizeof(fe<Fr_>)));
    VK_TRY(tmp.ensure(n * sizeof(Acc)));
    VK_TRY(domain_powers<Fr_>(ctx, inverse ? fe_inv_bin<Fr_>(w) : w, n / 2, tw.as<fe<Fr_>>()));
    const unsigned g = (unsigned)((n + 255) / 256), g2 = (unsigned)((n / 2 + 255) / 256);
    VK_LAUNCH(ctx, "fk_bitrev", (k_bitrev<Acc>), g, 256, 0, a.as<Acc>(), tmp.as<Acc>(), (uint32_t)n, lg);
    for (uint32_t half = 1; half < n; half <<= 1)
        VK_LAUNCH(ctx, "fk_pt_stage", (k_pt_stage<C, Fr_>), g2, 256, 0, tmp.as<Acc>(), (uint32_t)n, half,
                  tw.as<fe<Fr_>>(), (uint32_t)(n / (2 * half)));
    if (inverse)
        VK_LAUNCH(ctx, "fk_pt_scale", (k_pt_scale<C, Fr_>), g, 256, 0, tmp.as<Acc>(), (uint32_t)n,
                  (const fe<Fr_>*)nullptr, fe_inv_bin<Fr_>(mont_from_u64<Fr_>(n)));
    VK_CHECK_HIP(hipMemcpyAsync(a.p, tmp.p, n * sizeof(Acc), hipMemcpyDeviceToDevice, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));  // tw / tmp go back to the pool
    return VC_OK;
}
template <class Fr_>
static int fr_fft(vc_ctx* ctx, DevBuf& a, size_t n, bool inverse) {
    if (n <= 1) return VC_OK;
    const int lg = lg2_of(n);
    const fe<Fr_> w = group_gen_t<Fr_>(n, fr_generator<Fr_>());
    DevBuf tw(ctx), tmp(ctx);
    VK_TRY(tw.ensure(n / 2 * sizeof(fe<Fr_>)));
    VK_TRY(tmp.ensure(n * sizeof(fe<Fr_>)));
    VK_TRY(domain_powers<Fr_>(ctx, inverse ? fe_inv_bin<Fr_>(w) : w, n / 2, tw.as<fe<Fr_>>()));
    const unsigned g = (unsigned)((n + 255) / 256), g2 = (unsigned)((n / 2 + 255) / 256);
    VK_LAUNCH(ctx, "fk_bitrev", (k_bitrev<fe<Fr_>>), g, 256, 0, a.as<fe<Fr_>>(), tmp.as<fe<Fr_>>(), (uint32_t)n, lg);
    for (uint32_t half = 1; half < n; half <<= 1)
        VK_LAUNCH(ctx, "fk_fr_stage", (k_fr_stage<Fr_>), g2, 256, 0, tmp.as<fe<Fr_>>(), (uint32_t)n, half,
                  tw.as<fe<Fr_>>(), (uint32_t)(n / (2 * half)));
    if (inverse)
        VK_LAUNCH(ctx, "fk_fr_scale", (k_fr_scale<Fr_>), g, 256, 0, tmp.as<fe<Fr_>>(), (uint32_t)n,
                  fe_inv_bin<Fr_>(mont_from_u64<Fr_>(n)));
    VK_CHECK_HIP(hipMemcpyAsync(a.p, tmp.p, n * sizeof(fe<Fr_>), hipMemcpyDeviceToDevice, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

// mode 0: the reference's prove_all_points exactly; mode 1: the FK proofs it was meant to return
template <class C, class Fr_>
static int fk_all_t(vc_ctx* ctx, Table* t, size_t size, const uint64_t* evals, size_t ne, int mode,
                    uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_y, size_t* count) {
    using Acc = typename C::Acc;
    if (!is_pow2(size) || t->n < size) return VC_E_INVALID;
    if (ne == 0) return VC_E_DOMAIN;  // the reference: coeffs[degree] of the zero polynomial panics
    const int NL = aff_limbs64(ctx->curve);
    // the Lagrange SRS as projective points
    DevBuf L(ctx);
    VK_TRY(L.ensure(size * sizeof(Acc)));
    VK_LAUNCH(ctx, "fk_aff_to_acc", (k_aff_to_acc<C>), (size + 255) / 256, 256, 0, t->bases.as<typename C::Aff>(),
              t->inf.as<uint8_t>(), (uint32_t)size, L.as<Acc>());
    auto upload_evals = [&](DevBuf& dst, size_t n) -> int {  // evals padded with zeros to n, Montgomery
        DevBuf raw(ctx);
        VK_TRY(dst.ensure(n * sizeof(fe<Fr_>)));
        VK_TRY(raw.ensure(n * 32));
        const size_t m = std::min(ne, n);
        VK_CHECK_HIP(hipMemcpyAsync(raw.p, evals, m * 32, hipMemcpyHostToDevice, ctx->stream));
        VK_TRY(canon_to_mont_dev<Fr_>(ctx, raw.p, n, m, dst.as<fe<Fr_>>()));
        VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        return VC_OK;
    };
    DevBuf out(ctx);  // the D output points
    size_t D = 0;
    if (mode == 0) {
        // data.interpolate() over the data's own domain (LagrangeBasis::from_vec: next_pow2(len))
        size_t m = 1;
        while (m < ne) m <<= 1;
        DevBuf cf(ctx);
        VK_TRY(upload_evals(cf, m));
        VK_TRY(fr_fft<Fr_>(ctx, cf, m, true));
        std::vector<fe<Fr_>> coeffs(m);
        VK_CHECK_HIP(hipMemcpy(coeffs.data(), cf.p, m * sizeof(fe<Fr_>), hipMemcpyDeviceToHost));
        size_t deg = m;
        while (deg > 0 && fe_is_zero<Fr_>(coeffs[deg - 1])) deg--;
        if (deg == 0) return VC_E_DOMAIN;  // zero polynomial: coeffs[degree] out of bounds
        const size_t d = deg - 1;          // poly.degree()
        D = 1;
        while (D < 2 * d) D <<= 1;  // D::new(degree * 2)
        if (D > ne || d > size) return VC_E_DOMAIN;  // data[i] / g1[0..degree] out of bounds
        // c_hat = [c_d, 0^(d+1), c_0 .. c_{d-1}], resized to the domain by fft_in_place
        std::vector<fe<Fr_>> chat(D, fe_zero<Fr_>());
        std::vector<fe<Fr_>> full;
        full.push_back(coeffs[d]);
        full.insert(full.end(), d + 1, fe_zero<Fr_>());
        full.insert(full.end(), coeffs.begin(), coeffs.begin() + d);
        for (size_t i = 0; i < D && i < full.size(); i++) chat[i] = full[i];
        DevBuf yv(ctx);
        VK_TRY(yv.ensure(D * sizeof(fe<Fr_>)));
        VK_CHECK_HIP(hipMemcpy(yv.p, chat.data(), D * sizeof(fe<Fr_>), hipMemcpyHostToDevice));
        VK_TRY(fr_fft<Fr_>(ctx, yv, D, false));
        // g1 = ifft(lagrange_commitments) over the key's domain; s_hat = reverse(g1[0..d]) || O
        VK_TRY((pt_fft<C, Fr_>(ctx, L, size, true)));
        VK_TRY(out.ensure(D * sizeof(Acc)));
        VK_LAUNCH(ctx, "fk_gather", (k_pt_gather<C>), (D + 255) / 256, 256, 0, L.as<Acc>(), (uint32_t)D,
                  (int64_t)d - 1, (int64_t)-1, (uint32_t)d, out.as<Acc>());
        VK_TRY((pt_fft<C, Fr_>(ctx, out, D, false)));  // v
        VK_LAUNCH(ctx, "fk_pt_scale", (k_pt_scale<C, Fr_>), (D + 255) / 256, 256, 0, out.as<Acc>(), (uint32_t)D,
                  yv.as<fe<Fr_>>(), fe_zero<Fr_>());  // u = v .* y
        VK_TRY((pt_fft<C, Fr_>(ctx, out, D, true)));    // h_hat
    } else if (mode == 1) {
        const size_t n = size;
        D = n;
        if (ne > n) return VC_E_RANGE;
        DevBuf c2(ctx);
        VK_TRY(upload_evals(c2, 2 * n));  // zero-padded to 2n; the first n entries are the data
        // coefficients: iFFT over the key domain of the first n entries (the rest stays zero)
        {
            DevBuf cn(ctx);
            VK_TRY(cn.ensure(n * sizeof(fe<Fr_>)));
            VK_CHECK_HIP(hipMemcpyAsync(cn.p, c2.p, n * sizeof(fe<Fr_>), hipMemcpyDeviceToDevice, ctx->stream));
            VK_TRY(fr_fft<Fr_>(ctx, cn, n, true));
            VK_CHECK_HIP(hipMemcpyAsync(c2.p, cn.p, n * sizeof(fe<Fr_>), hipMemcpyDeviceToDevice, ctx->stream));
        }
        VK_TRY(fr_fft<Fr_>(ctx, c2, 2 * n, false));
        // monomial SRS S = fft(L) (setup made L = ifft(S)); S'[i] = S[n - 2 - i] for i <= n - 2
        VK_TRY((pt_fft<C, Fr_>(ctx, L, n, false)));
        DevBuf V(ctx);
        VK_TRY(V.ensure(2 * n * sizeof(Acc)));
        VK_LAUNCH(ctx, "fk_gather", (k_pt_gather<C>), (2 * n + 255) / 256, 256, 0, L.as<Acc>(), (uint32_t)(2 * n),
                  (int64_t)n - 2, (int64_t)-1, (uint32_t)(n - 1), V.as<Acc>());
        VK_TRY((pt_fft<C, Fr_>(ctx, V, 2 * n, false)));
        VK_LAUNCH(ctx, "fk_pt_scale", (k_pt_scale<C, Fr_>), (2 * n + 255) / 256, 256, 0, V.as<Acc>(),
                  (uint32_t)(2 * n), c2.as<fe<Fr_>>(), fe_zero<Fr_>());
        VK_TRY((pt_fft<C, Fr_>(ctx, V, 2 * n, true)));  // the Toeplitz product, h_j at j + n - 1
        VK_TRY(out.ensure(n * sizeof(Acc)));
        VK_LAUNCH(ctx, "fk_gather", (k_pt_gather<C>), (n + 255) / 256, 256, 0, V.as<Acc>(), (uint32_t)n,
                  (int64_t)n - 1, (int64_t)1, (uint32_t)n, out.as<Acc>());
        VK_TRY((pt_fft<C, Fr_>(ctx, out, n, false)));  // proofs at w^i
    } else {
        return VC_E_INVALID;
    }
    DevBuf dxy(ctx), dinf(ctx);
    VK_TRY(dxy.ensure(D * 2 * NL * 8));
    VK_TRY(dinf.ensure(D));
    VK_TRY(normalize_to_canon(ctx, ctx->curve, out.p, D, dxy.p, dinf.as<uint8_t>()));
    VK_CHECK_HIP(hipMemcpy(out_xy, dxy.p, D * 2 * NL * 8, hipMemcpyDeviceToHost));
    VK_CHECK_HIP(hipMemcpy(out_inf, dinf.p, D, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < D; i++)
        for (int k = 0; k < 4; k++) out_y[4 * i + k] = i < ne ? evals[4 * i + k] : 0;
    *count = D;
    return VC_OK;
}

// ---------------------------------------------------------------- multiproof kernels
// one block per z group: q_z[k] = (S_z[k] - S_z[z]) * inv[k] (k != z),
// q_z[z] = -w^-z sum_{k != z} q_z[k] w^k   (divide_by_vanishing, lagrange_basis.rs:91-119)
// 1/(w^k - w^z) = w^-z / (w^(k-z) - 1) = pw_inv[z] inv1[(k - z) mod N]: the per-domain cached
// inv1 table replaces a Z x N denominator pass and its batch inversion (and host round trip)
__global__ void __launch_bounds__(256) k_mp_quot(const fe<F>* __restrict__ S, const fe<F>* __restrict__ inv1,
                                                const fe<F>* __restrict__ pw, const fe<F>* __restrict__ pw_inv,
                                                const uint32_t* __restrict__ zval, size_t N, fe<F>* __restrict__ Q) {
    __shared__ fe<F> sh[256];
    uint32_t zi = blockIdx.x;
    uint32_t z = zval[zi];
    const fe<F>* Sz = S + (size_t)zi * N;
    fe<F> fz = Sz[z];
    const fe<F> wmz = pw_inv[z];
    fe<F> acc = fe_zero<F>();
    for (size_t k = threadIdx.x; k < N; k += 256) {
        fe<F> q = fe_zero<F>();
        if (k != z) {
            q = fe_mul<F>(fe_mul<F>(fe_sub<F>(Sz[k], fz), wmz), inv1[(k + N - z) & (N - 1)]);
            acc = fe_add<F>(acc, fe_mul<F>(q, pw[k]));
        }
        Q[(size_t)zi * N + k] = q;
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) sh[threadIdx.x] = fe_add<F>(sh[threadIdx.x], sh[threadIdx.x + h]);
        __syncthreads();
    }
    if (threadIdx.x == 0) Q[(size_t)zi * N + z] = fe_neg<F>(fe_mul<F>(sh[0], pw_inv[z]));
}

// g[k] = sum_z Q[z][k] ; h[k] = sum_z invt[z] S[z][k] ; hmg = h - g (when invt_z and hmg are given)
// g[k] = sum_z Q[z][k], h[k] = sum_z invt_z[z] S[z][k]: a block per MP_CB_K columns, its 256
// threads split the Z rows MP_CB_R ways (row-groups strided by MP_CB_R), partials added in LDS --
// the one-thread-per-column form ran 256 dependent multiplies per thread on 4 waves (~0.15 ms of
// the multiproof finish at N = 256)
constexpr uint32_t MP_CB_K = 16, MP_CB_R = 16;
__global__ void __launch_bounds__(256) k_mp_combine(const fe<F>* __restrict__ S, const fe<F>* __restrict__ Q,
                                                    const fe<F>* __restrict__ invt_z, size_t N, uint32_t Z,
                                                    fe<F>* __restrict__ g, fe<F>* __restrict__ h,
                                                    fe<F>* __restrict__ hmg) {
    __shared__ fe<F> pg[MP_CB_R][MP_CB_K], ph[MP_CB_R][MP_CB_K];
    const uint32_t kc = threadIdx.x % MP_CB_K, rg = threadIdx.x / MP_CB_K;
    const size_t k = (size_t)blockIdx.x * MP_CB_K + kc;
    fe<F> gg = fe_zero<F>(), hh = fe_zero<F>();
    if (k < N)
        for (uint32_t zi = rg; zi < Z; zi += MP_CB_R) {
            gg = fe_add<F>(gg, Q[(size_t)zi * N + k]);
            if (invt_z) hh = fe_add<F>(hh, fe_mul<F>(invt_z[zi], S[(size_t)zi * N + k]));
        }
    pg[rg][kc] = gg;
    ph[rg][kc] = hh;
    __syncthreads();
    if (rg == 0 && k < N) {
        for (uint32_t j = 1; j < MP_CB_R; j++) {
            gg = fe_add<F>(gg, pg[j][kc]);
            if (invt_z) hh = fe_add<F>(hh, ph[j][kc]);
        }
        g[k] = gg;
        if (invt_z) h[k] = hh;
        if (invt_z && hmg) hmg[k] = fe_sub<F>(hh, gg);
    }
}

// ---------------------------------------------------------------- to_data_item (a13)
__global__ void k_to_data_item(const fe<BN254Fq>* __restrict__ xy, const uint8_t* __restrict__ inf, size_t n,
                               fe<F>* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = to_data_item_canon(xy[2 * i], xy[2 * i + 1], inf[i] != 0);
}

}  // namespace vk

using namespace vk;

// ---------------------------------------------------------------- C ABI
namespace {
struct Guard {
    vc_ctx* c;
    std::lock_guard<std::recursive_mutex> lk;
    explicit Guard(vc_ctx* ctx) : c(ctx), lk(ctx->mu) { (void)hipSetDevice(ctx->device); }
    ~Guard() {
        if (c->timing) c->collect_timers();
    }
};
bool proof_ok(const vc_ipa_proof* p) { return p && p->l_xy && p->r_xy && p->l_inf && p->r_inf; }
}  // namespace

namespace vk {
int to_data_item_device(vc_ctx* ctx, const void* d_xy, const uint8_t* d_inf, size_t n, void* d_items) {
    if (n == 0) return VC_OK;
    VK_LAUNCH(ctx, "to_data_item", k_to_data_item, (n + 255) / 256, 256, 0, static_cast<const fe<BN254Fq>*>(d_xy),
              d_inf, n, static_cast<fe<F>*>(d_items));
    return VC_OK;
}
}  // namespace vk
extern "C" {

int vc_to_data_item_batch(vc_ctx* ctx, const uint64_t* xy, const uint8_t* inf, size_t n, uint64_t* out) {
    if (!ctx || (n && (!xy || !inf || !out))) return VC_E_INVALID;
    if (ctx->curve != VC_CURVE_BN254) return VC_E_INVALID;
    Guard g(ctx);
    if (n == 0) return VC_OK;
    DevBuf dxy(ctx), dinf(ctx), dout(ctx);
    VK_TRY(dxy.ensure(n * 64));
    VK_TRY(dinf.ensure(n));
    VK_TRY(dout.ensure(n * 32));
    VK_CHECK_HIP(hipMemcpyAsync(dxy.p, xy, n * 64, hipMemcpyHostToDevice, ctx->stream));
    VK_CHECK_HIP(hipMemcpyAsync(dinf.p, inf, n, hipMemcpyHostToDevice, ctx->stream));
    VK_LAUNCH(ctx, "to_data_item", k_to_data_item, (n + 255) / 256, 256, 0, dxy.as<fe<BN254Fq>>(), dinf.as<uint8_t>(),
              n, dout.as<fe<F>>());
    VK_CHECK_HIP(hipMemcpyAsync(out, dout.p, n * 32, hipMemcpyDeviceToHost, ctx->stream));
    VK_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VC_OK;
}

int vc_ipa_commit(vc_ctx* ctx, int table, size_t N, const uint64_t* data, size_t batch, uint64_t* out_xy,
                  uint8_t* out_inf) {
    return vc_msm_batch(ctx, table, N, data, batch, 0, out_xy, out_inf);
}

int vc_ipa_prove(vc_ctx* ctx, int table, size_t N, const uint64_t* data, const uint64_t* com_xy,
                 const uint8_t* com_inf, const uint64_t* points, size_t batch, vc_transcript** trs,
                 vc_ipa_proof* proofs) {
    if (!ctx || !data || !com_xy || !com_inf || !points || !proofs || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    for (size_t p = 0; p < batch; p++)
        if (!proof_ok(&proofs[p])) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    std::vector<std::vector<Fr>> d(batch, std::vector<Fr>(N));
    std::vector<Acc> coms(batch);
    std::vector<Fr> pts(batch);
    for (size_t p = 0; p < batch; p++) {
        for (size_t i = 0; i < N; i++) d[p][i] = fr_of(data + (p * N + i) * 4);
        coms[p] = acc_of(com_xy + 8 * p, com_inf[p]);
        pts[p] = fr_of(points + 4 * p);
    }
    return ipa_prove_impl(ctx, t, N, d, coms, pts, trs, proofs);
}

int vc_ipa_verify(vc_ctx* ctx, int table, size_t N, const uint64_t* com_xy, uint8_t com_inf, const uint64_t* point,
                  const vc_ipa_proof* proof, vc_transcript* tr, int* result) {
    if (!ctx || !point || !proof_ok(proof) || !result || (!com_xy && !com_inf) || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    uint64_t zero[8] = {0};
    return ipa_verify_impl(ctx, t, N, acc_of(com_inf ? zero : com_xy, com_inf), fr_of(point), proof, tr, result);
}

// ---------------------------------------------------------------- IPA commitment proof
// prove_commitment (ipa/mod.rs:199-234): the IPA rounds with neither the evaluation vector b
// nor q. Same representation as ipa_prove_impl -- the folded generators are coefficients over
// the first n CRS points -- so each round is one batch of 2B width-n fixed-base commits.
int vc_ipa_prove_commitment(vc_ctx* ctx, int table, size_t n, const uint64_t* data, const uint64_t* com_xy,
                            const uint8_t* com_inf, size_t batch, vc_ipa_proof* proofs) {
    if (!ctx || !data || !com_xy || !com_inf || !proofs || ctx->curve != VC_CURVE_BN254) return VC_E_INVALID;
    // n = data.max() + 1; the assert in vec_add_and_distribute (utils.rs:37) fires on any
    // odd split above 1, i.e. unless n is a power of two
    if (!is_pow2(n)) return VC_E_INVALID;
    size_t K = 0;
    while ((1ull << K) < n) K++;
    for (size_t p = 0; p < batch; p++)
        if (!proof_ok(&proofs[p]) || proofs[p].rounds < K) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    if (t->n < n) return VC_E_INVALID;  // key.g[0..max + 1] out of bounds
    std::vector<std::vector<Fr>> a(batch, std::vector<Fr>(n));
    std::vector<std::vector<Fr>> coeff(batch, std::vector<Fr>(n, fe_one<F>()));
    std::vector<vc_transcript*> trs(batch);
    for (size_t p = 0; p < batch; p++) {
        for (size_t i = 0; i < n; i++) a[p][i] = fr_of(data + (p * n + i) * 4);
        trs[p] = vc_transcript_new("ipa");
        transcript_append_point(trs[p], com_xy + 8 * p, com_inf[p], "C");
        (void)transcript_digest(trs[p], "x");
    }
    std::vector<Fr> sc(2 * batch * n);
    std::vector<uint64_t> oxy(2 * batch * 8);
    std::vector<uint8_t> oinf(2 * batch);
    int st = VC_OK;
    for (size_t r = 0; r < K && st == VC_OK; r++) {
        const size_t m = n >> r, half = m / 2;
        for (size_t p = 0; p < batch; p++) {
            Fr* sL = &sc[(2 * p) * n];
            Fr* sR = &sc[(2 * p + 1) * n];
            for (size_t i = 0; i < n; i++) {
                size_t j = i % m;
                // L = <gens_R, data_L>, R = <gens_L, data_R>
                sL[i] = j >= half ? fe_mul<F>(a[p][j - half], coeff[p][i]) : fe_zero<F>();
                sR[i] = j < half ? fe_mul<F>(a[p][j + half], coeff[p][i]) : fe_zero<F>();
            }
        }
        st = commit_batch(ctx, t, n, sc.data(), 2 * batch, oxy.data(), oinf.data());
        if (st != VC_OK) break;
        for (size_t p = 0; p < batch; p++) {
            const uint64_t* Lxy = &oxy[(2 * p) * 8];
            const uint64_t* Rxy = &oxy[(2 * p + 1) * 8];
            memcpy(proofs[p].l_xy + r * 8, Lxy, 64);
            memcpy(proofs[p].r_xy + r * 8, Rxy, 64);
            proofs[p].l_inf[r] = oinf[2 * p];
            proofs[p].r_inf[r] = oinf[2 * p + 1];
            transcript_append_point(trs[p], Lxy, oinf[2 * p], "L");
            transcript_append_point(trs[p], Rxy, oinf[2 * p + 1], "R");
            Fr x = transcript_digest(trs[p], "x");
            // data <- data_L + x data_R ; gens <- gens_R + x gens_L (coefficients)
            for (size_t j = 0; j < half; j++) a[p][j] = fe_add<F>(a[p][j], fe_mul<F>(x, a[p][j + half]));
            a[p].resize(half);
            for (size_t i = 0; i < n; i++)
                if ((i % m) < half) coeff[p][i] = fe_mul<F>(coeff[p][i], x);
        }
    }
    for (size_t p = 0; p < batch; p++) {
        if (st == VC_OK) {
            proofs[p].rounds = K;
            canon_of(a[p][0], proofs[p].tip);
            memset(proofs[p].y, 0, sizeof(proofs[p].y));
        }
        vc_transcript_free(trs[p]);
    }
    return st;
}

// verify_commitment_proof (ipa/mod.rs:237-265): c_K = L_K + x_K c_{K-1} + x_K^2 R_K unrolled to
// (prod x) C + sum_k P_k (L_k + x_k^2 R_k), P_k = prod_{j>k} x_j (one small variable-base MSM),
// checked against tip * <g[0..2^K], points_coeffs> (one fixed-base commit): their difference
// must be the identity.
int vc_ipa_verify_commitment_proof(vc_ctx* ctx, int table, const uint64_t* com_xy, uint8_t com_inf,
                                   const vc_ipa_proof* pr, int* result) {
    if (!ctx || !proof_ok(pr) || !result || (!com_xy && !com_inf) || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    const size_t K = pr->rounds;
    if (K >= 40) return VC_E_INVALID;
    const size_t n = 1ull << K;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    if (t->n < n) return VC_E_INVALID;  // key.g[0..2^rounds] out of bounds
    uint64_t zero[8] = {0};
    const uint64_t* cxy = com_inf ? zero : com_xy;
    vc_transcript* tr = vc_transcript_new("ipa");
    transcript_append_point(tr, cxy, com_inf, "C");
    (void)transcript_digest(tr, "x");
    std::vector<Fr> xs(K);
    for (size_t k = 0; k < K; k++) {
        transcript_append_point(tr, pr->l_xy + 8 * k, pr->l_inf[k], "L");
        transcript_append_point(tr, pr->r_xy + 8 * k, pr->r_inf[k], "R");
        xs[k] = transcript_digest(tr, "x");
    }
    vc_transcript_free(tr);
    std::vector<Fr> s(1, fe_one<F>());
    for (size_t k = 0; k < K; k++) {
        std::vector<Fr> ns(2 * s.size());
        for (size_t i = 0; i < s.size(); i++) {
            ns[2 * i] = fe_mul<F>(s[i], xs[k]);
            ns[2 * i + 1] = s[i];
        }
        s.swap(ns);
    }
    Fr tip = fr_of(pr->tip);
    std::vector<Fr> fs(n);
    for (size_t i = 0; i < n; i++) fs[i] = fe_neg<F>(fe_mul<F>(tip, s[i]));
    uint64_t axy[8];
    uint8_t ainf;
    VK_TRY(commit_batch(ctx, t, n, fs.data(), 1, axy, &ainf));
    std::vector<uint64_t> vxy(8 * (1 + 2 * K));
    std::vector<uint8_t> vinf(1 + 2 * K);
    std::vector<Fr> vs(1 + 2 * K);
    memcpy(&vxy[0], cxy, 64);
    vinf[0] = com_inf;
    Fr P = fe_one<F>();
    for (size_t k = K; k-- > 0;) {
        memcpy(&vxy[8 * (1 + 2 * k)], pr->l_xy + 8 * k, 64);
        memcpy(&vxy[8 * (2 + 2 * k)], pr->r_xy + 8 * k, 64);
        vinf[1 + 2 * k] = pr->l_inf[k];
        vinf[2 + 2 * k] = pr->r_inf[k];
        vs[1 + 2 * k] = P;
        vs[2 + 2 * k] = fe_mul<F>(P, fe_sqr<F>(xs[k]));
        P = fe_mul<F>(P, xs[k]);
    }
    vs[0] = P;
    Acc vb;
    VK_TRY(msm_points(ctx, vxy.data(), vinf.data(), vs, &vb));
    Acc tot = C::add(acc_of(axy, ainf), vb);
    *result = C::is_zero(tot) ? 1 : 0;
    return VC_OK;
}

int vc_kzg_setup(vc_ctx* ctx, size_t max_items, const uint64_t* secret, int* table_id, size_t* size) {
    if (!ctx || !secret || !table_id || max_items == 0) return VC_E_INVALID;
    Guard g(ctx);
    size_t n = 1;
    while (n < max_items) n <<= 1;
    DevBuf acc(ctx);
    Table* t = new Table();
    int st = VC_OK;
    if (ctx->curve == VC_CURVE_BN254) {
        st = acc.ensure(n * sizeof(BN254G1::Acc));
        BN254G1::Aff gen;
        uint64_t gxy[8] = {1, 0, 0, 0, 2, 0, 0, 0};
        gen.x = canon_to_mont<BN254Fq>(gxy);
        gen.y = canon_to_mont<BN254Fq>(gxy + 4);
        if (st == VC_OK)
            st = kzg_srs_dev<BN254G1, BN254Fr>(ctx, max_items, n, canon_to_mont<BN254Fr>(secret),
                                               group_gen_t<BN254Fr>(n, 5), gen, acc.as<BN254G1::Acc>());
    } else if (ctx->curve == VC_CURVE_BLS12_381) {
        st = acc.ensure(n * sizeof(BLS381G1::Acc));
        BLS381G1::Aff gen;
        const uint64_t gx[6] = {0xfb3af00adb22c6bbull, 0x6c55e83ff97a1aefull, 0xa14e3a3f171bac58ull,
                                0xc3688c4f9774b905ull, 0x2695638c4fa9ac0full, 0x17f1d3a73197d794ull};
        const uint64_t gy[6] = {0x0caa232946c5e7e1ull, 0xd03cc744a2888ae4ull, 0x00db18cb2c04b3edull,
                                0xfcf5e095d5d00af6ull, 0xa09e30ed741d8ae4ull, 0x08b3f481e3aaa0f1ull};
        gen.x = canon_to_mont<BLS381Fq>(gx);
        gen.y = canon_to_mont<BLS381Fq>(gy);
        if (st == VC_OK)
            st = kzg_srs_dev<BLS381G1, BLS381Fr>(ctx, max_items, n, canon_to_mont<BLS381Fr>(secret),
                                                 group_gen_t<BLS381Fr>(n, 7), gen, acc.as<BLS381G1::Acc>());
    } else {
        st = VC_E_INVALID;
    }
    if (st == VC_OK) st = table_from_acc(ctx, t, acc.p, n);
    if (st != VC_OK) {
        delete t;
        return st;
    }
    t->subgroup = 1;  // l_j(s) * G
    ctx->tables.push_back(t);
    *table_id = (int)ctx->tables.size() - 1;
    if (size) *size = n;
    return VC_OK;
}

int vc_kzg_prove(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                 uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y) {
    if (!ctx || (max && !evals) || !point || !proof_xy || !proof_inf || !y) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    if (ctx->curve == VC_CURVE_BN254)
        return kzg_prove_t<BN254G1, BN254Fr>(ctx, t, size, evals, max, point, proof_xy, proof_inf, y, nullptr);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return kzg_prove_t<BLS381G1, BLS381Fr>(ctx, t, size, evals, max, point, proof_xy, proof_inf, y, nullptr);
    return VC_E_INVALID;
}

int vc_kzg_prove_device(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                        const uint64_t* point, uint64_t* proof_xy, uint8_t* proof_inf, uint64_t* y) {
    if (!ctx || (max && !d_evals) || !point || !proof_xy || !proof_inf || !y) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    const uint64_t* ev = reinterpret_cast<const uint64_t*>(d_evals);
    if (ctx->curve == VC_CURVE_BN254)
        return kzg_prove_t<BN254G1, BN254Fr>(ctx, t, size, ev, max, point, proof_xy, proof_inf, y, nullptr, true);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return kzg_prove_t<BLS381G1, BLS381Fr>(ctx, t, size, ev, max, point, proof_xy, proof_inf, y, nullptr, true);
    return VC_E_INVALID;
}

int vc_kzg_commit_prove_device(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                               const uint64_t* point, uint64_t* com_xy, uint8_t* com_inf, uint64_t* proof_xy,
                               uint8_t* proof_inf, uint64_t* y) {
    if (!ctx || (max && !d_evals) || !point || !com_xy || !com_inf || !proof_xy || !proof_inf || !y)
        return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    const uint64_t* ev = reinterpret_cast<const uint64_t*>(d_evals);
    if (ctx->curve == VC_CURVE_BN254)
        return kzg_prove_t<BN254G1, BN254Fr>(ctx, t, size, ev, max, point, proof_xy, proof_inf, y, nullptr, true, 0, 1,
                                             nullptr, com_xy, com_inf);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return kzg_prove_t<BLS381G1, BLS381Fr>(ctx, t, size, ev, max, point, proof_xy, proof_inf, y, nullptr, true, 0,
                                               1, nullptr, com_xy, com_inf);
    return VC_E_INVALID;
}

int vc_kzg_prove_device_part(vc_ctx* ctx, int table, size_t size, const void* d_evals, size_t max,
                             const uint64_t* point, int part, int parts, uint32_t* out_acc, uint64_t* y) {
    if (!ctx || (max && !d_evals) || !point || !out_acc || !y || parts < 1 || part < 0 || part >= parts)
        return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    const uint64_t* ev = reinterpret_cast<const uint64_t*>(d_evals);
    if (ctx->curve == VC_CURVE_BN254)
        return kzg_prove_t<BN254G1, BN254Fr>(ctx, t, size, ev, max, point, nullptr, nullptr, y, nullptr, true, part,
                                             parts, out_acc);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return kzg_prove_t<BLS381G1, BLS381Fr>(ctx, t, size, ev, max, point, nullptr, nullptr, y, nullptr, true,
                                               part, parts, out_acc);
    return VC_E_INVALID;
}

int vc_kzg_prove_all_points(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t n_evals, int mode,
                            uint64_t* out_xy, uint8_t* out_inf, uint64_t* out_y, size_t* count) {
    if (!ctx || (n_evals && !evals) || !out_xy || !out_inf || !out_y || !count) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    if (ctx->curve == VC_CURVE_BN254)
        return fk_all_t<BN254G1, BN254Fr>(ctx, t, size, evals, n_evals, mode, out_xy, out_inf, out_y, count);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return fk_all_t<BLS381G1, BLS381Fr>(ctx, t, size, evals, n_evals, mode, out_xy, out_inf, out_y, count);
    return VC_E_INVALID;
}

int vc_kzg_quotient(vc_ctx* ctx, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                    uint64_t* q_out, uint64_t* y) {
    if (!ctx || (max && !evals) || !point || !q_out || !y) return VC_E_INVALID;
    Guard g(ctx);
    if (ctx->curve == VC_CURVE_BN254)
        return kzg_prove_t<BN254G1, BN254Fr>(ctx, nullptr, size, evals, max, point, nullptr, nullptr, y, q_out);
    if (ctx->curve == VC_CURVE_BLS12_381)
        return kzg_prove_t<BLS381G1, BLS381Fr>(ctx, nullptr, size, evals, max, point, nullptr, nullptr, y, q_out);
    return VC_E_INVALID;
}

}  // extern "C"

namespace vk {
// ---------------------------------------------------------------- range-sharded KZG open
// One member's share of KZG::prove_point (kzg/mod.rs:136-154) split by index range (SURVEY 8(e)
// C4): the member uploads only f on [lo, hi), computes q there, and its MSM covers the SRS points
// [lo, hi) (a point range on the table's radix copies). The global sum of each case leaves as one
// field partial (phase 1), the members' total comes back (phase 2). vc_group_kzg_prove drives it.
struct KzgShare {
    vc_ctx* ctx = nullptr;
    Table* t = nullptr;
    size_t n = 0, lo = 0, L = 0, nvalid = 0, m = 0;
    bool in_domain = false;
    uint32_t point[8] = {0}, omega[8] = {0};  // Montgomery Fr words
    uint64_t y_in[4] = {0};                   // in domain: y = f_m (canonical)
    DevBuf f, q, inv, part;
    explicit KzgShare(vc_ctx* c) : ctx(c), f(c), q(c), inv(c), part(c) {}
};

template <class C_, class Fr_>
static int kzg_share_begin_t(vc_ctx* ctx, Table* t, size_t size, const uint64_t* evals, size_t max,
                             const uint64_t* point, size_t lo, size_t hi, KzgShare* s, uint64_t* partial) {
    using Fe = fe<Fr_>;
    if (!is_pow2(size) || max > size || lo > hi || hi > size) return VC_E_INVALID;
    if (t->n < size) return VC_E_RANGE;
    s->ctx = ctx;
    s->t = t;
    s->n = size;
    s->lo = lo;
    s->L = hi - lo;
    s->nvalid = max > lo ? std::min(max, hi) - lo : 0;
    const Fe pm = canon_to_mont<Fr_>(point);
    const Fe omega = group_gen_t<Fr_>(size, fr_generator<Fr_>());
    memcpy(s->point, pm.v, 32);
    memcpy(s->omega, omega.v, 32);
    // prove_point: `point <= size` -> the in-domain branch with index to_usize(point)
    const Fe pc = fe_from_mont<Fr_>(pm);
    bool small = true;
    for (int i = 2; i < Fr_::N; i++) small &= pc.v[i] == 0;
    const uint64_t pv = (uint64_t)pc.v[0] | ((uint64_t)pc.v[1] << 32);
    s->in_domain = small && pv <= size;
    if (s->in_domain && pv == size) return VC_E_DOMAIN;  // vanishing_at(size) out of bounds
    s->m = s->in_domain ? (size_t)pv : 0;
    Fe fm = fe_zero<Fr_>();
    if (s->in_domain && s->m < max) {  // y = evaluate(point): the stored value, or 0 in [max, size]
        memcpy(s->y_in, evals + 4 * s->m, 32);
        fm = canon_to_mont<Fr_>(evals + 4 * s->m);
    }
    const size_t L = std::max<size_t>(s->L, 1);
    VK_TRY(s->f.ensure(L * 32));
    VK_TRY(s->q.ensure(L * 32));
    VK_TRY(s->inv.ensure(L * 32));
    if (s->nvalid)
        VK_CHECK_HIP(hipMemcpyAsync(s->q.p, evals + 4 * lo, s->nvalid * 32, hipMemcpyHostToDevice, ctx->stream));
    VK_TRY(canon_to_mont_dev<Fr_>(ctx, s->q.p, s->L, s->nvalid, s->f.as<Fe>()));
    Fe part;
    VK_TRY(kzg_range_part<Fr_>(ctx, size, s->f.as<Fe>(), s->nvalid, lo, s->L, pm, omega, s->in_domain, s->m, fm,
                               s->q.as<Fe>(), s->inv.as<Fe>(), s->part, &part));
    memcpy(partial, part.v, 32);
    return VC_OK;
}

template <class C_, class Fr_>
static int kzg_share_finish_t(KzgShare* s, const uint64_t* total, uint32_t* out_acc, uint64_t* y) {
    using Fe = fe<Fr_>;
    vc_ctx* ctx = s->ctx;
    Fe tot, pm, omega, ym = fe_zero<Fr_>();
    memcpy(tot.v, total, 32);
    memcpy(pm.v, s->point, 32);
    memcpy(omega.v, s->omega, 32);
    VK_TRY(kzg_range_finish<Fr_>(ctx, s->n, s->f.as<Fe>(), s->nvalid, s->lo, s->L, pm, omega, s->in_domain, s->m, tot,
                                 s->q.as<Fe>(), s->inv.as<Fe>(), &ym));
    if (s->in_domain) memcpy(y, s->y_in, 32);
    else mont_to_canon<Fr_>(ym, y);
    if (s->L == 0) {  // an empty share adds the identity
        typename C_::Acc z = C_::zero();
        memcpy(out_acc, &z, sizeof z);
        return VC_OK;
    }
    return msm_run(ctx, s->t, s->lo, s->q.p, s->L, 1, out_acc);
}

int kzg_share_begin(vc_ctx* ctx, int table, size_t size, const uint64_t* evals, size_t max, const uint64_t* point,
                    size_t lo, size_t hi, KzgShare** out, uint64_t* partial) {
    if (!ctx || !out || !point || !partial || (max && !evals)) return VC_E_INVALID;
    *out = nullptr;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    KzgShare* s = new KzgShare(ctx);
    int st = VC_E_INVALID;
    if (ctx->curve == VC_CURVE_BN254)
        st = kzg_share_begin_t<BN254G1, BN254Fr>(ctx, t, size, evals, max, point, lo, hi, s, partial);
    else if (ctx->curve == VC_CURVE_BLS12_381)
        st = kzg_share_begin_t<BLS381G1, BLS381Fr>(ctx, t, size, evals, max, point, lo, hi, s, partial);
    if (st != VC_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        delete s;  // (the pooled buffers return to the pool under the lock held here)
        return st;
    }
    *out = s;
    return VC_OK;
}

int kzg_share_finish(KzgShare* s, const uint64_t* total, uint32_t* out_acc, uint64_t* y) {
    if (!s || !total || !out_acc || !y) return VC_E_INVALID;
    Guard g(s->ctx);
    if (s->ctx->curve == VC_CURVE_BN254) return kzg_share_finish_t<BN254G1, BN254Fr>(s, total, out_acc, y);
    return kzg_share_finish_t<BLS381G1, BLS381Fr>(s, total, out_acc, y);
}

void kzg_share_free(KzgShare* s) {
    if (!s) return;
    {
        Guard g(s->ctx);  // the pooled buffers go back to their context's pool under its lock
        (void)hipStreamSynchronize(s->ctx->stream);
        s->f.release();
        s->q.release();
        s->inv.release();
        s->part.release();
    }
    delete s;
}

// sum of G range partials (Montgomery Fr words of the context's scalar field)
int kzg_share_sum(int curve, const uint64_t* parts, int G, uint64_t* total) {
    if (curve == VC_CURVE_BN254) {
        fe<BN254Fr> a = fe_zero<BN254Fr>(), b;
        for (int k = 0; k < G; k++) {
            memcpy(b.v, parts + 4 * (size_t)k, 32);
            a = fe_add<BN254Fr>(a, b);
        }
        memcpy(total, a.v, 32);
        return VC_OK;
    }
    if (curve == VC_CURVE_BLS12_381) {
        fe<BLS381Fr> a = fe_zero<BLS381Fr>(), b;
        for (int k = 0; k < G; k++) {
            memcpy(b.v, parts + 4 * (size_t)k, 32);
            a = fe_add<BLS381Fr>(a, b);
        }
        memcpy(total, a.v, 32);
        return VC_OK;
    }
    return VC_E_INVALID;
}

}  // namespace vk

// ---------------------------------------------------------------- multiproof (a11)
namespace vk {

struct MpPrep {
    Fr r, t;
    std::vector<Fr> rpow;
};

// the multiproof transcript's records "C" ++ compressed(C_i) ++ "z" ++ le64(z_i) ++ "y" ++ le(y_i)
// (multiproof.rs:106-113) for queries [lo, hi) into out: 75 bytes at offset 75 i, so the records
// are written straight into the transcript on up to 16 host threads (the point compression is the
// costly part); the SHA-256 over them stays serial
static void mp_records(const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                       size_t lo, size_t hi, uint8_t* out) {
    constexpr size_t REC = 75;
    static const uint64_t zero[8] = {0};
    for (size_t i = lo; i < hi; i++) {
        uint8_t* o = out + REC * (i - lo);
        o[0] = 'C';
        compress_g1(com_inf[i] ? zero : com_xy + 8 * i, com_inf[i] != 0, o + 1);
        o[33] = 'z';
        for (int k = 0; k < 8; k++) o[34 + k] = (uint8_t)(z[i] >> (8 * k));
        o[42] = 'y';
        memcpy(o + 43, y + 4 * i, 32);
    }
}

static std::vector<Fr> invert_domain_at(const Fr& t, size_t N) {  // utils.rs:57-62 (integer i)
    std::vector<Fr> d(N);
    for (size_t i = 0; i < N; i++) d[i] = fe_sub<F>(t, fr_u64(i));
    return host_batch_inv(d);
}

// ---- multiproof prover in three phases (multiproof.rs:99-176), so the Q x N field phase can
// be sharded over GPUs with one exchange:
//   mp_begin       host: transcript over all (C, z, y) and the challenge r        (:106-114)
//   mp_accumulate  device, per query shard [first, first + Qs): dense per-z sums
//                  S[z][k] = sum_{i: z_i = z} r^i f_i[k]  (canonical, N x N)      (:116-127)
//   mp_finish      device + host: sum of the shards' S, quotients, g, D, t, h, E and the
//                  inner proof                                                     (:129-175)
// Grouping queries by z and summing per group first is the same field arithmetic as the
// reference's per-group LagrangeBasis sums; rows of z with no query are zero and add nothing.
// pool_ok = false: the call's own filler thread feeds the hash (scheme_host.cpp
// transcript_digest_records) -- mp_prove_many's transcript workers and vc_multiproof_begin, whose
// callers run several transcripts at once: on the shared host pool their record filling queued
// on the pool's one-loop lock. No transcript is returned on error (VC_E_OOM if the hashing threw).
static int mp_begin(size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                    const uint64_t* y, vc_transcript** tr_out, Fr* r_out, bool pool_ok = true) {
    *tr_out = nullptr;
    if (!is_pow2(N) || Q == 0) return VC_E_INVALID;
    for (size_t i = 0; i < Q; i++)
        if (z[i] >= N) return VC_E_DOMAIN;
    // the records stream into the hash (never stored whole: transcript_digest_records)
    vc_transcript* tr = vc_transcript_new("multiproof");
    try {
        *r_out = transcript_digest_records(
            tr, Q, 75, [&](size_t lo, size_t hi, uint8_t* out) { mp_records(com_xy, com_inf, z, y, lo, hi, out); },
            "r", pool_ok && Q >= 8192);
    } catch (...) {  // the filler thread's failure, rethrown by the digest
        vc_transcript_free(tr);
        return VC_E_OOM;
    }
    *tr_out = tr;
    return VC_OK;
}

// distinct query points, sorted; VC_E_DOMAIN for a z outside the domain (the reference indexes
// the Lagrange evaluations with it and panics). The accumulate / finish entry points take z
// from the caller again, so every path validates here (a bitmap of N, not of max z).
static int mp_points(size_t N, size_t Q, const uint64_t* z, std::vector<uint32_t>* out) {
    if (N == 0 || N > (size_t(1) << 28)) return VC_E_INVALID;  // BN254 Fr has 2-adicity 28
    std::vector<uint8_t> seen(N, 0);
    for (size_t i = 0; i < Q; i++) {
        if (z[i] >= N) return VC_E_DOMAIN;
        seen[z[i]] = 1;
    }
    out->clear();
    for (size_t k = 0; k < N; k++)
        if (seen[k]) out->push_back((uint32_t)k);
    return VC_OK;
}

// rp[i] = r^(first + i) as radix-2^29 Montgomery limbs (x R', R' = 2^261, ff29.hpp), canonical, at
// a stride of MP_RP_WORDS words (the chunk kernel reads them as uniform scalar loads)
using P29 = F29BN254Fr;
constexpr uint32_t MP_RP_WORDS = 16;
__global__ void k_mp_rpow(Fr r, size_t first, size_t n, uint32_t* __restrict__ rp) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr acc = fe_one<F>(), b = r;
    size_t e = first + i;
    while (e) {
        if (e & 1) acc = fe_mul<F>(acc, b);
        e >>= 1;
        if (e) b = fe_sqr<F>(b);
    }
    const f29<P29> v = canon29<P29>(from_mont32<P29, F>(acc));
#pragma unroll
    for (int j = 0; j < P29::L; j++) rp[i * MP_RP_WORDS + j] = v.v[j];
}

// one block per (k block, chunk c of <= CH queries of one z): partial[c][k] =
// sum over sorted positions [be[2c], be[2c+1]) of r^i f_i[k] (f canonical; partial canonical).
// HBM-bound stream of the Q x N evaluations (the r^i are uniform over a block). Radix-2^29 with
// lazy reduction: the products f_i[k] (r^i R') of LZ queries add into 17 unsigned 64-bit columns
// (<= 9 products of < 2^58 per query and column) and ONE Montgomery reduction (9 rows, <= 9 more
// products per column) serves them: (9 LZ + 9) 2^58 + 2^35 < 2^64 for LZ <= 6 -- ~100-120
// instructions per element instead of a full 32-bit-limb multiply (~270) and an add. A block
// result is below (LZ p^2 / R' + p) = (1 + LZ 2^-7) p; the block results are added with one
// conditional subtraction each, so the running total stays below 2 p over a chunk of CH / LZ
// blocks, and a last one makes it canonical.
// Shapes (LZ x CH, A/B knob VKZG_MP_SHAPE): 3 x 16 (round 4's first), 4 x 16, 4 x 32, 6 x 24.
constexpr uint32_t MP_LZ_MAX = 6;
struct MpShape {
    uint32_t lz, ch;
};
// one block of <= LZ queries: products into the columns, one Montgomery reduction
template <uint32_t LZ>
__device__ __forceinline__ f29<P29> mp_block(const uint4 (&v)[LZ][2], const uint32_t (&qi)[LZ], uint32_t nq,
                                             const uint32_t* __restrict__ rp) {
    static_assert(LZ <= MP_LZ_MAX, "column bound");
    constexpr int L = P29::L;
    uint64_t t[2 * L];  // 2L - 1 product columns and the reduction's top carry
#pragma unroll
    for (int x = 0; x < 2 * L; x++) t[x] = 0;
#pragma unroll
    for (uint32_t j = 0; j < LZ; j++) {
        if (j >= nq) break;
        const uint32_t w[8] = {v[j][0].x, v[j][0].y, v[j][0].z, v[j][0].w, v[j][1].x, v[j][1].y, v[j][1].z, v[j][1].w};
        const f29<P29> a = unpack29<P29>(w);
        const uint32_t* b = rp + (size_t)qi[j] * MP_RP_WORDS;
#pragma unroll
        for (int y = 0; y < L; y++) {
            const uint32_t by = b[y];
#pragma unroll
            for (int x = 0; x < L; x++) t[x + y] += (uint64_t)a.v[x] * by;
        }
    }
    // Montgomery reduction of the columns (separated operand scanning): t / R' mod p
#pragma unroll
    for (int i = 0; i < L; i++) {
        const uint32_t m = ((uint32_t)t[i] * P29::inv) & M29;
#pragma unroll
        for (int j = 0; j < L; j++) t[i + j] += (uint64_t)m * P29::p(j);
        t[i + 1] += t[i] >> 29;
    }
    f29<P29> r;  // columns L .. 2L - 1 are the reduced value (as sqr29)
#pragma unroll
    for (int j = L; j < 2 * L - 1; j++) {
        t[j + 1] += t[j] >> 29;
        r.v[j - L] = (uint32_t)t[j] & M29;
    }
    r.v[L - 1] = (uint32_t)t[2 * L - 1];
    return r;
}

// NT = 1: non-temporal loads (the evaluations are read once per proof; A/B knob VKZG_MP_NT)
template <int NT, uint32_t LZ>
__device__ __forceinline__ void mp_load(const uint32_t* __restrict__ f, const uint32_t* __restrict__ order, uint32_t u,
                                        uint32_t nq, size_t N, size_t k, uint4 (&v)[LZ][2], uint32_t (&qi)[LZ]) {
#pragma unroll
    for (uint32_t j = 0; j < LZ; j++) {
        qi[j] = j < nq ? order[u + j] : 0u;
        if (j < nq) {
            const uint4* src = reinterpret_cast<const uint4*>(f + ((size_t)qi[j] * N + k) * 8);
            if constexpr (NT) {
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
                const u32x4 a = __builtin_nontemporal_load(s4), b = __builtin_nontemporal_load(s4 + 1);
                v[j][0] = make_uint4(a.x, a.y, a.z, a.w);
                v[j][1] = make_uint4(b.x, b.y, b.z, b.w);
            } else {
                v[j][0] = src[0];
                v[j][1] = src[1];
            }
        }
    }
}

// PF = 1: the next block's loads are issued before the current block's arithmetic, so every lane
// keeps LZ x 32 B in flight while it multiplies (A/B knob VKZG_MP_PF)
template <int NT, uint32_t LZ, uint32_t CH, int PF = 0>
__global__ void __launch_bounds__(256) k_mp_chunk(const uint32_t* __restrict__ f, const uint32_t* __restrict__ rp,
                                                 const uint32_t* __restrict__ order, const uint32_t* __restrict__ be,
                                                 size_t N, uint32_t kblk, Fr* __restrict__ partial) {
    const uint32_t c = blockIdx.x / kblk;  // 1-D grid: chunks can outnumber gridDim.y's 65535
    const size_t k = (size_t)(blockIdx.x % kblk) * blockDim.x + threadIdx.x;
    if (k >= N) return;
    const uint32_t u0 = be[2 * c], cnt = be[2 * c + 1] - u0;
    f29<P29> total = zero29<P29>();
    uint4 v[LZ][2];
    uint32_t qi[LZ];
    if constexpr (PF) {
        if (cnt > 0) mp_load<NT, LZ>(f, order, u0, min(cnt, LZ), N, k, v, qi);
    }
#pragma unroll
    for (uint32_t h = 0; h < CH; h += LZ) {
        if (h >= cnt) break;
        const uint32_t nq = min(cnt - h, LZ);
        if constexpr (PF) {
            uint4 w[LZ][2];
            uint32_t qw[LZ];
            if (h + LZ < cnt) mp_load<NT, LZ>(f, order, u0 + h + LZ, min(cnt - h - LZ, LZ), N, k, w, qw);
            const f29<P29> r = mp_block<LZ>(v, qi, nq, rp);
            total = csub29<P29>(carry29<P29>(add29_raw<P29>(total, r)));
#pragma unroll
            for (uint32_t j = 0; j < LZ; j++) {
                v[j][0] = w[j][0];
                v[j][1] = w[j][1];
                qi[j] = qw[j];
            }
        } else {
            mp_load<NT, LZ>(f, order, u0 + h, nq, N, k, v, qi);
            const f29<P29> r = mp_block<LZ>(v, qi, nq, rp);
            total = csub29<P29>(carry29<P29>(add29_raw<P29>(total, r)));
        }
    }
    total = csub29<P29>(carry29<P29>(total));
    pack29<P29>(total, partial[(size_t)c * N + k].v);
}

// S[row][k] = sum of the partials of the row's chunks [zc[row], zc[row+1])
__global__ void k_mp_chunk_reduce(const Fr* __restrict__ partial, const uint32_t* __restrict__ zc, size_t N,
                                  uint32_t kblk, Fr* __restrict__ S) {
    const uint32_t zz = blockIdx.x / kblk;
    const size_t k = (size_t)(blockIdx.x % kblk) * blockDim.x + threadIdx.x;
    if (k >= N) return;
    Fr acc = fe_zero<F>();
    for (uint32_t c = zc[zz]; c < zc[zz + 1]; c++) acc = fe_add<F>(acc, partial[(size_t)c * N + k]);
    S[(size_t)zz * N + k] = acc;
}

// rows of S are the distinct query points zval (sorted, over ALL queries -- every shard
// uses the same rows so the shards' S add up); Z = zval.size().
// The shard's plan depends on z alone (not on the challenge r): rows, the counting sort of the
// queries by row, chunks of <= CH queries inside a row, and their uploads -- so mp_begin_accumulate
// builds it while the host transcript that yields r runs on another thread.
struct MpPlan {
    size_t Qs = 0, first = 0, Z = 0;
    uint32_t nch = 0;
    std::vector<uint32_t> order, be, zc;  // alive until mp_run's sync (async uploads)
    DevBuf d_rp, d_order, d_be, d_zc, d_part;
    explicit MpPlan(vc_ctx* ctx) : d_rp(ctx), d_order(ctx), d_be(ctx), d_zc(ctx), d_part(ctx) {}
};
// block / chunk shape of k_mp_chunk (VKZG_MP_SHAPE: 0 = 3 x 16, 1 = 4 x 16, 2 = 4 x 32, 3 = 6 x 24);
// 4 x 16 by default: 0.125-0.129 ms against 0.128-0.131 for 3 x 16 (profiles/r04/mp_shape_ab.txt)
static int mp_shape_index() {
    static const int shape_env = getenv("VKZG_MP_SHAPE") ? atoi(getenv("VKZG_MP_SHAPE")) : 1;
    return shape_env >= 0 && shape_env < 4 ? shape_env : 1;
}
static int mp_plan(vc_ctx* ctx, size_t N, size_t Qs, const uint64_t* z, size_t first, const std::vector<uint32_t>& zval,
                   MpPlan* pl) {
    hipStream_t st = ctx->stream;
    const size_t Z = zval.size();
    pl->Qs = Qs;
    pl->first = first;
    pl->Z = Z;
    if (Qs == 0) return VC_OK;
    // row of each query: a table over the domain (z < N, checked by mp_points over all queries)
    std::vector<uint32_t> row_of(N, 0xffffffffu), row(Qs);
    for (size_t k = 0; k < Z; k++) row_of[zval[k]] = (uint32_t)k;
    for (size_t i = 0; i < Qs; i++) {
        if (z[i] >= N || row_of[z[i]] == 0xffffffffu) return VC_E_DOMAIN;
        row[i] = row_of[z[i]];
    }
    static const MpShape shapes[4] = {{3, 16}, {4, 16}, {4, 32}, {6, 24}};
    const uint32_t MP_CHUNK = shapes[mp_shape_index()].ch;
    // counting sort of the shard's queries by row, then chunks of <= MP_CHUNK queries
    std::vector<uint32_t> cnt(Z + 1, 0);
    pl->order.resize(Qs);
    for (size_t i = 0; i < Qs; i++) cnt[row[i] + 1]++;
    for (size_t k = 0; k < Z; k++) cnt[k + 1] += cnt[k];
    {
        std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
        for (size_t i = 0; i < Qs; i++) pl->order[pos[row[i]]++] = (uint32_t)i;
    }
    // chunks of <= MP_CHUNK queries inside one row; zc[row] = first chunk of the row
    pl->be.clear();
    pl->zc.assign(Z + 1, 0);
    for (size_t k = 0; k < Z; k++) {
        pl->zc[k] = (uint32_t)(pl->be.size() / 2);
        for (uint32_t u = cnt[k]; u < cnt[k + 1]; u += MP_CHUNK) {
            pl->be.push_back(u);
            pl->be.push_back(std::min<uint32_t>(u + MP_CHUNK, cnt[k + 1]));
        }
    }
    pl->nch = (uint32_t)(pl->be.size() / 2);
    pl->zc[Z] = pl->nch;
    VK_TRY(pl->d_rp.ensure(Qs * MP_RP_WORDS * 4));
    VK_TRY(pl->d_order.ensure(Qs * 4));
    VK_TRY(pl->d_be.ensure(pl->be.size() * 4));
    VK_TRY(pl->d_zc.ensure((Z + 1) * 4));
    VK_TRY(pl->d_part.ensure(std::max<size_t>(pl->nch, 1) * N * 32));
    VK_CHECK_HIP(hipMemcpyAsync(pl->d_order.p, pl->order.data(), Qs * 4, hipMemcpyHostToDevice, st));
    VK_CHECK_HIP(hipMemcpyAsync(pl->d_be.p, pl->be.data(), pl->be.size() * 4, hipMemcpyHostToDevice, st));
    VK_CHECK_HIP(hipMemcpyAsync(pl->d_zc.p, pl->zc.data(), (Z + 1) * 4, hipMemcpyHostToDevice, st));
    return VC_OK;
}
static int mp_run(vc_ctx* ctx, size_t N, const void* d_data, const Fr& r, MpPlan& pl, void* d_S) {
    hipStream_t st = ctx->stream;
    const size_t Qs = pl.Qs, Z = pl.Z;
    if (Qs == 0) {  // an empty shard contributes zero sums (synchronous like every ABI call)
        VK_CHECK_HIP(hipMemsetAsync(d_S, 0, Z * N * 32, st));
        VK_CHECK_HIP(hipStreamSynchronize(st));
        return VC_OK;
    }
    VK_LAUNCH(ctx, "mp_rpow", k_mp_rpow, (Qs + 255) / 256, 256, 0, r, pl.first, Qs, pl.d_rp.as<uint32_t>());
    const uint32_t kblk = (uint32_t)((N + 255) / 256);
    // non-temporal loads by default: 0.119-0.121 ms (4.43-4.51 TB/s) against 0.125-0.127 at 2^16 x 256
    // (profiles/r04/mp_nt_ab.txt)
    static const int nt_env = getenv("VKZG_MP_NT") ? atoi(getenv("VKZG_MP_NT")) : 1;
    using KFn = void (*)(const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*, size_t, uint32_t, Fr*);
    static const int pf_env = getenv("VKZG_MP_PF") ? atoi(getenv("VKZG_MP_PF")) : 0;
    static const KFn kerns[3][4] = {
        {k_mp_chunk<0, 3, 16>, k_mp_chunk<0, 4, 16>, k_mp_chunk<0, 4, 32>, k_mp_chunk<0, 6, 24>},
        {k_mp_chunk<1, 3, 16>, k_mp_chunk<1, 4, 16>, k_mp_chunk<1, 4, 32>, k_mp_chunk<1, 6, 24>},
        {k_mp_chunk<1, 3, 16, 1>, k_mp_chunk<1, 4, 16, 1>, k_mp_chunk<1, 4, 32, 1>, k_mp_chunk<1, 6, 24, 1>}};
    const KFn kern = kerns[pf_env ? 2 : nt_env ? 1 : 0][mp_shape_index()];
    VK_LAUNCH(ctx, "mp_chunk", kern, (size_t)pl.nch * kblk, 256, 0, reinterpret_cast<const uint32_t*>(d_data),
              pl.d_rp.as<uint32_t>(), pl.d_order.as<uint32_t>(), pl.d_be.as<uint32_t>(), N, kblk, pl.d_part.as<Fr>());
    VK_LAUNCH(ctx, "mp_chunk_reduce", k_mp_chunk_reduce, Z * kblk, 256, 0, pl.d_part.as<Fr>(), pl.d_zc.as<uint32_t>(),
              N, kblk, reinterpret_cast<Fr*>(d_S));
    VK_CHECK_HIP(hipStreamSynchronize(st));  // the plan's host vectors may die after this
    return VC_OK;
}
static int mp_accumulate(vc_ctx* ctx, size_t N, size_t Qs, const void* d_data, const uint64_t* z, const Fr& r,
                         size_t first, const std::vector<uint32_t>& zval, void* d_S) {
    MpPlan pl(ctx);
    const int st = mp_plan(ctx, N, Qs, z, first, zval, &pl);
    if (st != VC_OK) {
        (void)hipStreamSynchronize(ctx->stream);  // uploads from the plan's vectors may be queued
        return st;
    }
    return mp_run(ctx, N, d_data, r, pl, d_S);
}

// mp_begin on a helper thread while this thread runs `overlap` (the shard's plan; mp_prove also
// the evaluations' upload): the serial SHA-256 transcript is the longest host step of a multiproof
// (2.6 ms at Q = 2^16), and neither the plan nor the upload needs its challenge. Falls back to
// running both in turn if no thread can be started.
template <class Fn>
static int mp_begin_overlapped(size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                               const uint64_t* y, vc_transcript** tr_out, Fr* r_out, Fn overlap) {
    int st_b = VC_E_INVALID, st_o = VC_OK;
    *tr_out = nullptr;
    auto guarded = [&]() -> int {  // the helper must be joined whatever the overlap does
        try {
            return overlap();
        } catch (...) {
            return VC_E_OOM;
        }
    };
    // the overlapped transcript fills its records on its own filler thread, not the host pool the
    // overlapped planning uses: single proof 3.99-4.15 -> 3.84-3.89 ms (`profiles/r04/mp_begin_pool/`;
    // VKZG_MP_BEGIN_POOL=1 restores the pool, A/B probe)
    static const bool pool = getenv("VKZG_MP_BEGIN_POOL") && atoi(getenv("VKZG_MP_BEGIN_POOL")) != 0;
    std::thread th;
    try {
        th = std::thread([&] {
            try {
                st_b = mp_begin(N, Q, com_xy, com_inf, z, y, tr_out, r_out, pool);
            } catch (...) {  // nothing may leave a thread function
                st_b = VC_E_OOM;
            }
        });
    } catch (const std::system_error&) {  // no thread: one after the other
        st_b = mp_begin(N, Q, com_xy, com_inf, z, y, tr_out, r_out);
        if (st_b == VC_OK) st_o = guarded();
    }
    if (th.joinable()) {
        st_o = guarded();
        th.join();
    }
    if (st_b != VC_OK || st_o != VC_OK) {
        if (*tr_out) vc_transcript_free(*tr_out);
        *tr_out = nullptr;
        return st_b != VC_OK ? st_b : st_o;
    }
    return VC_OK;
}

int mp_rows(size_t N, size_t Q, const uint64_t* z, size_t* rows) {
    if (!z || !rows || !is_pow2(N) || Q == 0) return VC_E_INVALID;
    std::vector<uint32_t> zval;
    VK_TRY(mp_points(N, Q, z, &zval));
    *rows = zval.size();
    return VC_OK;
}

// begin + accumulate of one query shard [first, first + Qs) with the transcript overlapped (the
// single-proof paths: mp_prove, vc_multiproof_prove_sharded)
int mp_begin_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                        const uint64_t* z, const uint64_t* y, size_t first, size_t Qs, const void* d_data, void* d_S,
                        vc_transcript** tr_out, uint64_t* r_out) {
    if (tr_out) *tr_out = nullptr;  // no transcript on any error return (vc_scheme.h)
    if (!ctx || !com_xy || !com_inf || !z || !y || !d_S || !tr_out || !r_out || (Qs && !d_data) || first > Q ||
        Qs > Q - first || ctx->curve != VC_CURVE_BN254 || !is_pow2(N) || Q == 0)
        return VC_E_INVALID;
    std::vector<uint32_t> zval;
    VK_TRY(mp_points(N, Q, z, &zval));
    Guard g(ctx);
    MpPlan pl(ctx);
    Fr r;
    const int st = mp_begin_overlapped(N, Q, com_xy, com_inf, z, y, tr_out, &r,
                                       [&] { return mp_plan(ctx, N, Qs, z + first, first, zval, &pl); });
    if (st != VC_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        return st;
    }
    canon_of(r, r_out);
    const int st2 = mp_run(ctx, N, d_data, r, pl, d_S);
    if (st2 != VC_OK) {
        vc_transcript_free(*tr_out);
        *tr_out = nullptr;
    }
    return st2;
}

// S = sum over G shards (canonical) -> Montgomery
__global__ void k_mp_sum_parts(const Fr* __restrict__ parts, int G, size_t NN, Fr* __restrict__ S) {
    size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= NN) return;
    Fr acc = parts[g];
    for (int k = 1; k < G; k++) acc = fe_add<F>(acc, parts[(size_t)k * NN + g]);
    S[g] = fe_to_mont<F>(acc);
}

static int mp_finish(vc_ctx* ctx, int scheme, Table* t, size_t N, const std::vector<uint32_t>& zval,
                     const void* d_S_parts, int G, vc_transcript* tr, uint64_t* d_xy, uint8_t* d_inf,
                     vc_ipa_proof* ipa_proof, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!is_pow2(N) || G < 1 || zval.empty()) return VC_E_INVALID;
    hipStream_t st = ctx->stream;
    // VKZG_VERBOSE: phase laps on stderr (with a stream sync at each: diagnostics only)
    static const bool verbose = getenv("VKZG_VERBOSE") != nullptr;
    auto tic = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!verbose) return;
        (void)hipStreamSynchronize(st);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[mp_finish] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tic).count());
        tic = now;
    };
    const uint32_t Z = (uint32_t)zval.size();
    DevBuf d_zv(ctx), d_S(ctx), d_Q(ctx), d_g(ctx), d_h(ctx), d_it(ctx);
    VK_TRY(d_zv.ensure(Z * 4));
    VK_TRY(d_S.ensure((size_t)Z * N * 32));
    VK_TRY(d_Q.ensure((size_t)Z * N * 32));
    VK_TRY(d_g.ensure(N * 32));
    VK_TRY(d_h.ensure(N * 32));
    VK_TRY(d_it.ensure(Z * 32));
    VK_CHECK_HIP(hipMemcpyAsync(d_zv.p, zval.data(), Z * 4, hipMemcpyHostToDevice, st));
    VK_LAUNCH(ctx, "mp_sum_parts", k_mp_sum_parts, ((size_t)Z * N + 255) / 256, 256, 0,
              reinterpret_cast<const Fr*>(d_S_parts), G, (size_t)Z * N, d_S.as<Fr>());
    const fe<F>*pw = nullptr, *pwi = nullptr, *inv1 = nullptr;
    VK_TRY(domain_tables<F>(ctx, bn254_group_gen(N), N, &pw, &pwi, &inv1));
    VK_LAUNCH(ctx, "mp_quot", k_mp_quot, Z, 256, 0, d_S.as<fe<F>>(), inv1, pw, pwi, d_zv.as<uint32_t>(), N,
              d_Q.as<fe<F>>());
    VK_LAUNCH(ctx, "mp_combine", k_mp_combine, (N + MP_CB_K - 1) / MP_CB_K, 256, 0, d_S.as<fe<F>>(), d_Q.as<fe<F>>(),
              (const fe<F>*)nullptr, N, Z, d_g.as<fe<F>>(), d_h.as<fe<F>>(), (fe<F>*)nullptr);
    // D = commit(g) and E = commit(h) read g / h in device memory (Montgomery scalars) on the latency
    // path, which completes by polled flags: no read-back of g or h and no stream wait; h - g (the
    // inner proof's data) is made on the device and copied into page-locked memory ahead of the E
    // commit, so it is on the host when E's flags are
    auto commit_dev = [&](const void* d_sc, uint64_t* xy, uint8_t* inf) -> int {
        VK_TRY(ctx->ws[WS_MISC].ensure(65));
        uint8_t* dxy_ = ctx->ws[WS_MISC].as<uint8_t>();
        bool on_host = false;
        VK_TRY(msm_batch_run(ctx, t, N, d_sc, 1, 1, dxy_, dxy_ + 64, xy, inf, &on_host, nullptr, nullptr));
        if (on_host) return VC_OK;
        uint8_t tmp[65];
        VK_CHECK_HIP(hipMemcpyAsync(tmp, dxy_, 65, hipMemcpyDeviceToHost, st));
        VK_CHECK_HIP(hipStreamSynchronize(st));
        memcpy(xy, tmp, 64);
        *inf = tmp[64];
        return VC_OK;
    };
    lap("sums, quotients, g");
    uint64_t dxy[8];
    uint8_t dinf;
    VK_TRY(commit_dev(d_g.p, dxy, &dinf));
    lap("D");
    transcript_append_point(tr, dxy, dinf, "D");
    Fr tt = transcript_digest(tr, "t");
    std::vector<Fr> invs = invert_domain_at(tt, N);  // 1/(t - z), z an integer (utils.rs:57-62)
    std::vector<Fr> invz(Z);
    for (uint32_t k = 0; k < Z; k++) invz[k] = invs[zval[k]];
    VK_TRY(ctx->pin_mp.ensure(N * 32 + (size_t)Z * 32));
    uint8_t* pin_hmg = static_cast<uint8_t*>(ctx->pin_mp.p);
    memcpy(pin_hmg + N * 32, invz.data(), Z * 32);
    VK_CHECK_HIP(hipMemcpyAsync(d_it.p, pin_hmg + N * 32, Z * 32, hipMemcpyHostToDevice, st));
    DevBuf d_hmg(ctx);
    VK_TRY(d_hmg.ensure(N * 32));
    VK_LAUNCH(ctx, "mp_combine", k_mp_combine, (N + MP_CB_K - 1) / MP_CB_K, 256, 0, d_S.as<fe<F>>(), d_Q.as<fe<F>>(),
              d_it.as<fe<F>>(), N, Z, d_g.as<fe<F>>(), d_h.as<fe<F>>(), d_hmg.as<fe<F>>());
    VK_CHECK_HIP(hipMemcpyAsync(pin_hmg, d_hmg.p, N * 32, hipMemcpyDeviceToHost, st));
    lap("t, h");
    uint64_t exy[8];
    uint8_t einf;
    VK_TRY(commit_dev(d_h.p, exy, &einf));  // (its completion follows the copy above in the stream)
    lap("E");
    transcript_append_point(tr, exy, einf, "E");
    std::vector<Fr> hmg(N);
    memcpy(hmg.data(), pin_hmg, N * 32);
    Acc mc = C::add(acc_of(exy, einf), C::neg(acc_of(dxy, dinf)));
    memcpy(d_xy, dxy, 64);
    *d_inf = dinf;
    if (scheme == 0) {
        std::vector<std::vector<Fr>> dd(1, hmg);
        std::vector<Acc> cs(1, mc);
        std::vector<Fr> ps(1, tt);
        vc_transcript* trs[1] = {tr};
        const int s = ipa_prove_impl(ctx, t, N, dd, cs, ps, trs, ipa_proof);
        lap("inner IPA proof");
        return s;
    }
    std::vector<uint64_t> ev(N * 4);
    for (size_t k = 0; k < N; k++) canon_of(hmg[k], &ev[4 * k]);
    uint64_t tc[4];
    canon_of(tt, tc);
    return kzg_prove_t<BN254G1, BN254Fr>(ctx, t, N, ev.data(), N, tc, kzg_xy, kzg_inf, kzg_y, nullptr);
}

static int mp_prove(vc_ctx* ctx, int scheme, Table* t, size_t N, size_t Q, const uint64_t* data, const uint64_t* com_xy,
                    const uint8_t* com_inf, const uint64_t* z, const uint64_t* y, uint64_t* d_xy, uint8_t* d_inf,
                    vc_ipa_proof* ipa_proof, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y) {
    vc_transcript* tr = nullptr;
    Fr r;
    std::vector<uint32_t> zval;
    if (!is_pow2(N) || Q == 0) return VC_E_INVALID;
    VK_TRY(mp_points(N, Q, z, &zval));
    DevBuf d_data(ctx), d_S(ctx);
    MpPlan pl(ctx);
    // the 32 Q N bytes of evaluations cross PCIe and the shard is planned under the transcript
    int st = mp_begin_overlapped(N, Q, com_xy, com_inf, z, y, &tr, &r, [&]() -> int {
        VK_TRY(d_data.ensure(Q * N * 32));
        VK_TRY(d_S.ensure(zval.size() * N * 32));
        VK_CHECK_HIP(hipMemcpyAsync(d_data.p, data, Q * N * 32, hipMemcpyHostToDevice, ctx->stream));
        return mp_plan(ctx, N, Q, z, 0, zval, &pl);
    });
    if (st != VC_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        return st;
    }
    st = mp_run(ctx, N, d_data.p, r, pl, d_S.p);
    if (st == VC_OK)
        st = mp_finish(ctx, scheme, t, N, zval, d_S.p, 1, tr, d_xy, d_inf, ipa_proof, kzg_xy, kzg_inf, kzg_y);
    vc_transcript_free(tr);
    return st;
}

// P independent multiproofs of Q queries each (same N, one CRS / SRS) on one GPU, proof-parallel:
// the host transcripts (records + serial SHA-256, the part that bounds one proof) run on worker
// threads while the GPU accumulates every proof whose challenge r is ready; each later stage then
// runs ONCE for all P proofs -- one batched D commit, one batched E commit and, for IPA, one
// batched inner proof (its 8 latency-bound rounds shared by the P proofs) -- instead of P times.
// Each proof is the one mp_prove gives for its queries. Arrays are [P][Q] (com_xy [P][Q][8],
// y [P][Q][4]); d_data [P][Q][N] canonical on the device; outputs [P].
static int mp_prove_many(vc_ctx* ctx, int scheme, Table* t, size_t N, size_t Q, size_t P, const uint8_t* d_data,
                         const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                         uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy,
                         uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!is_pow2(N) || Q == 0) return VC_E_INVALID;
    if (P == 0) return VC_OK;
    struct Begun {
        vc_transcript* tr = nullptr;
        Fr r;
        std::vector<uint32_t> zval;
        int st = VC_E_INVALID;
        bool done = false;
    };
    std::vector<Begun> B(P);
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<size_t> next{0};
    std::atomic<bool> cancel{false};  // set once phase 2 fails: the workers start no further transcript
    // one proof per worker at a time, each filled serially (no nested host pool): T workers share
    // the host's CPUs instead of queueing on the pool's one-loop lock
    const unsigned T = (unsigned)std::min<size_t>(P, std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2)));
    std::vector<std::thread> workers;
    for (unsigned k = 0; k < T; k++)
        workers.emplace_back([&] {
            for (size_t p; !cancel.load(std::memory_order_relaxed) && (p = next.fetch_add(1)) < P;) {
                Begun b;
                try {  // nothing may leave a thread function
                    b.st = mp_begin(N, Q, com_xy + p * Q * 8, com_inf + p * Q, z + p * Q, y + p * Q * 4, &b.tr,
                                    &b.r, false);
                    if (b.st == VC_OK) b.st = mp_points(N, Q, z + p * Q, &b.zval);
                } catch (...) {
                    b.st = VC_E_OOM;
                }
                std::lock_guard<std::mutex> lk(mu);
                B[p] = std::move(b);
                B[p].done = true;
                cv.notify_all();
            }
        });
    auto free_all = [&] {
        for (auto& w : workers) w.join();
        workers.clear();
        for (auto& b : B)
            if (b.tr) vc_transcript_free(b.tr);
    };
    // phase 2: per-point sums of each proof as soon as its transcript is done (GPU, in order)
    std::vector<std::unique_ptr<DevBuf>> S(P);
    int st = VC_OK;
    for (size_t p = 0; p < P && st == VC_OK; p++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return B[p].done; });
        }
        if ((st = B[p].st) != VC_OK) break;
        S[p] = std::make_unique<DevBuf>(ctx);
        st = S[p]->ensure(B[p].zval.size() * N * 32);
        if (st == VC_OK)
            st = mp_accumulate(ctx, N, Q, d_data + p * Q * N * 32, z + p * Q, B[p].r, 0, B[p].zval, S[p]->p);
    }
    if (st != VC_OK) cancel.store(true);
    for (auto& w : workers) w.join();
    workers.clear();
    if (st != VC_OK) {
        free_all();
        return st;
    }
    // phase 3: quotients and g of every proof, then D for all P in one batched commit
    hipStream_t hs = ctx->stream;
    const fe<F>*pw = nullptr, *pwi = nullptr, *inv1 = nullptr;
    st = domain_tables<F>(ctx, bn254_group_gen(N), N, &pw, &pwi, &inv1);
    std::vector<std::unique_ptr<DevBuf>> Sm(P), Qb(P), zv(P), it(P);
    DevBuf d_g(ctx), d_h(ctx);
    if (st == VC_OK) st = d_g.ensure(P * N * 32);
    if (st == VC_OK) st = d_h.ensure(P * N * 32);
    for (size_t p = 0; p < P && st == VC_OK; p++) {
        const uint32_t Z = (uint32_t)B[p].zval.size();
        Sm[p] = std::make_unique<DevBuf>(ctx);
        Qb[p] = std::make_unique<DevBuf>(ctx);
        zv[p] = std::make_unique<DevBuf>(ctx);
        it[p] = std::make_unique<DevBuf>(ctx);
        if ((st = Sm[p]->ensure((size_t)Z * N * 32)) != VC_OK || (st = Qb[p]->ensure((size_t)Z * N * 32)) != VC_OK ||
            (st = zv[p]->ensure(Z * 4)) != VC_OK || (st = it[p]->ensure(Z * 32)) != VC_OK)
            break;
        auto launch = [&]() -> int {
            VK_CHECK_HIP(hipMemcpyAsync(zv[p]->p, B[p].zval.data(), Z * 4, hipMemcpyHostToDevice, hs));
            VK_LAUNCH(ctx, "mp_sum_parts", k_mp_sum_parts, ((size_t)Z * N + 255) / 256, 256, 0, S[p]->as<Fr>(), 1,
                      (size_t)Z * N, Sm[p]->as<Fr>());
            VK_LAUNCH(ctx, "mp_quot", k_mp_quot, Z, 256, 0, Sm[p]->as<fe<F>>(), inv1, pw, pwi, zv[p]->as<uint32_t>(), N,
                      Qb[p]->as<fe<F>>());
            VK_LAUNCH(ctx, "mp_combine", k_mp_combine, (N + MP_CB_K - 1) / MP_CB_K, 256, 0, Sm[p]->as<fe<F>>(), Qb[p]->as<fe<F>>(),
                      (const fe<F>*)nullptr, N, Z, d_g.as<fe<F>>() + p * N, d_h.as<fe<F>>() + p * N,
                      (fe<F>*)nullptr);
            return VC_OK;
        };
        st = launch();
    }
    std::vector<Fr> g(P * N), h(P * N);
    std::vector<uint64_t> dxy(P * 8), exy(P * 8);
    std::vector<uint8_t> dinf(P), einf(P);
    std::vector<Fr> tt(P);
    if (st == VC_OK && hipMemcpyAsync(g.data(), d_g.p, P * N * 32, hipMemcpyDeviceToHost, hs) != hipSuccess) st = VC_E_HIP;
    if (st == VC_OK && hipStreamSynchronize(hs) != hipSuccess) st = VC_E_HIP;
    if (st == VC_OK) st = commit_batch(ctx, t, N, g.data(), P, dxy.data(), dinf.data());
    // t of every proof, then h and E for all P
    for (size_t p = 0; p < P && st == VC_OK; p++) {
        transcript_append_point(B[p].tr, &dxy[p * 8], dinf[p], "D");
        tt[p] = transcript_digest(B[p].tr, "t");
        const std::vector<Fr> invs = invert_domain_at(tt[p], N);  // 1/(t - z), z an integer (utils.rs:57-62)
        const uint32_t Z = (uint32_t)B[p].zval.size();
        std::vector<Fr> invz(Z);
        for (uint32_t k = 0; k < Z; k++) invz[k] = invs[B[p].zval[k]];
        if (hipMemcpyAsync(it[p]->p, invz.data(), Z * 32, hipMemcpyHostToDevice, hs) != hipSuccess) {
            st = VC_E_HIP;
            break;
        }
        auto launch = [&]() -> int {
            VK_LAUNCH(ctx, "mp_combine", k_mp_combine, (N + MP_CB_K - 1) / MP_CB_K, 256, 0, Sm[p]->as<fe<F>>(), Qb[p]->as<fe<F>>(),
                      it[p]->as<fe<F>>(), N, Z, d_g.as<fe<F>>() + p * N, d_h.as<fe<F>>() + p * N,
                      (fe<F>*)nullptr);
            return VC_OK;
        };
        st = launch();
        if (st == VC_OK && hipStreamSynchronize(hs) != hipSuccess) st = VC_E_HIP;  // invz dies here
    }
    if (st == VC_OK && hipMemcpyAsync(h.data(), d_h.p, P * N * 32, hipMemcpyDeviceToHost, hs) != hipSuccess) st = VC_E_HIP;
    if (st == VC_OK && hipStreamSynchronize(hs) != hipSuccess) st = VC_E_HIP;
    if (st == VC_OK) st = commit_batch(ctx, t, N, h.data(), P, exy.data(), einf.data());
    std::vector<std::vector<Fr>> hmg(P, std::vector<Fr>(N));
    std::vector<Acc> mc(P);
    for (size_t p = 0; p < P && st == VC_OK; p++) {
        transcript_append_point(B[p].tr, &exy[p * 8], einf[p], "E");
        for (size_t k = 0; k < N; k++) hmg[p][k] = fe_sub<F>(h[p * N + k], g[p * N + k]);
        mc[p] = C::add(acc_of(&exy[p * 8], einf[p]), C::neg(acc_of(&dxy[p * 8], dinf[p])));
        memcpy(d_xy + p * 8, &dxy[p * 8], 64);
        d_inf[p] = dinf[p];
    }
    // the inner proofs: one batched IPA (each proof with its own transcript), or P KZG openings
    if (st == VC_OK && scheme == 0) {
        std::vector<vc_transcript*> trs(P);
        for (size_t p = 0; p < P; p++) trs[p] = B[p].tr;
        st = ipa_prove_impl(ctx, t, N, hmg, mc, tt, trs.data(), ipa_proofs);
    }
    for (size_t p = 0; st == VC_OK && scheme == 1 && p < P; p++) {
        std::vector<uint64_t> ev(N * 4);
        for (size_t k = 0; k < N; k++) canon_of(hmg[p][k], &ev[4 * k]);
        uint64_t tc[4];
        canon_of(tt[p], tc);
        st = kzg_prove_t<BN254G1, BN254Fr>(ctx, t, N, ev.data(), N, tc, kzg_xy + p * 8, kzg_inf + p, kzg_y + p * 4,
                                          nullptr);
    }
    free_all();
    return st;
}

// E - D and t of verify_multiproof (:178-215); tr returned positioned after "E"
static int mp_claim(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                    const uint64_t* y, const uint64_t* d_xy, uint8_t d_inf, Acc* claim, Fr* t_out,
                    vc_transcript** tr_out) {
    if (!is_pow2(N) || N > (size_t(1) << 28)) return VC_E_INVALID;  // tables below are sized by N
    for (size_t i = 0; i < Q; i++)
        if (z[i] >= N) return VC_E_DOMAIN;
    const double c0 = verify_timing() ? verify_clock_us() : 0.0;
    vc_transcript* tr = nullptr;
    Fr r;
    // the e-coefficient MSM's points (the Q commitments) are uploaded and checked on the GPU while
    // the host transcript runs (mp_begin_overlapped) once the transcript is long enough to pay for
    // the helper thread (Q = 32768: verify 2.37-2.52 -> 2.28 ms; neutral at 4096)
    const bool filled = Q >= 8192;
    if (Q == 0) {  // no queries: the transcript of the labels alone (mp_begin wants Q > 0)
        tr = vc_transcript_new("multiproof");
        r = transcript_digest(tr, "r");
    } else if (filled) {
        VK_TRY(mp_begin_overlapped(N, Q, com_xy, com_inf, z, y, &tr, &r,
                                   [&] { return bases_fill(ctx, &ctx->scratch, com_xy, com_inf, Q); }));
    } else {
        VK_TRY(mp_begin(N, Q, com_xy, com_inf, z, y, &tr, &r));
    }
    vc_transcript_append_point(tr, d_xy, d_inf, "D");
    Fr tt = transcript_digest(tr, "t");
    std::vector<Fr> invs = invert_domain_at(tt, N);
    std::vector<Fr> coef(Q);
    // coef_i = r^i / (t - z_i): contiguous slices on the host pool, each starting from r^lo
    // (2 Q multiplies: ~2.5 ms serial at Q = 2^15)
    auto fill = [&](size_t lo, size_t hi) {
        Fr rp = fe_pow_u64<F>(r, lo);
        for (size_t i = lo; i < hi; i++) {
            coef[i] = fe_mul<F>(rp, invs[z[i]]);
            rp = fe_mul<F>(rp, r);
        }
    };
    if (Q < 4096 || host_pool().size() == 1) {
        fill(0, Q);
    } else {
        const unsigned T = host_pool().size();
        host_pool().run([&](unsigned k) { fill(Q * k / T, Q * (k + 1) / T); });
    }
    const double c1 = verify_timing() ? verify_clock_us() : 0.0;
    Acc e;
    int st = msm_points(ctx, com_xy, com_inf, coef, &e, filled);
    if (st != VC_OK) {
        vc_transcript_free(tr);
        return st;
    }
    if (verify_timing())
        fprintf(stderr, "mp_claim Q=%zu transcript+coef_us=%.1f e_msm_us=%.1f\n", Q, c1 - c0, verify_clock_us() - c1);
    uint64_t exy[8];
    uint8_t einf;
    aff_of(e, exy, &einf);
    vc_transcript_append_point(tr, exy, einf, "E");
    *claim = C::add(e, C::neg(acc_of(d_xy, d_inf)));
    *t_out = tt;
    *tr_out = tr;
    return VC_OK;
}

}  // namespace vk

extern "C" {

int vc_multiproof_prove(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, const uint64_t* data,
                        const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                        uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proof, uint64_t* kzg_xy, uint8_t* kzg_inf,
                        uint64_t* kzg_y) {
    if (!ctx || !data || !com_xy || !com_inf || !z || !y || !d_xy || !d_inf || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    if (scheme == 0 && !proof_ok(ipa_proof)) return VC_E_INVALID;
    if (scheme == 1 && (!kzg_xy || !kzg_inf || !kzg_y)) return VC_E_INVALID;
    if (scheme != 0 && scheme != 1) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    return mp_prove(ctx, scheme, t, N, Q, data, com_xy, com_inf, z, y, d_xy, d_inf, ipa_proof, kzg_xy, kzg_inf, kzg_y);
}

int vc_multiproof_prove_many(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, size_t P, const void* d_data,
                             const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z, const uint64_t* y,
                             uint64_t* d_xy, uint8_t* d_inf, vc_ipa_proof* ipa_proofs, uint64_t* kzg_xy,
                             uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!ctx || (P && (!d_data || !com_xy || !com_inf || !z || !y || !d_xy || !d_inf)) ||
        ctx->curve != VC_CURVE_BN254 || (scheme != 0 && scheme != 1))
        return VC_E_INVALID;
    for (size_t p = 0; scheme == 0 && p < P; p++)
        if (!ipa_proofs || !proof_ok(&ipa_proofs[p])) return VC_E_INVALID;
    if (scheme == 1 && P && (!kzg_xy || !kzg_inf || !kzg_y)) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    return mp_prove_many(ctx, scheme, t, N, Q, P, static_cast<const uint8_t*>(d_data), com_xy, com_inf, z, y, d_xy,
                         d_inf, ipa_proofs, kzg_xy, kzg_inf, kzg_y);
}

int vc_multiproof_begin(size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf, const uint64_t* z,
                        const uint64_t* y, vc_transcript** tr_out, uint64_t* r_out, size_t* rows) {
    if (!com_xy || !com_inf || !z || !y || !tr_out || !r_out || !rows) return VC_E_INVALID;
    vc_transcript* tr = nullptr;
    Fr r;
    VK_TRY(mp_begin(N, Q, com_xy, com_inf, z, y, &tr, &r, false));  // (callers overlap several)
    canon_of(r, r_out);
    std::vector<uint32_t> zval;
    const int zst = mp_points(N, Q, z, &zval);  // z itself was validated by mp_begin
    if (zst != VC_OK) {
        vc_transcript_free(tr);
        return zst;
    }
    *rows = zval.size();
    *tr_out = tr;
    return VC_OK;
}

int vc_multiproof_rows(size_t N, size_t Q, const uint64_t* z, size_t* rows) { return mp_rows(N, Q, z, rows); }

int vc_multiproof_begin_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                                   const uint64_t* z, const uint64_t* y, size_t first, size_t Qs, const void* d_data,
                                   void* d_S, vc_transcript** transcript, uint64_t* r) {
    return mp_begin_accumulate(ctx, N, Q, com_xy, com_inf, z, y, first, Qs, d_data, d_S, transcript, r);
}

int vc_multiproof_accumulate(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* z, size_t first, size_t Qs,
                             const void* d_data, const uint64_t* r, void* d_S) {
    if (!ctx || !z || !r || !d_S || (Qs && !d_data) || first > Q || Qs > Q - first || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    if (!is_pow2(N) || Q == 0) return VC_E_INVALID;
    Guard g(ctx);
    std::vector<uint32_t> zval;
    VK_TRY(mp_points(N, Q, z, &zval));
    return mp_accumulate(ctx, N, Qs, d_data, z + first, fr_of(r), first, zval, d_S);
}

int vc_multiproof_finish(vc_ctx* ctx, int scheme, int table, size_t N, size_t Q, const uint64_t* z,
                         const void* d_S_parts, int G, vc_transcript* tr, uint64_t* d_xy, uint8_t* d_inf,
                         vc_ipa_proof* ipa_proof, uint64_t* kzg_xy, uint8_t* kzg_inf, uint64_t* kzg_y) {
    if (!ctx || !z || !d_S_parts || G < 1 || !tr || !d_xy || !d_inf || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    if (scheme == 0 && !proof_ok(ipa_proof)) return VC_E_INVALID;
    if (scheme == 1 && (!kzg_xy || !kzg_inf || !kzg_y)) return VC_E_INVALID;
    if (scheme != 0 && scheme != 1) return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    std::vector<uint32_t> zval;
    VK_TRY(mp_points(N, Q, z, &zval));
    return mp_finish(ctx, scheme, t, N, zval, d_S_parts, G, tr, d_xy, d_inf, ipa_proof, kzg_xy, kzg_inf,
                     kzg_y);
}

int vc_multiproof_verify_ipa(vc_ctx* ctx, int table, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                             const uint64_t* z, const uint64_t* y, const uint64_t* d_xy, uint8_t d_inf,
                             const vc_ipa_proof* proof, int* result) {
    if (!ctx || !com_xy || !com_inf || !z || !y || !d_xy || !proof_ok(proof) || !result || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    Guard g(ctx);
    Table* t = ctx->table(table);
    if (!t) return VC_E_TABLE;
    Acc claim;
    Fr tt;
    vc_transcript* tr = nullptr;
    VK_TRY(mp_claim(ctx, N, Q, com_xy, com_inf, z, y, d_xy, d_inf, &claim, &tt, &tr));
    int st = ipa_verify_impl(ctx, t, N, claim, tt, proof, tr, result);
    vc_transcript_free(tr);
    return st;
}

int vc_multiproof_kzg_claim(vc_ctx* ctx, size_t N, size_t Q, const uint64_t* com_xy, const uint8_t* com_inf,
                            const uint64_t* z, const uint64_t* y, const uint64_t* d_xy, uint8_t d_inf, uint64_t* c_xy,
                            uint8_t* c_inf, uint64_t* t_out) {
    if (!ctx || !com_xy || !com_inf || !z || !y || !d_xy || !c_xy || !c_inf || !t_out || ctx->curve != VC_CURVE_BN254)
        return VC_E_INVALID;
    Guard g(ctx);
    Acc claim;
    Fr tt;
    vc_transcript* tr = nullptr;
    VK_TRY(mp_claim(ctx, N, Q, com_xy, com_inf, z, y, d_xy, d_inf, &claim, &tt, &tr));
    vc_transcript_free(tr);
    aff_of(claim, c_xy, c_inf);
    canon_of(tt, t_out);
    return VC_OK;
}

}  // extern "C"
