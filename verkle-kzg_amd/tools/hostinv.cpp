// Host Montgomery inversion variants for BLS12-381 Fq (the last serial step of every MSM call:
// acc_to_affine): the library's host fe_inv_bin (since round 5 the divstep inverse, fe_inv_host in
// csrc/ff.hpp), the 32-bit-limb binary Euclid and the standalone 64-bit-limb binary Euclid it
// replaced. Measured on the GPU box's host: Fermat with a 5-bit window 15 us, 32-bit binary 13.2
// us, 64-bit binary 7.4 us, divsteps 1.2 us (tools/hostops.cpp, profiles/r05/host_ops/).
// build: hipcc -O3 --offload-arch=gfx950 -I.. hostinv.cpp -o hostinv   (host code only)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include "../csrc/ff.hpp"
using namespace vk;
typedef unsigned __int128 u128;

template <class F>
fe<F> inv_old(const fe<F>& a_mont) {
    fe<F> u = a_mont, v, x1 = fe_zero<F>(), x2 = fe_zero<F>();
    for (int i = 0; i < F::N; i++) v.v[i] = F::p(i);
    x1.v[0] = 1;
    if (fe_is_zero<F>(u)) return fe_zero<F>();
    while (!fe_is_one_raw<F>(u) && !fe_is_one_raw<F>(v)) {
        while ((u.v[0] & 1) == 0) { fe_shr1<F>(u, 0); uint32_t c = (x1.v[0] & 1) ? fe_add_p_raw<F>(x1) : 0u; fe_shr1<F>(x1, c); }
        while ((v.v[0] & 1) == 0) { fe_shr1<F>(v, 0); uint32_t c = (x2.v[0] & 1) ? fe_add_p_raw<F>(x2) : 0u; fe_shr1<F>(x2, c); }
        if (fe_geq_raw<F>(u, v)) { fe_sub_raw<F>(u, v); x1 = fe_sub<F>(x1, x2); } else { fe_sub_raw<F>(v, u); x2 = fe_sub<F>(x2, x1); }
    }
    fe<F> r = fe_is_one_raw<F>(u) ? x1 : x2;
    fe<F> r2; for (int i = 0; i < F::N; i++) r2.v[i] = F::r2(i);
    return fe_mul<F>(fe_mul<F>(r, r2), r2);
}

// 64-bit limbs: u, v odd-reduction binary Euclid; x1, x2 kept in [0, p)
template <int M>
struct B64 {
    uint64_t p[M];
    static bool one(const uint64_t* a) { if (a[0] != 1) return false; for (int i = 1; i < M; i++) if (a[i]) return false; return true; }
    static void shr1(uint64_t* a, uint64_t top) { for (int i = 0; i < M - 1; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 63); a[M - 1] = (a[M - 1] >> 1) | (top << 63); }
    uint64_t addp(uint64_t* a) const { u128 c = 0; for (int i = 0; i < M; i++) { c += (u128)a[i] + p[i]; a[i] = (uint64_t)c; c >>= 64; } return (uint64_t)c; }
    static bool geq(const uint64_t* a, const uint64_t* b) { for (int i = M - 1; i >= 0; i--) if (a[i] != b[i]) return a[i] > b[i]; return true; }
    static void sub(uint64_t* a, const uint64_t* b) { uint64_t br = 0; for (int i = 0; i < M; i++) { u128 d = (u128)a[i] - b[i] - br; a[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; } }
    void subm(uint64_t* a, const uint64_t* b) const { if (geq(a, b)) sub(a, b); else { uint64_t t[M]; memcpy(t, b, sizeof t); sub(t, a); memcpy(a, p, sizeof t); sub(a, t); } }
    void inv(const uint64_t* a, uint64_t* out) const {
        uint64_t u[M], v[M], x1[M] = {1}, x2[M] = {0};
        memcpy(u, a, sizeof u); memcpy(v, p, sizeof v);
        while (!one(u) && !one(v)) {
            while ((u[0] & 1) == 0) { shr1(u, 0); uint64_t c = (x1[0] & 1) ? addp(x1) : 0; shr1(x1, c); }
            while ((v[0] & 1) == 0) { shr1(v, 0); uint64_t c = (x2[0] & 1) ? addp(x2) : 0; shr1(x2, c); }
            if (geq(u, v)) { sub(u, v); subm(x1, x2); } else { sub(v, u); subm(x2, x1); }
        }
        memcpy(out, one(u) ? x1 : x2, sizeof u);
    }
};

int main() {
    using F = BLS381Fq;
    B64<6> b;
    for (int i = 0; i < 6; i++) b.p[i] = (uint64_t)F::p(2 * i) | ((uint64_t)F::p(2 * i + 1) << 32);
    fe<F> a = fe_one<F>();
    for (int i = 0; i < F::N; i++) a.v[i] = 0x12345678u * (i + 1);
    a.v[F::N - 1] &= 0x0fffffff;
    a = fe_to_mont<F>(a);
    fe<F> r2; for (int i = 0; i < F::N; i++) r2.v[i] = F::r2(i);
    const int K = 2000;
    fe<F> y = a, z = a, w = a, m = a;
    auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) m = fe_mul<F>(m, a);
    auto t1 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) y = fe_inv_bin<F>(fe_add<F>(y, a));
    auto t2 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) z = inv_old<F>(fe_add<F>(z, a));
    auto t3 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) {
        fe<F> s = fe_add<F>(w, a), r;
        b.inv(reinterpret_cast<const uint64_t*>(s.v), reinterpret_cast<uint64_t*>(r.v));
        w = fe_mul<F>(fe_mul<F>(r, r2), r2);
    }
    auto t4 = std::chrono::steady_clock::now();
    auto us = [](auto a_, auto b_) { return std::chrono::duration<double, std::micro>(b_ - a_).count(); };
    printf("{\"mul_ns\": %.1f, \"library_fe_inv_bin_us\": %.2f, \"binary32_us\": %.2f, \"binary64_us\": %.2f, \"agree\": %d}\n",
           us(t0, t1) * 1e3 / K, us(t1, t2) / K, us(t2, t3) / K, us(t3, t4) / K,
           (int)(fe_eq<F>(y, z) && fe_eq<F>(z, w)) + (int)(m.v[0] == 12345));
}
