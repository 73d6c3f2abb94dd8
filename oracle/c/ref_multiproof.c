/* ORACLE (test infrastructure + CPU baseline only; never linked into the product).
 *
 * Plain-C restatement of the field phases of prove_multiproof
 * (/root/reference/vector-commit/src/multiproof.rs:99-176) over BN254 Fr, with the reference's own
 * thread structure -- the CPU baseline of configs[4] (C5):
 *   r_pows = powers_of(r, Q)                          (utils.rs:44-55, serial)
 *   scaled_i = data_i * r^i                           (:117-121, rayon par_iter over queries)
 *   per distinct point z: total_z = sum scaled_i,     (:124-146, rayon par_bridge over points)
 *       q_z = total_z.divide_by_vanishing(z)          (lagrange_basis.rs:91-119: two field
 *                                                      divisions per i, arkworks Div = inverse)
 *   g = sum_z q_z                                     (:148-150, serial)
 *   inv = invert_domain_at(t, N)                      (utils.rs:57-62, batch inversion)
 *   h = sum_z sum_i scaled_i * inv[z]                 (:160-165, serial)
 * r and t (transcript challenges), the commitments D / E and the inner proof are the caller's
 * (oracle/pyoracle/mpcheck.py assembles the whole proof; bench.py times the parts).
 * Inversions use the binary extended Euclid algorithm on Montgomery residues (what arkworks'
 * Fp::inverse runs), not Fermat. Pinned by tests/test_oracle.py against the Python restatement
 * (oracle/pyoracle/protocol.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

#define NL 4
/* BN254 scalar field r */
static const u64 P_[NL] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
#include "ref_field.h"

/* ---- binary extended Euclid inverse of a Montgomery residue a R (Guide to ECC alg. 2.22 in the
 * Montgomery domain, as arkworks 0.4 Fp::inverse): returns a^-1 R. */
static int big_is_one(const u64* a) { return a[0] == 1 && !(a[1] | a[2] | a[3]); }
static int big_is_even(const u64* a) { return (a[0] & 1) == 0; }
static void big_shr1(u64* a) {
    for (int i = 0; i < NL - 1; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 63);
    a[NL - 1] >>= 1;
}
static int big_geq(const u64* a, const u64* b) {
    for (int i = NL - 1; i >= 0; i--) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return 0;
    }
    return 1;
}
static void big_sub(u64* a, const u64* b) {
    u64 br = 0;
    for (int i = 0; i < NL; i++) {
        u128 d = (u128)a[i] - b[i] - br;
        a[i] = (u64)d;
        br = (u64)(d >> 64) ? 1 : 0;
    }
}
/* x / 2 mod p for x < p */
static void half_mod(fe* x) {
    if (x->v[0] & 1) {
        u64 c = 0;
        for (int i = 0; i < NL; i++) {
            u128 s = (u128)x->v[i] + P_[i] + c;
            x->v[i] = (u64)s;
            c = (u64)(s >> 64);
        }
        big_shr1(x->v);
        x->v[NL - 1] |= c << 63;
    } else {
        big_shr1(x->v);
    }
}
static void finv_euclid(fe* r, const fe* a) {
    u64 u[NL], v[NL];
    memcpy(u, a->v, sizeof u);
    memcpy(v, P_, sizeof v);
    fe b = R2_, c = {{0}};  /* b = R^2: the result stays in Montgomery form */
    while (!big_is_one(u) && !big_is_one(v)) {
        while (big_is_even(u)) {
            big_shr1(u);
            half_mod(&b);
        }
        while (big_is_even(v)) {
            big_shr1(v);
            half_mod(&c);
        }
        if (big_geq(u, v)) {
            big_sub(u, v);
            fsub(&b, &b, &c);
        } else {
            big_sub(v, u);
            fsub(&c, &c, &b);
        }
    }
    *r = big_is_one(u) ? b : c;
}

static void fpow_small(fe* r, const fe* a, u64 e) { /* ark pow([e]): MSB-first square-and-multiply */
    fe acc = ONE_;
    int started = 0;
    for (int b = 63; b >= 0; b--) {
        if (started) fmul(&acc, &acc, &acc);
        if ((e >> b) & 1) {
            fmul(&acc, &acc, a);
            started = 1;
        }
    }
    *r = acc;
}

typedef struct {
    size_t N, Q;
    const u64* data;  /* Q x N canonical */
    const u64* z;     /* Q */
    const fe* rp;     /* Q powers of r */
    fe* scaled;       /* Q x N */
    const fe* omega;
    const fe* van;
    const fe* van_inv;
    /* grouping: distinct points and their query lists */
    size_t npts;
    const u64* pts;
    const size_t* qstart;  /* npts + 1 */
    const size_t* qidx;    /* Q, queries grouped by point */
    fe* quot;              /* npts x N */
    size_t lo, hi;         /* query range (scale) / point range (quotients) */
} mp_job;

static void* scale_job(void* arg) {
    mp_job* j = (mp_job*)arg;
    for (size_t i = j->lo; i < j->hi; i++)
        for (size_t k = 0; k < j->N; k++) {
            fe e;
            to_mont(&e, j->data + (i * j->N + k) * 4);
            fmul(&j->scaled[i * j->N + k], &e, &j->rp[i]);
        }
    return NULL;
}

static void* quot_job(void* arg) {
    mp_job* j = (mp_job*)arg;
    const size_t N = j->N;
    fe* total = (fe*)malloc(sizeof(fe) * N);
    for (size_t p = j->lo; p < j->hi; p++) {
        memset(total, 0, sizeof(fe) * N);
        for (size_t s = j->qstart[p]; s < j->qstart[p + 1]; s++) {
            const fe* src = j->scaled + j->qidx[s] * N;
            for (size_t k = 0; k < N; k++) fadd(&total[k], &total[k], &src[k]);
        }
        const size_t index = (size_t)j->pts[p];
        fe* q = j->quot + p * N;
        memset(q, 0, sizeof(fe) * N);
        fe index_f;
        fpow_small(&index_f, j->omega, index);
        const fe eval = total[index];  /* max = N: every index is < max */
        for (size_t i = 0; i < N; i++) {
            if (i == index) continue;
            fe i_f, sub, den, inv, t;
            fpow_small(&i_f, j->omega, i);
            fsub(&sub, &total[i], &eval);
            fsub(&den, &i_f, &index_f);
            finv_euclid(&inv, &den);
            fmul(&q[i], &sub, &inv);
            fmul(&t, &sub, &j->van[index]);
            fmul(&t, &t, &j->van_inv[i]);
            fsub(&den, &index_f, &i_f);
            finv_euclid(&inv, &den);
            fmul(&t, &t, &inv);
            fadd(&q[index], &q[index], &t);
        }
    }
    free(total);
    return NULL;
}

static void run_threads(void* (*fn)(void*), mp_job* base, size_t count, int T) {
    if ((size_t)T > count) T = count ? (int)count : 1;
    mp_job* jobs = (mp_job*)calloc(T, sizeof(mp_job));
    pthread_t* th = (pthread_t*)calloc(T, sizeof(pthread_t));
    for (int t = 0; t < T; t++) {
        jobs[t] = *base;
        jobs[t].lo = count * t / T;
        jobs[t].hi = count * (t + 1) / T;
    }
    for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
    fn(&jobs[0]);
    for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

/* Two-phase form (prove_multiproof needs g before the transcript yields t, and h after it):
 * bn254fr_mp_g runs :117-150 (scaling, grouped quotients, g) and keeps the scaled data and the
 * grouping; bn254fr_mp_h runs :155-165 (invert_domain_at(t), h) on them; bn254fr_mp_free releases.
 * N = domain size (power of two, every query's data has N values), z[i] < N; r, omega canonical.
 * g_out: N x 4 canonical. Returns the state, or NULL on a bad argument. */
typedef struct {
    size_t N, Q, npts;
    u64* pts;
    size_t* qstart;
    size_t* qidx;
    fe* scaled;
} mp_state;

void* bn254fr_mp_g(size_t N, size_t Q, const u64* data, const u64* z, const u64* r_c, const u64* omega_c,
                   int nthreads, u64* g_out) {
    init();
    if (N == 0 || (N & (N - 1)) || Q == 0) return NULL;
    for (size_t i = 0; i < Q; i++)
        if (z[i] >= N) return NULL;
    const int T = nthreads < 1 ? 1 : nthreads;
    fe r, omega;
    to_mont(&r, r_c);
    to_mont(&omega, omega_c);
    /* precompute.rs:47-58: van[i] = N / w^i, van_inv = 1 / van */
    fe* van = (fe*)malloc(sizeof(fe) * N);
    fe* van_inv = (fe*)malloc(sizeof(fe) * N);
    fe nf;
    {
        u64 nn[NL] = {N, 0, 0, 0};
        to_mont(&nf, nn);
    }
    for (size_t i = 0; i < N; i++) {
        fe w, wi;
        fpow_small(&w, &omega, i);
        finv_euclid(&wi, &w);
        fmul(&van[i], &nf, &wi);
        finv_euclid(&van_inv[i], &van[i]);
    }
    fe* rp = (fe*)malloc(sizeof(fe) * Q);
    rp[0] = ONE_;
    for (size_t i = 1; i < Q; i++) fmul(&rp[i], &rp[i - 1], &r);
    fe* scaled = (fe*)malloc(sizeof(fe) * Q * N);
    mp_job jb;
    memset(&jb, 0, sizeof jb);
    jb.N = N;
    jb.Q = Q;
    jb.data = data;
    jb.z = z;
    jb.rp = rp;
    jb.scaled = scaled;
    jb.omega = &omega;
    jb.van = van;
    jb.van_inv = van_inv;
    run_threads(scale_job, &jb, Q, T);
    /* group by point (counting sort over z < N) */
    size_t* cnt = (size_t*)calloc(N + 1, sizeof(size_t));
    for (size_t i = 0; i < Q; i++) cnt[z[i] + 1]++;
    u64* pts = (u64*)malloc(sizeof(u64) * N);
    size_t* qstart = (size_t*)malloc(sizeof(size_t) * (N + 1));
    size_t npts = 0, acc = 0;
    for (size_t v = 0; v < N; v++)
        if (cnt[v + 1]) {
            pts[npts] = v;
            qstart[npts] = acc;
            acc += cnt[v + 1];
            npts++;
        }
    qstart[npts] = acc;
    size_t* pos = (size_t*)calloc(N, sizeof(size_t));
    size_t* slot = (size_t*)malloc(sizeof(size_t) * N);
    for (size_t p = 0; p < npts; p++) slot[pts[p]] = qstart[p];
    size_t* qidx = (size_t*)malloc(sizeof(size_t) * Q);
    for (size_t i = 0; i < Q; i++) qidx[slot[z[i]] + pos[z[i]]++] = i;
    fe* quot = (fe*)malloc(sizeof(fe) * npts * N);
    jb.npts = npts;
    jb.pts = pts;
    jb.qstart = qstart;
    jb.qidx = qidx;
    jb.quot = quot;
    run_threads(quot_job, &jb, npts, T);
    fe* g = (fe*)calloc(N, sizeof(fe));
    for (size_t p = 0; p < npts; p++)
        for (size_t k = 0; k < N; k++) fadd(&g[k], &g[k], &quot[p * N + k]);
    for (size_t k = 0; k < N; k++) from_mont(g_out + 4 * k, &g[k]);
    free(g), free(quot), free(slot), free(pos), free(cnt), free(rp), free(van_inv), free(van);
    mp_state* st = (mp_state*)calloc(1, sizeof(mp_state));
    st->N = N;
    st->Q = Q;
    st->npts = npts;
    st->pts = pts;
    st->qstart = qstart;
    st->qidx = qidx;
    st->scaled = scaled;
    return st;
}

/* t canonical; h_out: N x 4 canonical. Returns 0, or -1 when t - i = 0 for some i < N. */
int bn254fr_mp_h(void* state, const u64* t_c, u64* h_out) {
    mp_state* st = (mp_state*)state;
    const size_t N = st->N;
    if (N == 0) return -1;
    fe t;
    to_mont(&t, t_c);
    /* invert_domain_at(t, N): 1 / (t - i), batch inversion (one inversion + 3 (N - 1) products) */
    fe* inv = (fe*)malloc(sizeof(fe) * N);
    fe* pre = (fe*)malloc(sizeof(fe) * N);
    int bad = 0;
    for (size_t i = 0; i < N; i++) {
        u64 ii[NL] = {i, 0, 0, 0};
        fe fi;
        to_mont(&fi, ii);
        fsub(&inv[i], &t, &fi);
        if (fiszero(&inv[i])) bad = 1;
    }
    if (bad) {
        free(inv), free(pre);
        return -1;
    }
    pre[0] = inv[0];
    for (size_t i = 1; i < N; i++) fmul(&pre[i], &pre[i - 1], &inv[i]);
    fe run;
    finv_euclid(&run, &pre[N - 1]);
    for (size_t i = N; i-- > 1;) {
        fe orig = inv[i];
        fmul(&inv[i], &run, &pre[i - 1]);
        fmul(&run, &run, &orig);
    }
    inv[0] = run;
    fe* h = (fe*)calloc(N, sizeof(fe));
    for (size_t p = 0; p < st->npts; p++)
        for (size_t s = st->qstart[p]; s < st->qstart[p + 1]; s++) {
            const fe* src = st->scaled + st->qidx[s] * N;
            for (size_t k = 0; k < N; k++) {
                fe m;
                fmul(&m, &src[k], &inv[st->pts[p]]);
                fadd(&h[k], &h[k], &m);
            }
        }
    for (size_t k = 0; k < N; k++) from_mont(h_out + 4 * k, &h[k]);
    free(h), free(pre), free(inv);
    return 0;
}

void bn254fr_mp_free(void* state) {
    mp_state* st = (mp_state*)state;
    if (!st) return;
    free(st->pts), free(st->qstart), free(st->qidx), free(st->scaled);
    free(st);
}

/* One-call form: g and h for given r and t. Returns 0, or -1 on a bad argument. */
int bn254fr_mp_field_phases(size_t N, size_t Q, const u64* data, const u64* z, const u64* r_c, const u64* t_c,
                            const u64* omega_c, int nthreads, u64* g_out, u64* h_out) {
    void* st = bn254fr_mp_g(N, Q, data, z, r_c, omega_c, nthreads, g_out);
    if (!st) return -1;
    int rc = bn254fr_mp_h(st, t_c, h_out);
    bn254fr_mp_free(st);
    return rc;
}
