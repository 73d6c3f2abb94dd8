/* ORACLE (test infrastructure + CPU baseline only; never linked into the product).
 *
 * Plain-C restatement of the reference MSM `utils::inner_product`
 * (/root/reference/vector-commit/src/utils.rs:16-19):
 *     a.iter().zip(b).map(|(P, s)| P * s).sum()
 * i.e. one full double-and-add scalar multiplication per term (arkworks 0.4
 * `sw_double_and_add_projective` / `mul_bigint`: MSB-first over the canonical
 * scalar bits, leading zeros skipped, general projective add of the base), then a
 * sequential fold from zero.  64-bit-limb Montgomery (CIOS) field arithmetic
 * with unsigned __int128, like arkworks' own backend.
 *
 * Compiled once per curve (-DCURVE_BN254 / -DCURVE_BLS12_381 / -DCURVE_BANDERSNATCH)
 * into oracle/_build/libref_oracle.so; symbols are prefixed with the curve name.
 * Optional pthread split of the terms (the sum is commutative, so the affine
 * result is identical to the sequential fold); cores used = nthreads.
 *
 * Pinned by tests/test_oracle.py against the Python big-int oracle
 * (oracle/pyoracle), itself pinned by generator / r*G = O KATs.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;


#if defined(CURVE_BN254)
#define NL 4
#define PFX(x) bn254_##x
#define SW 1
#define COEFF_B 3
static const u64 P_[NL] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
#elif defined(CURVE_BLS12_381)
#define NL 6
#define PFX(x) bls12_381_##x
#define SW 1
#define COEFF_B 4
static const u64 P_[NL] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                           0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
#elif defined(CURVE_BANDERSNATCH)
#define NL 4
#define PFX(x) bandersnatch_##x
#define SW 0
/* base field = BLS12-381 Fr */
static const u64 P_[NL] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
/* d = 45022363124591815672509500913686876175488063829319466900776701791074614335719, a = -5 */
static const u64 D_CANON[NL] = {0xb369f2f5188d58e7ULL, 0xcb66677177e54f92ULL, 0xc66e3bf86be3b6d8ULL, 0x6389c12633c267cbULL};
#else
#error "define a curve"
#endif

#include "ref_field.h"

#if SW
/* ------------------------------------------------ short Weierstrass a=0, Jacobian */
typedef struct { fe x, y, z; } pt;
static void pzero(pt* p) { memset(p, 0, sizeof *p); p->y = ONE_; }
static int piszero(const pt* p) { return fiszero(&p->z); }
static void pdbl(pt* r, const pt* p) {
    if (piszero(p)) { *r = *p; return; }
    fe A, B, C, D, E, F, t;
    fmul(&A, &p->x, &p->x);
    fmul(&B, &p->y, &p->y);
    fmul(&C, &B, &B);
    fadd(&t, &p->x, &B);
    fmul(&t, &t, &t);
    fsub(&t, &t, &A);
    fsub(&t, &t, &C);
    fadd(&D, &t, &t);
    fadd(&E, &A, &A);
    fadd(&E, &E, &A);
    fmul(&F, &E, &E);
    pt o;
    fsub(&o.x, &F, &D);
    fsub(&o.x, &o.x, &D);
    fsub(&t, &D, &o.x);
    fmul(&t, &E, &t);
    fe c8;
    fadd(&c8, &C, &C);
    fadd(&c8, &c8, &c8);
    fadd(&c8, &c8, &c8);
    fsub(&o.y, &t, &c8);
    fmul(&o.z, &p->y, &p->z);
    fadd(&o.z, &o.z, &o.z);
    *r = o;
}
static void padd(pt* r, const pt* p, const pt* q) {
    if (piszero(p)) { *r = *q; return; }
    if (piszero(q)) { *r = *p; return; }
    fe z1z1, z2z2, u1, u2, s1, s2, t;
    fmul(&z1z1, &p->z, &p->z);
    fmul(&z2z2, &q->z, &q->z);
    fmul(&u1, &p->x, &z2z2);
    fmul(&u2, &q->x, &z1z1);
    fmul(&t, &q->z, &z2z2);
    fmul(&s1, &p->y, &t);
    fmul(&t, &p->z, &z1z1);
    fmul(&s2, &q->y, &t);
    if (feq(&u1, &u2)) {
        if (feq(&s1, &s2)) { pdbl(r, p); return; }
        pzero(r);
        return;
    }
    fe h, i, j, rr, v;
    fsub(&h, &u2, &u1);
    fadd(&i, &h, &h);
    fmul(&i, &i, &i);
    fmul(&j, &h, &i);
    fsub(&rr, &s2, &s1);
    fadd(&rr, &rr, &rr);
    fmul(&v, &u1, &i);
    pt o;
    fmul(&o.x, &rr, &rr);
    fsub(&o.x, &o.x, &j);
    fsub(&o.x, &o.x, &v);
    fsub(&o.x, &o.x, &v);
    fsub(&t, &v, &o.x);
    fmul(&t, &rr, &t);
    fmul(&s1, &s1, &j);
    fadd(&s1, &s1, &s1);
    fsub(&o.y, &t, &s1);
    fadd(&t, &p->z, &q->z);
    fmul(&t, &t, &t);
    fsub(&t, &t, &z1z1);
    fsub(&t, &t, &z2z2);
    fmul(&o.z, &t, &h);
    *r = o;
}
static void pload(pt* r, const u64* xy, int inf) {
    if (inf) { pzero(r); return; }
    to_mont(&r->x, xy);
    to_mont(&r->y, xy + NL);
    r->z = ONE_;
}
static void pstore(u64* xy, uint8_t* inf, const pt* p) {
    if (piszero(p)) {
        memset(xy, 0, 2 * NL * sizeof(u64));
        *inf = 1;
        return;
    }
    fe zi, zi2, zi3, x, y;
    finv(&zi, &p->z);
    fmul(&zi2, &zi, &zi);
    fmul(&zi3, &zi2, &zi);
    fmul(&x, &p->x, &zi2);
    fmul(&y, &p->y, &zi3);
    from_mont(xy, &x);
    from_mont(xy + NL, &y);
    *inf = 0;
}
/* mixed add, p Jacobian + (x2, y2) affine Montgomery (madd-2007-bl, 7M + 4S): the bucket add of
 * the Pippenger baseline below (arkworks' buckets also add affine bases into projective sums) */
static void pmadd(pt* r, const pt* p, const fe* x2, const fe* y2) {
    if (piszero(p)) { r->x = *x2; r->y = *y2; r->z = ONE_; return; }
    fe z1z1, u2, s2, t;
    fmul(&z1z1, &p->z, &p->z);
    fmul(&u2, x2, &z1z1);
    fmul(&t, &p->z, &z1z1);
    fmul(&s2, y2, &t);
    if (feq(&u2, &p->x)) {
        if (feq(&s2, &p->y)) { pdbl(r, p); return; }
        pzero(r);
        return;
    }
    fe h, hh, i, j, rr, v;
    fsub(&h, &u2, &p->x);
    fmul(&hh, &h, &h);
    fadd(&i, &hh, &hh);
    fadd(&i, &i, &i);
    fmul(&j, &h, &i);
    fsub(&rr, &s2, &p->y);
    fadd(&rr, &rr, &rr);
    fmul(&v, &p->x, &i);
    pt o;
    fmul(&o.x, &rr, &rr);
    fsub(&o.x, &o.x, &j);
    fsub(&o.x, &o.x, &v);
    fsub(&o.x, &o.x, &v);
    fsub(&t, &v, &o.x);
    fmul(&t, &rr, &t);
    fmul(&s2, &p->y, &j);
    fadd(&s2, &s2, &s2);
    fsub(&o.y, &t, &s2);
    fadd(&t, &p->z, &h);
    fmul(&t, &t, &t);
    fsub(&t, &t, &z1z1);
    fsub(&o.z, &t, &hh);
    *r = o;
}
typedef struct { fe x, y; int inf; } aff;
static void aload(aff* a, const u64* xy, int inf) {
    a->inf = inf;
    if (inf) return;
    to_mont(&a->x, xy);
    to_mont(&a->y, xy + NL);
}
static void aadd(pt* r, const pt* p, const aff* a, int neg) {
    if (a->inf) { *r = *p; return; }
    if (!neg) { pmadd(r, p, &a->x, &a->y); return; }
    fe ny, z = {{0}};
    fsub(&ny, &z, &a->y);
    pmadd(r, p, &a->x, &ny);
}
#else
/* ------------------------------------------------ twisted Edwards a=-5, extended (X,Y,T,Z) */
typedef struct { fe x, y, t, z; } pt;
static fe D_;
static void pzero(pt* p) { memset(p, 0, sizeof *p); p->y = ONE_; p->z = ONE_; }
static void padd(pt* r, const pt* p, const pt* q) {
    /* add-2008-hwcd (unified, complete for a non-square, d non-square) */
    fe A, B, C, Dd, E, F, G, H, t1, t2;
    fmul(&A, &p->x, &q->x);
    fmul(&B, &p->y, &q->y);
    fmul(&C, &p->t, &q->t);
    fmul(&C, &C, &D_);
    fmul(&Dd, &p->z, &q->z);
    fadd(&t1, &p->x, &p->y);
    fadd(&t2, &q->x, &q->y);
    fmul(&E, &t1, &t2);
    fsub(&E, &E, &A);
    fsub(&E, &E, &B);
    fsub(&F, &Dd, &C);
    fadd(&G, &Dd, &C);
    /* H = B - a*A = B + 5A */
    fadd(&t1, &A, &A);
    fadd(&t1, &t1, &t1);
    fadd(&t1, &t1, &A);
    fadd(&H, &B, &t1);
    pt o;
    fmul(&o.x, &E, &F);
    fmul(&o.y, &G, &H);
    fmul(&o.t, &E, &H);
    fmul(&o.z, &F, &G);
    *r = o;
}
static void pdbl(pt* r, const pt* p) { padd(r, p, p); }
static void pload(pt* r, const u64* xy, int inf) {
    if (inf) { pzero(r); return; }
    to_mont(&r->x, xy);
    to_mont(&r->y, xy + NL);
    fmul(&r->t, &r->x, &r->y);
    r->z = ONE_;
}
static void pstore(u64* xy, uint8_t* inf, const pt* p) {
    fe zi, x, y;
    finv(&zi, &p->z);
    fmul(&x, &p->x, &zi);
    fmul(&y, &p->y, &zi);
    from_mont(xy, &x);
    from_mont(xy + NL, &y);
    /* identity is (0, 1); y is canonical here */
    u64 one_c[NL] = {1};
    *inf = (fiszero(&x) && memcmp(xy + NL, one_c, sizeof one_c) == 0) ? 1 : 0;
}
#endif

#if !SW
typedef struct { pt p; int inf; } aff;  /* extended with Z = 1 (T = x y) */
static void aload(aff* a, const u64* xy, int inf) {
    a->inf = inf;
    if (!inf) pload(&a->p, xy, 0);
}
static void aadd(pt* r, const pt* p, const aff* a, int neg) {
    if (a->inf) { *r = *p; return; }
    if (!neg) { padd(r, p, &a->p); return; }
    pt q = a->p;
    fe z = {{0}};
    fsub(&q.x, &z, &q.x);
    fsub(&q.t, &z, &q.t);
    padd(r, p, &q);
}
#endif

/* arkworks mul_bigint: MSB-first, leading zeros skipped */
static void pmul(pt* r, const pt* base, const u64* k /*4 limbs canonical*/) {
    pt acc;
    pzero(&acc);
    int started = 0;
    for (int i = 3; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            int bit = (k[i] >> b) & 1;
            if (!started && !bit) continue;
            started = 1;
            pdbl(&acc, &acc);
            if (bit) padd(&acc, &acc, base);
        }
    *r = acc;
}

typedef struct {
    const u64* bases;
    const uint8_t* inf;
    const u64* scalars;
    size_t lo, hi;
    pt acc;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    pt acc;
    pzero(&acc);
    for (size_t i = j->lo; i < j->hi; i++) {
        pt b, m;
        pload(&b, j->bases + i * 2 * NL, j->inf ? j->inf[i] : 0);
        pmul(&m, &b, j->scalars + i * 4);
        padd(&acc, &acc, &m);
    }
    j->acc = acc;
    return NULL;
}

/* naive MSM; bases: n x (x[NL], y[NL]) canonical LE u64; scalars: n x 4 u64 canonical (< r) */
int PFX(ref_msm)(const u64* bases, const uint8_t* inf, const u64* scalars, size_t n, int nthreads,
                 u64* out_xy, uint8_t* out_inf) {
    init();
#if !SW
    to_mont(&D_, D_CANON);
#endif
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    job_t* jobs = (job_t*)calloc(nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t].bases = bases;
        jobs[t].inf = inf;
        jobs[t].scalars = scalars;
        jobs[t].lo = n * t / nthreads;
        jobs[t].hi = n * (t + 1) / nthreads;
    }
    if (nthreads == 1) run_job(&jobs[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    pt acc;
    pzero(&acc);
    for (int t = 0; t < nthreads; t++) padd(&acc, &acc, &jobs[t].acc);
    pstore(out_xy, out_inf, &acc);
    free(jobs);
    free(th);
    return 0;
}

/* ------------------------------------------------ Pippenger baseline (SURVEY 8(d) "fair CPU bound")
 * The same MSM by the bucket method on T threads: thread t runs a whole Pippenger over its point
 * chunk [n t / T, n (t + 1) / T) -- signed c-bit digits (c ~ 0.69 log2(m) + 2, arkworks'
 * ln_without_floats + 2), mixed bucket adds of affine bases, running-sum bucket reduction, Horner
 * over windows -- and the T chunk sums are added. Exact group arithmetic: the affine result equals
 * ref_msm's. Not a restatement of a reference line; it is the all-core CPU bound a fair
 * comparison needs beside the 1-core naive port above. */
static int pip_window(size_t m) {
    int lg = 0;
    while (((size_t)1 << (lg + 1)) <= m) lg++;
    int c = lg * 69 / 100 + 2;
    if (c < 2) c = 2;
    if (c > 16) c = 16;
    return c;
}

static void pip_chunk(const u64* bases, const uint8_t* inf, const u64* scalars, size_t lo, size_t hi, pt* out) {
    pzero(out);
    const size_t m = hi - lo;
    if (m == 0) return;
    const int c = pip_window(m);
    const int W = (256 + 1 + c - 1) / c;  /* one spare bit absorbs the last carry */
    const u64 mask = ((u64)1 << c) - 1;
    const int64_t half = (int64_t)1 << (c - 1);
    int32_t* dig = (int32_t*)malloc(sizeof(int32_t) * m * W);
    aff* pts = (aff*)malloc(sizeof(aff) * m);
    for (size_t i = 0; i < m; i++) {
        aload(&pts[i], bases + (lo + i) * 2 * NL, inf ? inf[lo + i] : 0);
        const u64* k = scalars + (lo + i) * 4;
        int64_t carry = 0;
        for (int w = 0; w < W; w++) {
            const int b0 = w * c;
            u64 raw = 0;
            if (b0 < 256) {
                const int q = b0 / 64, s = b0 % 64;
                raw = k[q] >> s;
                if (s && q + 1 < 4) raw |= k[q + 1] << (64 - s);
            }
            int64_t d = (int64_t)(raw & mask) + carry;
            if (d > half) {
                d -= (int64_t)1 << c;
                carry = 1;
            } else {
                carry = 0;
            }
            dig[i * W + w] = (int32_t)d;
        }
    }
    const size_t NB = (size_t)1 << (c - 1);
    pt* bk = (pt*)malloc(sizeof(pt) * NB);
    for (int w = W - 1; w >= 0; w--) {
        for (int k = 0; k < c && w < W - 1; k++) pdbl(out, out);
        for (size_t b = 0; b < NB; b++) pzero(&bk[b]);
        for (size_t i = 0; i < m; i++) {
            const int32_t d = dig[i * W + w];
            if (d > 0) aadd(&bk[d - 1], &bk[d - 1], &pts[i], 0);
            else if (d < 0) aadd(&bk[-d - 1], &bk[-d - 1], &pts[i], 1);
        }
        pt run, sum;
        pzero(&run);
        pzero(&sum);
        for (size_t b = NB; b-- > 0;) {
            padd(&run, &run, &bk[b]);
            padd(&sum, &sum, &run);
        }
        padd(out, out, &sum);
    }
    free(bk);
    free(pts);
    free(dig);
}

typedef struct {
    const u64* bases;
    const uint8_t* inf;
    const u64* scalars;
    size_t lo, hi;     /* point chunk (pip_msm) or commit range (pip_msm_batch) */
    size_t width;      /* 0: one chunk; else commits of `width` terms over bases[0, width) */
    u64* out_xy;
    uint8_t* out_inf;
    pt acc;
} pjob_t;

static void* pip_job(void* arg) {
    pjob_t* j = (pjob_t*)arg;
    if (j->width == 0) {
        pip_chunk(j->bases, j->inf, j->scalars, j->lo, j->hi, &j->acc);
        return NULL;
    }
    for (size_t g = j->lo; g < j->hi; g++) {
        pt r;
        pip_chunk(j->bases, j->inf, j->scalars + g * j->width * 4, 0, j->width, &r);
        pstore(j->out_xy + g * 2 * NL, j->out_inf + g, &r);
    }
    return NULL;
}

static void pip_run(pjob_t* jobs, int T) {
    pthread_t* th = (pthread_t*)calloc(T, sizeof(pthread_t));
    for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, pip_job, &jobs[t]);
    pip_job(&jobs[0]);
    for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
    free(th);
}

int PFX(pip_msm)(const u64* bases, const uint8_t* inf, const u64* scalars, size_t n, int nthreads, u64* out_xy,
                 uint8_t* out_inf) {
    init();
#if !SW
    to_mont(&D_, D_CANON);
#endif
    int T = nthreads < 1 ? 1 : nthreads;
    if ((size_t)T > n / 64) T = n / 64 ? (int)(n / 64) : 1;  /* at least 64 points per chunk */
    pjob_t* jobs = (pjob_t*)calloc(T, sizeof(pjob_t));
    for (int t = 0; t < T; t++) {
        jobs[t].bases = bases;
        jobs[t].inf = inf;
        jobs[t].scalars = scalars;
        jobs[t].lo = n * t / T;
        jobs[t].hi = n * (t + 1) / T;
    }
    pip_run(jobs, T);
    pt acc;
    pzero(&acc);
    for (int t = 0; t < T; t++) padd(&acc, &acc, &jobs[t].acc);
    pstore(out_xy, out_inf, &acc);
    free(jobs);
    return 0;
}

/* `batch` commits of width terms each over bases[0, width) (scalars batch x width), commits split
 * over T threads (the batched-commit baseline) */
int PFX(pip_msm_batch)(const u64* bases, const uint8_t* inf, const u64* scalars, size_t width, size_t batch,
                       int nthreads, u64* out_xy, uint8_t* out_inf) {
    init();
#if !SW
    to_mont(&D_, D_CANON);
#endif
    if (width == 0) return -1;
    int T = nthreads < 1 ? 1 : nthreads;
    if ((size_t)T > batch) T = batch ? (int)batch : 1;
    pjob_t* jobs = (pjob_t*)calloc(T, sizeof(pjob_t));
    for (int t = 0; t < T; t++) {
        jobs[t].bases = bases;
        jobs[t].inf = inf;
        jobs[t].scalars = scalars;
        jobs[t].lo = batch * t / T;
        jobs[t].hi = batch * (t + 1) / T;
        jobs[t].width = width;
        jobs[t].out_xy = out_xy;
        jobs[t].out_inf = out_inf;
    }
    pip_run(jobs, T);
    free(jobs);
    return 0;
}

/* on-curve check of canonical affine points (used to validate generated inputs) */
int PFX(ref_on_curve)(const u64* bases, size_t n) {
    init();
#if !SW
    to_mont(&D_, D_CANON);
#endif
    for (size_t i = 0; i < n; i++) {
        fe x, y, x2, y2, l, r;
        to_mont(&x, bases + i * 2 * NL);
        to_mont(&y, bases + i * 2 * NL + NL);
        fmul(&x2, &x, &x);
        fmul(&y2, &y, &y);
#if SW
        fe b = {{0}};
        b.v[0] = COEFF_B;
        to_mont(&b, b.v);
        fmul(&l, &x2, &x);
        fadd(&l, &l, &b);
        if (!feq(&l, &y2)) return 0;
        (void)r;
#else
        /* -5 x^2 + y^2 == 1 + d x^2 y^2 */
        fe five = {{0}};
        five.v[0] = 5;
        to_mont(&five, five.v);
        fmul(&l, &x2, &five);
        fsub(&l, &y2, &l);
        fmul(&r, &x2, &y2);
        fmul(&r, &r, &D_);
        fadd(&r, &r, &ONE_);
        if (!feq(&l, &r)) return 0;
#endif
    }
    return 1;
}
