/* ORACLE (test infrastructure + CPU baseline only). 64-bit-limb Montgomery field arithmetic
 * (CIOS with unsigned __int128, like arkworks' own backend), shared by ref_curve.c and
 * ref_multiproof.c. The includer defines NL (u64 limbs) and `static const u64 P_[NL]`. */
#ifndef REF_FIELD_H
#define REF_FIELD_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

typedef struct { u64 v[NL]; } fe;

static u64 INV_;   /* -p^{-1} mod 2^64 */
static fe R2_;     /* R^2 mod p */
static fe ONE_;    /* R mod p (Montgomery one) */
static int inited_;

static int geq_p(const u64* a) {
    for (int i = NL - 1; i >= 0; i--) {
        if (a[i] > P_[i]) return 1;
        if (a[i] < P_[i]) return 0;
    }
    return 1;
}
static void sub_p(u64* a) {
    u64 br = 0;
    for (int i = 0; i < NL; i++) {
        u128 d = (u128)a[i] - P_[i] - br;
        a[i] = (u64)d;
        br = (u64)(d >> 64) ? 1 : 0;
    }
}
static void fadd(fe* r, const fe* a, const fe* b) {
    u64 c = 0;
    u64 t[NL];
    for (int i = 0; i < NL; i++) {
        u128 s = (u128)a->v[i] + b->v[i] + c;
        t[i] = (u64)s;
        c = (u64)(s >> 64);
    }
    if (c || geq_p(t)) sub_p(t);
    memcpy(r->v, t, sizeof t);
}
static void fsub(fe* r, const fe* a, const fe* b) {
    u64 br = 0;
    u64 t[NL];
    for (int i = 0; i < NL; i++) {
        u128 d = (u128)a->v[i] - b->v[i] - br;
        t[i] = (u64)d;
        br = (u64)(d >> 64) ? 1 : 0;
    }
    if (br) {
        u64 c = 0;
        for (int i = 0; i < NL; i++) {
            u128 s = (u128)t[i] + P_[i] + c;
            t[i] = (u64)s;
            c = (u64)(s >> 64);
        }
    }
    memcpy(r->v, t, sizeof t);
}
static void fmul(fe* r, const fe* a, const fe* b) {
    u64 t[NL + 2];
    memset(t, 0, sizeof t);
    for (int i = 0; i < NL; i++) {
        u64 C = 0;
        for (int j = 0; j < NL; j++) {
            u128 s = (u128)a->v[j] * b->v[i] + t[j] + C;
            t[j] = (u64)s;
            C = (u64)(s >> 64);
        }
        u128 s = (u128)t[NL] + C;
        t[NL] = (u64)s;
        t[NL + 1] = (u64)(s >> 64);
        u64 m = t[0] * INV_;
        s = (u128)m * P_[0] + t[0];
        C = (u64)(s >> 64);
        for (int j = 1; j < NL; j++) {
            s = (u128)m * P_[j] + t[j] + C;
            t[j - 1] = (u64)s;
            C = (u64)(s >> 64);
        }
        s = (u128)t[NL] + C;
        t[NL - 1] = (u64)s;
        t[NL] = t[NL + 1] + (u64)(s >> 64);
    }
    if (t[NL] || geq_p(t)) sub_p(t);
    memcpy(r->v, t, NL * sizeof(u64));
}
static int fiszero(const fe* a) {
    u64 o = 0;
    for (int i = 0; i < NL; i++) o |= a->v[i];
    return o == 0;
}
static int feq(const fe* a, const fe* b) { return memcmp(a->v, b->v, sizeof a->v) == 0; }
static void to_mont(fe* r, const u64* canon) {
    fe a;
    memcpy(a.v, canon, sizeof a.v);
    fmul(r, &a, &R2_);
}
static void from_mont(u64* canon, const fe* a) {
    fe one = {{0}};
    one.v[0] = 1;
    fe t;
    fmul(&t, a, &one);
    memcpy(canon, t.v, sizeof t.v);
}
/* a^(p-2) */
static void finv(fe* r, const fe* a) {
    u64 e[NL];
    memcpy(e, P_, sizeof e);
    e[0] -= 2; /* p is odd and > 2: no borrow */
    fe acc = ONE_;
    for (int i = NL - 1; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            fmul(&acc, &acc, &acc);
            if ((e[i] >> b) & 1) fmul(&acc, &acc, a);
        }
    *r = acc;
}
static void init(void) {
    if (inited_) return;
    u64 inv = 1;
    for (int i = 0; i < 7; i++) inv *= 2 - P_[0] * inv;
    INV_ = (u64)0 - inv;
    /* R mod p and R^2 mod p by doubling */
    fe x = {{0}};
    x.v[0] = 1;
    for (int i = 0; i < 64 * NL * 2; i++) {
        fadd(&x, &x, &x);
        if (i == 64 * NL - 1) ONE_ = x;
    }
    R2_ = x;
    inited_ = 1;
}

#endif /* REF_FIELD_H */
