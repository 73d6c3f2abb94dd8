// Host 6x64 Montgomery multiply variants (BLS12-381 Fq) for the MSM host Horner pass.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
typedef unsigned __int128 u128;
static constexpr uint64_t P[6] = {0xb9feffffffffaaabULL,0x1eabfffeb153ffffULL,0x6730d2a0f6b0f624ULL,0x64774b84f38512bfULL,0x4b1ba7b6434bacd7ULL,0x1a0111ea397fe69aULL};
static constexpr uint64_t INV = 0x89f3fffcfffcfffdULL;
// variant A: as in ff.hpp new
static inline void mulA(uint64_t* r, const uint64_t* pa, const uint64_t* pb) {
    constexpr int M = 6;
    uint64_t t[M + 1] = {0};
#pragma unroll
    for (int i = 0; i < M; i++) {
        uint64_t C = 0;
#pragma unroll
        for (int j = 0; j < M; j++) { u128 s = (u128)pa[j] * pb[i] + t[j] + C; t[j] = (uint64_t)s; C = (uint64_t)(s >> 64); }
        t[M] += C;
        const uint64_t m = t[0] * INV;
        u128 s = (u128)m * P[0] + t[0];
        C = (uint64_t)(s >> 64);
#pragma unroll
        for (int j = 1; j < M; j++) { s = (u128)m * P[j] + t[j] + C; t[j - 1] = (uint64_t)s; C = (uint64_t)(s >> 64); }
        t[M - 1] = t[M] + C;
        t[M] = 0;
    }
    uint64_t d[M]; uint64_t br = 0;
#pragma unroll
    for (int j = 0; j < M; j++) { u128 s = (u128)t[j] - P[j] - br; d[j] = (uint64_t)s; br = (uint64_t)(s >> 64) & 1; }
    uint64_t mask = 0 - br;
#pragma unroll
    for (int j = 0; j < M; j++) r[j] = (t[j] & mask) | (d[j] & ~mask);
}
// variant B: product-then-reduce interleaved with branchless select
static inline void mulB(uint64_t* r, const uint64_t* a, const uint64_t* b) {
    uint64_t t0=0,t1=0,t2=0,t3=0,t4=0,t5=0,t6=0;
    uint64_t T[7];
#define ROW(i) { \
    u128 s; uint64_t C; \
    s = (u128)a[0]*b[i] + t0; t0=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)a[1]*b[i] + t1 + C; t1=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)a[2]*b[i] + t2 + C; t2=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)a[3]*b[i] + t3 + C; t3=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)a[4]*b[i] + t4 + C; t4=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)a[5]*b[i] + t5 + C; t5=(uint64_t)s; C=(uint64_t)(s>>64); \
    t6 += C; \
    uint64_t m = t0*INV; \
    s = (u128)m*P[0] + t0; C=(uint64_t)(s>>64); \
    s = (u128)m*P[1] + t1 + C; t0=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)m*P[2] + t2 + C; t1=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)m*P[3] + t3 + C; t2=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)m*P[4] + t4 + C; t3=(uint64_t)s; C=(uint64_t)(s>>64); \
    s = (u128)m*P[5] + t5 + C; t4=(uint64_t)s; C=(uint64_t)(s>>64); \
    t5 = t6 + C; t6 = 0; }
    ROW(0) ROW(1) ROW(2) ROW(3) ROW(4) ROW(5)
    uint64_t t[6]={t0,t1,t2,t3,t4,t5}, d[6]; uint64_t br=0;
    for (int j=0;j<6;j++){ u128 s=(u128)t[j]-P[j]-br; d[j]=(uint64_t)s; br=(uint64_t)(s>>64)&1; }
    uint64_t mask = 0 - br;
    for (int j=0;j<6;j++) r[j] = (t[j] & mask) | (d[j] & ~mask);
}
template <class F> double bench(F f) {
    uint64_t x[6] = {1,2,3,4,5,6}, y[6] = {7,8,9,10,11,0x123};
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int k = 0; k < 1000000; k++) f(x, x, y);
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::nano>(t1 - t0).count() / 1e6 + (x[0] & 1) * 1e-9;
}
int main() {
    printf("A %.1f ns  B %.1f ns\n", bench(mulA), bench(mulB));
    uint64_t x[6]={1,2,3,4,5,6}, y[6]={7,8,9,10,11,0x123}, r1[6], r2[6];
    for(int k=0;k<100;k++){ mulA(r1,x,y); mulB(r2,x,y); if (memcmp(r1,r2,48)) { printf("mismatch\n"); return 1;} memcpy(x,r1,48);} 
    printf("match\n");
}
