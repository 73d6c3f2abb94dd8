// Issue cost per wave64 instruction class on gfx950 (per-SIMD throughput at 1 / 2 / 4 waves per
// SIMD): 8 independent instructions with 8 distinct destinations per group, no dependencies.
// Complements issueprobe.hip (the multiply's classes). Prints JSON lines; the clock is taken
// from the v_mad_u64_u32 reference (4 cycles) at the same occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define G8(op) R8(op " v10, %0, v20\n\t" op " v11, %1, v21\n\t" op " v12, %0, v22\n\t" op " v13, %1, v23\n\t" \
                  op " v14, %0, v24\n\t" op " v15, %1, v25\n\t" op " v16, %0, v26\n\t" op " v17, %1, v27\n\t")
#define G8_3(op) R8(op " v10, %0, v20, v30\n\t" op " v11, %1, v21, v31\n\t" op " v12, %0, v22, v32\n\t" \
                    op " v13, %1, v23, v33\n\t" op " v14, %0, v24, v34\n\t" op " v15, %1, v25, v35\n\t"   \
                    op " v16, %0, v26, v36\n\t" op " v17, %1, v27, v37\n\t")
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17"
#define CLOB64 "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v40", "v41", "v42", "v43", "v44", "v45", \
               "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55"

template <int KIND>
__global__ void k_issue(uint32_t* out, long long* cyc, int iters) {
    uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
    for (int i = 0; i < iters; i++) {
        if constexpr (KIND == 0)
            asm volatile(R8("v_mad_u64_u32 v[40:41], s[98:99], %0, %1, v[20:21]\n\t"
                            "v_mad_u64_u32 v[42:43], s[98:99], %0, %1, v[22:23]\n\t"
                            "v_mad_u64_u32 v[44:45], s[98:99], %0, %1, v[24:25]\n\t"
                            "v_mad_u64_u32 v[46:47], s[98:99], %0, %1, v[26:27]\n\t"
                            "v_mad_u64_u32 v[48:49], s[98:99], %0, %1, v[28:29]\n\t"
                            "v_mad_u64_u32 v[50:51], s[98:99], %0, %1, v[20:21]\n\t"
                            "v_mad_u64_u32 v[52:53], s[98:99], %0, %1, v[22:23]\n\t"
                            "v_mad_u64_u32 v[54:55], s[98:99], %0, %1, v[24:25]\n\t") ::"v"(a), "v"(b) : CLOB64, "s98", "s99");
        else if constexpr (KIND == 1) asm volatile(G8("v_add_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 2) asm volatile(G8("v_and_b32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 3) asm volatile(G8("v_lshrrev_b32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 4) asm volatile(G8("v_sub_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 5) asm volatile(G8_3("v_add3_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 6) asm volatile(G8_3("v_alignbit_b32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 7) asm volatile(G8_3("v_and_or_b32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 8) asm volatile(G8_3("v_bfe_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 9) asm volatile(G8_3("v_lshl_add_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 10) asm volatile(G8("v_mul_lo_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 11) asm volatile(G8("v_mul_hi_u32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 12) asm volatile(G8_3("v_mad_u32_u24") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 13)
            asm volatile(R8("v_lshrrev_b64 v[40:41], 29, v[20:21]\n\t"
                            "v_lshrrev_b64 v[42:43], 29, v[22:23]\n\t"
                            "v_lshrrev_b64 v[44:45], 29, v[24:25]\n\t"
                            "v_lshrrev_b64 v[46:47], 29, v[26:27]\n\t"
                            "v_lshrrev_b64 v[48:49], 29, v[28:29]\n\t"
                            "v_lshrrev_b64 v[50:51], 29, v[30:31]\n\t"
                            "v_lshrrev_b64 v[52:53], 29, v[32:33]\n\t"
                            "v_lshrrev_b64 v[54:55], 29, v[34:35]\n\t") ::"v"(a), "v"(b) : CLOB64);
        else if constexpr (KIND == 14)
            asm volatile(R8("v_lshl_add_u64 v[40:41], v[20:21], 0, v[30:31]\n\t"
                            "v_lshl_add_u64 v[42:43], v[22:23], 0, v[32:33]\n\t"
                            "v_lshl_add_u64 v[44:45], v[24:25], 0, v[34:35]\n\t"
                            "v_lshl_add_u64 v[46:47], v[26:27], 0, v[36:37]\n\t"
                            "v_lshl_add_u64 v[48:49], v[20:21], 0, v[30:31]\n\t"
                            "v_lshl_add_u64 v[50:51], v[22:23], 0, v[32:33]\n\t"
                            "v_lshl_add_u64 v[52:53], v[24:25], 0, v[34:35]\n\t"
                            "v_lshl_add_u64 v[54:55], v[26:27], 0, v[36:37]\n\t") ::"v"(a), "v"(b) : CLOB64);
        else if constexpr (KIND == 15) asm volatile(G8("v_add_co_u32") ::"v"(a), "v"(b) : CLOB, "vcc");
        else if constexpr (KIND == 16) asm volatile(G8("v_mul_u32_u24") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 17)
            asm volatile(R8("v_mov_b64 v[40:41], v[20:21]\n\t"
                            "v_mov_b64 v[42:43], v[22:23]\n\t"
                            "v_mov_b64 v[44:45], v[24:25]\n\t"
                            "v_mov_b64 v[46:47], v[26:27]\n\t"
                            "v_mov_b64 v[48:49], v[28:29]\n\t"
                            "v_mov_b64 v[50:51], v[30:31]\n\t"
                            "v_mov_b64 v[52:53], v[32:33]\n\t"
                            "v_mov_b64 v[54:55], v[34:35]\n\t") ::"v"(a), "v"(b) : CLOB64);
        else if constexpr (KIND == 18) asm volatile(G8("v_or_b32") ::"v"(a), "v"(b) : CLOB);
        else if constexpr (KIND == 19) asm volatile(G8("v_max_u32") ::"v"(a), "v"(b) : CLOB);
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = 0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

template <int KIND>
double run(int blocks, int threads) {
    uint32_t* out;
    long long* cyc;
    const int iters = 4000;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    (void)hipMalloc(&cyc, 8);
    k_issue<KIND><<<blocks, threads>>>(out, cyc, 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_issue<KIND><<<blocks, threads>>>(out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    (void)hipFree(cyc);
    return ms / ((double)iters * 64 * blocks * threads / 64 / 1024);  // ms per instruction per SIMD
}

int main() {
    const char* names[] = {"v_mad_u64_u32", "v_add_u32", "v_and_b32", "v_lshrrev_b32", "v_sub_u32", "v_add3_u32",
                           "v_alignbit_b32", "v_and_or_b32", "v_bfe_u32", "v_lshl_add_u32", "v_mul_lo_u32",
                           "v_mul_hi_u32", "v_mad_u32_u24", "v_lshrrev_b64", "v_lshl_add_u64", "v_add_co_u32",
                           "v_mul_u32_u24", "v_mov_b64", "v_or_b32", "v_max_u32"};
    for (int wps : {1, 2, 4}) {
        double t[20];
        t[0] = run<0>(256 * wps, 256); t[1] = run<1>(256 * wps, 256); t[2] = run<2>(256 * wps, 256);
        t[3] = run<3>(256 * wps, 256); t[4] = run<4>(256 * wps, 256); t[5] = run<5>(256 * wps, 256);
        t[6] = run<6>(256 * wps, 256); t[7] = run<7>(256 * wps, 256); t[8] = run<8>(256 * wps, 256);
        t[9] = run<9>(256 * wps, 256); t[10] = run<10>(256 * wps, 256); t[11] = run<11>(256 * wps, 256);
        t[12] = run<12>(256 * wps, 256); t[13] = run<13>(256 * wps, 256); t[14] = run<14>(256 * wps, 256);
        t[15] = run<15>(256 * wps, 256); t[16] = run<16>(256 * wps, 256); t[17] = run<17>(256 * wps, 256);
        t[18] = run<18>(256 * wps, 256); t[19] = run<19>(256 * wps, 256);
        for (int k = 0; k < 20; k++)
            printf("{\"inst\":\"%s\",\"waves_per_simd\":%d,\"cycles_rel_mad4\":%.2f}\n", names[k], wps, 4.0 * t[k] / t[0]);
    }
    return 0;
}
