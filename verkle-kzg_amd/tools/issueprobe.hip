// Issue cost of the multiply's instruction classes on gfx950: cycles per wave-instruction for
// blocks of independent v_mad_u64_u32, VCC add-with-carry chains, independent adds and
// v_mul_lo_u32, at 1 / 2 / 4 waves per SIMD (per-SIMD throughput). Prints JSON lines.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
template <int KIND>
__global__ void k_issue(uint32_t* out, long long* cyc, int iters) {
    uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3, c = a ^ b;
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        if constexpr (KIND == 0) {
            asm volatile(R8("v_mad_u64_u32 v[10:11], s[98:99], %0, %1, v[20:21]\n\t"
                            "v_mad_u64_u32 v[12:13], s[98:99], %0, %1, v[22:23]\n\t"
                            "v_mad_u64_u32 v[14:15], s[98:99], %0, %1, v[24:25]\n\t"
                            "v_mad_u64_u32 v[16:17], s[98:99], %0, %1, v[26:27]\n\t"
                            "v_mad_u64_u32 v[18:19], s[98:99], %0, %1, v[28:29]\n\t"
                            "v_mad_u64_u32 v[30:31], s[98:99], %0, %1, v[20:21]\n\t"
                            "v_mad_u64_u32 v[32:33], s[98:99], %0, %1, v[22:23]\n\t"
                            "v_mad_u64_u32 v[34:35], s[98:99], %0, %1, v[24:25]\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19",
                           "v30", "v31", "v32", "v33", "v34", "v35", "s98", "s99");
        } else if constexpr (KIND == 1) {
            asm volatile(R8("v_add_co_u32 v10, vcc, %0, v20\n\t"
                            "v_addc_co_u32 v11, vcc, %1, v21, vcc\n\t"
                            "v_addc_co_u32 v12, vcc, %0, v22, vcc\n\t"
                            "v_addc_co_u32 v13, vcc, %1, v23, vcc\n\t"
                            "v_addc_co_u32 v14, vcc, %0, v24, vcc\n\t"
                            "v_addc_co_u32 v15, vcc, %1, v25, vcc\n\t"
                            "v_addc_co_u32 v16, vcc, %0, v26, vcc\n\t"
                            "v_addc_co_u32 v17, vcc, %1, v27, vcc\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "vcc");
        } else if constexpr (KIND == 2) {
            asm volatile(R8("v_add_u32 v10, %0, v20\n\t"
                            "v_add_u32 v11, %1, v21\n\t"
                            "v_add_u32 v12, %0, v22\n\t"
                            "v_add_u32 v13, %1, v23\n\t"
                            "v_add_u32 v14, %0, v24\n\t"
                            "v_add_u32 v15, %1, v25\n\t"
                            "v_add_u32 v16, %0, v26\n\t"
                            "v_add_u32 v17, %1, v27\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        } else if constexpr (KIND == 4) {
            asm volatile(R8("v_lshrrev_b64 v[10:11], 29, v[20:21]\n\t"
                            "v_lshrrev_b64 v[12:13], 29, v[22:23]\n\t"
                            "v_lshrrev_b64 v[14:15], 29, v[24:25]\n\t"
                            "v_lshrrev_b64 v[16:17], 29, v[26:27]\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        } else if constexpr (KIND == 5) {
            asm volatile(R8("v_lshl_add_u64 v[10:11], v[20:21], 0, v[30:31]\n\t"
                            "v_lshl_add_u64 v[12:13], v[22:23], 0, v[32:33]\n\t"
                            "v_lshl_add_u64 v[14:15], v[24:25], 0, v[34:35]\n\t"
                            "v_lshl_add_u64 v[16:17], v[26:27], 0, v[36:37]\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        } else if constexpr (KIND == 6) {
            asm volatile(R8("v_alignbit_b32 v10, %0, v20, 29\n\t"
                            "v_alignbit_b32 v11, %1, v21, 29\n\t"
                            "v_alignbit_b32 v12, %0, v22, 29\n\t"
                            "v_alignbit_b32 v13, %1, v23, 29\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13");
        } else if constexpr (KIND == 7) {
            asm volatile(R8("v_add3_u32 v10, %0, v20, v30\n\t"
                            "v_add3_u32 v11, %1, v21, v31\n\t"
                            "v_add3_u32 v12, %0, v22, v32\n\t"
                            "v_add3_u32 v13, %1, v23, v33\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13");
        } else if constexpr (KIND == 8) {
            asm volatile(R8("v_mad_u32_u24 v10, %0, v20, v30\n\t"
                            "v_mad_u32_u24 v11, %1, v21, v31\n\t"
                            "v_mad_u32_u24 v12, %0, v22, v32\n\t"
                            "v_mad_u32_u24 v13, %1, v23, v33\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13");
        } else if constexpr (KIND == 9) {
            asm volatile(R8("v_mul_hi_u32 v10, %0, v20\n\t"
                            "v_mul_hi_u32 v11, %1, v21\n\t"
                            "v_mul_hi_u32 v12, %0, v22\n\t"
                            "v_mul_hi_u32 v13, %1, v23\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13");
        } else if constexpr (KIND == 10) {
            asm volatile(R8("v_fma_f64 v[10:11], v[20:21], v[22:23], v[24:25]\n\t"
                            "v_fma_f64 v[12:13], v[20:21], v[22:23], v[26:27]\n\t"
                            "v_fma_f64 v[14:15], v[20:21], v[22:23], v[28:29]\n\t"
                            "v_fma_f64 v[16:17], v[20:21], v[22:23], v[30:31]\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        } else if constexpr (KIND == 11) {
            asm volatile(R8("v_pk_mad_u16 v10, %0, v20, v30\n\t"
                            "v_pk_mad_u16 v11, %1, v21, v31\n\t"
                            "v_pk_mad_u16 v12, %0, v22, v32\n\t"
                            "v_pk_mad_u16 v13, %1, v23, v33\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13");
        } else {
            asm volatile(R8("v_mul_lo_u32 v10, %0, v20\n\t"
                            "v_mul_lo_u32 v11, %1, v21\n\t"
                            "v_mul_lo_u32 v12, %0, v22\n\t"
                            "v_mul_lo_u32 v13, %1, v23\n\t"
                            "v_mul_lo_u32 v14, %0, v24\n\t"
                            "v_mul_lo_u32 v15, %1, v25\n\t"
                            "v_mul_lo_u32 v16, %0, v26\n\t"
                            "v_mul_lo_u32 v17, %1, v27\n\t")
                         :: "v"(a), "v"(b) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int KIND>
void run(const char* name, int blocks, int threads) {
    uint32_t* out;
    long long* cyc;
    const int iters = 2000;
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
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double inst = (double)iters * (KIND >= 4 && KIND != 12 ? 32 : 64);  // per wave
    const double waves_per_simd = (double)blocks * threads / 64 / 1024;
    printf("{\"probe\":\"%s\",\"waves_per_simd\":%.2f,\"cycles_per_inst_one_wave\":%.2f,"
           "\"simd_cycles_per_inst\":%.2f}\n",
           name, waves_per_simd, c / inst, ms * 1e-3 * 2.4e9 / (inst * waves_per_simd));
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    const char* names[] = {"v_mad_u64_u32 x8 independent", "v_add_co/addc chain", "v_add_u32 independent",
                           "v_mul_lo_u32 independent", "v_lshrrev_b64", "v_lshl_add_u64", "v_alignbit_b32",
                           "v_add3_u32", "v_mad_u32_u24", "v_mul_hi_u32", "v_fma_f64", "v_pk_mad_u16"};
    for (int wps : {1, 2, 4}) {
        run<0>(names[0], 256 * wps, 256);
        run<1>(names[1], 256 * wps, 256);
        run<2>(names[2], 256 * wps, 256);
        run<3>(names[3], 256 * wps, 256);
        run<4>(names[4], 256 * wps, 256);
        run<5>(names[5], 256 * wps, 256);
        run<6>(names[6], 256 * wps, 256);
        run<7>(names[7], 256 * wps, 256);
        run<8>(names[8], 256 * wps, 256);
        run<9>(names[9], 256 * wps, 256);
        run<10>(names[10], 256 * wps, 256);
        run<11>(names[11], 256 * wps, 256);
    }
    return 0;
}
