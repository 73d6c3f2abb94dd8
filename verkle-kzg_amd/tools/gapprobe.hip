// Dispatch-gap probe: K dependent kernels of ~20 us each back to back on one stream, launched
// directly vs replayed from a captured hipGraph; prints the per-kernel overhead of each.
// build: hipcc --offload-arch=gfx950 -O2 gapprobe.hip -o gapprobe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void spin(float* buf, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = buf[i];
    for (int k = 0; k < iters; k++) v = v * 1.0000001f + 0.5f;
    buf[i] = v;
}

int main() {
    const int K = 12, blocks = 2048, iters = 4000;
    float* buf = nullptr;
    CK(hipMalloc(&buf, blocks * 256 * sizeof(float)));
    CK(hipMemset(buf, 0, blocks * 256 * sizeof(float)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // one kernel alone
    float one = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a, st));
        hipLaunchKernelGGL(spin, dim3(blocks), dim3(256), 0, st, buf, iters);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&one, a, b));
    }
    // K in a stream
    float direct = 0;
    double host_us = 0;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(a, st));
        for (int k = 0; k < K; k++) hipLaunchKernelGGL(spin, dim3(blocks), dim3(256), 0, st, buf, iters);
        CK(hipEventRecord(b, st));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&direct, a, b));
        host_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    // the same K captured once and replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(spin, dim3(blocks), dim3(256), 0, st, buf, iters);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float graph = 0;
    double ghost_us = 0;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(a, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(b, st));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&graph, a, b));
        ghost_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    printf("{\"kernel_us\": %.1f, \"K\": %d, \"direct_us\": %.1f, \"direct_gap_us\": %.2f, \"direct_host_enqueue_us\": %.1f, "
           "\"graph_us\": %.1f, \"graph_gap_us\": %.2f, \"graph_host_enqueue_us\": %.1f}\n",
           one * 1e3, K, direct * 1e3, (direct - K * one) * 1e3 / (K - 1), host_us, graph * 1e3,
           (graph - K * one) * 1e3 / (K - 1), ghost_us);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(buf));
    return 0;
}
