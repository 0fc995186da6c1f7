// Wave dispatch rate probe: how fast does the chip start one-wave blocks?
// Launches N blocks of 64 threads (empty body, or a body that touches LDS of
// the tile gather's size) and reports blocks per microsecond (hipEvents).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(64) void k_empty(int *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1;
}
__global__ __launch_bounds__(64) void k_lds(int *out) {
    __shared__ float s[1920]; // 7680 B, the tile gather's per-wave LDS
    s[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    if (s[63 - threadIdx.x] < -1.f) out[0] = 1;
}
// a wave that lives ~T cycles (spins on s_memrealtime, 100 MHz ticks)
__global__ __launch_bounds__(64) void k_wait(int *out, unsigned long long ticks) {
    __shared__ float s[1920];
    s[threadIdx.x] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {}
    if (s[threadIdx.x] < -1.f) out[0] = 1;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 69000;
    int *d;
    hipMalloc(&d, 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int kind = 0; kind < 5; ++kind) {
        const unsigned long long ticks = kind == 2 ? 100ull : kind == 3 ? 500ull : 1000ull; // 1, 5, 10 us
        auto launch = [&] {
            if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(n), dim3(64), 0, 0, d);
            else if (kind == 1) hipLaunchKernelGGL(k_lds, dim3(n), dim3(64), 0, 0, d);
            else hipLaunchKernelGGL(k_wait, dim3(n), dim3(64), 0, 0, d, ticks);
        };
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000.0 / 10.0;
        const char *names[] = {"empty", "lds7680", "wait1us", "wait5us", "wait10us"};
        printf("%-9s blocks %d: %.1f us per launch, %.0f blocks/us\n", names[kind], n, us, n / us);
    }
    return 0;
}
