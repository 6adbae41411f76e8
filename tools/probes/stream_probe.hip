// Diagnostic (not part of the library): do two streams' kernels overlap?  Per iteration, a 4096-wave
// kernel on one stream vs two 2048-wave kernels on two non-blocking streams (each wave spins
// spin_us; dynamic LDS per workgroup as k_env's c3 instance).
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/probes/stream_probe tools/probes/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k_spin(int* out, int spin_ticks) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = (int)blockIdx.x;
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) out[blockIdx.x] = lds[63];
}

int main() {
    int* buf;
    hipMalloc(&buf, 1 << 20);
    hipStream_t s[4];
    for (int i = 0; i < 4; i++) hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 100;
    for (int lds : {0, 9216})
        for (int spin : {1000, 1500})
            for (int G : {1, 2, 4}) {
                const int waves = 4096 / G;
                auto step = [&]() {
                    for (int j = 0; j < G; j++) hipLaunchKernelGGL(k_spin, dim3(waves), dim3(64), lds, s[j], buf, spin);
                };
                for (int i = 0; i < 10; i++) step();
                hipDeviceSynchronize();
                hipEventRecord(a, 0);
                for (int i = 0; i < iters; i++) step();
                for (int j = 0; j < G; j++) hipStreamSynchronize(s[j]);
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                printf("{\"lds\": %d, \"spin_us\": %.0f, \"streams\": %d, \"us_per_iter\": %.2f}\n", lds, spin / 100.0, G,
                       1e3 * ms / iters);
            }
    return 0;
}
