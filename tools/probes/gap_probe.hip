// Diagnostic (not part of the library): per-launch cost of back-to-back kernels on one stream, as a
// function of the dirty bytes each launch leaves in L2 and the store policy.  4096 one-wave workgroups
// (the c3 grid); each wave spins for `spin_ns` (s_memrealtime, 100 MHz) and stores `bytes_per_wave`
// bytes (dwordx4 per lane) as normal, nontemporal or write-through (sc1) stores.
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/probes/gap_probe tools/probes/gap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int POLICY>
__global__ __launch_bounds__(64) void k_probe(int* out, int bytes_per_wave, int spin_ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (spin_ticks > 0)
        while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) __builtin_amdgcn_s_sleep(2);
    char* base = (char*)out + (size_t)blockIdx.x * bytes_per_wave;
    const int n = bytes_per_wave / 16;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes_per_wave, 0x00020000);
    for (int i = threadIdx.x; i < n; i += 64) {
        const i32x4 v = {i, (int)blockIdx.x, 1, 2};
        if (POLICY == 0) *(i32x4*)(base + 16 * i) = v;
        else if (POLICY == 1) __builtin_nontemporal_store(v, (i32x4*)(base + 16 * i));
        else __builtin_amdgcn_raw_buffer_store_b128(v, r, 16 * i, 0, 16);  // sc1: write-through
    }
}

int main(int argc, char** argv) {
    const int waves = 4096, iters = 200;
    const int spins[] = {0, 1000};            // 0 / 10 us
    const int sizes[] = {0, 1024, 4096, 16384};  // bytes per wave: 0, 4, 16, 64 MB per launch
    int* buf;
    hipMalloc(&buf, (size_t)waves * 16384);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int spin : spins)
        for (int sz : sizes)
            for (int pol = 0; pol < 3; pol++) {
                if (sz == 0 && pol > 0) continue;
                auto launch = [&]() {
                    if (pol == 0) hipLaunchKernelGGL(k_probe<0>, dim3(waves), dim3(64), 0, s, buf, sz, spin);
                    else if (pol == 1) hipLaunchKernelGGL(k_probe<1>, dim3(waves), dim3(64), 0, s, buf, sz, spin);
                    else hipLaunchKernelGGL(k_probe<2>, dim3(waves), dim3(64), 0, s, buf, sz, spin);
                };
                for (int i = 0; i < 20; i++) launch();
                hipEventRecord(a, s);
                for (int i = 0; i < iters; i++) launch();
                hipEventRecord(b, s);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                printf("{\"spin_us\": %.1f, \"mb_per_launch\": %.1f, \"policy\": \"%s\", \"us_per_launch\": %.2f}\n", spin / 100.0,
                       (double)sz * waves / 1e6, pol == 0 ? "normal" : pol == 1 ? "nt" : "sc1", 1e3 * ms / iters);
            }
    return 0;
}
