// Diagnostic (not part of the library): how long a 4096-wave grid takes to START — the first
// to the last wave's start (s_memrealtime, 100 MHz) — as a function of the dynamic LDS per workgroup, the
// waves per workgroup and the VGPRs a wave allocates (a c3 single-step launch's waves start over 3-5 us).
// Each wave stamps its start, then spins `spin` ticks so the grid is resident at once (4 waves per SIMD).
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/probes/spread_probe tools/probes/spread_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int VG>
__global__ __launch_bounds__(256) void k_spread(unsigned long long* out, int spin) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (VG) {  // keep ~VG VGPRs live (the c3 kernels allocate 128 / 69)
        int v[VG > 0 ? VG : 1];
#pragma unroll
        for (int i = 0; i < VG; i++) v[i] = (int)threadIdx.x * (i + 3);
#pragma unroll
        for (int i = 0; i < VG; i++) asm volatile("" : "+v"(v[i]));
        int acc = 0;
#pragma unroll
        for (int i = 0; i < VG; i++) acc ^= v[i];
        if (acc == 0x7fffffff) lds[threadIdx.x] = acc;
    }
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin) __builtin_amdgcn_s_sleep(2);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t0;
}

int main() {
    const int waves = 4096;
    unsigned long long* d;
    hipMalloc(&d, waves * 8);
    std::vector<unsigned long long> h(waves);
    hipFuncSetAttribute((const void*)k_spread<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipFuncSetAttribute((const void*)k_spread<100>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    for (int i = 0; i < 2000; i++) hipLaunchKernelGGL(k_spread<0>, dim3(waves), dim3(64), 0, 0, d, 0);  // clocks up
    hipDeviceSynchronize();
    for (int vg : {0, 100})
        for (int wpg : {1, 4})
            for (int lds : {0, 10240, 40960}) {
                if (wpg == 1 && lds > 10240) continue;
                if (wpg == 4 && lds == 10240) continue;
                std::vector<double> sp;
                for (int rep = 0; rep < 5; rep++) {
                    auto k = vg ? k_spread<100> : k_spread<0>;
                    hipLaunchKernelGGL(k, dim3(waves / wpg), dim3(64 * wpg), lds, 0, d, 2000);  // 20 us resident
                    hipDeviceSynchronize();
                    hipMemcpy(h.data(), d, waves * 8, hipMemcpyDeviceToHost);
                    const auto mm = std::minmax_element(h.begin(), h.end());
                    sp.push_back((*mm.second - *mm.first) / 100.0);
                }
                std::sort(sp.begin(), sp.end());
                printf("{\"vgprs\": \"%s\", \"waves_per_wg\": %d, \"lds_per_wg\": %d, \"start_spread_us\": {\"min\": %.2f, \"median\": %.2f, \"max\": %.2f}}\n",
                       vg ? "~100" : "few", wpg, lds, sp[0], sp[2], sp[4]);
            }
    return 0;
}
