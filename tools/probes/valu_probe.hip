// VALU issue-rate probe (gfx950): cycles per wave64 VALU instruction as a function of the EXEC mask
// (how many lanes, which half) and of the waves resident per SIMD.  Each wave runs N iterations of
// 16 independent v_add_u32 / v_mul_hi_u32 / v_xor3_b32 in inline asm under `if (lane < lanes)` (or
// lanes >= 32 only); s_memtime around the loop, per-wave cycles written out.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

template <int OP>
__global__ __launch_bounds__(64) void probe(int iters, int lanes, int hiHalf, unsigned long long* out, int* sink) {
    const int l = threadIdx.x;
    int a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
    const int b = (int)blockIdx.x | 1;
    const bool on = hiHalf ? (l >= 64 - lanes) : (l < lanes);
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (on) {
        for (int i = 0; i < iters; i++) {
#define ONE(x)                                                                                    \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));                        \
    else if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));                \
    else if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));              \
    else asm volatile("v_readlane_b32 s0, %0, 1" : : "v"(x) : "s0");
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) out[blockIdx.x] = t1 - t0;
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff) sink[l] = 1;
}

int main(int argc, char** argv) {
    const int iters = 2000;
    int* sink;
    unsigned long long* out;
    const int maxBlocks = 256 * 4 * 8;
    hipMalloc(&sink, 256);
    hipMalloc(&out, maxBlocks * 8);
    std::vector<unsigned long long> h(maxBlocks);
    const char* names[] = {"v_add_u32", "v_mul_hi_u32", "v_xor_b32", "v_readlane_b32"};
    for (int op = 0; op < 4; op++)
        for (int wps : {1, 2, 4, 8})
            for (int lanes : {64, 32, 8, 1})
                for (int hi = 0; hi < (lanes == 32 ? 2 : 1); hi++) {
                    const int blocks = 256 * 4 * wps;
                    auto k = op == 0 ? probe<0> : op == 1 ? probe<1> : op == 2 ? probe<2> : probe<3>;
                    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, iters, lanes, hi, out, sink);
                    hipDeviceSynchronize();
                    hipEvent_t e0, e1;
                    hipEventCreate(&e0);
                    hipEventCreate(&e1);
                    hipEventRecord(e0);
                    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, iters, lanes, hi, out, sink);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    hipMemcpy(h.data(), out, blocks * 8, hipMemcpyDeviceToHost);
                    std::sort(h.begin(), h.begin() + blocks);
                    const double med = (double)h[blocks / 2];
                    const double n = 16.0 * iters;
                    // s_memtime counts at the shader clock; kernel time gives the chip-level rate
                    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"lanes\": %d, \"high_half\": %d, \"memtime_per_inst_per_wave\": %.3f, "
                           "\"kernel_ms\": %.4f, \"wave_insts_per_simd_per_ns\": %.4f}\n",
                           names[op], wps, lanes, hi, med / n, ms, blocks * n / 1024.0 / (ms * 1e6));
                }
    return 0;
}
