// EXEC-mask probe (gfx950): chip-wide issue rate of one VALU instruction kind, 4 waves per SIMD,
// as a function of the active-lane set: all 64, the first n lanes, or n lanes spread over the wave.
// Each wave runs ITERS x 16 independent copies in inline asm under `if (active)`.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY(INS)                                                                                   \
    for (int i = 0; i < iters; i++) {                                                               \
        asm volatile(INS : "+v"(a0) : "v"(b)); asm volatile(INS : "+v"(a1) : "v"(b));               \
        asm volatile(INS : "+v"(a2) : "v"(b)); asm volatile(INS : "+v"(a3) : "v"(b));               \
        asm volatile(INS : "+v"(a4) : "v"(b)); asm volatile(INS : "+v"(a5) : "v"(b));               \
        asm volatile(INS : "+v"(a6) : "v"(b)); asm volatile(INS : "+v"(a7) : "v"(b));               \
        asm volatile(INS : "+v"(a0) : "v"(b)); asm volatile(INS : "+v"(a1) : "v"(b));               \
        asm volatile(INS : "+v"(a2) : "v"(b)); asm volatile(INS : "+v"(a3) : "v"(b));               \
        asm volatile(INS : "+v"(a4) : "v"(b)); asm volatile(INS : "+v"(a5) : "v"(b));               \
        asm volatile(INS : "+v"(a6) : "v"(b)); asm volatile(INS : "+v"(a7) : "v"(b));               \
    }

template <int OP>
__global__ __launch_bounds__(64) void probe(int iters, unsigned long long mask, int* sink) {
    const int l = threadIdx.x;
    int a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
    const int b = (int)blockIdx.x | 1;
    if ((mask >> l) & 1ull) {
        if constexpr (OP == 0) { BODY("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 1) { BODY("v_mul_lo_u32 %0, %0, %1") }
        if constexpr (OP == 2) { BODY("v_mul_hi_u32 %0, %0, %1") }
        if constexpr (OP == 3) { BODY("v_bcnt_u32_b32 %0, %0, %1") }
        if constexpr (OP == 4) { BODY("v_lshlrev_b32 %0, %1, %0") }
        if constexpr (OP == 5) { BODY("v_cndmask_b32 %0, %0, %1, vcc") }
        if constexpr (OP == 6) { BODY("v_ffbl_b32 %0, %1") }
        if constexpr (OP == 7) { BODY("v_readfirstlane_b32 s0, %1\n v_mov_b32 %0, s0") }
        if constexpr (OP == 8) { BODY("v_mad_u32_u24 %0, %0, %1, %0") }
        if constexpr (OP == 9) { BODY("v_bfe_u32 %0, %0, %1, 5") }
    }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff) sink[l] = 1;
}

int main() {
    const int iters = 2000, blocks = 256 * 4 * 4;  // 4 waves per SIMD
    int* sink;
    hipMalloc(&sink, 256);
    const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_bcnt_u32_b32", "v_lshlrev_b32", "v_cndmask_b32",
                           "v_ffbl_b32", "v_readfirstlane_b32+v_mov", "v_mad_u32_u24", "v_bfe_u32"};
    struct M { const char* name; unsigned long long m; } masks[] = {
        {"all64", ~0ull}, {"first48", (1ull << 48) - 1}, {"first32", 0xFFFFFFFFull}, {"first16", 0xFFFFull},
        {"first8", 0xFFull}, {"first1", 1ull}, {"spread8", 0x0101010101010101ull}, {"spread4_q", 0x0001000100010001ull},
        {"last32", 0xFFFFFFFF00000000ull}, {"odd32", 0xAAAAAAAAAAAAAAAAull}};
    for (int op = 0; op < 10; op++)
        for (auto& mk : masks) {
            void (*k)(int, unsigned long long, int*) =
                op == 0 ? probe<0> : op == 1 ? probe<1> : op == 2 ? probe<2> : op == 3 ? probe<3> : op == 4 ? probe<4>
                : op == 5 ? probe<5> : op == 6 ? probe<6> : op == 7 ? probe<7> : op == 8 ? probe<8> : probe<9>;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, iters, mk.m, sink);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, iters, mk.m, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double n = 16.0 * iters * blocks;
            printf("{\"op\": \"%s\", \"exec\": \"%s\", \"ms\": %.4f, \"wave_insts_per_simd_per_ns\": %.4f}\n", names[op], mk.name, ms,
                   n / 1024.0 / (ms * 1e6));
        }
    return 0;
}
