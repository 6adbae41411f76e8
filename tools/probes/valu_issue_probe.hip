// VALU issue-rate probe for the issue roofline: SIMD cycles per wave64 VALU
// instruction, per instruction class, at 1 / 2 / 4 waves per SIMD (k_env's c3 occupancy is 4), with a
// full or an 8-lane EXEC mask.  Each wave runs 8 independent accumulators through ITERS x 16
// instructions of one opcode (inline asm, so nothing is folded); s_memtime (shader cycles) and
// s_memrealtime (100 MHz) are stamped around the loop together with the wave's HW_ID / XCC_ID.  The
// host groups the waves by SIMD and divides the SIMD's issued instructions by the span from its first
// wave's start to its last wave's end: cycles per instruction per SIMD (the issue interval), and the
// shader clock from the two time bases.  Diagnostic only (tools/issue_roofline.py reads the output).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

constexpr int ITERS = 4000;
struct Stamp {
    unsigned long long t0, t1, r0, r1;
    unsigned hw, xcc, pad0, pad1;
};

template <int OP>
__global__ __launch_bounds__(64) void probe(int lanes, Stamp* out, int* sink) {
    const int l = threadIdx.x;
    int a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
    const int b = (int)blockIdx.x | 1;
    const bool on = l < lanes;
    const unsigned long long sm = __builtin_amdgcn_read_exec() ^ (unsigned long long)(blockIdx.x & 7);  // a lane mask in SGPRs
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (on) {
        for (int i = 0; i < ITERS; i++) {
#define ONE(x)                                                                                                 \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));                            \
    else if constexpr (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));                       \
    else if constexpr (OP == 2) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x));                             \
    else if constexpr (OP == 3) asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(x));                              \
    else if constexpr (OP == 4) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(x) : "v"(b));                \
    else if constexpr (OP == 5) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));              \
    else if constexpr (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));                    \
    else if constexpr (OP == 7) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));                    \
    else if constexpr (OP == 8) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(b));               \
    else if constexpr (OP == 9) asm volatile("v_readlane_b32 s0, %0, 1" : : "v"(x) : "s0");                    \
    else if constexpr (OP == 10) asm volatile("v_readfirstlane_b32 s0, %0" : : "v"(x) : "s0");                 \
    else if constexpr (OP == 11) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(b));                    \
    else if constexpr (OP == 12) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(b));                 \
    else if constexpr (OP == 13) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(x), "v"(b) : "vcc");          \
    else if constexpr (OP == 14) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(sm)); \
    else if constexpr (OP == 15) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(b), "v"(l));           \
    else if constexpr (OP == 16) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b));                          \
    else if constexpr (OP == 17) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");     \
    else if constexpr (OP == 18) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(b));                      \
    else if constexpr (OP == 19) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(b));                      \
    else if constexpr (OP == 21) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(x) : "v"(b));             \
    else if constexpr (OP == 22) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(b));     \
    else if constexpr (OP == 23) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b));                 \
    else if constexpr (OP == 24) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b));               \
    else if constexpr (OP == 25) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));                      \
    else if constexpr (OP == 26) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));                  \
    else asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(b));
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
#undef ONE
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (l == 0) {
        Stamp s;
        s.t0 = t0;
        s.t1 = t1;
        s.r0 = r0;
        s.r1 = r1;
        s.hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        s.xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));
        out[blockIdx.x] = s;
    }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff) sink[l] = 1;
}

// 64-bit-result opcodes (register pairs): OP 0 v_mad_u64_u32, 1 v_lshl_add_u64, 2 v_lshrrev_b64
template <int OP>
__global__ __launch_bounds__(64) void probe64(int lanes, Stamp* out, int* sink) {
    const int l = threadIdx.x;
    unsigned long long a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
    const int b = (int)blockIdx.x | 1;
    const bool on = l < lanes;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (on) {
        for (int i = 0; i < ITERS; i++) {
#define ONE(x)                                                                                              \
    if constexpr (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x) : "v"(b) : "vcc");    \
    else if constexpr (OP == 1) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(x));                      \
    else asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x));
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
#undef ONE
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (l == 0) {
        Stamp s;
        s.t0 = t0;
        s.t1 = t1;
        s.r0 = r0;
        s.r1 = r1;
        s.hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        s.xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));
        out[blockIdx.x] = s;
    }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffffull) sink[l] = 1;
}

typedef void (*Kern)(int, Stamp*, int*);
static Kern kern(int op) {
    switch (op) {
        case 0: return probe<0>;
        case 1: return probe<1>;
        case 2: return probe<2>;
        case 3: return probe<3>;
        case 4: return probe<4>;
        case 5: return probe<5>;
        case 6: return probe<6>;
        case 7: return probe<7>;
        case 8: return probe<8>;
        case 9: return probe<9>;
        case 10: return probe<10>;
        case 11: return probe<11>;
        case 12: return probe<12>;
        case 13: return probe<13>;
        case 14: return probe<14>;
        case 15: return probe<15>;
        case 16: return probe<16>;
        case 17: return probe<17>;
        case 18: return probe<18>;
        case 19: return probe<19>;
        case 20: return probe<20>;
        case 21: return probe<21>;
        case 22: return probe<22>;
        case 23: return probe<23>;
        case 24: return probe<24>;
        case 25: return probe<25>;
        case 26: return probe<26>;
        case 27: return probe64<0>;
        case 28: return probe64<1>;
        default: return probe64<2>;
    }
}

int main(int argc, char** argv) {
    const char* names[] = {"v_add_u32", "v_xor_b32", "v_lshlrev_b32", "v_bfe_u32", "v_and_or_b32", "v_cndmask_b32",
                           "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_readlane_b32", "v_readfirstlane_b32",
                           "v_perm_b32", "v_bcnt_u32_b32", "v_cmp_gt_u32", "v_cndmask_b32_e64_sgpr", "v_bfi_b32",
                           "v_mov_b32", "v_add_co_u32", "v_sub_u32", "v_max_u32", "v_or_b32", "v_alignbit_b32",
                           "v_bitop3_b32", "v_add3_u32", "v_lshl_or_b32", "v_and_b32", "v_mul_u32_u24", "v_mad_u64_u32",
                           "v_lshl_add_u64", "v_lshrrev_b64"};
    const int nops = 30;
    int only = -1;
    if (argc > 1) only = atoi(argv[1]);
    int* sink;
    Stamp* out;
    const int maxBlocks = 1024 * 4;
    if (hipMalloc(&sink, 256) != hipSuccess || hipMalloc(&out, maxBlocks * sizeof(Stamp)) != hipSuccess) return 1;
    std::vector<Stamp> h(maxBlocks);
    // clocks up: ~2 s of back-to-back probe launches first (MI355X_MICROARCH.md, DVFS)
    for (int i = 0; i < 8000; i++) hipLaunchKernelGGL(kern(0), dim3(4096), dim3(64), 0, 0, 64, out, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (int op = 0; op < nops; op++)
        for (int wps : {1, 2, 4})
            for (int lanes : {64, 8}) {
                if (only >= 0 && op != only && op != 0) continue;
                const int blocks = 1024 * wps;
                hipLaunchKernelGGL(kern(op), dim3(blocks), dim3(64), 0, 0, lanes, out, sink);
                hipLaunchKernelGGL(kern(op), dim3(blocks), dim3(64), 0, 0, lanes, out, sink);
                if (hipDeviceSynchronize() != hipSuccess) return 3;
                if (hipMemcpy(h.data(), out, blocks * sizeof(Stamp), hipMemcpyDeviceToHost) != hipSuccess) return 4;
                // per SIMD: waves, span [first start, last end], instructions issued
                std::map<unsigned long long, std::vector<int>> bySimd;
                for (int i = 0; i < blocks; i++) {
                    const unsigned hw = h[i].hw;
                    const unsigned long long key = ((unsigned long long)(h[i].xcc & 15) << 32) | (hw & 0xFFF0u);  // SE/SH/CU/SIMD
                    bySimd[key].push_back(i);
                }
                std::vector<double> cyc;
                std::vector<double> clk;
                std::map<int, int> occ;
                for (auto& kv : bySimd) {
                    unsigned long long s0 = ~0ull, s1 = 0;
                    for (int i : kv.second) {
                        s0 = std::min(s0, h[i].t0);
                        s1 = std::max(s1, h[i].t1);
                        clk.push_back((double)(h[i].t1 - h[i].t0) / (double)(h[i].r1 - h[i].r0) * 0.1);  // GHz
                    }
                    occ[(int)kv.second.size()]++;
                    cyc.push_back((double)(s1 - s0) / ((double)kv.second.size() * ITERS * 16.0));
                }
                std::sort(cyc.begin(), cyc.end());
                std::sort(clk.begin(), clk.end());
                int modal = 0, best = 0;
                for (auto& kv : occ)
                    if (kv.second > best) best = kv.second, modal = kv.first;
                printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"lanes\": %d, \"simds\": %zu, \"modal_waves_on_a_simd\": %d, "
                       "\"cycles_per_inst_per_simd\": {\"p10\": %.3f, \"median\": %.3f, \"p90\": %.3f}, \"clock_ghz\": %.3f}\n",
                       names[op], wps, lanes, cyc.size(), modal, cyc[cyc.size() / 10], cyc[cyc.size() / 2], cyc[cyc.size() * 9 / 10],
                       clk[clk.size() / 2]);
                fflush(stdout);
            }
    return 0;
}
