// EXEC-density probe (gfx950): SIMD cycles per wave64 VALU instruction as a function of how many
// lanes are active, at 4 waves per SIMD (k_env c3's occupancy), for a 2-cycle op (v_add_u32) and
// 4-cycle ops (v_lshlrev_b32, v_mul_lo_u32, v_cmp_gt_u32 + v_cndmask, v_readfirstlane_b32); and a mixed
// SIMD (waves alternately dense and 8-lane sparse) to see whether a sparse wave slows its neighbours.
// Same method as valu_issue_probe.hip (per-SIMD issued instructions / span, s_memtime cycles).
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

constexpr int ITERS = 4000;
struct Stamp {
    unsigned long long t0, t1;
    unsigned hw, xcc;
};

template <int OP>
__global__ __launch_bounds__(64) void probe(int lanes, int mixed, Stamp* out, int* sink) {
    const int l = threadIdx.x;
    int a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
    const int b = (int)blockIdx.x | 1;
    const int myLanes = (mixed && (blockIdx.x & 1)) ? 64 : lanes;
    const bool on = l < myLanes;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (on) {
        for (int i = 0; i < ITERS; i++) {
#define ONE(x)                                                                                 \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));            \
    else if constexpr (OP == 1) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x));             \
    else if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));    \
    else if constexpr (OP == 3) asm volatile("v_readfirstlane_b32 s0, %0" : : "v"(x) : "s0");  \
    else asm volatile("v_cmp_gt_u32 s[0:1], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(x) : "v"(b) : "s0", "s1");
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
            ONE(a0) ONE(a1) ONE(a2) ONE(a3) ONE(a4) ONE(a5) ONE(a6) ONE(a7)
#undef ONE
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) {
        Stamp s;
        s.t0 = t0;
        s.t1 = t1;
        s.hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        s.xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));
        out[blockIdx.x] = s;
    }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff) sink[l] = 1;
}

typedef void (*Kern)(int, int, Stamp*, int*);
int main() {
    const Kern ks[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>};
    const char* names[] = {"v_add_u32", "v_lshlrev_b32", "v_mul_lo_u32", "v_readfirstlane_b32", "v_cmp+v_cndmask"};
    const int insts[] = {1, 1, 1, 1, 2};
    int* sink;
    Stamp* out;
    const int blocks = 4096;  // 4 waves per SIMD
    if (hipMalloc(&sink, 256) != hipSuccess || hipMalloc(&out, blocks * sizeof(Stamp)) != hipSuccess) return 1;
    std::vector<Stamp> h(blocks);
    for (int i = 0; i < 4000; i++) hipLaunchKernelGGL(ks[0], dim3(blocks), dim3(64), 0, 0, 64, 0, out, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (int op = 0; op < 5; op++)
        for (int mixed = 0; mixed < 2; mixed++)
            for (int lanes : {64, 48, 33, 32, 24, 17, 16, 12, 9, 8, 4, 1}) {
                if (mixed && lanes != 8 && lanes != 32) continue;
                for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(ks[op], dim3(blocks), dim3(64), 0, 0, lanes, mixed, out, sink);
                if (hipDeviceSynchronize() != hipSuccess) return 3;
                if (hipMemcpy(h.data(), out, blocks * sizeof(Stamp), hipMemcpyDeviceToHost) != hipSuccess) return 4;
                std::map<unsigned long long, std::vector<int>> bySimd;
                for (int i = 0; i < blocks; i++)
                    bySimd[((unsigned long long)(h[i].xcc & 15) << 32) | (h[i].hw & 0xFFF0u)].push_back(i);
                std::vector<double> cyc;
                for (auto& kv : bySimd) {
                    unsigned long long s0 = ~0ull, s1 = 0;
                    for (int i : kv.second) {
                        s0 = std::min(s0, h[i].t0);
                        s1 = std::max(s1, h[i].t1);
                    }
                    cyc.push_back((double)(s1 - s0) / ((double)kv.second.size() * ITERS * 16.0 * insts[op]));
                }
                std::sort(cyc.begin(), cyc.end());
                printf("{\"op\": \"%s\", \"lanes\": %d, \"mixed_with_dense_waves\": %d, \"cycles_per_inst_per_simd\": "
                       "{\"p10\": %.3f, \"median\": %.3f, \"p90\": %.3f}}\n",
                       names[op], lanes, mixed, cyc[cyc.size() / 10], cyc[cyc.size() / 2], cyc[cyc.size() * 9 / 10]);
                fflush(stdout);
            }
    return 0;
}
