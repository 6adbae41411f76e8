// mrts_kernels.hip — gfx950 kernels for the vectorised microRTS env step.
//
// One 64-lane wavefront (= one workgroup) owns one game.  The game's units live in LDS as
// struct-of-arrays in PhysicalGameState list order (slot order == LinkedList order), with a
// cell -> slot occupancy map (one live unit per cell is an engine invariant:
// PhysicalGameState.addUnit, reference src/rts/PhysicalGameState.java:189-201).  The Java
// semantics are order-dependent (rows in cell order, fillWithNones in list order, conflict scans
// and cycle() execution in LinkedHashMap insertion order), so every ORDERED decision runs
// wave-uniformly (all lanes agree, scalar branches), while every order-free sub-problem
// (row fetch + decode, legality, conflict flags, ready ranking, death compaction, visibility,
// observation planes, legal-action masks) runs lane-parallel with ballots and DPP reductions.
// No MFMA: integer/indexing work.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "mrts_internal.h"

using namespace mrts;

#define DEV __device__ __forceinline__

namespace {

constexpr uint16_t EMPTY = 0xFFFF, WALL = 0xFFFE;
constexpr int INF = 0x7FFFFFFF;
enum { T_NONE = 0, T_MOVE = 1, T_HARVEST = 2, T_RETURN = 3, T_PRODUCE = 4, T_ATTACK = 5 };
enum { MODE_STEP = 0, MODE_RESET = 1, MODE_MASKS = 2, MODE_PLAYOUT = 3, MODE_TRACE = 4 };

// Diagnostic build only (-DMRTS_PHASE_TIMING, tools/phase_timing.py): per-phase shader-clock cycles
// summed over games; not compiled into libmrts.so.
#ifdef MRTS_PHASE_TIMING
constexpr int PH_GAMES = 1 << 16;
constexpr int NPH = 32;  // phase slots
__device__ unsigned long long g_phase[NPH * PH_GAMES];  // [phase][game], no contention
__device__ unsigned long long g_span[11 * PH_GAMES];    // last launch: [game] start / end, s_memrealtime (100 MHz),
                                                       // placement: HW_ID | XCC_ID << 32 | nu at start << 40 | nu at end << 48
#ifdef MRTS_SPAN_ONLY
// per-game start / end / placement plus 8 milestones (lane 0 stores s_memrealtime to g_span block
// 3 + mileOf(phase id)); no per-phase accumulation.  Each stamp costs an lgkmcnt drain and a store.
constexpr int NMILE = 8;
constexpr int mileOf(int ph) {
#ifdef MRTS_MILES_STEP  // multi-step analysis (tools/single_step_anatomy.py MILES=step): 0 = iteration start (after the
                        // view snapshot hand-off), 1 = the rows unpacked + issue index (selfPlayFast) instead of the load
    return ph == 0 ? 0 : ph == 22 ? 1 : ph == 1 ? 2 : ph == 3 ? 3 : ph == 4 ? 4 : ph == 5 ? 5 : ph == 6 ? 6 : ph == 9 ? 7 : -1;
#else
    return ph == 20 ? 0 : ph == 21 ? 1 : ph == 1 ? 2 : ph == 3 ? 3 : ph == 4 ? 4 : ph == 5 ? 5 : ph == 6 ? 6 : ph == 9 ? 7 : -1;
#endif
}
#ifdef MRTS_NO_MILESTONES  // start / end / placement only (tools/launch_gap.py)
#define PHASE_IN(acc, tt, i) \
    do {                     \
    } while (0)
#else
#define PHASE_IN(acc, tt, i)                                                                      \
    do {                                                                                          \
        if (mileOf(i) >= 0 && threadIdx.x == 0 && (int)blockIdx.x < PH_GAMES)                      \
            g_span[(3 + mileOf(i)) * PH_GAMES + blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#endif
#else
#define PHASE_IN(acc, tt, i)                          \
    do {                                              \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        (acc)[i] += t_ - (tt);                        \
        (tt) = t_;                                    \
    } while (0)
#endif
#define PHASE(i) PHASE_IN(G.phAcc, G.tph_, i)  // in the kernel body
#define MPHASE(i) PHASE_IN(phAcc, tph_, i)     // inside Game methods
#else
#define PHASE(i) \
    do {         \
    } while (0)
#define MPHASE(i) \
    do {          \
    } while (0)
#endif
// Diagnostic build only (-DMRTS_ABLATE, tools/ablate_price.py): g_ablate bit b runs phase b twice
// (idempotently, inputs laundered so the copies cannot be merged) — the marginal cost of a phase in
// the real, contended kernel.  Never loaded by the package.
#ifdef MRTS_ABLATE
__device__ uint32_t g_ablate;
__device__ unsigned long long g_dbg[4];  // diagnostics: [0] PO render items, [1] PO renders, [2] delta renders
template <class T>
DEV T launder(T v) {
    asm volatile("" : "+v"(v));
    return v;
}
template <class T>
DEV void keepv(T v) {
    asm volatile("" ::"v"(v));
}
#define ABL(b) ((G_AB >> (b)) & 1u)
enum { AB_LOAD = 0, AB_OBS = 1, AB_STORE = 2, AB_MASKBITS = 3, AB_RECORD = 4, AB_POLICY = 5, AB_ACCEPT = 6,
       AB_LEGAL = 7, AB_OUTCOME = 8, AB_INDEX = 9, AB_GONE = 10, AB_TABLES = 11, AB_RANK = 12, AB_DECODE = 13,
       AB_ISSUE = 14, AB_CYCLERANK = 15,
       // skips (outputs nothing in the step reads back): the observation, the mask record stores
       AB_SKIP_OBS = 16, AB_SKIP_RECORD = 17,
       // PO observation split: everything but the stores (values kept alive) / only the stores (zeros)
       AB_PO_NOSTORE = 18, AB_PO_ZEROSTORE = 19,
       // PO observation pieces skipped: sight-disk painting, the last-writer cell map, the render record
       AB_PO_NOPAINT = 20, AB_PO_NOSCELL = 21, AB_PO_NORECORD = 22, AB_PO_NOSNAPSHOT = 23, AB_COUNT = 24 };
#endif
enum { GT_SELFPLAY = 0, GT_AGENT_VS_BOT = 1, GT_BOT_VS_BOT = 2, GT_PLAYOUT = 3 };  // game_kind & 15
// per-player counters of this step's issued pairs, as the TraceEntry holds them (after issueSafe's
// legality rewrite, before issue()'s conflict cancellations): HARVEST, RETURN, ATTACK, and PRODUCE
// of a Worker / a Base or Barracks / a Light, Heavy or Ranged
enum { RC_HARVEST = 0, RC_RETURN = 1, RC_ATTACK = 2, RC_PROD_WORKER = 3, RC_PROD_BUILDING = 4, RC_PROD_COMBAT = 5, RC_N = 6 };
DEV int prodCategory(uint32_t typeFlags) {  // the reward functions' name tests (DevUtt.flags N_*)
    return (typeFlags & N_WORKER) ? RC_PROD_WORKER : (typeFlags & N_BUILDING) ? RC_PROD_BUILDING
                                                   : (typeFlags & N_COMBAT) ? RC_PROD_COMBAT : -1;
}
enum { GK_PASSIVE = 0, GK_RANDOM_BIASED = 1 };                    // AI kinds (bits 4-7 ai1, 8-11 ai2)
enum : uint32_t {
    E_CAPACITY = 1u << 0, E_ADDUNIT = 1u << 1, E_PRODUCE_TYPE = 1u << 2, E_OLDER = 1u << 3,
    E_NEG_RES = 1u << 4, E_COLLISION = 1u << 5, E_RECORD = 1u << 6
};
// MODE_TRACE per-game result word (KDyn.trace_out)
enum : uint32_t { TR_ISSUED = 1u, TR_GAMEOVER = 2u, TR_NO_UNIT = 4u };

DEV int lane_id() { return (int)threadIdx.x; }
// branch-probability hints: cold paths (more than 64 units, auto-reset, conflict resolution, the
// general mask writer, reward bookkeeping the benchmark does not request) are laid out away from the
// hot straight-line code, which then packs into fewer instruction-cache lines
#define MRTS_LIKELY(x) __builtin_expect(!!(x), 1)
#define MRTS_UNLIKELY(x) __builtin_expect(!!(x), 0)
// Output stores.  WT = streaming (`nt`) stores, so output lines do not sit dirty in the XCD's L2
// until the end-of-kernel write-back.  Builtins, not inline asm: the wait-count and store-data
// hazard passes must see the stores.  MRTS_WT bits (measured on c3 / c5 / --mask-mode full,
// profiles/r12_summary.md): 1 full-observability planes (c3 +4.5 %, full masks +3 %: on),
// 2 delta mask records + policy rows (c3 -1.3 %), 4 full-rewrite mask chunks (-15 %),
// 8 state block (neutral), 16 partial-observability planes (c5 -18 %).  Round 2: write-through
// (`sc1`) buffer stores leave no line in the XCD's L2, so the next step's state and action-row
// reads (the same game runs on the same XCD every launch: tools/xcd_placement.py) keep theirs:
// 32 full-observability planes (c3 +3.2 %), 128 partially observable planes (c5 +3.4 %), 64 delta
// mask records (byte-granular partial lines: c3 -5 %, off).  profiles/round2_store_policy.md.
#ifndef MRTS_MULTI_NOPRIO
#define MRTS_MULTI_NOPRIO 0
#endif
// 0: multi-step launches take the unit-count thresholds only, not the rank among the SIMD's waves (A/B)
#ifndef MRTS_SIMD_RANK
#define MRTS_SIMD_RANK 1
#endif
// 1: the rank also on c5's partially observable kernel (measured -4 %: its games outrank their own
// helper waves, which then reach the handoff barriers late; round3q)
// the rank's remaining-work estimate: (units + own idle units + MRTS_RANK_C) x steps left.  One game
// alone on a SIMD takes ~ a + b x units per step with a / b ~ 75 units (E = 1024 span data), so the
// steps left dominate: the games that fell behind issue first (c3, same box, 3 runs each: C = 0
// 315.5 / 285.3 M at K = 200 / 20, C = 75 334.4 / 285.5 M, C = 150 334.1 / 280.7, C = 400 333.6 / 284.5;
// later, with balanced placement and the byte image, C = 4000 vs 400: K = 20 kernel 11.95 vs 12.08 us
// per step over 4 pairs, K = 200 equal — a game one step behind always outranks, units break ties)
#ifndef MRTS_RANK_C
#define MRTS_RANK_C 4000
#endif
// 0: multi-step launches keep game g on block g (no balanced placement, A/B builds)
#ifndef MRTS_BALANCE
#define MRTS_BALANCE 1
#endif
// k_env's step body reads KDyn through the laundered pointer too (round 6: SGPR spills 153 -> 136, no VGPR spills,
// but c3 / c5 / c2 +-0 to -0.6 %: the re-read fields wait on scalar loads where the spilled ones were a readlane)
#ifndef MRTS_BODY_LAUNDER
#define MRTS_BODY_LAUNDER 0
#endif
#ifndef MRTS_BAL_MIN_ITER
#define MRTS_BAL_MIN_ITER 64
#endif
// c5 (partially observable 32x32 self-play with helper waves) placed the same way: the dispatcher puts the game
// waves of blocks b and b + n / 2 on one SIMD (round 6 span data, profiles/round6/placement_c5.json); c5 +0.6 %
#ifndef MRTS_BALANCE_PO
#define MRTS_BALANCE_PO 1
#endif
#ifndef MRTS_BAL_PO_GS
#define MRTS_BAL_PO_GS 2
#endif
// the cost a game posts for the next placement: 0 = its unit count, 1 = units + own idle units at the launch's
// last step (the estimate the SIMD rank uses: a step's decode / issue / mask / policy work grows with the idle
// ones; round 6: c3 K = 20 kernel -0.6 %, c5 +0.4 % over 0; the estimate averaged over the launch's steps was worse)
#ifndef MRTS_BAL_COST_IDLE
#define MRTS_BAL_COST_IDLE 1
#endif
// 1: rollout timing events ride on the kernel dispatch (hipExtLaunchKernelGGL); 0: separate records
#ifndef MRTS_EXT_EVENTS
#define MRTS_EXT_EVENTS 1
#endif
#ifndef MRTS_SIMD_RANK_PO
#define MRTS_SIMD_RANK_PO 0
#endif
#ifndef MRTS_SAMPLE_UNIFIED
#define MRTS_SAMPLE_UNIFIED 1
#endif
#ifndef MRTS_PO_ROWS  // PO maps up to 32 wide: the ranged attack bits from unit row bitmaps too (round 6)
#define MRTS_PO_ROWS 1
#endif
#ifndef MRTS_MASK_QUADS  // c3: each idle unit's mask bits computed by a quad of lanes, one per direction (round 6)
#define MRTS_MASK_QUADS 1
#endif
#ifndef MRTS_REC_LANES  // delta mask records stored lane-parallel (storeRecordsLanes, round 5); 0 = by their own lanes
#define MRTS_REC_LANES 1
#endif
#ifndef MRTS_PHILOX_UNROLL
#define MRTS_PHILOX_UNROLL 1
#endif
#ifndef MRTS_POS_CHECKED  // selfPlayFast's issueBatch skips the position pairs acceptChain settled (round 5)
#define MRTS_POS_CHECKED 1
#endif
#ifndef MRTS_SAMPLE32  // the sampler's type / produce-type picks in 32-bit operations, the packed word direct (round 5)
#define MRTS_SAMPLE32 1
#endif
#ifndef MRTS_PO_VRES  // PO self-play: the views' base reservations in their own bitmap (round 6: measured -0.5 %, off)
#define MRTS_PO_VRES 0
#endif
#ifndef MRTS_QUADS_PO  // the quads on the partially observable 32x32 instances too (round 6)
#define MRTS_QUADS_PO 1
#endif
#ifndef MRTS_WALK32  // the cost walks on the 32x32 partially observable instances too, base reservations included (round 6)
#define MRTS_WALK32 1
#endif
#ifndef MRTS_INDEX_WALK  // buildIndex's PRODUCE costs by a walk over their lanes (round 5); 0 = wave reductions
#define MRTS_INDEX_WALK 1
#endif
#ifndef MRTS_PICK_SPLIT  // the sampler's direction picks as 32-bit picks apart from the attack pick (round 5)
#define MRTS_PICK_SPLIT 1
#endif
#ifndef MRTS_ETA_FLAT  // cycleLanes' ready test with the branch-free duration lookup (round 5)
#define MRTS_ETA_FLAT 1
#endif
#ifndef MRTS_DECODE_FWD  // selfPlayFast decodes forwarded words directly (decodeFwd, round 5)
#define MRTS_DECODE_FWD 1
#endif
#ifndef MRTS_CONF_LDS  // acceptChainReg's parallel-path conflict test through an LDS copy of the reservations (round 5)
#define MRTS_CONF_LDS 1
#endif
#ifndef MRTS_XOR3  // Philox's xors as one three-input bit op (round 5); 0 = plain C
#define MRTS_XOR3 1
#endif
// c2's helper-wave launches: the game wave issues at priority >= 1, ahead of its helper wave (at 0) — round 6:
// c2 +1.6 % / +0.4 % (two rounds of interleaved runs; the helper at 3 instead: -4.5 %); on c5 +0.5 % / -0.6 %, so
// c5 keeps its unit-count priorities (which already put most of its games above their helpers: without any
// priority c5 lost 9 %)
#ifndef MRTS_GAME_OVER_HELPER
#define MRTS_GAME_OVER_HELPER 1
#endif
#ifndef MRTS_HELPER_PRIO
#define MRTS_HELPER_PRIO 0
#endif
// 1: partially observable multi-step launches without the render helper wave (A/B builds only).  Round 4
// had made it the default after its full-size soak found 2 of 2048 c5 games with one stale observation value
// for a unit that died in the observed step; round 5 found the cause (the renders read the dead unit's
// fields by readlane inside their divergent chunk loop, from a lane that was off there — writeObsPOFast)
// and the helper is back on.
#ifndef MRTS_PO_FAST  // partially observable self-play games through selfPlayFast (round 5); 0 = the generic path
#define MRTS_PO_FAST 1
#endif
#ifndef MRTS_RESP_RING  // the per-step Responses ring (mrts_set_step_responses); 0 = A/B builds without it
#define MRTS_RESP_RING 1
#endif
#ifndef MRTS_NO_PO_HELPER
#define MRTS_NO_PO_HELPER 0
#endif
// issue-priority thresholds on a game's unit count (k_env): 1 / 2 / 3 from T1 / T2 / T3 units
// (units + own idle units; measured against units alone at 24 / 30 / 36: c3 +1.8 % at K = 200,
// +0.8 % at K = 20)
#ifndef MRTS_PRIO_IDLE
#define MRTS_PRIO_IDLE 1
#endif
#ifndef MRTS_PRIO_T1
#define MRTS_PRIO_T1 29
#endif
#ifndef MRTS_PRIO_T2
#define MRTS_PRIO_T2 35
#endif
#ifndef MRTS_PRIO_T3
#define MRTS_PRIO_T3 41
#endif
#ifndef MRTS_WT
#define MRTS_WT 161
#endif
typedef int32_t i32x4v __attribute__((ext_vector_type(4)));
typedef int32_t i32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef int32_t i32x3u __attribute__((ext_vector_type(3), aligned(4)));
template <bool WT>
DEV void st4(void* p, int a, int b, int c, int d) {  // 16-byte aligned
    const i32x4v v = {a, b, c, d};
    if (WT) __builtin_nontemporal_store(v, (i32x4v*)p);
    else *(i32x4v*)p = v;
}
template <bool WT>
DEV void st4u(void* p, int a, int b, int c, int d) {  // 4-byte aligned
    const i32x4u v = {a, b, c, d};
    if (WT) __builtin_nontemporal_store(v, (i32x4u*)p);
    else *(i32x4u*)p = v;
}
template <bool WT>
DEV void st3u(void* p, int a, int b, int c) {  // 4-byte aligned
    const i32x3u v = {a, b, c};
    if (WT) __builtin_nontemporal_store(v, (i32x3u*)p);
    else *(i32x3u*)p = v;
}
template <bool WT>
DEV void st1(int32_t* p, int a) {
    if (WT) __builtin_nontemporal_store(a, p);
    else *p = a;
}
constexpr bool WT_OBS = (MRTS_WT & 1) != 0, WT_MASK = (MRTS_WT & 2) != 0, WT_FULLMASK = (MRTS_WT & 4) != 0,
               WT_STATE = (MRTS_WT & 8) != 0, WT_POOBS = (MRTS_WT & 16) != 0;
// MRTS_WT bit 32: full-observability planes as write-through (`sc1`) buffer stores, which leave no
// line in the XCD's L2 (MI355X_MICROARCH.md, store flavours), so the next step's state and action
// reads keep their L2 lines; `rsrc` = a raw buffer over the stored region (gfx9 descriptor word 3)
constexpr bool SC1_OBS = (MRTS_WT & 32) != 0;
// MRTS_WT bit 64: delta mask records (and zero records) likewise; bit 128: partially observable planes
constexpr bool SC1_MASK = (MRTS_WT & 64) != 0, SC1_POOBS = (MRTS_WT & 128) != 0;
DEV __amdgpu_buffer_rsrc_t bufRsrc(void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
}
DEV void st4sc1(__amdgpu_buffer_rsrc_t r, uint32_t byteOff, int a, int b, int c, int d) {
    const i32x4v v = {a, b, c, d};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)byteOff, 0, 16);
}
DEV int ux(uint32_t c) { return (int)(c & 0xFF); }
DEV int uy(uint32_t c) { return (int)((c >> 8) & 0xFF); }
DEV int utyp(uint32_t c) { return (int)((c >> 16) & 0xF); }
DEV int uplay(uint32_t c) { return (int)((c >> 20) & 3) - 1; }
DEV uint32_t pack_uc(int x, int y, int t, int p) {
    return (uint32_t)x | ((uint32_t)y << 8) | ((uint32_t)t << 16) | ((uint32_t)(p + 1) << 20);
}
DEV int ua_type(uint32_t a) { return (int)(a & 0xF); }
DEV int ua_ut(uint32_t a) { return (int)((a >> 4) & 0xF); }
DEV int ua_tx(uint32_t a) { return (int)((a >> 8) & 0xFF); }
DEV int ua_ty(uint32_t a) { return (int)((a >> 16) & 0xFF); }
DEV uint32_t pack_ua(int t, int ut, int tx, int ty) {
    return (uint32_t)t | ((uint32_t)ut << 4) | ((uint32_t)tx << 8) | ((uint32_t)ty << 16);
}
// UnitAction.DIRECTION_OFFSET_X/Y (rts/UnitAction.java:94-100); invalid directions move nowhere
DEV int dxo(int d) { return d == 1 ? 1 : (d == 3 ? -1 : 0); }
DEV int dyo(int d) { return d == 0 ? -1 : (d == 2 ? 1 : 0); }
DEV int clampdir(int d) { return (d >= 0 && d <= 3) ? d : ACT_INVALID; }

// Diagnostic build only (-DMRTS_LANE_AUDIT, `make audit`; tests/test_zz_lane_audit.py): every cross-lane read
// checks at run time that the lanes it reads are active where it executes — a readlane's source lane, every lane
// for the DPP reductions and ballots (which the code treats as whole-wave) — and records the source line of a
// violation in g_laneAudit (one vector store per lane, its own slot).  A readlane of an inactive lane returns
// whatever its register last held (the round-4 soak's stale PO value).  Not in libmrts.so.
#ifdef MRTS_LANE_AUDIT
__device__ int32_t g_laneAudit[256];
DEV void laneAuditHit(int line, int kind) { g_laneAudit[threadIdx.x & 255] = line | (kind << 24); }
DEV bool laneOn(int k) { return (__builtin_amdgcn_read_exec() >> k) & 1ull; }
DEV bool waveOn() { return __builtin_amdgcn_read_exec() == ~0ull; }
DEV int rlAudit(int v, int k, int line) {
    if (!laneOn(k)) laneAuditHit(line, 1);
    return __builtin_amdgcn_readlane(v, k);
}
#define rl(v, k) rlAudit((v), (k), __LINE__)
#define LANE_AUDIT_WAVE(kind)                              \
    do {                                                   \
        if (!waveOn()) laneAuditHit(__LINE__, (kind));     \
    } while (0)
#else
DEV int rl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
#define LANE_AUDIT_WAVE(kind) ((void)0)
#endif
// four int32 values (each within int16) as four packed int16
DEV uint2 pk16(int4 w) {
    return make_uint2(((uint32_t)w.x & 0xFFFFu) | ((uint32_t)w.y << 16), ((uint32_t)w.z & 0xFFFFu) | ((uint32_t)w.w << 16));
}
DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
DEV uint32_t uniu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
#ifdef MRTS_LANE_AUDIT
#define ballot(p) ballotAudit((p), __LINE__)
DEV uint64_t ballotAudit(bool p, int line) {
    if (!waveOn()) laneAuditHit(line, 3);
    return __ballot(p);
}
#else
DEV uint64_t ballot(bool p) { return __ballot(p); }
#endif
DEV int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
// A game is one wave and its LDS is private to that wave: LDS operations of one wave execute in
// order, so a wave-scope fence (a compiler barrier, no instruction) orders them across lanes.
DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Whole-wave reductions with DPP (GFX9 row_bcast forms): quad swaps, half-row and row mirrors
// reduce each 16-lane row; row_bcast:15/31 chain the rows; lane 63 holds the result.
template <bool MIN>
DEV int wave_reduce(int v) {
    LANE_AUDIT_WAVE(2);
    const int id = MIN ? INF : 0;
    auto op = [](int a, int b) { return MIN ? min(a, b) : a + b; };
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x140, 0xF, 0xF, false));  // row_mirror
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return rl(v, 63);
}
// Inclusive prefix sum over the wave's lanes with DPP: row_shr 1/2/4/8 scan each 16-lane row
// (lanes shifted in from outside the row read 0), row_bcast:15 / :31 carry the row totals.
DEV int wave_incl_sum(int v) {
    LANE_AUDIT_WAVE(2);
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
DEV int wave_min(int v) { return wave_reduce<true>(v); }
DEV int wave_sum(int v) { return wave_reduce<false>(v); }

// java.util.Random (48-bit LCG, JDK 8) — GameState.r / UnitAction.r / Sampler.generator, per game
struct JRand {
    uint64_t s;
    DEV int next(int bits) {
        s = (s * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int)(uint32_t)(s >> (48 - bits));
    }
    DEV int nextInt(int bound) {
        if ((bound & -bound) == bound) return (int)(((int64_t)bound * (int64_t)next(31)) >> 31);
        int bits, val;
        do {
            bits = next(31);
            val = bits % bound;
        } while ((int)((uint32_t)bits - (uint32_t)val + (uint32_t)(bound - 1)) < 0);
        return val;
    }
    DEV double nextDouble() { return (double)(((int64_t)next(26) << 27) + next(27)) * (1.0 / 9007199254740992.0); }
};
DEV uint64_t rng_of(int lo, int hi) { return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32); }

// Snapshot byte per unit for PartiallyObservableGameState views (rts/PartiallyObservableGameState.java:35-54):
// bit p = unit is in player p's snapshot list; bits 2-4 / 5-7 = (snapshot UAA action type + 1), 0 = none.
DEV int snap_in(uint32_t b, int p) { return (b >> p) & 1; }
DEV int snap_act(uint32_t b, int p) { return (int)((b >> (2 + 3 * p)) & 7); }

// The unit-type table is read with lane-varying indices all over the step; an LDS copy turns those
// global loads into LDS reads.
constexpr int UTT_WORDS = (int)(sizeof(DevUtt) / 4);
constexpr int UTT_LDS = (int)((sizeof(DevUtt) + 15) & ~(size_t)15);
static_assert(sizeof(DevUtt) % 4 == 0 && UTT_WORDS <= 192, "DevUtt copy: 3 words per lane");

// a ^ b ^ k in one VALU instruction (gfx950's three-input bit op, truth table 0x96; the compiler emits
// two v_xor_b32 for it).  k MUST be wave-uniform (a Philox key word, in an SGPR): the "s" constraint would
// silently readfirstlane a per-lane value.  Other targets (ARCH overridden) take the plain C form.
DEV uint32_t xor3s(uint32_t a, uint32_t b, uint32_t k) {
#if MRTS_XOR3 && defined(__gfx950__)
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "s"(k));
    return d;
#else
    return a ^ b ^ k;
#endif
}
// Philox4x32-10, the ten rounds unrolled (rolled, the loop carried two v_mov per round and the xors
// were not fused: 8 VALU per round against 4)
DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#if MRTS_PHILOX_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = xor3s((uint32_t)(p1 >> 32), c[1], k0), n1 = (uint32_t)p1;
        const uint32_t n2 = xor3s((uint32_t)(p0 >> 32), c[3], k1), n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
DEV int pickBit(uint32_t r, uint64_t bitsv, int n) {
    const uint64_t m = n >= 64 ? ~0ull : ((1ull << n) - 1);
    bitsv &= m;
    const int cnt = __popcll(bitsv);
    if (cnt == 0) return -1;
    int k = (int)(((uint64_t)r * (uint32_t)cnt) >> 32);
    while (k--) bitsv &= bitsv - 1;
    return __builtin_ctzll(bitsv);
}
// one cell's action from its mask bits (lo/hi: mask slots 1..K-1 -> bit i-1), Philox counter
// (slot id, step, cell, 0)
// Masked-uniform random policy of one cell (the bench / rollout agent): mask slots 1..K-1 as bits
// (lo: slots 1..64, hi: 65..), Philox4x32-10 with key = seed, counter = (slot id, step, cell, 0)
DEV uint32_t packFwdFree(const int32_t a[7]) {  // = packFwd (defined with the forwarded words below)
    return ((uint32_t)a[0] & 7u) | (((uint32_t)(a[1] + 1) & 7u) << 3) | (((uint32_t)(a[2] + 1) & 7u) << 6) |
           (((uint32_t)(a[3] + 1) & 7u) << 9) | (((uint32_t)(a[4] + 1) & 7u) << 12) | (((uint32_t)(a[5] + 1) & 15u) << 15) |
           (((uint32_t)(a[6] + 1) & 127u) << 19);
}
// pickBit of a field of at most 32 bits (already masked): the same pick in 32-bit operations
DEV int pickBit32(uint32_t r, uint32_t bitsv) {
    const int cnt = __popc(bitsv);
    if (cnt == 0) return -1;
    int k = (int)__umulhi(r, (uint32_t)cnt);
    while (k--) bitsv &= bitsv - 1;
    return __builtin_ctz(bitsv);
}
// packFwd of a row with every value 0 (each parameter field holds value + 1)
constexpr uint32_t FWD_ZERO = (1u << 3) | (1u << 6) | (1u << 9) | (1u << 12) | (1u << 15) | (1u << 19);
// packed (optional): packFwd(a) of the drawn row, built from the picks (no field repacking)
DEV void sampleBitsRaw(uint64_t seed, uint32_t step, uint32_t slotId, int ntypes, int K, uint64_t lo, uint64_t hi, int c,
                       int32_t a[7], uint32_t* packed = nullptr) {
#if MRTS_SAMPLE_UNIFIED && MRTS_SAMPLE32
    uint32_t ctr[4] = {slotId, step, (uint32_t)c, 0u};
    philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    // mask slots 1..K-1 as bits of lo:hi (slot k -> bit k - 1): the type field is bits 0..5, the produce
    // types bits 22.., the direction fields bits 6 + 4 (t - 1).., the attack window bits 22 + ntypes..
    const int t = pickBit32(ctr[0], (uint32_t)lo & 63u);
    int pv = 0, ut = 0;
    if (MRTS_PICK_SPLIT && t > 0 && t < 5) {
        // a direction: 4 bits at 2 + 4 t (below 32) — one 32-bit pick
        pv = pickBit32(ctr[1], ((uint32_t)lo >> (2 + 4 * t)) & 15u);
    } else if (t > 0) {
        // the attack window: K - 23 - ntypes bits from 22 + ntypes (across lo / hi); without
        // MRTS_PICK_SPLIT every type's field in this one 64-bit pick
        const int b = t == 5 ? 22 + ntypes : 2 + 4 * t, n = t == 5 ? K - 23 - ntypes : 4;
        uint64_t v = b >= 64 ? hi >> (b - 64) : ((lo >> b) | (hi << (64 - b)));
        v &= n >= 64 ? ~0ull : ((1ull << n) - 1);
        pv = pickBit(ctr[1], v, 64);
    }
    if (t == 4) ut = pickBit32(ctr[2], (uint32_t)(lo >> 22) & ((1u << ntypes) - 1u));
    a[0] = t > 0 ? t : 0;
    a[1] = t == 1 ? pv : 0;
    a[2] = t == 2 ? pv : 0;
    a[3] = t == 3 ? pv : 0;
    a[4] = t == 4 ? pv : 0;
    a[5] = ut;
    a[6] = t == 5 ? pv : 0;
    if (packed)
        *packed = FWD_ZERO + (uint32_t)(t > 0 ? t : 0) + (t > 0 ? (uint32_t)pv << (t == 5 ? 19 : 3 * t) : 0u) +
                  ((uint32_t)ut << 15);
#else
    for (int k = 0; k < 7; k++) a[k] = 0;
    uint32_t ctr[4] = {slotId, step, (uint32_t)c, 0u};
    philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    auto field = [&](int off, int n) -> uint64_t {  // mask slots [off, off+n) (off >= 1)
        const int b = off - 1;
        uint64_t v;
        if (b >= 64) v = hi >> (b - 64);
        else v = (lo >> b) | (b ? (hi << (64 - b)) : 0ull);
        return n >= 64 ? v : (v & ((1ull << n) - 1));
    };
    const int t = pickBit(ctr[0], field(1, 6), 6);
    if (t < 0) {
        if (packed) *packed = FWD_ZERO;
        return;
    }
    a[0] = t;
#if MRTS_SAMPLE_UNIFIED
    // the parameter of type t from ONE pick over that type's field (move / harvest / return / produce
    // direction: 4 slots at 7 + 4 (t - 1); attack: the K - 23 - ntypes slots after the unit types), not
    // one pick per case: the lanes of a wave hold several types, and a switch runs its cases one after
    // the other.  Same words of the same Philox block, same picks: identical rows.
    if (t > 0) {
        const int off = t == 5 ? 23 + ntypes : 3 + 4 * t, n = t == 5 ? K - 23 - ntypes : 4;
        const int pv = pickBit(ctr[1], field(off, n), n);
        a[1] = t == 1 ? pv : 0;
        a[2] = t == 2 ? pv : 0;
        a[3] = t == 3 ? pv : 0;
        a[4] = t == 4 ? pv : 0;
        a[6] = t == 5 ? pv : 0;
    }
    if (t == 4) a[5] = pickBit(ctr[2], field(23, ntypes), ntypes);
#else
    switch (t) {
        case 1: a[1] = pickBit(ctr[1], field(7, 4), 4); break;
        case 2: a[2] = pickBit(ctr[1], field(11, 4), 4); break;
        case 3: a[3] = pickBit(ctr[1], field(15, 4), 4); break;
        case 4:
            a[4] = pickBit(ctr[1], field(19, 4), 4);
            a[5] = pickBit(ctr[2], field(23, ntypes), ntypes);
            break;
        case 5: {
            const int off = 23 + ntypes, n = K - off;
            a[6] = pickBit(ctr[1], field(off, n), n);
        } break;
    }
#endif
    if (packed) *packed = packFwdFree(a);
#endif
}

// Unmasked uniform random row (BASELINE config c2) of cell c of slot id slotId:
// type in [0, 6), the four directions in [0, 4), produce type in [0, ntypes), attack window index
// in [0, natt) — rows that reach every illegal -> NONE path of issueSafe.  Philox4x32-10, key =
// seed, counter = (slot id, step, cell, UNIFORM_TAG); ranges by multiply-shift of the 32-bit words.
constexpr uint32_t UNIFORM_TAG = 0x554E4946u;  // "UNIF": a stream apart from the masked policy's (word 3 = 0)
DEV void uniformRow(uint64_t seed, uint32_t step, uint32_t slotId, int c, int ntypes, int natt, int32_t a[7]) {
    uint32_t ctr[4] = {slotId, step, (uint32_t)c, UNIFORM_TAG};
    philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    auto below = [](uint32_t r, int n) { return (int)(((uint64_t)r * (uint32_t)n) >> 32); };
    a[0] = below(ctr[0], 6);
    a[1] = (int)(ctr[1] & 3u);
    a[2] = (int)((ctr[1] >> 2) & 3u);
    a[3] = (int)((ctr[1] >> 4) & 3u);
    a[4] = (int)((ctr[1] >> 6) & 3u);
    a[5] = below(ctr[2], ntypes);
    a[6] = below(ctr[3], natt);
}

// Forwarded action word (H_FWD / stateFwdOff): the 7 values of a fused-policy row, which the sampler
// draws as type 0..5 and parameters -1..(field size - 1): type 3 bits, the four directions 3 bits
// each, produce type 4 bits, attack index 7 bits, each parameter stored + 1.
DEV uint32_t packFwd(const int32_t a[7]) {
    return ((uint32_t)a[0] & 7u) | (((uint32_t)(a[1] + 1) & 7u) << 3) | (((uint32_t)(a[2] + 1) & 7u) << 6) |
           (((uint32_t)(a[3] + 1) & 7u) << 9) | (((uint32_t)(a[4] + 1) & 7u) << 12) | (((uint32_t)(a[5] + 1) & 15u) << 15) |
           (((uint32_t)(a[6] + 1) & 127u) << 19);
}
DEV void unpackFwd(uint32_t w, int32_t a[7]) {
    a[0] = (int32_t)(w & 7u);
    a[1] = (int32_t)((w >> 3) & 7u) - 1;
    a[2] = (int32_t)((w >> 6) & 7u) - 1;
    a[3] = (int32_t)((w >> 9) & 7u) - 1;
    a[4] = (int32_t)((w >> 12) & 7u) - 1;
    a[5] = (int32_t)((w >> 15) & 15u) - 1;
    a[6] = (int32_t)((w >> 19) & 127u) - 1;
}

// The kernel's KDyn argument as a pointer into the constant (kernarg) address space.  The multi-step
// loop makes it opaque once per iteration (freshLane), so the compiler re-reads a field with a scalar
// load (SMEM) where the step uses it, instead of loading every field at kernel entry and keeping it
// live across the loop: that spilled ~240 SGPRs into VGPR lanes, and every reload was a v_readlane —
// a VALU instruction in a VALU-issue-bound kernel (MRTS_DYN_LAUNDER = 0: the old form).
#ifndef MRTS_DYN_LAUNDER
#define MRTS_DYN_LAUNDER 1
#endif
typedef const __attribute__((address_space(4))) KDyn* KDynPtr;
// k_env's KDyn argument: its third kernel argument, after the two pointers, at byte 16 of the kernarg
// segment.  The offset is laundered (not the address: an address escaping into asm makes the compiler
// copy the whole argument to scratch memory first).
static_assert(alignof(KDyn) <= 8, "k_env(int32_t*, const KStatic*, KDyn): KDyn at kernarg byte 16");
DEV KDynPtr kdynArg(bool launder) {
    int z = 0;
    if (launder) asm volatile("" : "+s"(z));
    return (KDynPtr)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + 16 + z);
}
// One sight disk (dx^2 + dy^2 <= sr^2) ORed into per-row bitmaps of a W-wide map ((W + 31) / 32 words a
// row): one atomicOr per covered row word.  dlo / dhi: the unit-type table's half-widths for sr <= 15
// (host-computed, DevUtt::diskLo/Hi); a larger sight takes the integer square root per row.
DEV void paintDiskRows(uint32_t* rows, int H, int W, int x, int y, int sr, uint32_t dlo, uint32_t dhi) {
    const int WPR = (W + 31) >> 5;
    for (int dy = -sr; dy <= sr; dy++) {
        const int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        const int ady = dy < 0 ? -dy : dy;
        int w;
        if (sr <= 15) {
            w = (int)(((ady < 8 ? dlo : dhi) >> (4 * (ady & 7))) & 0xFu);
        } else {
            const int lim = sr * sr - dy * dy;
            w = (int)__builtin_sqrtf((float)lim);
            while (w * w > lim) w--;
            while ((w + 1) * (w + 1) <= lim) w++;
        }
        const int x0 = max(0, x - w), x1 = min(W - 1, x + w);
        for (int k = x0 >> 5; k <= (x1 >> 5); k++) {
            const int lo = max(x0, 32 * k) - 32 * k, hi = min(x1, 32 * k + 31) - 32 * k;
            const uint32_t b = (hi - lo == 31) ? 0xFFFFFFFFu : (((1u << (hi - lo + 1)) - 1u) << lo);
            atomicOr(&rows[yy * WPR + k], b);
        }
    }
}

struct Game {
#define D (*Dp)
    const KStatic& P;
    KDynPtr Dp;  // the kernel argument itself (kernarg memory): fields load on demand
    const DevUtt& U;
    int g, H, W, HW, CAP;
    int K, NT, R;  // mask slots per cell, unit types, attack window (2 * max range + 1): table values or constants
    bool po;
    bool iter;        // a multi-step kernel (KDyn.n_iter iterations per launch)
    int32_t* stBase;  // the state blocks (a leading kernel argument: preloaded into SGPRs)
    int stWords;      // words per state block (a constant in a specialised kernel)
    uint32_t* uc;    // unit core: x | y<<8 | type<<16 | (player+1)<<20 | dead<<31
    uint32_t* ua;    // assignment: type | utype<<4 | tx<<8 | ty<<16 | PRESENT/READY/PA/DEC/BAD
    int32_t* at;     // assignment issue time (UnitActionAssignment.time)
    int32_t* as;     // assignment insertion sequence number (LinkedHashMap order)
    uint32_t* bits;  // running ResourceUsage positions, indices [-W, HW+W)
    uint32_t* scell; // PO: last snapshot unit per cell (slot+1, 0 = none)
    uint32_t* vis;   // PO: 2 x H rows x ceil(W/32) words of sight-disk bitmaps (after scell)
    // PO delta rendering (poDeltaShape maps only, after vis): the previous render's sight rows [view][2][H]
    // and dead-unit chunks [view][NCW], this view's dirty chunk bits [NCW] and chunk list [HW / 4]
    uint32_t* poVis;
    uint32_t* poPend;
    uint32_t* poDirty;
    uint32_t* vis2;  // writeObsPOFast2: view 1's sight rows [2][H]
    uint16_t* poList;
    int32_t* rseq;   // ready-list scratch (64)
    uint32_t* mprev; // previous mask row sets, [2][maskWords(HW)] (delta mask writes)
    int32_t* rwc;    // reward counters [player][RC_*] of the pairs issued this step
    int32_t* hdr;    // [32]: header words 0..15 (H_*) + HX_* extras
    int16_t* hp;
    int16_t* res;
    int16_t* par;    // UnitAction.parameter (direction / NONE duration)
    uint16_t* cell;  // cell -> slot, EMPTY or WALL
    uint16_t* rslot; // ready-list scratch (64)
    uint8_t* snap;   // PO snapshot bits
    // wave-uniform scalars (only ever modified in uniform control flow)
    int time, nu, pres0, pres1, seq, deaths;
    // Cold per-game scalars live in LDS (`hdr`), not in SGPRs: the header words H_* (steps, error
    // flags, cancel counter, kind, the three java.util.Random states) plus the HX_* extras below.
    // issue index (valid while ixValid): `bits` = target cells (+W) of present MOVE/PRODUCE
    // assignments, whether any exists, per player the largest present PRODUCE cost (-1 = none) and
    // the sum of present PRODUCE costs
#ifdef MRTS_PHASE_TIMING
    uint64_t tph_;
#ifndef MRTS_SPAN_ONLY
    uint64_t phAcc[NPH];  // per-phase cycles (registers: constant indices), flushed at kernel end
#endif
#endif
#ifdef MRTS_ABLATE
    uint32_t G_AB = 0;
    DEV bool ab(int b) const { return (G_AB >> b) & 1u; }
#endif
    // lane id for the step code: threadIdx.x passed through an opaque (volatile asm) copy at the start
    // of every iteration of a multi-step launch, so that lane-derived values are recomputed per
    // iteration instead of being hoisted out of the loop and held in VGPRs across it (the loop alone
    // took k_env from 67 to 166 VGPRs: 3 waves per SIMD instead of the 4 the benchmark needs)
    // Only the multi-step kernels (iter, a compile-time constant after inlining) pay for it.
    int lidv;
    DEV int lid() const {
        if (!iter) return (int)threadIdx.x;
        __builtin_assume(lidv >= 0 && lidv < 64);
        return lidv;
    }
    DEV void freshLane() {
        if (iter) asm volatile("" : "=v"(lidv) : "0"((int)threadIdx.x));
        // multi-step kernels: the kernel argument's address made opaque again each step, so the fields
        // and addresses derived from it are re-read (SMEM) in the phase that uses them rather than held
        // across the step in spilled SGPRs (each reload a v_readlane)
        if (iter && MRTS_DYN_LAUNDER) Dp = kdynArg(true);
    }
    // the helper wave of a HELP launch (threads 64..127) runs Game methods as lanes 0..63
    DEV void helperLane() { asm volatile("" : "=v"(lidv) : "0"((int)threadIdx.x - 64)); }
    bool ixValid;
    bool anyMP;
    // the PRODUCE costs of the issue index, the batch and the candidates summed by a walk over their
    // lanes instead of whole-wave reductions (the masked-policy 16x16 instances: few PRODUCE lanes;
    // c2's uniform rows make many, where the reductions are cheaper; round 5)
    bool walk;
    uint32_t lcu, lua;     // load(): lane l's unit core / assignment words (units 0..63) as loaded
    uint32_t lfwd;         // load(): lane l's forwarded action word (KDyn.fwd_read)
    bool fwdOn;            // this game's forwarded action words are current (H_FWD == fwd_stamp - 1)
    bool fwdWritten;       // this launch wrote the forwarded action words (store() stamps H_FWD)
    uint32_t lkey, lsnap;  // PO delta: lane l's hp | resources << 16 as loaded, its previous render's snapshot byte
    bool poLds;            // the last PO render (writeObsPOFast2) left its whole record in LDS as well
    // multi-step launch: this is the launch's last iteration (the state block's internal copies — the
    // mask row sets, the forwarded words — are stored then only); the first (the terrain plane,
    // static, is written by the first observation write of the launch only).  One step: both.
    bool lastIt, firstIt;
    uint64_t killedLanes;  // cycle(): ready-list lanes whose unit was killed earlier in the cycle
    int curP;              // player whose pa is being issued
    // CloserToEnemyBase/Unit: each player's first Base before the step (x | y << 8, -1 = none) and
    // the smallest squared distance from the OTHER player's mobile units to it, before the step
    int readySlot;         // per lane: the unit slot of ready item lid() (-1 outside cycle)
    uint32_t polStep;      // the fused policy's Philox step (D.pol_step, + 1 per iteration of a multi-step launch)
    uint32_t uniStep;      // the fused uniform policy's step (D.uni_step, likewise)
    // helper-wave launch (k_env HELP): this iteration's uniform rows, drawn by the helper wave,
    // packed (packFwd) per [player slot][cell]; null = draw them here (fetchRow)
    const uint32_t* helpRows = nullptr;
    // helper-wave launch, partially observable (k_env HELP && FPO): where writeMasksLanes leaves this
    // step's mask records, policy rows and vacated cells for the helper to store (null = store them here)
    uint32_t* recOut = nullptr;
    int maxProd0, maxProd1, sumProd0, sumProd1;

    // h, w, hw, cap: the map dimensions — compile-time constants in a specialised kernel (every LDS
    // array offset then folds to an immediate), else the kernel arguments
    DEV Game(const KStatic& p, const KDyn& d /* k_env's argument D; other fields read through kdynArg */, int32_t* stb, int stw, uint8_t* smem, int h, int w, int hw, int cap, bool partial,
             int k, int nt, int r, bool iterating = false, int game = -1, bool walk = false)
        : P(p), Dp(kdynArg(false)), U(*(const DevUtt*)smem), g(game >= 0 ? game : (int)blockIdx.x), H(h), W(w), HW(hw), CAP(cap), K(k), NT(nt), R(r),
          po(partial), iter(iterating), stBase(stb), stWords(stw), walk(walk) {
        uint8_t* q = smem + UTT_LDS;  // the unit-type table copy comes first (see copyUtt)
        uc = (uint32_t*)q; q += 4 * CAP;
        ua = (uint32_t*)q; q += 4 * CAP;
        at = (int32_t*)q; q += 4 * CAP;
        as = (int32_t*)q; q += 4 * CAP;
        bits = (uint32_t*)q; q += 4 * ((HW + 2 * W + 31) / 32);
        rseq = (int32_t*)q; q += 4 * 64;
        mprev = (uint32_t*)q; q += 8 * maskWords(HW);
        rwc = (int32_t*)q; q += 4 * 16;
        hdr = (int32_t*)q; q += 4 * 32;
        hp = (int16_t*)q; q += 2 * CAP;
        res = (int16_t*)q; q += 2 * CAP;
        par = (int16_t*)q; q += 2 * CAP;
        cell = (uint16_t*)q; q += 2 * HW;
        rslot = (uint16_t*)q; q += 2 * 64;
        snap = (uint8_t*)q; q += (CAP + 3) & ~3;
        scell = (uint32_t*)q;  // PO only, last: the offsets above do not depend on it
        vis = scell + HW;
        poVis = vis + 2 * H * ((W + 31) / 32);
        poPend = poVis + 4 * H;
        poDirty = poPend + 2 * poChunkWords(HW);  // [view][dirty, next pending bits] (view 1: writeObsPOFast2)
        vis2 = poDirty + 4 * poChunkWords(HW);
        poList = (uint16_t*)(vis2 + 2 * H);  // up to 2 x HW / 4 entries
        ixValid = false;
        fwdOn = false;
        fwdWritten = false;
        lfwd = 0;
        poLds = false;
        lastIt = true;
        firstIt = true;
        polStep = d.pol_step;
        uniStep = d.uni_step;
        freshLane();
    }
    // HX_*: snapshot sequence limits (PO), CloserToEnemy* base positions / old minimum distances
    enum { HX_SNAP = 16, HX_BASE = 18, HX_OLDSQ = 20, HX_POVALID = 22 };
    DEV int hget(int i) const { return uni(hdr[i]); }
    DEV void hset(int i, int v) const {
        if (lid() == 0) hdr[i] = v;
    }
    DEV void addErr(uint32_t bits) const {
        if (lid() == 0) hdr[H_ERR] |= (int32_t)bits;
    }
    DEV uint32_t errFlags() const { return (uint32_t)hget(H_ERR); }
    DEV JRand rngLoad(int i) const { return JRand{rng_of(hget(i), hget(i + 1))}; }
    DEV void rngStore(int i, const JRand& r) const {
        hset(i, (int)(uint32_t)r.s);
        hset(i + 1, (int)(uint32_t)(r.s >> 32));
    }
    DEV int pres(int p) const { return p == 0 ? pres0 : pres1; }
    DEV void addPres(int p, int v) {
        if (p == 0) pres0 += v;
        else pres1 += v;
    }
    DEV bool inb(int x, int y) const { return x >= 0 && x < W && y >= 0 && y < H; }
    DEV const int32_t* tmpl() const { return P.tmpl + P.tmpl_off[g]; }
    DEV int32_t* st() const { return stBase + (size_t)g * stWords; }

    // UnitAction.ETA (rts/UnitAction.java:307-329)
    DEV int eta(int t, int prm, int ut, int unitType) const {
        switch (t) {
            case T_NONE: return prm;
            case T_MOVE: return U.moveT[unitType];
            case T_ATTACK: return U.attackT[unitType];
            case T_HARVEST: return U.harvestT[unitType];
            case T_RETURN: return U.moveT[unitType];  // RETURN lasts moveTime (:321-322)
            case T_PRODUCE: return U.produceT[ut];
        }
        return 0;
    }
    // eta without the per-type branches (lane-varying t: the switch ran each case under its own exec mask):
    // produceT, moveT, attackT, harvestT are consecutive MAX_TYPES arrays of DevUtt, so the duration is one
    // LDS read at [array(t)][t == PRODUCE ? ut : unitType]; NONE keeps its parameter, unknown types 0
    DEV int etaFlat(int t, int prm, int ut, int unitType) const {
        static_assert(offsetof(DevUtt, moveT) == offsetof(DevUtt, produceT) + 4 * MAX_TYPES &&
                          offsetof(DevUtt, attackT) == offsetof(DevUtt, produceT) + 8 * MAX_TYPES &&
                          offsetof(DevUtt, harvestT) == offsetof(DevUtt, produceT) + 12 * MAX_TYPES,
                      "DevUtt duration arrays");
        // array per type (4 bits each): MOVE moveT (1), HARVEST harvestT (3), RETURN moveT (1), PRODUCE produceT (0),
        // ATTACK attackT (2)
        const int arr = (int)((0x201310u >> (4 * (t & 7))) & 15u);
        const int v = U.produceT[arr * MAX_TYPES + (t == T_PRODUCE ? ut : unitType)];
        return t == T_NONE ? prm : (t <= T_ATTACK ? v : 0);
    }
    DEV int etaSlot(int s) const {
        const uint32_t a = ua[s];
        return eta(ua_type(a), par[s], ua_ut(a), utyp(uc[s]));
    }

    // ------------------------------------------------------------------ state load / store
    DEV void setTerrainWord(int w, uint32_t v) {  // 4 terrain bytes -> cells 4w..4w+3
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (4 * w + b < HW) cell[4 * w + b] = ((v >> (8 * b)) & 0xFFu) ? WALL : EMPTY;
    }
    DEV void initCells() {  // terrain walls from the map template
        const int32_t* t = tmpl() + T_TERR;
        for (int w = lid(); w < (HW + 3) / 4; w += 64) setTerrainWord(w, (uint32_t)t[w]);
        wsync();
    }
    DEV void copyUtt() {  // the LDS copy of the unit-type table, when load() does not fetch it
        const int32_t* ug = (const int32_t*)&P.utt;
        int32_t* ul = (int32_t*)&U;
        for (int i = lid(); i < UTT_WORDS; i += 64) ul[i] = ug[i];
        wsync();
    }
    DEV void storeTerrain() {  // the template's terrain words into the state block (at reset)
        const int32_t* t = tmpl() + T_TERR;
        int32_t* d = st() + stateTerrOff(CAP, HW);
        for (int w = lid(); w < (HW + 3) / 4; w += 64) d[w] = t[w];
    }
    DEV uint32_t* prevG() const { return (uint32_t*)(st() + H_WORDS + N_ARRAYS * CAP); }
    DEV void loadPrev() {  // previous mask row sets (delta mask writes), when not fetched by load()
        const uint32_t* pg = prevG();
        for (int i = lid(); i < 2 * maskWords(HW); i += 64) mprev[i] = pg[i];
        wsync();
    }
    DEV void placeUnits() {
        for (int i = lid(); i < nu; i += 64) {
            const uint32_t c = uc[i];
            if (!(c & UC_DEAD)) cell[uy(c) * W + ux(c)] = (uint16_t)i;
        }
        wsync();
    }
    DEV void loadHeader(const int32_t* s) { loadHeader(lid() < H_WORDS ? s[lid()] : 0); }
    DEV void loadHeader(int hv) {  // hv = header word lid() (lanes < H_WORDS)
        time = rl(hv, H_TIME);
        nu = rl(hv, H_NU);
        pres0 = rl(hv, H_RES0);
        pres1 = rl(hv, H_RES1);
        seq = rl(hv, H_SEQ);
        deaths = 0;
        const int l = lid();
        if (l < H_WORDS) hdr[l] = hv;
        else if (l < 32) hdr[l] = (l >= HX_BASE && l < HX_BASE + 2) ? -1 : (l >= HX_OLDSQ && l < HX_OLDSQ + 2) ? INF : 0;
    }
    // One global round trip: header, unit rows 0..63 (speculative — CAP >= 64), the terrain and the
    // previous mask row sets are all in flight before the first wait.
    DEV void load(bool wantPrev) {
        const int32_t* s = st();
        const int32_t* arr = s + H_WORDS;
        const int32_t* terr = s + stateTerrOff(CAP, HW);
        const int l = lid();
        const int TW = (HW + 3) / 4, PW = 2 * maskWords(HW);
        const int hv = l < H_WORDS ? s[l] : 0;
        const int32_t* ug = (const int32_t*)&P.utt;
        const int32_t u0 = ug[l], u1 = l + 64 < UTT_WORDS ? ug[l + 64] : 0, u2 = l + 128 < UTT_WORDS ? ug[l + 128] : 0;
        int32_t r[N_ARRAYS];
#pragma unroll
        for (int a = 0; a < N_ARRAYS; a++) r[a] = arr[a * CAP + l];
        const uint32_t tw = l < TW ? (uint32_t)terr[l] : 0u;
        const uint32_t pv = (wantPrev && l < PW) ? (uint32_t)arr[N_ARRAYS * CAP + l] : 0u;
        // forwarded action words (speculative: used only if H_FWD, in this same round, matches)
        const uint32_t fw = D.fwd_read ? (uint32_t)s[stateFwdOff(CAP, HW) + l] : 0u;
        // PO delta: the previous render's record, in the same memory round
        const bool poRec = po && D.obs_delta && D.po_prev && poDeltaShape(H, W);
        const int32_t* pr = poRec ? D.po_prev + (size_t)g * D.po_words : nullptr;
        const int NCW = poChunkWords(HW), SW = poSnapWords(CAP);
        int32_t prv0 = 0, prsb = 0, prvv = 0, prv2 = 0, prpd = 0;
        if (poRec) {
            prv0 = pr[0];
            prsb = pr[1 + (l >> 2)];
            prvv = l < 4 * H ? pr[1 + SW + l] : 0;
            prv2 = l + 64 < 4 * H ? pr[1 + SW + l + 64] : 0;
            prpd = l < 2 * NCW ? pr[1 + SW + 4 * H + l] : 0;
        }
        loadHeader(hv);
        MPHASE(20);
        lcu = (uint32_t)r[A_UC];
        lua = (uint32_t)r[A_UA];
        lfwd = fw;
        fwdOn = D.fwd_read && (uint32_t)rl(hv, H_FWD) == D.fwd_stamp - 1u;
        if (poRec) {
            lkey = (uint32_t)(uint16_t)r[A_HP] | ((uint32_t)(uint16_t)r[A_RES] << 16);
            lsnap = ((uint32_t)prsb >> (8 * (l & 3))) & 0xFFu;
            if (l < 4 * H) poVis[l] = (uint32_t)prvv;
            if (l + 64 < 4 * H) poVis[l + 64] = (uint32_t)prv2;
            if (l < 2 * NCW) poPend[l] = (uint32_t)prpd;
            if (l == 0) hdr[HX_POVALID] = prv0;
        }
        {
            int32_t* ul = (int32_t*)&U;
            ul[l] = u0;
            if (l + 64 < UTT_WORDS) ul[l + 64] = u1;
            if (l + 128 < UTT_WORDS) ul[l + 128] = u2;
        }
        if (l < nu) {
            uc[l] = (uint32_t)r[A_UC];
            hp[l] = (int16_t)r[A_HP];
            res[l] = (int16_t)r[A_RES];
            ua[l] = (uint32_t)r[A_UA];
            par[l] = (int16_t)r[A_PAR];
            at[l] = r[A_AT];
            as[l] = r[A_AS];
        }
        for (int i = l + 64; i < nu; i += 64) {
            uc[i] = (uint32_t)arr[A_UC * CAP + i];
            hp[i] = (int16_t)arr[A_HP * CAP + i];
            res[i] = (int16_t)arr[A_RES * CAP + i];
            ua[i] = (uint32_t)arr[A_UA * CAP + i];
            par[i] = (int16_t)arr[A_PAR * CAP + i];
            at[i] = arr[A_AT * CAP + i];
            as[i] = arr[A_AS * CAP + i];
        }
        if (l < TW) setTerrainWord(l, tw);
        for (int w = l + 64; w < TW; w += 64) setTerrainWord(w, (uint32_t)terr[w]);
        if (wantPrev) {
            if (l < PW) mprev[l] = pv;
            for (int i = l + 64; i < PW; i += 64) mprev[i] = prevG()[i];
        }
        wsync();
        MPHASE(21);
        placeUnits();
    }
    DEV void store() {
        int32_t* s = st();
        const int l = lid();
        int hv = l < H_WORDS ? hdr[l] : 0;
        switch (l) {
            case H_TIME: hv = time; break;
            case H_NU: hv = nu; break;
            case H_RES0: hv = pres0; break;
            case H_RES1: hv = pres1; break;
            case H_SEQ: hv = seq; break;
            case H_FWD: hv = fwdWritten ? (int)D.fwd_stamp : 0; break;
        }
        if (l < H_WORDS) st1<WT_STATE>(s + l, hv);
        int32_t* arr = s + H_WORDS;
        for (int i = l; i < nu; i += 64) {
            st1<WT_STATE>(arr + A_UC * CAP + i, (int32_t)uc[i]);
            st1<WT_STATE>(arr + A_HP * CAP + i, hp[i]);
            st1<WT_STATE>(arr + A_RES * CAP + i, res[i]);
            st1<WT_STATE>(arr + A_UA * CAP + i, (int32_t)ua[i]);
            st1<WT_STATE>(arr + A_PAR * CAP + i, par[i]);
            st1<WT_STATE>(arr + A_AT * CAP + i, at[i]);
            st1<WT_STATE>(arr + A_AS * CAP + i, as[i]);
        }
    }
    // Between two iterations of a multi-step launch (KDyn.n_iter): the state stays in LDS, so the
    // registers load() would set are re-derived from it — lane l's unit words, the forwarded action
    // word the previous iteration sampled (lfwd, kept in its register), the per-step header extras.
    DEV void nextStep() {
        freshLane();
        const int l = lid();
        wsync();
        lcu = uc[l];  // l < 64 <= CAP; selfPlayFast ignores lanes >= nu
        lua = ua[l];
        fwdOn = fwdWritten;
        // without forwarded words (more than 64 units) the next decode reads the rows the previous
        // iteration's policy stored to the action tensor, and a PO render that kept no LDS copy of
        // its record makes the next one re-read it: this wave's own plain stores, read back on the
        // same CU — a workgroup-scope fence (the stores' vmcnt drain, which also waits for the
        // iteration's observation stores: only when needed — c5 paid ~6 us per step draining them
        // every step; an agent-scope __threadfence would also write back the XCD's L2: 4x slower)
        const bool poRec = po && D.obs_delta && D.po_prev && poDeltaShape(H, W);
        const bool poReload = poRec && !poLds;  // a render that kept no LDS copy: re-read the record
        if (poReload || (!fwdWritten && !D.uni_actions)) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        fwdWritten = false;
        poLds = false;
        hset(H_NU, nu);  // "the loaded unit count" of this iteration (PO delta render)
        if (poRec && !poReload) {  // the previous render's record from its LDS copies
            lkey = (uint32_t)(uint16_t)hp[l] | ((uint32_t)(uint16_t)res[l] << 16);
            lsnap = snap[l];  // after the compaction = the record's snapshot bytes; before clearSnap
        } else if (poReload) {  // the previous render's record, as load() takes it
            const int32_t* pr = D.po_prev + (size_t)g * D.po_words;
            const int NCW = poChunkWords(HW), SW = poSnapWords(CAP);
            const int32_t prv0 = pr[0], prsb = pr[1 + (l >> 2)];
            const int32_t prvv = l < 4 * H ? pr[1 + SW + l] : 0, prv2 = l + 64 < 4 * H ? pr[1 + SW + l + 64] : 0;
            const int32_t prpd = l < 2 * NCW ? pr[1 + SW + 4 * H + l] : 0;
            lkey = (uint32_t)(uint16_t)hp[l] | ((uint32_t)(uint16_t)res[l] << 16);
            lsnap = ((uint32_t)prsb >> (8 * (l & 3))) & 0xFFu;
            if (l < 4 * H) poVis[l] = (uint32_t)prvv;
            if (l + 64 < 4 * H) poVis[l + 64] = (uint32_t)prv2;
            if (l < 2 * NCW) poPend[l] = (uint32_t)prpd;
            if (l == 0) hdr[HX_POVALID] = prv0;
        }
        ixValid = false;
        deaths = 0;
        polStep++;
        uniStep++;
        // (HX_POVALID stays: it is the PO render record's "views rendered", set by poRecordSnaps)
        if (l >= H_WORDS && l < 32 && l != HX_POVALID)
            hdr[l] = (l >= HX_BASE && l < HX_BASE + 2) ? -1 : (l >= HX_OLDSQ && l < HX_OLDSQ + 2) ? INF : 0;
        wsync();
    }
    // new GameState(PhysicalGameState.load(map)) — JNIGridnetClient.reset (tests/JNIGridnetClient.java:239-241).
    // envSteps is NOT part of it: VecClient.reset (tests/JNIGridnetVecClient.java:179-211) never touches
    // envSteps[]; only the auto-reset path zeroes it (:229,264-265,285).
    DEV void resetFromTemplate() {
        const int32_t* t = tmpl();
        const int nu_t = t[T_NU];
        time = 0;
        seq = 0;
        deaths = 0;
        pres0 = t[T_RES0];
        pres1 = t[T_RES1];
        nu = nu_t;
        const int32_t* tu = t + tmplUnits(HW);
        for (int i = lid(); i < nu_t; i += 64) {
            uc[i] = (uint32_t)tu[i];
            hp[i] = (int16_t)tu[nu_t + i];
            res[i] = (int16_t)tu[2 * nu_t + i];
            ua[i] = 0;
            par[i] = -1;
            at[i] = 0;
            as[i] = 0;
        }
        wsync();
        for (int c = lid(); c < HW; c += 64)
            if (cell[c] != WALL) cell[c] = EMPTY;
        wsync();
        placeUnits();
    }

    // ------------------------------------------------------------------ row fetch + decode
    // UnitAction.fromVectorAction (rts/UnitAction.java:675-709) for every idle unit of the external
    // player(s), lane-parallel, in ONE round of global loads: a pure function of (row, unit).  The
    // decoded action is parked in the unit's empty assignment fields with UA_DEC.
    // JNIGridnetClientSelfPlay.gameStep's two issueSafe passes (tests/JNIGridnetClientSelfPlay.java:
    // 159-189) for a game whose units fit one wave, under full observability: predecode, then per
    // player the acceptance chain (PlayerAction.fromVectorAction), issueSafe of the accepted rows in
    // cell order and fillWithNones(gs, p, 1) in list order — the same sequence as predecode + decode +
    // issuePlayer, with each lane's own unit fields (load()'s registers) instead of LDS re-reads.
    // Between steps no unit is dead; decoded rows are never parked in LDS (every idle unit's
    // assignment is written by its issue or its fill).
    // Partially observable games too (round 5; all units in one wave, snapBothOk): Java decodes each player's
    // rows against that player's view (JNIGridnetClientSelfPlay.java:159-189, PlayerAction.fromVectorAction
    // on the PartiallyObservableGameState), which holds every own unit (sight covers its own cell) with the
    // assignments it has when the view is made — so the decode, fillWithNones and issueSafe are the full
    // state's; only the pa's base reservations come from the view (the assignments of the units in it,
    // baseReservations(p)), and the views' snapshots are taken in order: both memberships + view 0's
    // assignments before player 0 issues (snapshotBoth, or the helper wave's bytes: snapTaken), view 1's
    // assignments after (snapshotActions(1)).  The generic predecode + decode path did the same, slower.
    DEV void selfPlayFast(const int32_t* rows0, const int32_t* rows1, int s0, bool snapTaken = false) {
        const int l = lid();
        const uint32_t cu = lcu;
        const int pl = l < nu ? uplay(cu) : -1;
        const bool idle = pl >= 0 && !(lua & UA_PRESENT);
        int32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
        if (fwdOn) {
            // the previous launch's fused policy sampled this unit's row (the values it wrote to the
            // action tensor at this cell) and forwarded it in the state block (decoded below)
            if (!MRTS_DECODE_FWD && idle) unpackFwd(lfwd, a);
        } else if (idle) {
            fetchRow(pl == 0 ? rows0 : rows1, s0 + pl, uy(cu) * W + ux(cu), a);
        }
        const bool useIx = !po && (HW + 2 * W + 31) / 32 <= 64;  // PO: the view's reservations (baseReservations)
        if (useIx) buildIndex();  // while the rows are in flight
        // PO (round 6): each view's base reservations go to a bitmap of their own in the top words of `scell` (free
        // during the issue: the general render's scratch map is done with; a helper wave's packs and cell map end at
        // word 896 of 32x32's 1,024), so the issue index in `bits` stays valid across both players' issues instead of
        // being rebuilt after each view's acceptance chain
        const int NBv = (HW + 2 * W + 31) / 32;
        uint32_t* const vres = (MRTS_PO_VRES && po && NBv <= 64 && HW - NBv >= (HW == 1024 ? 896 : 0)) ? scell + (HW - NBv) : nullptr;
#ifdef MRTS_ABLATE
        if (useIx && ab(AB_INDEX)) buildIndex();
#endif
        MPHASE(22);
        int t = 0, pr = -1, ut = 0, tx = 0, ty = 0;
        bool bad = false;
#ifdef MRTS_ABLATE
        if (ab(AB_DECODE) && idle) {
            int32_t b2[7];
            for (int k = 0; k < 7; k++) b2[k] = launder(a[k]);
            int t2 = 0, pr2 = -1, ut2 = 0, tx2 = 0, ty2 = 0;
            const bool bad2 = decodeFields(launder(cu), b2, t2, pr2, ut2, tx2, ty2);
            keepv(t2 + pr2 + ut2 + tx2 + ty2 + (int)bad2);
        }
#endif
        if (idle) bad = (MRTS_DECODE_FWD && fwdOn) ? decodeFwd(cu, lfwd, t, pr, ut, tx, ty) : decodeFields(cu, a, t, pr, ut, tx, ty);
        if (ballot(bad)) addErr(E_PRODUCE_TYPE);
        const uint32_t adec = pack_ua(t, ut, tx, ty);
        const int c = uy(cu) * W + ux(cu);
        MPHASE(1);
        for (int p = 0; p < 2; p++) {
            if (po) {  // the views, in Java's order (see above)
                if (p == 0) {
                    if (!snapTaken) snapshotBoth();
                } else {
                    snapshotActions(1);
                }
            }
            int run0, run1;
            if (useIx) {
                if (!ixValid) buildIndex();
                run0 = sumProd0;
                run1 = sumProd1;
            } else {
                baseReservations(p, run0, run1, vres);
            }
            curP = p;
            const bool mine = idle && pl == p;
            const bool cand = mine && !bad;
            const uint64_t m = ballot(cand);
            bool isPA = false;
            if (m) {
                const int rank = cellRank(m, cand, c);
#ifdef MRTS_ABLATE
                if (ab(AB_RANK)) keepv(cellRank(m, cand, launder(c)));
                if (ab(AB_ACCEPT)) {
                    int r0 = run0, r1 = run1, ir = 0;
                    const uint64_t a2 = acceptChain(p, r0, r1, cand, launder(rank), __popcll(m), launder(t), launder(pr),
                                                    launder(c), launder(adec), true, ir);
                    keepv(ir + (int)a2 + r0 + r1);
                }
#endif
                MPHASE(23);
                int irank = 0;
                const uint64_t acc = acceptChain(p, run0, run1, cand, rank, __popcll(m), t, pr, c, adec, useIx || vres, irank, vres);
                MPHASE(2);
                isPA = (acc >> l) & 1ull;
                int tt = 0, prm = 0, ttx = 0, tty = 0, tut = 0;
                if (isPA) {
                    tt = t;
                    prm = pr;
                    ttx = tx;
                    tty = ty;
                    tut = ut;
#ifdef MRTS_ABLATE
                    if (ab(AB_LEGAL)) {
                        int a1 = launder(t), a2 = launder(pr), a3 = launder(tx), a4 = launder(ty), a5 = launder(ut);
                        legality(l, launder(cu), a1, a2, a3, a4, a5);
                        keepv(a1 + a2 + a3 + a4 + a5);
                    }
#endif
                    // A forwarded row was sampled by the fused policy from this unit's mask record, which
                    // the previous step wrote from this same state (no cycle in between): its type bit
                    // and parameter bits are members of getUnitActions' list (a PRODUCE's free
                    // directions x affordable types is a full product), and issuing the other player's
                    // pairs changes nothing the test reads (positions, hp, resources move only in
                    // cycle) — so issueSafe's legality test returns the row unchanged and is skipped.
                    // Any other row (the caller's tensor, the uniform policy) is tested.
                    if (!fwdOn) legality(l, cu, tt, prm, ttx, tty, tut);
                }
                wsync();
                MPHASE(24);
                if (acc) issueBatch(isPA, irank, __popcll(acc), l, tt, prm, ttx, tty, tut, false, &cu, nullptr, MRTS_POS_CHECKED);
            }
            // fillWithNones(gs, p, 1): p's idle units left without an action, list order
            const bool fill = mine && !isPA;
            const uint64_t mf = ballot(fill);
            if (fill) {
                ua[l] = pack_ua(T_NONE, 0, 0, 0) | UA_PRESENT;
                par[l] = 1;
                at[l] = time;
                as[l] = seq + lanes_below(mf);
            }
            seq += __popcll(mf);
            wsync();
            MPHASE(3);
        }
    }
    // Row of cell c of slot `slot` (rows = that slot's rows): the action tensor's, or, in a fused
    // uniform-policy step (KDyn.uni_actions), the Philox row the launch also writes there
    // (writeUniformRows) — drawn again in registers instead of read back.
    DEV void fetchRow(const int32_t* rows, int slot, int c, int32_t a[7]) const {
        if (helpRows) {  // the helper wave drew this step's rows (self-play: slot & 1 = player)
            unpackFwd(helpRows[(slot & 1) * HW + c], a);
            return;
        }
        if (D.uni_actions) {
            uniformRow(D.uni_seed, uniStep, D.uni_slot_base + (uint32_t)slot, c, NT, K - 23 - NT, a);
            return;
        }
        const int32_t* r = rows + (size_t)c * 7;
#pragma unroll
        for (int k = 0; k < 7; k++) a[k] = r[k];
    }
    // the fused uniform policy's output: every row of this game's slots, as k_policy_uniform writes them
    DEV void writeUniformRows(int slot0, int nslots) const {
        for (int i = 0; i < nslots; i++)
            for (int c = lid(); c < HW; c += 64) {
                int32_t a[7];
                uniformRow(D.uni_seed, uniStep, D.uni_slot_base + (uint32_t)(slot0 + i), c, NT, K - 23 - NT, a);
                int32_t* dst = D.uni_actions + ((size_t)(slot0 + i) * HW + c) * 7;
                st4u<false>(dst, a[0], a[1], a[2], a[3]);
                st3u<false>(dst + 4, a[4], a[5], a[6]);
            }
    }
    DEV void predecode(const int32_t* rows0, const int32_t* rows1, int only, int s0, int s1) {
        bool bad_any = false;
        const int l = lid();
        // units 0..63: rows requested first, the issue index (LDS only) is built while they are in
        // flight, then decoded
        int32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
        bool act = false;
        if (l < nu) {
            const uint32_t cu = uc[l];
            const int pl = uplay(cu);
            act = !(pl < 0 || (ua[l] & UA_PRESENT) || (only >= 0 && pl != only));
            if (act) {
                // units 0..63 of a self-play game: the fused policy's forwarded word when current
                // (as selfPlayFast), else the action tensor
                if (fwdOn) unpackFwd(lfwd, a);
                else fetchRow(pl == 0 ? rows0 : rows1, pl == 0 ? s0 : s1, uy(cu) * W + ux(cu), a);
            }
        }
        if (!po && (HW + 2 * W + 31) / 32 <= 64) buildIndex();
        if (act) bad_any |= decodeRow(l, a);
        for (int o = l + 64; o < nu; o += 64) {
            const uint32_t cu = uc[o];
            const int pl = uplay(cu);
            if (pl < 0 || (ua[o] & UA_PRESENT) || (only >= 0 && pl != only)) continue;
            int32_t b[7];
            fetchRow(pl == 0 ? rows0 : rows1, pl == 0 ? s0 : s1, uy(cu) * W + ux(cu), b);
            bad_any |= decodeRow(o, b);
        }
        if (ballot(bad_any)) addErr(E_PRODUCE_TYPE);
        wsync();
    }
    // UnitAction.fromVectorAction of row a for unit o; returns "produce type out of range"
    DEV bool decodeRow(int o, const int32_t a[7]) {
        int t, pr, ut, tx, ty;
        const bool bad = decodeFields(uc[o], a, t, pr, ut, tx, ty);
        ua[o] = pack_ua(t, ut, tx, ty) | UA_DEC | (bad ? UA_BAD : 0u);
        par[o] = (int16_t)pr;
        return bad;
    }
    // UnitAction.fromVectorAction (rts/UnitAction.java:675-709) of row components a[0..6] for a unit
    // with core word cu
    // Branch-free (selects only): the lanes of one wave hold rows of every type, and a divergent switch
    // runs each present case's instructions for the whole wave.
    // decodeFields(cu, unpackFwd(w)) straight from a forwarded action word: the direction field picked by
    // the type with one bit-field extract instead of unpacking all seven values and selecting among them
    DEV bool decodeFwd(uint32_t cu, uint32_t w, int& t, int& pr, int& ut, int& tx, int& ty) const {
        const int ctr = R / 2;
        const int x = ux(cu), y = uy(cu);
        const int a0 = (int)(w & 7u);
        t = a0 <= 5 ? a0 : ACT_INVALID;
        const bool dirT = t >= T_MOVE && t <= T_PRODUCE;
        const int d = (int)__builtin_amdgcn_ubfe(w, 3u * (uint32_t)(dirT ? t : T_PRODUCE), 3u) - 1;  // a[t] (a[4] otherwise)
        pr = dirT ? clampdir(d) : -1;
        const bool prod = t == T_PRODUCE;
        const int a5 = (int)((w >> 15) & 15u) - 1, a6 = (int)((w >> 19) & 127u) - 1;
        const bool badType = a5 < 0 || a5 >= NT;
        ut = (prod && !badType) ? a5 : 0;
        const int ax = x + (a6 % R - ctr), ay = y + (a6 / R - ctr);
        const bool att = t == T_ATTACK, on = inb(ax, ay);
        tx = att ? (on ? ax : 255) : 0;
        ty = att ? (on ? ay : 255) : 0;
        return prod && badType;
    }
    DEV bool decodeFields(uint32_t cu, const int32_t a[7], int& t, int& pr, int& ut, int& tx, int& ty) const {
        const int ctr = R / 2;
        const int x = ux(cu), y = uy(cu);
        t = (a[0] >= 0 && a[0] <= 5) ? a[0] : ACT_INVALID;
        // MOVE / HARVEST / RETURN / PRODUCE: the direction of that type's component
        const int d = t == T_MOVE ? a[1] : t == T_HARVEST ? a[2] : t == T_RETURN ? a[3] : a[4];
        pr = (t >= T_MOVE && t <= T_PRODUCE) ? clampdir(d) : -1;
        // PRODUCE: utt.getUnitType(int) throws for a type outside the table (:697)
        const bool prod = t == T_PRODUCE;
        const bool badType = a[5] < 0 || a[5] >= NT;
        ut = (prod && !badType) ? a[5] : 0;
        // ATTACK: the target cell of the window index, off-map -> never legal
        const int ax = x + (a[6] % R - ctr), ay = y + (a[6] / R - ctr);
        const bool att = t == T_ATTACK, on = inb(ax, ay);
        tx = att ? (on ? ax : 255) : 0;
        ty = att ? (on ? ay : 255) : 0;
        return prod && badType;
    }

    // ------------------------------------------------------------------ Java row layout
    // PlayerAction.fromVectorAction over Java rows [pos, 7 comps] in list order (rts/PlayerAction.java:
    // 384-417): a row counts iff an own unit with no assignment stands at (pos % W, pos / W); rows may
    // name a unit twice (both can be accepted).  Accepted pairs go, in order, to the game's scratch.
    // Returns the pair count.
    DEV int rowsDecode(int p, const int32_t* rows) {
        int run0, run1;
        baseReservations(p, run0, run1);
        const int l = lid();
        uint32_t* pairs = D.pairs + (size_t)g * D.n_rows * 2;
        int npairs = 0;
        bool badAny = false;
        for (int r0 = 0; r0 < D.n_rows; r0 += 64) {
            const int r = r0 + l;
            int32_t a[8] = {-1, 0, 0, 0, 0, 0, 0, 0};
            if (r < D.n_rows)
#pragma unroll
                for (int k = 0; k < 8; k++) a[k] = rows[(size_t)r * 8 + k];
            const int pos = a[0];
            bool cand = false;
            int s = 0, t = 0, pr = 0, ut = 0, tx = 0, ty = 0;
            uint32_t cu = 0;
            if (pos >= 0 && pos < HW) {
                s = cell[pos];
                if (s < CAP) {
                    cu = uc[s];
                    cand = uplay(cu) == p && !(ua[s] & UA_PRESENT);
                }
            }
            if (cand) {
                const bool bad = decodeFields(cu, a + 1, t, pr, ut, tx, ty);
                badAny |= bad;
                cand = !bad;  // Java throws here (UnitAction.java:697): reported as E_PRODUCE_TYPE
            }
            const uint64_t m = ballot(cand);
            if (m == 0) continue;
            const uint32_t av = pack_ua(t, ut, 0, 0);
            int irank = 0;
            const uint64_t acc = acceptChain(p, run0, run1, cand, cand ? lanes_below(m) : -1, __popcll(m), t, pr, pos, av, false, irank);
            if ((acc >> l) & 1ull) {
                const int idx = npairs + lanes_below(acc);
                pairs[(size_t)idx * 2] = (uint32_t)s | ((uint32_t)t << 16) | ((uint32_t)ut << 20);
                pairs[(size_t)idx * 2 + 1] = (uint32_t)(uint16_t)pr | ((uint32_t)tx << 16) | ((uint32_t)ty << 24);
            }
            npairs += __popcll(acc);
        }
        if (ballot(badAny)) addErr(E_PRODUCE_TYPE);
        __threadfence();  // the pairs are read back (by other lanes) in rowsIssue
        return npairs;
    }
    // issueSafe(pa) for the pairs of rowsDecode + fillWithNones(gs, p, fillDur) (PlayerAction.java:217-235)
    DEV void rowsIssue(int p, int npairs, int fillDur) {
        curP = p;
        const uint32_t* pairs = D.pairs + (size_t)g * D.n_rows * 2;
        for (int b0 = 0; b0 < npairs; b0 += 64) {
            const int k = b0 + lid();
            const bool act = k < npairs;
            int s = 0, t = 0, prm = 0, tx = 0, ty = 0, ut = 0;
            if (act) {
                const uint32_t w0 = pairs[(size_t)k * 2], w1 = pairs[(size_t)k * 2 + 1];
                s = (int)(w0 & 0xFFFFu);
                t = (int)((w0 >> 16) & 0xFu);
                ut = (int)((w0 >> 20) & 0xFu);
                prm = (int)(int16_t)(w1 & 0xFFFFu);
                tx = (int)((w1 >> 16) & 0xFFu);
                ty = (int)(w1 >> 24);
                legality(s, t, prm, tx, ty, ut);
            }
            wsync();
            issueBatch(act, lid(), min(64, npairs - b0), s, t, prm, tx, ty, ut, true);
        }
        issueFills(p, fillDur);
    }

    // ------------------------------------------------------------------ trace replay (MODE_TRACE)
    // issueSafe(pa) (rts/GameState.java:338-408) of player p's pairs of a trace entry, as
    // TestTracesIntegrity.testTrace builds them (test/microrts/TestTracesIntegrity.java:101-121): rows
    // [player, x, y, type, parameter, target x, target y, unit type], the player's rows in the given
    // order.  Each action's legality is judged on the trace's own Unit object, whose fields equal those
    // of the state's unit at (x, y) whenever the replay is in sync; that unit is then the one issued —
    // the first unit at (x, y) in list order (GameState.java:356-382; one unit per cell).  No fillWithNones.
    // Returns issue()'s value: a pair was put with a type other than NONE.
    DEV bool traceIssue(int p, const int32_t* rows, int n, uint32_t& flags) {
        curP = p;
        bool put = false;
        bool missing = false;
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int r = r0 + lid();
            int32_t a[8] = {-1, 0, 0, 0, 0, 0, 0, 0};
            if (r < n)
#pragma unroll
                for (int k = 0; k < 8; k++) a[k] = rows[(size_t)r * 8 + k];
            bool act = a[0] == p;
            int s = 0;
            if (act) {
                s = inb(a[1], a[2]) ? (int)cell[a[2] * W + a[1]] : EMPTY;
                if (s >= CAP) {  // no unit there: Java prints "Inconsistent order" and issues the trace's unit
                    missing = true;
                    act = false;
                }
            }
            int t = a[3], prm = a[4], tx = 0, ty = 0, ut = 0;
            if (act) {
                if (t < T_NONE || t > T_ATTACK) t = ACT_INVALID;  // never in getUnitActions: NONE(0)
                const bool dir = t >= T_MOVE && t <= T_PRODUCE;
                if (dir && (prm < 0 || prm > 3)) prm = 4;  // not a direction: never legal
                if (t == T_PRODUCE) ut = a[7];              // the host checked 0 <= ut < ntypes
                if (t == T_ATTACK) {
                    const bool on = inb(a[5], a[6]);
                    tx = on ? a[5] : 255;
                    ty = on ? a[6] : 255;
                }
                legality(s, t, prm, tx, ty, ut);
            }
            const uint64_t m = ballot(act);
            wsync();
            if (m) issueBatch(act, act ? lanes_below(m) : 0, __popcll(m), s, t, prm, tx, ty, ut, true, nullptr, &put);
        }
        if (ballot(missing)) flags |= TR_NO_UNIT;
        return put;
    }

    // Base reservations of every current assignment the deciding view holds (PlayerAction.java:387-394,
    // merged as ResourceUsage.java:92-97); in a PO view only snapshot units' assignments count.
    // tgt: the bitmap to fill (null: `bits`, which then no longer holds the issue index)
    DEV void baseReservations(int p, int& r0, int& r1, uint32_t* tgt = nullptr) {
        const int NB = (HW + 2 * W + 31) / 32;
        uint32_t* const bits = tgt ? tgt : this->bits;
        if (!tgt) ixValid = false;  // `bits` now holds this view's set
        for (int i = lid(); i < NB; i += 64) bits[i] = 0;
        wsync();
        int s0 = 0, s1 = 0, w0 = 0, w1 = 0;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            int key = -1;  // walk: a PRODUCE's cost | player << 16
            if (o < nu) {
                const uint32_t a = ua[o];
                const int t = ua_type(a);
                if ((a & UA_PRESENT) && (!po || snap_in(snap[o], p)) && (t == T_MOVE || t == T_PRODUCE)) {
                    const uint32_t c = uc[o];
                    const int d = par[o];
                    const int pos = (uy(c) + dyo(d)) * W + ux(c) + dxo(d) + W;
                    atomicOr(&bits[pos >> 5], 1u << (pos & 31));
                    if (t == T_PRODUCE) {
                        key = U.cost[ua_ut(a)] | ((uplay(c) == 0 ? 0 : 1) << 16);
                        if (uplay(c) == 0) s0 += U.cost[ua_ut(a)];
                        else s1 += U.cost[ua_ut(a)];
                    }
                }
            }
            if (walk) {  // the few PRODUCE lanes: one lane read each (buildIndex's walk)
                for (uint64_t mm = ballot(key >= 0); mm; mm &= mm - 1) {
                    const int kv = uni(rl(key, __builtin_ctzll(mm)));
                    if ((kv >> 16) == 0) w0 += kv & 0xFFFF;
                    else w1 += kv & 0xFFFF;
                }
            }
        }
        if (walk) {
            r0 = w0;
            r1 = w1;
        } else {
            r0 = wave_sum(s0);
            r1 = wave_sum(s1);
        }
        wsync();
    }

    // PlayerAction.fromVectorAction (rts/PlayerAction.java:384-417): decoded rows in ascending cell
    // order; accepted iff ua.ru.consistentWith(running ru) (rts/ResourceUsage.java:31-50).  Only the
    // acceptance chain is serial; accepted units get UA_PA.
    // issueNow (self-play, all units in one wave): the accepted rows are issued straight from the
    // chain's registers — issueSafe(pa) of the same pairs in the same (cell) order as issuePlayer
    DEV void decode(int p, bool issueNow = false) {
        int run0, run1;
        // full observability: the base reservations are the issue index (every present MOVE/PRODUCE
        // target + per-player PRODUCE cost sums), kept current across issue batches
        const bool useIx = !po && (HW + 2 * W + 31) / 32 <= 64;
        if (useIx) {
            if (!ixValid) buildIndex();
            run0 = sumProd0;
            run1 = sumProd1;
        } else {
            baseReservations(p, run0, run1);
        }
        MPHASE(13);
        if (MRTS_LIKELY(nu <= 64)) {
            decodeUnits(p, run0, run1, useIx, issueNow);
            return;
        }
        ixValid = false;  // the chain below adds to `bits`
        for (int c0 = 0; c0 < HW; c0 += 64) {
            const int c = c0 + lid();
            const int s = c < HW ? cell[c] : EMPTY;
            uint32_t a = 0;
            bool cand = false;
            if (s < CAP) {
                a = ua[s];
                cand = uplay(uc[s]) == p && (a & UA_DEC) && !(a & (UA_PRESENT | UA_BAD));
            }
            const uint64_t m = ballot(cand);
            if (m == 0) continue;
            const int t = ua_type(a), pr = par[s < CAP ? s : 0];
            int irank = 0;
            const uint64_t acc = acceptChain(p, run0, run1, cand, cand ? lanes_below(m) : -1, __popcll(m), t, pr, c, a, false, irank);
            if ((acc >> lid()) & 1ull) ua[s] = a | UA_PA;
            wsync();
        }
    }
    // Unit-parallel form (all units in one wave): the candidates' ascending-cell order is a rank
    // computed in registers, so the serial part is the acceptance chain alone.
    DEV void decodeUnits(int p, int& run0, int& run1, bool keepBits, bool issueNow) {
        const int o = lid();
        uint32_t a = 0, cu = 0;
        bool cand = false;
        if (o < nu) {
            cu = uc[o];
            a = ua[o];
            cand = !(cu & UC_DEAD) && uplay(cu) == p && (a & UA_DEC) && !(a & (UA_PRESENT | UA_BAD));
        }
        const uint64_t m = ballot(cand);
        if (m == 0) {
            if (issueNow) {
                curP = p;
                issueFills(p, 1);
            }
            return;
        }
        const int c = uy(cu) * W + ux(cu);
        const int pr = o < nu ? par[o] : 0;
        MPHASE(12);
        const int rank = cellRank(m, cand, c);
        MPHASE(14);
        int irank = 0;
        const uint64_t acc = acceptChain(p, run0, run1, cand, rank, __popcll(m), ua_type(a), pr, c, a, keepBits, irank);
        const bool isPA = (acc >> o) & 1ull;
        if (!issueNow) {
            if (isPA) ua[o] = a | UA_PA;
            wsync();
            return;
        }
        MPHASE(2);
        // issuePlayer(p, 1, false) of the accepted lanes (issuePA's legality + issueBatch, then the fills)
        curP = p;
        int t = 0, prm = 0, tx = 0, ty = 0, ut = 0;
        if (isPA) {
            t = ua_type(a);
            prm = pr;
            tx = ua_tx(a);
            ty = ua_ty(a);
            ut = ua_ut(a);
            // forwarded fused-policy rows (every decoded row here when fwdOn: all units in one wave)
            // are members of getUnitActions' list — see selfPlayFast; the masks, and so the rows,
            // come from the full state in partially observable games too (JNIGridnetClient.java:210-223)
            if (!fwdOn) legality(o, t, prm, tx, ty, ut);
        }
        wsync();
        if (acc) issueBatch(isPA, irank, __popcll(acc), o, t, prm, tx, ty, ut);
        issueFills(p, 1);
    }
    // rank of each candidate lane among the candidates m by cell c (cells are distinct)
    DEV int cellRank(uint64_t m, bool cand, int c) const {
        int rank = 0;
        for (uint64_t mm = m; mm; mm &= mm - 1) rank += rl(c, __builtin_ctzll(mm)) < c;
        return cand ? rank : -1;
    }
    // acceptChain with the reservation bitmap held one word per lane (readlane instead of LDS reads).
    // The candidates' (usesPos, cost, position) keys are first permuted into rank order (lane r holds
    // rank r's key, via rseq), so each chain step is one readlane and a few scalar tests.  The other
    // player's running sum cannot change during p's chain: if it blocks (ResourceUsage.java:38-46),
    // every candidate is rejected.
    DEV uint64_t acceptChainReg(int p, int& run0, int& run1, int rank, int n, bool usesPos, int tpos, int cost, int NB,
                                bool keepBits, int& irank, uint32_t* RB) {
        const int l = lid();
        {
            // Parallel form for the common case: when no candidate's used position is reserved already,
            // no two candidates use the same position, and the base reservations plus every candidate's
            // cost fit the player's resources, each sequential consistentWith test below passes (the
            // running sum only grows by accepted costs, so every prefix fits too) — accept them all.
            const int runQ = p == 0 ? run1 : run0, presQ = p == 0 ? pres1 : pres0, presP = p == 0 ? pres0 : pres1;
            const int runP = p == 0 ? run0 : run1;
            const bool cand = rank >= 0, up = cand && usesPos;
            if (!(runQ != 0 && runQ > 0 && runQ > presQ)) {
                bool conf = false;
                if (MRTS_CONF_LDS) {
                    // reserved already, or used by another candidate: each candidate ORs its position into a
                    // copy of the reservation words (rseq, free here) and is in conflict when the bit was set —
                    // by the base reservations or by another candidate (one of each equal pair sees it)
                    uint32_t* cp = (uint32_t*)rseq;
                    if (l < NB) cp[l] = RB[l];
                    wsync();
                    if (up) conf = (atomicOr(&cp[tpos >> 5], 1u << (tpos & 31)) >> (tpos & 31)) & 1u;
                    wsync();
                } else {
                    conf = up && ((RB[tpos >> 5] >> (tpos & 31)) & 1u);
                    for (uint64_t mm = ballot(up); mm; mm &= mm - 1) {
                        const int k = __builtin_ctzll(mm);
                        const int tk = rl(tpos, k);  // read in uniform flow: lane k itself is off inside the test below
                        if (up && k != l && tk == tpos) conf = true;
                    }
                }
                int sumc = 0;
                if (walk) {  // the candidates' PRODUCE costs (a few lanes): one lane read each
                    for (uint64_t mm = ballot(cand && cost > 0); mm; mm &= mm - 1) sumc += uni(rl(cost, __builtin_ctzll(mm)));
                } else if (ballot(cand && cost > 0)) {
                    sumc = wave_sum(cand ? cost : 0);
                }
                if (!ballot(conf) && runP + sumc <= presP) {
                    if (p == 0) run0 = runP + sumc;
                    else run1 = runP + sumc;
                    if (!keepBits && up) atomicOr(&RB[tpos >> 5], 1u << (tpos & 31));
                    if (cand) irank = rank;
                    wsync();
                    return ballot(cand);
                }
            }
        }
        uint32_t bv = l < NB ? RB[l] : 0u;
        if (rank >= 0) rseq[rank] = (int)(((uint32_t)usesPos << 31) | ((uint32_t)cost << 16) | ((uint32_t)tpos & 0xFFFFu));
        wsync();
        const int keyR = l < n ? rseq[l] : 0;
        const int runQ = p == 0 ? run1 : run0, presQ = p == 0 ? pres1 : pres0, presP = p == 0 ? pres0 : pres1;
        int runP = p == 0 ? run0 : run1;
        uint64_t accR = 0;  // accepted, bit r = rank r
        if (!(runQ != 0 && runQ > 0 && runQ > presQ)) {
            for (int r = 0; r < n; r++) {
                const uint32_t key = uniu((uint32_t)rl(keyR, r));
                const int bi = (int)(key & 0xFFFFu), cst = (int)((key >> 16) & 0x7FFFu);
                const bool up = key >> 31;
                bool ok = true;
                if (up) ok = !(((uint32_t)rl((int)bv, bi >> 5) >> (bi & 31)) & 1u);
                if (runP != 0) {
                    const int sum = cst + runP;
                    if (sum > 0 && sum > presP) ok = false;
                }
                if (ok) {
                    if (up && l == (bi >> 5)) bv |= 1u << (bi & 31);
                    runP += cst;
                    accR |= 1ull << r;
                }
            }
        }
        if (p == 0) run0 = runP;
        else run1 = runP;
        wsync();  // rseq is read again by the next chain
        if (!keepBits && l < NB) RB[l] = bv;
        const bool isAcc = rank >= 0 && ((accR >> rank) & 1ull);
        if (isAcc) irank = __popcll(accR & ((1ull << rank) - 1ull));
        return ballot(isAcc);
    }
    // ua.ru.consistentWith(running ru) for the n candidates in rank order (PlayerAction.java:400-415);
    // returns the accepted lanes
    // keepBits: `bits` is left as it was (the chain's additions stay in registers)
    // irank: each accepted lane's rank among the accepted (the pa's issue order)
    DEV uint64_t acceptChain(int p, int& run0, int& run1, bool cand, int rank, int n, int t, int pr, int c, uint32_t a,
                             bool keepBits, int& irank, uint32_t* RB = nullptr) {
        const bool usesPos = cand && (t == T_MOVE || t == T_PRODUCE);
        const int tpos = c + dyo(pr) * W + dxo(pr) + W;  // ResourceUsage position (UnitAction.java:254-291)
        const int cost = (cand && t == T_PRODUCE) ? U.cost[ua_ut(a)] : 0;
        const int NB = (HW + 2 * W + 31) / 32;
        if (NB <= 64) return acceptChainReg(p, run0, run1, rank, n, usesPos, tpos, cost, NB, keepBits, irank, RB ? RB : bits);
        uint64_t acc = 0;
        int nacc = 0;
        for (int r = 0; r < n; r++) {
            const int k = __builtin_ctzll(ballot(rank == r));
            const bool up = rl(usesPos, k);
            const int bi = rl(tpos, k), cst = rl(cost, k);
            bool ok = true;
            if (up) ok = !((uniu(bits[bi >> 5]) >> (bi & 31)) & 1u);
            if (run0 != 0) {
                const int sum = (p == 0 ? cst : 0) + run0;
                if (sum > 0 && sum > pres0) ok = false;
            }
            if (run1 != 0) {
                const int sum = (p == 1 ? cst : 0) + run1;
                if (sum > 0 && sum > pres1) ok = false;
            }
            if (ok) {
                if (up && lid() == 0) bits[bi >> 5] |= 1u << (bi & 31);
                if (p == 0) run0 += cst;
                else run1 += cst;
                acc |= 1ull << k;
                if (lid() == k) irank = nacc;
                nacc++;
            }
        }
        return acc;
    }

    // ------------------------------------------------------------------ issueSafe / issue
    // Unit.canExecuteAction (rts/units/Unit.java:531-534) = membership in getUnitActions
    // (:382-522) under UnitAction.equals (rts/UnitAction.java:191-208); an illegal action becomes
    // NONE(ETA(original)) (rts/GameState.java:347-354).  Lane-local.
    DEV void legality(int s, int& t, int& prm, int& tx, int& ty, int& ut) const { legality(s, uc[s], t, prm, tx, ty, ut); }
    DEV void legality(int s, uint32_t cu, int& t, int& prm, int& tx, int& ty, int& ut) const {
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const uint32_t fl = U.flags[typ];
        bool legal = false;
        int etaOrig = 0;
        switch (t) {
            case T_NONE: legal = true; break;
            case T_MOVE:
                etaOrig = U.moveT[typ];
                if ((fl & F_MOVE) && prm < 4) {
                    const int nx = x + dxo(prm), ny = y + dyo(prm);
                    legal = inb(nx, ny) && cell[ny * W + nx] == EMPTY;
                }
                break;
            case T_HARVEST:
                etaOrig = U.harvestT[typ];
                if ((fl & F_HARVEST) && res[s] == 0 && prm < 4) {
                    const int nx = x + dxo(prm), ny = y + dyo(prm);
                    if (inb(nx, ny)) {
                        const int n = cell[ny * W + nx];
                        legal = n < CAP && (U.flags[utyp(uc[n])] & F_RESOURCE);
                    }
                }
                break;
            case T_RETURN:
                etaOrig = U.moveT[typ];
                if ((fl & F_HARVEST) && res[s] > 0 && prm < 4) {
                    const int nx = x + dxo(prm), ny = y + dyo(prm);
                    if (inb(nx, ny)) {
                        const int n = cell[ny * W + nx];
                        legal = n < CAP && (U.flags[utyp(uc[n])] & F_STOCKPILE) && uplay(uc[n]) == pl;
                    }
                }
                break;
            case T_PRODUCE: {
                etaOrig = U.produceT[ut];
                bool produces = false;
                for (int i = 0; i < U.nprod[typ]; i++) produces |= (U.prod[typ][i] == ut);
                if (produces && prm < 4 && pres(pl) >= U.cost[ut]) {
                    const int nx = x + dxo(prm), ny = y + dyo(prm);
                    legal = inb(nx, ny) && cell[ny * W + nx] == EMPTY;
                }
            } break;
            case T_ATTACK:
                etaOrig = U.attackT[typ];
                if ((fl & F_ATTACK) && tx != 255) {
                    const int n = cell[ty * W + tx];
                    if (n < CAP) {
                        const int tp = uplay(uc[n]);
                        if (tp >= 0 && tp != pl) {
                            const int dx = tx - x, dy = ty - y, r = U.range[typ];
                            legal = (r == 1) ? (abs(dx) + abs(dy) == 1) : (dx * dx + dy * dy <= r * r);
                        }
                    }
                }
                break;
            default: etaOrig = 0; break;  // unknown type: ETA 0 (UnitAction.java:328)
        }
        if (!legal) {
            t = T_NONE;
            prm = etaOrig;
            tx = ty = ut = 0;
        } else if (t == T_ATTACK) {
            prm = -1;
        }
    }

    // Does present assignment o conflict with a new MOVE/PRODUCE (target ntgt, producer player pl,
    // cost ncost) — !old.ru.consistentWith(new ru) (GameState.java:264, ResourceUsage.java:31-50)
    DEV bool conflicts(int o, int ntgt, bool nProduce, int ncost, int pl) const {
        const uint32_t a = ua[o];
        if (!(a & UA_PRESENT)) return false;
        const int ot = ua_type(a);
        if (ot != T_MOVE && ot != T_PRODUCE) return false;
        const uint32_t oc = uc[o];
        const int od = par[o];
        if (((uy(oc) + dyo(od)) * W + ux(oc) + dxo(od)) == ntgt) return true;
        if (nProduce) {
            const int ores = (ot == T_PRODUCE && uplay(oc) == pl) ? U.cost[ua_ut(a)] : 0;
            const int sum = ores + ncost;
            if (sum > 0 && sum > pres(pl)) return true;
        }
        return false;
    }

    // GameState.issue for one pair (rts/GameState.java:252-326), wave-uniform arguments.  Returns the
    // type of the action put into the map (NONE when a conflict cancelled the new one).
    DEV int issueOne(int s, int t, int prm, int tx, int ty, int ut) {
        if (t == T_MOVE || t == T_PRODUCE) {
            const uint32_t cu = uniu(uc[s]);
            const int pl = uplay(cu), typ = utyp(cu);
            const int ntgt = (uy(cu) + dyo(prm)) * W + ux(cu) + dxo(prm);
            const bool nProduce = (t == T_PRODUCE);
            const int ncost = nProduce ? U.cost[ut] : 0;
            bool any = false;
            for (int o0 = 0; o0 < nu; o0 += 64) {
                const int o = o0 + lid();
                any |= ballot(o < nu && conflicts(o, ntgt, nProduce, ncost, pl)) != 0;
            }
            int lastSeq = -1;
            bool orig = true;  // p still names pa's own Pair (GameState.java:296 replaces only the loop variable)
            const int tIn = t, utIn = ut;
            while (any) {  // rare: resolve the conflicting assignments in insertion order
                int best = INF;
                for (int o = lid(); o < nu; o += 64)
                    if (as[o] > lastSeq && conflicts(o, ntgt, nProduce, ncost, pl)) best = min(best, as[o]);
                best = wave_min(best);
                if (best == INF) break;
                int os = INF;
                for (int o = lid(); o < nu; o += 64)
                    if ((ua[o] & UA_PRESENT) && as[o] == best) os = o;
                os = wave_min(os);
                lastSeq = best;
                if (uni(at[os]) == time) {  // same-cycle conflict: policy (GameState.java:266-297)
                    bool cold = false, cnew = false;
                    if (U.crs == 2) {
                        JRand rc = rngLoad(H_RNG_CANCEL);
                        if (rc.nextInt(2) == 0) cnew = true;
                        else cold = true;
                        rngStore(H_RNG_CANCEL, rc);
                    } else if (U.crs == 3) {
                        const int cc = hget(H_CANCEL_CNT);
                        if ((cc % 2) == 0) cnew = true;
                        else cold = true;
                        hset(H_CANCEL_CNT, cc + 1);
                    } else {
                        cold = cnew = true;
                    }
                    const int d1 = uni(etaSlot(os));
                    const int d2 = eta(t, prm, ut, typ);
                    const int md = min(d1, d2);
                    if (cold) {
                        if (lid() == 0) {
                            ua[os] = pack_ua(T_NONE, 0, 0, 0) | UA_PRESENT;
                            par[os] = (int16_t)md;
                            if (po) {  // the mutated UAA object is shared with the PO snapshots holding it
                                uint32_t b = snap[os];
                                for (int q = 0; q < 2; q++)
                                    if (snap_in(b, q) && snap_act(b, q) && as[os] < hdr[HX_SNAP + q])
                                        b = (b & ~(7u << (2 + 3 * q))) | ((uint32_t)(T_NONE + 1) << (2 + 3 * q));
                                snap[os] = (uint8_t)b;
                            }
                        }
                    }
                    if (cnew) {
                        t = T_NONE;
                        prm = md;
                        tx = ty = ut = 0;
                        orig = false;
                    }
                    wsync();
                } else {  // older assignment: only the new one is cancelled (:298-317)
                    // p.m_b = NONE mutates pa's own Pair unless a cancel already replaced p: the
                    // TraceEntry (pa.clone() after issueSafe) then records NONE, not the PRODUCE
                    if (orig && tIn == T_PRODUCE && (D.reward_need & RN_COUNTS) && lid() == 0) {
                        const int pc = prodCategory(U.flags[utIn]);
                        if (pc >= 0) rwc[curP * RC_N + pc] -= 1;
                    }
                    orig = false;
                    addErr(E_OLDER);
                    t = T_NONE;
                    prm = -1;
                    tx = ty = ut = 0;
                }
            }
        }
        // a unit with an assignment here got it from an earlier pair of this pa (Java rows may name a
        // unit twice): LinkedHashMap.put replaces the value and keeps the entry's position
        const bool again = (uniu(ua[s]) & UA_PRESENT) != 0;
        if (lid() == 0) {
            ua[s] = pack_ua(t, ut, tx, ty) | UA_PRESENT;
            par[s] = (int16_t)prm;
            at[s] = time;
            if (!again) as[s] = seq;
        }
        if (!again) seq++;
        wsync();
        return t;
    }

    // Issue index over ALL units (GameState.issue checks every present assignment, :255-262); under
    // full observability it is also every view's base ResourceUsage (PlayerAction.java:387-394).
    DEV void buildIndex() {
#ifdef MRTS_PHASE_TIMING
#ifndef MRTS_SPAN_ONLY
        phAcc[15] += 1000;  // call counter (x1000 so the per-step mean shows)
#endif
#endif
        const int NB = (HW + 2 * W + 31) / 32;
        for (int i = lid(); i < NB; i += 64) bits[i] = 0;
        wsync();
        bool mp = false;
        if (walk) {
            // the present PRODUCEs' costs per player (largest, sum) by walking their few lanes: one lane read
            // each (cost | player << 16), scalar max / add, instead of four whole-wave reductions
            int mc0 = -1, mc1 = -1, s0 = 0, s1 = 0;
            for (int o0 = 0; o0 < nu; o0 += 64) {
                const int o = o0 + lid();
                int key = -1;
                if (o < nu) {
                    const uint32_t a = ua[o];
                    const int t = ua_type(a);
                    if ((a & UA_PRESENT) && (t == T_MOVE || t == T_PRODUCE)) {
                        mp = true;
                        const uint32_t c = uc[o];
                        const int d = par[o];
                        const int pos = (uy(c) + dyo(d)) * W + ux(c) + dxo(d) + W;
                        atomicOr(&bits[pos >> 5], 1u << (pos & 31));
                        if (t == T_PRODUCE) key = U.cost[ua_ut(a)] | ((uplay(c) == 0 ? 0 : 1) << 16);
                    }
                }
                for (uint64_t mm = ballot(key >= 0); mm; mm &= mm - 1) {
                    const int kv = uni(rl(key, __builtin_ctzll(mm)));
                    const int k = kv & 0xFFFF;
                    if ((kv >> 16) == 0) {
                        mc0 = max(mc0, k);
                        s0 += k;
                    } else {
                        mc1 = max(mc1, k);
                        s1 += k;
                    }
                }
            }
            anyMP = ballot(mp) != 0;
            maxProd0 = mc0;
            maxProd1 = mc1;
            sumProd0 = s0;
            sumProd1 = s1;
        } else {
            int mc0 = -1, mc1 = -1, s0 = 0, s1 = 0;
            for (int o = lid(); o < nu; o += 64) {
                const uint32_t a = ua[o];
                const int t = ua_type(a);
                if (!(a & UA_PRESENT) || (t != T_MOVE && t != T_PRODUCE)) continue;
                mp = true;
                const uint32_t c = uc[o];
                const int d = par[o];
                const int pos = (uy(c) + dyo(d)) * W + ux(c) + dxo(d) + W;
                atomicOr(&bits[pos >> 5], 1u << (pos & 31));
                if (t == T_PRODUCE) {
                    const int k = U.cost[ua_ut(a)];
                    if (uplay(c) == 0) {
                        mc0 = max(mc0, k);
                        s0 += k;
                    } else {
                        mc1 = max(mc1, k);
                        s1 += k;
                    }
                }
            }
            anyMP = ballot(mp) != 0;
            if (ballot(mc0 >= 0 || mc1 >= 0)) {  // any present PRODUCE (rare)
                maxProd0 = -wave_min(-mc0);
                maxProd1 = -wave_min(-mc1);
                sumProd0 = wave_sum(s0);
                sumProd1 = wave_sum(s1);
            } else {
                maxProd0 = maxProd1 = -1;
                sumProd0 = sumProd1 = 0;
            }
        }
        ixValid = true;
        wsync();
    }

    // GameState.issue (rts/GameState.java:252-326) for a batch of (unit s, action) lanes in rank order
    // 0..n-1.  When no new MOVE/PRODUCE conflicts with a present assignment or an earlier one of the
    // batch, every issue() takes its no-conflict branch and the batch is issued in parallel (seq =
    // seq + rank); otherwise the batch runs one pair at a time through issueOne.
    // checkDup (Java rows): a unit named by an earlier pair of this pa (same batch, or already issued)
    // forces the one-at-a-time path
    // cuKnown: the lane's unit core word uc[s] (already in a register), or null
    // putAny (trace replay): set when a pair is put with a type other than NONE — GameState.issue's
    // return value (:323-324)
    // posChecked: the batch's MOVE / PRODUCE positions are known to be distinct and unreserved (the rows
    // passed acceptChain's ResourceUsage test against this same index: selfPlayFast) — the pairwise
    // walk then visits the PRODUCE lanes only, for the cost sums (round 5: it read four values per MOVE
    // lane per batch)
    DEV void issueBatch(bool act, int rank, int n, int s, int t, int prm, int tx, int ty, int ut, bool checkDup = false,
                        const uint32_t* cuKnown = nullptr, bool* putAny = nullptr, bool posChecked = false) {
        const bool mp = act && (t == T_MOVE || t == T_PRODUCE);
        const bool np = act && t == T_PRODUCE;
        if (MRTS_UNLIKELY(D.reward_need & RN_COUNTS)) {  // the pairs as the TraceEntry records them (legality applied)
            const int pc = np ? prodCategory(U.flags[ut]) : -1;
            auto cnt = [](bool b) { return (int)__popcll(ballot(b)); };
            const int c[RC_N] = {cnt(act && t == T_HARVEST), cnt(act && t == T_RETURN), cnt(act && t == T_ATTACK),
                                 cnt(pc == RC_PROD_WORKER), cnt(pc == RC_PROD_BUILDING), cnt(pc == RC_PROD_COMBAT)};
            if (lid() == 0)
#pragma unroll
                for (int k = 0; k < RC_N; k++) rwc[curP * RC_N + k] += c[k];
        }
        const uint64_t mpm = ballot(mp);
        bool conf = false;
        if (checkDup) {
            if (act && (ua[s] & UA_PRESENT)) conf = true;
            for (uint64_t mm = ballot(act); mm; mm &= mm - 1) {
                const int k = __builtin_ctzll(mm);
                const int sk = rl(s, k), rk = rl(rank, k);  // uniform flow (no readlane under a lane test)
                if (act && sk == s && rk < rank) conf = true;
            }
        }
        int ntgt = 0, ncost = 0, pl = 0;
        if (mpm) {
            if (!ixValid) buildIndex();
            if (mp) {
                const uint32_t cu = cuKnown ? *cuKnown : uc[s];
                pl = uplay(cu);
                ntgt = (uy(cu) + dyo(prm)) * W + ux(cu) + dxo(prm);
                ncost = np ? U.cost[ut] : 0;
                const int pr = pl == 0 ? pres0 : pres1;
                if ((bits[(ntgt + W) >> 5] >> ((ntgt + W) & 31)) & 1u) conf = true;
                if (np) {
                    if (anyMP && ncost > 0 && ncost > pr) conf = true;
                    const int mc = pl == 0 ? maxProd0 : maxProd1;
                    if (mc >= 0 && mc + ncost > 0 && mc + ncost > pr) conf = true;
                }
            }
            if (posChecked && ballot(np && ncost > 0 && ncost > (pl == 0 ? pres0 : pres1))) {
                // a PRODUCE whose cost alone exceeds the resources conflicts with any earlier MOVE / PRODUCE
                // of the batch (consistentWith: 0 + cost > resources) — the walk below skips the MOVEs
                const int minRank = wave_min(mp ? rank : INF);
                if (np && ncost > 0 && ncost > (pl == 0 ? pres0 : pres1) && minRank < rank) conf = true;
            }
            for (uint64_t mm = posChecked ? ballot(np) : mpm; mm; mm &= mm - 1) {  // earlier MOVE/PRODUCE lanes of the batch
                const int k = __builtin_ctzll(mm);
                const int rk = rl(rank, k), tk = posChecked ? 0 : rl(ntgt, k), pk = rl(pl, k), ck = rl(np ? ncost : -1, k);
                if (mp && rk < rank) {
                    if (!posChecked && tk == ntgt) conf = true;
                    if (np) {
                        const int sum = ((ck >= 0 && pk == pl) ? ck : 0) + ncost;
                        if (sum > 0 && sum > (pl == 0 ? pres0 : pres1)) conf = true;
                    }
                }
            }
        }
        if (MRTS_LIKELY(ballot(conf) == 0)) {
            if (putAny && ballot(act && t != T_NONE)) *putAny = true;
            if (act) {
                ua[s] = pack_ua(t, ut, tx, ty) | UA_PRESENT;
                par[s] = (int16_t)prm;
                at[s] = time;
                as[s] = seq + rank;
                if (mp && ixValid) atomicOr(&bits[(ntgt + W) >> 5], 1u << ((ntgt + W) & 31));
            }
            seq += n;
            if (mpm) {
                anyMP = true;
                if (walk) {
                    // the batch's PRODUCEs (a few lanes): one lane read each, scalar max / add
                    for (uint64_t mm = ballot(np); mm; mm &= mm - 1) {
                        const int kv = uni(rl(ncost | (pl << 16), __builtin_ctzll(mm)));
                        const int k = kv & 0xFFFF;
                        if ((kv >> 16) == 0) {
                            maxProd0 = max(maxProd0, k);
                            sumProd0 += k;
                        } else if ((kv >> 16) == 1) {
                            maxProd1 = max(maxProd1, k);
                            sumProd1 += k;
                        }
                    }
                } else {
                    if (ballot(np)) {  // PRODUCE is rare: skip the four reductions otherwise
                        maxProd0 = max(maxProd0, -wave_min(np && pl == 0 ? -ncost : 1));
                        maxProd1 = max(maxProd1, -wave_min(np && pl == 1 ? -ncost : 1));
                        sumProd0 += wave_sum(np && pl == 0 ? ncost : 0);
                        sumProd1 += wave_sum(np && pl == 1 ? ncost : 0);
                    }
                }
            }
            wsync();
        } else {
#ifdef MRTS_PHASE_TIMING
#ifndef MRTS_SPAN_ONLY
            phAcc[11] += 1000;  // slow-path batches
#endif
#endif
            for (int r = 0; r < n; r++) {
                const int k = __builtin_ctzll(ballot(act && rank == r));
                const int put = issueOne(rl(s, k), rl(t, k), rl(prm, k), rl(tx, k), rl(ty, k), rl(ut, k));
                if (putAny && put != T_NONE) *putAny = true;
            }
            ixValid = false;
        }
    }

    // GameState.issueSafe(pa) (rts/GameState.java:338-408) of the lanes' decoded actions.
    DEV void issuePA(int s, bool isPA, int rank, int n) {
        int t = 0, prm = 0, tx = 0, ty = 0, ut = 0;
        if (isPA) {
            const uint32_t a = ua[s];
            t = ua_type(a);
            prm = par[s];
            tx = ua_tx(a);
            ty = ua_ty(a);
            ut = ua_ut(a);
            legality(s, t, prm, tx, ty, ut);
        }
        wsync();
        issueBatch(isPA, rank, n, s, t, prm, tx, ty, ut);
    }
    // Agent pa = [accepted rows in cell order] + PlayerAction.fillWithNones(gs, p, fillDur)
    // (rts/PlayerAction.java:217-235) in list order; AI pa (RandomBiasedAI / PassiveAI) = its units
    // in list order (listOrder).
    DEV void issuePlayer(int p, int fillDur, bool listOrder) {
        curP = p;
        if (!listOrder && nu <= 64) {
            const int o = lid();
            uint32_t cu = 0;
            bool isPA = false;
            if (o < nu) {
                cu = uc[o];
                isPA = !(cu & UC_DEAD) && uplay(cu) == p && (ua[o] & UA_PA);
            }
            const uint64_t m = ballot(isPA);
            if (m) issuePA(o, isPA, cellRank(m, isPA, uy(cu) * W + ux(cu)), __popcll(m));
        } else if (!listOrder) {
            for (int c0 = 0; c0 < HW; c0 += 64) {
                const int c = c0 + lid();
                const int s = c < HW ? cell[c] : EMPTY;
                const bool isPA = s < CAP && uplay(uc[s]) == p && (ua[s] & UA_PA);
                const uint64_t m = ballot(isPA);
                if (m) issuePA(s, isPA, lanes_below(m), __popcll(m));
            }
        } else {
            for (int o0 = 0; o0 < nu; o0 += 64) {
                const int o = o0 + lid();
                const bool isPA = o < nu && !(uc[o] & UC_DEAD) && uplay(uc[o]) == p && (ua[o] & UA_PA);
                const uint64_t m = ballot(isPA);
                if (m) issuePA(o, isPA, lanes_below(m), __popcll(m));
            }
        }
        issueFills(p, fillDur);
    }
    // the NONE fills never conflict (issue() checks MOVE/PRODUCE only): parallel, seq in list order
    DEV void issueFills(int p, int fillDur) {
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            bool fill = false;
            if (o < nu) {
                const uint32_t c = uc[o];
                fill = !(c & UC_DEAD) && uplay(c) == p && !(ua[o] & (UA_PRESENT | UA_PA));
            }
            const uint64_t m = ballot(fill);
            if (fill) {
                ua[o] = pack_ua(T_NONE, 0, 0, 0) | UA_PRESENT;
                par[o] = (int16_t)fillDur;
                at[o] = time;
                as[o] = seq + lanes_below(m);
            }
            seq += __popcll(m);
        }
        wsync();
    }

    // ------------------------------------------------------------------ RandomBiasedAI
    // RandomBiasedAI.getAction (ai/RandomBiasedAI.java:51-107): for every idle unit of b in list
    // order, getUnitActions(gs) (rts/units/Unit.java:382-522) weighted 5 (attack/harvest/return) or 1,
    // Sampler.weighted (util/Sampler.java:116-135) with the game's java.util.Random, then accepted iff
    // consistent with the running reservations, else that list's NONE(10).  The chosen actions are
    // parked with UA_PA and issued later in list order.  getUnitActions of an owned unit is the same
    // in every view (neighbours and range-3 targets are always inside its own sight radius), the
    // base reservations are the view's (PO: b's snapshot).
    DEV void randomBiased(int b) {
        bool anyIdle = false;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            anyIdle |= ballot(o < nu && !(uc[o] & UC_DEAD) && uplay(uc[o]) == b && !(ua[o] & UA_PRESENT)) != 0;
        }
        if (!anyIdle) return;  // canExecuteAnyAction (rts/GameState.java:416-423): empty pa, no draws
        int run0, run1;
        baseReservations(b, run0, run1);
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            uint64_t m = ballot(o < nu && !(uc[o] & UC_DEAD) && uplay(uc[o]) == b && !(ua[o] & UA_PRESENT));
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                pickRandomBiased(o0 + k, b, run0, run1);
            }
        }
    }
    DEV void pickRandomBiased(int s, int b, int& run0, int& run1) {
        const uint32_t cu = uniu(uc[s]);
        const int x = ux(cu), y = uy(cu), typ = utyp(cu);
        const uint32_t fl = U.flags[typ];
        const int carried = uni(res[s]);
        int nb[4];
        uint32_t atkDirs = 0, harvDirs = 0, retDirs = 0, freeDirs = 0;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int nx = x + dxo(d), ny = y + dyo(d);
            nb[d] = inb(nx, ny) ? uni(cell[ny * W + nx]) : WALL;
            if (nb[d] < CAP) {
                const uint32_t oc = uniu(uc[nb[d]]);
                const int op = uplay(oc);
                const uint32_t ofl = U.flags[utyp(oc)];
                if (op >= 0 && op != b) atkDirs |= 1u << d;
                if (ofl & F_RESOURCE) harvDirs |= 1u << d;
                if ((ofl & F_STOCKPILE) && op == b) retDirs |= 1u << d;
            } else if (nb[d] == EMPTY) {
                freeDirs |= 1u << d;
            }
        }
        const int r = U.range[typ];
        int nAtk = 0;
        if (fl & F_ATTACK) {
            if (r == 1) {
                nAtk = __popc(atkDirs);
            } else {
                for (int q0 = 0; q0 < nu; q0 += 64) {
                    const int q = q0 + lid();
                    bool in = false;
                    if (q < nu) {
                        const uint32_t qc = uc[q];
                        const int op = uplay(qc), dx = ux(qc) - x, dy = uy(qc) - y;
                        in = !(qc & UC_DEAD) && op >= 0 && op != b && dx * dx + dy * dy <= r * r;
                    }
                    nAtk += __popcll(ballot(in));
                }
            }
        }
        const int nHarv = (fl & F_HARVEST) && carried == 0 ? __popc(harvDirs) : 0;
        const int nRet = (fl & F_HARVEST) && carried > 0 ? __popc(retDirs) : 0;
        int nProd = 0;
        for (int i = 0; i < U.nprod[typ]; i++)
            if (pres(b) >= U.cost[U.prod[typ][i]]) nProd += __popc(freeDirs);
        const int nMove = (fl & F_MOVE) ? __popc(freeDirs) : 0;
        const int n5 = nAtk + nHarv + nRet, n1 = nProd + nMove + 1;
        double total = 0.0;
        for (int i = 0; i < n5; i++) total += 5.0;
        for (int i = 0; i < n1; i++) total += 1.0;
        JRand rs = rngLoad(H_RNG_SAMPLER);
        const double tmp = rs.nextDouble() * total;
        rngStore(H_RNG_SAMPLER, rs);
        int idx = -1;
        double accum = 0.0;
        for (int i = 0; i < n5 + n1; i++) {
            accum += i < n5 ? 5.0 : 1.0;
            if (accum >= tmp) {
                idx = i;
                break;
            }
        }
        auto nth = [](uint32_t m, int n) {  // n-th set bit (0-based)
            for (int i = 0; i < n; i++) m &= m - 1;
            return __builtin_ctz(m);
        };
        int t = T_NONE, prm = 10, ut = 0, tx = 0, ty = 0;
        if (idx < nAtk) {
            t = T_ATTACK;
            prm = -1;
            if (r == 1) {
                const int d = nth(atkDirs, idx);
                tx = x + dxo(d);
                ty = y + dyo(d);
            } else {  // idx-th enemy in list order inside the disk
                int seen = 0;
                for (int q0 = 0; q0 < nu; q0 += 64) {
                    const int q = q0 + lid();
                    uint32_t qc = 0;
                    bool in = false;
                    if (q < nu) {
                        qc = uc[q];
                        const int op = uplay(qc), dx = ux(qc) - x, dy = uy(qc) - y;
                        in = !(qc & UC_DEAD) && op >= 0 && op != b && dx * dx + dy * dy <= r * r;
                    }
                    const uint64_t mm = ballot(in);
                    const int cnt = __popcll(mm);
                    if (idx - seen < cnt) {
                        uint64_t z = mm;
                        for (int i = 0; i < idx - seen; i++) z &= z - 1;
                        const uint32_t tc = (uint32_t)rl((int)qc, __builtin_ctzll(z));
                        tx = ux(tc);
                        ty = uy(tc);
                        break;
                    }
                    seen += cnt;
                }
            }
        } else if (idx < nAtk + nHarv) {
            t = T_HARVEST;
            prm = nth(harvDirs, idx - nAtk);
        } else if (idx < n5) {
            t = T_RETURN;
            prm = nth(retDirs, idx - nAtk - nHarv);
        } else {
            int j = idx - n5;
            if (j < nProd) {
                for (int i = 0; i < U.nprod[typ]; i++) {
                    const int u2 = U.prod[typ][i];
                    if (pres(b) < U.cost[u2]) continue;
                    const int n = __popc(freeDirs);
                    if (j < n) {
                        t = T_PRODUCE;
                        ut = u2;
                        prm = nth(freeDirs, j);
                        break;
                    }
                    j -= n;
                }
            } else if (j < nProd + nMove) {
                t = T_MOVE;
                prm = nth(freeDirs, j - nProd);
            }
        }
        // ua.resourceUsage(u, pgs).consistentWith(pa.r, gs) (RandomBiasedAI.java:91)
        bool ok = true;
        int bi = 0, cst = 0;
        const bool up = (t == T_MOVE || t == T_PRODUCE);
        if (up) {
            bi = (y + dyo(prm)) * W + x + dxo(prm) + W;
            ok = !((uniu(bits[bi >> 5]) >> (bi & 31)) & 1u);
        }
        if (t == T_PRODUCE) cst = U.cost[ut];
        if (run0 != 0) {
            const int sum = (b == 0 ? cst : 0) + run0;
            if (sum > 0 && sum > pres0) ok = false;
        }
        if (run1 != 0) {
            const int sum = (b == 1 ? cst : 0) + run1;
            if (sum > 0 && sum > pres1) ok = false;
        }
        if (ok) {
            if (up && lid() == 0) bits[bi >> 5] |= 1u << (bi & 31);
            if (b == 0) run0 += cst;
            else run1 += cst;
        } else {
            t = T_NONE;
            prm = 10;
            ut = tx = ty = 0;
        }
        if (lid() == 0) {
            ua[s] = pack_ua(t, ut, tx, ty) | UA_PA;
            par[s] = (int16_t)prm;
        }
        wsync();
    }

    // ------------------------------------------------------------------ PO snapshot
    // new PartiallyObservableGameState(gs, p) (rts/PartiallyObservableGameState.java:35-54):
    // the list keeps p's units and every other unit whose cell p observes (`observable`, :61-71); the
    // assignment map is the live one at this moment (UAA objects shared).
    // Sight disks (dx^2 + dy^2 <= sightRadius^2 of the seeing unit's type) painted into per-row bitmaps:
    // lane = seeing unit, one atomicOr per covered row word; a cell is seen iff its bit is set.
    DEV void paintDisk(uint32_t* rows, uint32_t u) const {
        const int t = utyp(u);
        paintDiskRows(rows, H, W, ux(u), uy(u), U.sight[t], U.diskLo[t], U.diskHi[t]);
    }
    // paintDisk for every lane with `act` at once, maps with W <= 32 (one row word) and sight <= 15:
    // a uniform loop over dy up to the table's largest sight, one predicated atomicOr per row
    DEV void paintDisks(bool act, uint32_t u, uint32_t* rows) const {
        const int t = utyp(u), x = ux(u), y = uy(u);
        const int sr = act ? U.sight[t] : -1, SM = U.maxSight;
        const uint32_t dlo = act ? U.diskLo[t] : 0u, dhi = act ? U.diskHi[t] : 0u;
        for (int dy = -SM; dy <= SM; dy++) {
            const int yy = y + dy, ady = dy < 0 ? -dy : dy;
            const int w = (int)(((ady < 8 ? dlo : dhi) >> (4 * (ady & 7))) & 0xFu);
            const int x0 = max(0, x - w), x1 = min(W - 1, x + w);
            const uint32_t b = ((2u << (x1 - x0)) - 1u) << x0;  // columns x0..x1 (x1 - x0 = 31: 2u << 31 wraps to 0)
            if (ady <= sr && yy >= 0 && yy < H) atomicOr(&rows[yy], b);
        }
    }
    // paintDisks into two views at once: the same disk (same unit) ORed into view 0's rows when act0
    // and into view 1's when act1 (row buffers rows0 / rows1 chosen per lane)
    DEV void paintDisks2(bool act0, uint32_t* rows0, bool act1, uint32_t* rows1, uint32_t u) const {
        const bool act = act0 || act1;
        const int t = utyp(u), x = ux(u), y = uy(u);
        const int sr = act ? U.sight[t] : -1, SM = U.maxSight;
        const uint32_t dlo = act ? U.diskLo[t] : 0u, dhi = act ? U.diskHi[t] : 0u;
        for (int dy = -SM; dy <= SM; dy++) {
            const int yy = y + dy, ady = dy < 0 ? -dy : dy;
            const int w = (int)(((ady < 8 ? dlo : dhi) >> (4 * (ady & 7))) & 0xFu);
            const int x0 = max(0, x - w), x1 = min(W - 1, x + w);
            const uint32_t b = ((2u << (x1 - x0)) - 1u) << x0;
            const bool row = ady <= sr && yy >= 0 && yy < H;
            if (row && act0) atomicOr(&rows0[yy], b);
            if (row && act1) atomicOr(&rows1[yy], b);
        }
    }
    DEV bool seen(const uint32_t* rows, int x, int y) const {
        const int WPR = (W + 31) >> 5;
        return (rows[y * WPR + (x >> 5)] >> (x & 31)) & 1u;
    }
    // PartiallyObservableGameState (rts/PartiallyObservableGameState.java:35-71): the view keeps the
    // units inside the sight of player p's (live) units, with the assignments they hold now.  Lane =
    // unit, a uniform loop over the observers (few; painting disks costs more here).
    DEV void snapshot(int p) {
#ifdef MRTS_ABLATE
        if (ab(AB_PO_NOSNAPSHOT)) return;
#endif
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            uint32_t cu = 0;
            bool live = false;
            if (o < nu) {
                cu = uc[o];
                live = !(cu & UC_DEAD);
            }
            bool vis = live && uplay(cu) == p;
            const int x = ux(cu), y = uy(cu);
            for (int q0 = 0; q0 < nu; q0 += 64) {
                const int q = q0 + lid();
                uint32_t qc = q < nu ? uc[q] : UC_DEAD;
                const bool obs = !(qc & UC_DEAD) && uplay(qc) == p;
                // each observer's x | y << 8 | sight^2 << 16, looked up once per lane, so the serial
                // loop below is one readlane per observer (no dependent LDS read of the sight table)
                const int sr = obs ? U.sight[utyp(qc)] : 0;
                const uint32_t ow = (uint32_t)ux(qc) | ((uint32_t)uy(qc) << 8) | ((uint32_t)(sr * sr) << 16);
                uint64_t m = ballot(obs);
                // two observers per round: independent readlane -> test chains (the loop is latency-bound)
                while (m) {
                    const int k1 = __builtin_ctzll(m);
                    m &= m - 1;
                    const int k2 = m ? __builtin_ctzll(m) : k1;
                    m &= m ? m - 1 : 0ull;
                    const uint32_t w1 = (uint32_t)rl((int)ow, k1), w2 = (uint32_t)rl((int)ow, k2);
                    const int dx1 = (int)(w1 & 0xFFu) - x, dy1 = (int)((w1 >> 8) & 0xFFu) - y;
                    const int dx2 = (int)(w2 & 0xFFu) - x, dy2 = (int)((w2 >> 8) & 0xFFu) - y;
                    vis |= (dx1 * dx1 + dy1 * dy1 <= (int)(w1 >> 16)) | (dx2 * dx2 + dy2 * dy2 <= (int)(w2 >> 16));
                }
            }
            if (o < nu) {
                uint32_t b = snap[o] & ~(1u << p) & ~(7u << (2 + 3 * p));
                if (live && vis) {
                    b |= 1u << p;
                    const uint32_t a = ua[o];
                    if (a & UA_PRESENT) b |= (uint32_t)(ua_type(a) + 1) << (2 + 3 * p);
                }
                snap[o] = (uint8_t)b;
            }
        }
        hset(HX_SNAP + p, seq);
        wsync();
    }
    // Both views' membership at once (self-play, poFast2 shapes): lane = unit paints its sight disk
    // into its own player's row bitmap (the host table's half-widths: the cells dx^2 + dy^2 <= sight^2,
    // exactly snapshot()'s test), then a unit is in view p iff it is live and its cell's bit is set
    // in p's rows (own units cover their own cell).  View 0's assignment bits are taken now; view 1's
    // by snapshotActions(1) after player 0's pairs are issued (the views' unitActions copies are taken
    // at different times; positions and liveness do not change in between).  `vis` is scratch here
    // (the render clears it).
    DEV bool snapBothOk() const { return W <= 32 && H <= 32 && nu <= 64 && U.maxSight <= 15; }
    DEV void snapshotBoth() {
#ifdef MRTS_ABLATE
        if (ab(AB_PO_NOSNAPSHOT)) return;
#endif
        const int l = lid();
        uint32_t* const r0 = vis;
        uint32_t* const r1 = vis + H;
        if (l < 2 * H) vis[l] = 0;
        const bool inList = l < nu;
        const uint32_t cu = inList ? uc[l] : UC_DEAD;
        const bool live = !(cu & UC_DEAD);
        const int own = uplay(cu);
        wsync();
        paintDisks2(live && own == 0, r0, live && own == 1, r1, cu);
        wsync();
        if (inList) {
            const int x = ux(cu), y = uy(cu);
            const bool in0 = live && ((r0[y] >> x) & 1u), in1 = live && ((r1[y] >> x) & 1u);
            uint32_t b = (in0 ? 1u : 0u) | (in1 ? 2u : 0u);
            const uint32_t a = ua[l];
            if (in0 && (a & UA_PRESENT)) b |= (uint32_t)(ua_type(a) + 1) << 2;
            snap[l] = (uint8_t)b;
        }
        hset(HX_SNAP + 0, seq);
        wsync();
    }
    DEV void snapshotActions(int p) {  // view p's assignment bits now (membership from snapshotBoth)
#ifdef MRTS_ABLATE
        if (ab(AB_PO_NOSNAPSHOT)) return;
#endif
        const int l = lid();
        if (l < nu) {
            uint32_t b = snap[l] & ~(7u << (2 + 3 * p));
            const uint32_t a = ua[l];
            if (((b >> p) & 1u) && (a & UA_PRESENT)) b |= (uint32_t)(ua_type(a) + 1) << (2 + 3 * p);
            snap[l] = (uint8_t)b;
        }
        hset(HX_SNAP + p, seq);
        wsync();
    }
    DEV void clearSnap() {
        for (int o = lid(); o < CAP; o += 64) snap[o] = 0;
        wsync();
    }

    // ------------------------------------------------------------------ cycle
    DEV void kill(int k) {  // GameState.removeUnit (rts/GameState.java:79-82)
        killedLanes |= ballot(readySlot == k);
        if (lid() == 0) {
            const uint32_t c = uc[k];
            uc[k] = c | UC_DEAD;
            cell[uy(c) * W + ux(c)] = EMPTY;
            ua[k] &= ~UA_PRESENT;
        }
        deaths++;
        wsync();
    }
    // UnitAction.execute (rts/UnitAction.java:338-465) — also for units killed earlier in the loop
    DEV void execute(int s) { execute(s, uniu(uc[s]), uniu(ua[s]), uni(par[s])); }
    // cu / a / prm: the unit's core word, its assignment and parameter (wave-uniform)
    DEV void execute(int s, uint32_t cu, uint32_t a, int prm) {
        const bool dead = cu & UC_DEAD;
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const int t = ua_type(a);
        switch (t) {
            case T_MOVE: {
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (!dead) {
                    if (uni(cell[ny * W + nx]) != EMPTY) addErr(E_COLLISION);
                    if (lid() == 0) {
                        cell[y * W + x] = EMPTY;
                        cell[ny * W + nx] = (uint16_t)s;
                    }
                }
                if (lid() == 0) uc[s] = (cu & ~0xFFFFu) | (uint32_t)nx | ((uint32_t)ny << 8);
                wsync();
            } break;
            case T_ATTACK: {
                const int n = uni(cell[ua_ty(a) * W + ua_tx(a)]);
                if (n < CAP) {
                    int dmg = U.minD[typ];
                    if (U.minD[typ] != U.maxD[typ]) {
                        JRand rd = rngLoad(H_RNG_DAMAGE);
                        dmg = U.minD[typ] + rd.nextInt(1 + (U.maxD[typ] - U.minD[typ]));
                        rngStore(H_RNG_DAMAGE, rd);
                    }
                    const int nhp = uni(hp[n]) - dmg;
                    if (lid() == 0) hp[n] = (int16_t)nhp;
                    wsync();
                    if (nhp <= 0) kill(n);
                }
            } break;
            case T_HARVEST: {
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (inb(nx, ny)) {
                    const int n = uni(cell[ny * W + nx]);
                    if (n < CAP && (U.flags[utyp(uniu(uc[n]))] & F_RESOURCE) && (U.flags[typ] & F_HARVEST) && uni(res[s]) == 0) {
                        const int nr = uni(res[n]) - U.harvestAmt[typ];
                        if (lid() == 0) {
                            res[n] = (int16_t)nr;
                            res[s] = (int16_t)U.harvestAmt[typ];
                        }
                        wsync();
                        if (nr <= 0) kill(n);
                    }
                }
            } break;
            case T_RETURN: {
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (inb(nx, ny)) {
                    const int n = uni(cell[ny * W + nx]);
                    const int carried = uni(res[s]);
                    if (n < CAP && (U.flags[utyp(uniu(uc[n]))] & F_STOCKPILE) && carried > 0) {
                        addPres(pl, carried);
                        if (lid() == 0) res[s] = 0;
                        wsync();
                    }
                }
            } break;
            case T_PRODUCE: {
                const int ut = ua_ut(a);
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (pres(pl) - U.cost[ut] >= 0) {
                    if (uni(cell[ny * W + nx]) != EMPTY) {
                        addErr(E_ADDUNIT);  // PhysicalGameState.addUnit throws (:190-195)
                    } else if (nu >= CAP) {
                        addErr(E_CAPACITY);
                    } else {
                        if (lid() == 0) {
                            uc[nu] = pack_uc(nx, ny, ut, pl);
                            hp[nu] = (int16_t)U.hp[ut];
                            res[nu] = 0;
                            ua[nu] = 0;
                            par[nu] = -1;
                            cell[ny * W + nx] = (uint16_t)nu;
                            if (po) snap[nu] = 0;  // produced this step: in no snapshot
                        }
                        nu++;
                        addPres(pl, -U.cost[ut]);
                        wsync();
                    }
                } else {
                    addErr(E_NEG_RES);
                }
            } break;
            default: break;
        }
    }
    // GameState.cycle (rts/GameState.java:553-571): time++, snapshot the ready assignments
    // (ETA + issue time <= time) in insertion order, then remove + execute each in that order.
    DEV void cycle() {
        time++;
        ixValid = false;
        if (MRTS_LIKELY(nu <= 64)) {
            cycleLanes();
            return;
        }
        // gather the ready list into LDS (slot order), count R
        int R = 0;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            bool ready = false;
            if (o < nu) {
                const uint32_t a = ua[o];
                ready = (a & UA_PRESENT) && etaSlot(o) + at[o] <= time;
            }
            const uint64_t m = ballot(ready);
            const int idx = R + lanes_below(m);
            if (ready && idx < 64) {
                rslot[idx] = (uint16_t)o;
                rseq[idx] = as[o];
            }
            if (ready) ua[o] |= UA_READY;
            R += __popcll(m);
        }
        wsync();
        if (R == 0) return;
        if (R <= 64) {
            // rank by insertion sequence: lane k holds ready item k
            const int k = lid();
            const int myseq = k < R ? rseq[k] : INF;
            const int myslot = k < R ? rslot[k] : 0;
            int rank = 0;
            for (int j = 0; j < R; j++) rank += rl(myseq, j) < myseq;
            wsync();
            if (k < R) rslot[rank] = (uint16_t)myslot;
            wsync();
            // lane r now holds ready item r (insertion order).  Every ready assignment leaves the
            // map (ua's PRESENT/READY) before any executes: no execute reads another unit's flags.
            // NONE executes as a no-op, so only the other types run, one by one, from registers —
            // a unit's core word changes under another's execute only by a kill (tracked in `killed`).
            const int os = k < R ? rslot[k] : 0;
            uint32_t a = 0, cu = 0;
            int prm = 0;
            if (k < R) {
                a = ua[os];
                cu = uc[os];
                prm = par[os];
                ua[os] = a & ~(UA_READY | UA_PRESENT);
            }
            wsync();
            uint64_t work = ballot(k < R && ua_type(a) != T_NONE);
            killedLanes = 0;
            readySlot = k < R ? os : -1;
            while (work) {
                const int r = __builtin_ctzll(work);
                work &= work - 1;
                uint32_t c = uniu(rl((int)cu, r));
                if ((killedLanes >> r) & 1ull) c |= UC_DEAD;
                execute(rl(os, r), c, uniu(rl((int)a, r)) & ~(UA_READY | UA_PRESENT), rl(prm, r));
            }
            readySlot = -1;
        } else {  // > 64 ready assignments: repeated minimum search
            while (true) {
                int best = INF;
                for (int o = lid(); o < nu; o += 64)
                    if (ua[o] & UA_READY) best = min(best, as[o]);
                best = wave_min(best);
                if (best == INF) break;
                int os = INF;
                for (int o = lid(); o < nu; o += 64)
                    if ((ua[o] & UA_READY) && as[o] == best) os = o;
                os = wave_min(os);
                if (lid() == 0) ua[os] &= ~(UA_READY | UA_PRESENT);
                wsync();
                execute(os);
            }
        }
    }
    // cycle() with every unit in one wave: lane = unit.  Each ready assignment leaves the map first
    // (in parallel); NONE executes as a no-op, so only the other ready assignments are ordered — by
    // insertion sequence (unique), ranked in registers — and executed one by one from registers.
    DEV void cycleLanes() {
        const int l = lid();
        bool ready = false;
        uint32_t a = 0, cu = 0;
        int prm = 0, sq = 0;
        if (l < nu) {
            a = ua[l];
            cu = uc[l];
            prm = par[l];
            sq = as[l];
            const int t0 = at[l];
            if (a & UA_PRESENT) ready = (MRTS_ETA_FLAT ? etaFlat(ua_type(a), prm, ua_ut(a), utyp(cu)) : eta(ua_type(a), prm, ua_ut(a), utyp(cu))) + t0 <= time;
        }
        if (ready) ua[l] = a & ~(UA_READY | UA_PRESENT);
        const bool wk = ready && ua_type(a) != T_NONE;
        const uint64_t work = ballot(wk);
        wsync();
        if (!work) return;
        int rank = 0;
        for (uint64_t m = work; m; m &= m - 1) rank += rl(sq, __builtin_ctzll(m)) < sq;
        killedLanes = 0;
        readySlot = wk ? l : -1;
        const int nw = __popcll(work);
        for (int r = 0; r < nw; r++) {
            const int k = __builtin_ctzll(ballot(wk && rank == r));
            uint32_t c = uniu((uint32_t)rl((int)cu, k));
            if ((killedLanes >> k) & 1ull) c |= UC_DEAD;
            execute(k, c, uniu((uint32_t)rl((int)a, k)) & ~(UA_READY | UA_PRESENT), rl(prm, k));
        }
        readySlot = -1;
    }
    // PhysicalGameState.gameover/winner (rts/PhysicalGameState.java:334-387)
    DEV void outcome(bool& gameover, int& winner) {
        int c0 = 0, c1 = 0;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            const uint32_t c = o < nu ? uc[o] : UC_DEAD;
            const bool live = !(c & UC_DEAD);
            c0 += __popcll(ballot(live && uplay(c) == 0));
            c1 += __popcll(ballot(live && uplay(c) == 1));
        }
        gameover = (c0 + c1 == 0) || ((c0 > 0) != (c1 > 0));
        winner = (c0 > 0 && c1 == 0) ? 0 : ((c1 > 0 && c0 == 0) ? 1 : -1);
    }
    // GameState.isComplete (rts/GameState.java:148-157): every owned unit has an assignment
    DEV bool complete() const {
        bool idle = false;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            if (o < nu) {
                const uint32_t c = uc[o];
                idle |= !(c & UC_DEAD) && uplay(c) >= 0 && !(ua[o] & UA_PRESENT);
            }
        }
        return ballot(idle) == 0;
    }
    // order-preserving removal of dead slots (LinkedList.remove, PhysicalGameState.java:208-210)
    DEV void compact() {
        int base = 0;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            const bool alive = o < nu && !(uc[o] & UC_DEAD);
            const uint64_t m = ballot(alive);
            const int idx = base + lanes_below(m);
            uint32_t c = 0, a = 0, sb = 0;
            int32_t t0 = 0, t1 = 0;
            int16_t h = 0, r = 0, pr = 0;
            if (alive) {
                if (po) sb = snap[o];
                c = uc[o];
                a = ua[o];
                t0 = at[o];
                t1 = as[o];
                h = hp[o];
                r = res[o];
                pr = par[o];
            }
            wsync();
            if (alive) {
                if (po) snap[idx] = (uint8_t)sb;
                uc[idx] = c;
                ua[idx] = a;
                at[idx] = t0;
                as[idx] = t1;
                hp[idx] = h;
                res[idx] = r;
                par[idx] = pr;
            }
            wsync();
            base += __popcll(m);
        }
        nu = base;
        for (int c = lid(); c < HW; c += 64)
            if (cell[c] != WALL) cell[c] = EMPTY;
        wsync();
        placeUnits();
    }

    // ------------------------------------------------------------------ reward functions
    // CloserToEnemyBaseRewardFunction.java:16-60 (and the identical CloserToEnemyUnit text): the enemy
    // Base is the first unit of minplayer named "Base" in the pre-cycle list; distances are from
    // maxplayer's Light/Heavy/Ranged/Worker units.  Squared distances are exact integers and sqrt is
    // monotone, so min(sqrt) = sqrt(min).
    DEV bool mobileType(int t) const { return (U.flags[t] & (N_WORKER | N_COMBAT)) != 0; }  // Light/Heavy/Ranged/Worker
    DEV void closerBefore() {
        int b0 = -1, b1 = -1;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            const uint32_t c = o < nu ? uc[o] : UC_DEAD;
            const bool base = !(c & UC_DEAD) && (U.flags[utyp(c)] & N_BASE);
            const uint64_t m0 = ballot(base && uplay(c) == 0), m1 = ballot(base && uplay(c) == 1);
            if (b0 < 0 && m0) b0 = o0 + __builtin_ctzll(m0);
            if (b1 < 0 && m1) b1 = o0 + __builtin_ctzll(m1);
        }
        hset(HX_BASE, b0 >= 0 ? (int)(uniu(uc[b0]) & 0xFFFFu) : -1);
        hset(HX_BASE + 1, b1 >= 0 ? (int)(uniu(uc[b1]) & 0xFFFFu) : -1);
        int o0, o1;
        closerMin(o0, o1);
        hset(HX_OLDSQ, o0);
        hset(HX_OLDSQ + 1, o1);
    }
    // smallest squared distance of player p's mobile units to the other player's base (INF if none)
    DEV void closerMin(int& sq0, int& sq1) {
        const int basePos0 = hget(HX_BASE), basePos1 = hget(HX_BASE + 1);
        int m0 = INF, m1 = INF;
        for (int o = lid(); o < nu; o += 64) {
            const uint32_t c = uc[o];
            if ((c & UC_DEAD) || !mobileType(utyp(c))) continue;
            const int pl = uplay(c);
            const int bp = pl == 0 ? basePos1 : basePos0;
            if (pl < 0 || bp < 0) continue;
            const int dx = (bp & 0xFF) - ux(c), dy = (bp >> 8) - uy(c), d = dx * dx + dy * dy;
            if (pl == 0) m0 = min(m0, d);
            else m1 = min(m1, d);
        }
        sq0 = wave_min(m0);
        sq1 = wave_min(m1);
    }
    static DEV double closerDist(int sq) { return sq == INF ? 2000000000.0 : __builtin_sqrt((double)sq); }
    // computeReward of every a_rfs entry for the game's external slots (slot0 + i is player pl(i)),
    // written to reward / done [slot][R]; returns done of a_rfs[0] (drives the auto-reset,
    // JNIGridnetVecClient.java:247,272).  WinLoss: WinLossRewardFunction.java:16-24; ResourceGather:
    // ResourceGatherRewardFunction.java:22-42; ProduceWorker / ProduceBuilding / ProduceCombatUnit:
    // ProduceWorkerRewardFunction.java:20-30 (the other two: the same lines of their files); Attack:
    // AttackRewardFunction.java:20-36 (a legal attack always targets a minplayer unit of the pre-cycle
    // pgs).  Constants are float 1.
    // it: this launch's iteration (the step's place in the Responses ring, KDyn.resp_reward)
    DEV bool writeRewards(int slot0, int nslots, int pl0, int pl1, bool gameover, int winner, int it = 0) {
        const int R = D.n_rewards;
        int newSq0 = INF, newSq1 = INF;
        if (MRTS_UNLIKELY(D.reward_need & RN_CLOSER)) closerMin(newSq0, newSq1);
        bool resLeft = false;
        if (D.reward_need & RN_RESOURCES)
            for (int o0 = 0; o0 < nu; o0 += 64) {
                const int o = o0 + lid();
                resLeft |= ballot(o < nu && !(uc[o] & UC_DEAD) && (U.flags[utyp(uc[o])] & N_RESOURCE) && res[o] > 0) != 0;
            }
        const int k0 = (int)(D.reward_kinds4 & 15u);
        // the Responses ring (mrts_set_step_responses): reward / done point at the call's ring and each
        // iteration writes its own step there (resp_stride = n_slots * n_rewards; 0 = the plain buffers)
        const size_t ro = MRTS_RESP_RING ? (size_t)((uint32_t)it * (uint32_t)D.resp_stride) : 0;
        const bool done0 = k0 == RF_WINLOSS ? gameover : (k0 == RF_RESOURCE_GATHER ? !resLeft : false);
        const int L = lid();
        if (R == 1 && k0 == RF_WINLOSS) {  // WinLoss alone (the common case): a wave-uniform branch, no switch
            if (L < nslots) {
                const int p = L ? pl1 : pl0;
                if (D.reward) D.reward[ro + slot0 + L] = gameover ? (winner == p ? 1.0 : -1.0) : 0.0;
                if (D.done) D.done[ro + slot0 + L] = gameover ? 1 : 0;
            }
            return done0;
        }
        if (L < nslots * R && (D.reward || D.done)) {
            const int i = L / R, j = L - i * R;
            const int p = i ? pl1 : pl0;
            const int kind = (int)((D.reward_kinds4 >> (4 * j)) & 15u);
            double r = 0.0;
            bool d = false;
            switch (kind) {
                case RF_WINLOSS:
                    d = gameover;
                    r = gameover ? (winner == p ? 1.0 : -1.0) : 0.0;
                    break;
                case RF_RESOURCE_GATHER:
                    r = (double)(rwc[p * RC_N + RC_HARVEST] + rwc[p * RC_N + RC_RETURN]);
                    d = !resLeft;
                    break;
                case RF_PRODUCE_WORKER: r = (double)rwc[p * RC_N + RC_PROD_WORKER]; break;
                case RF_PRODUCE_BUILDING: r = (double)rwc[p * RC_N + RC_PROD_BUILDING]; break;
                case RF_PRODUCE_COMBAT_UNIT: r = (double)rwc[p * RC_N + RC_PROD_COMBAT]; break;
                case RF_ATTACK: r = (double)rwc[p * RC_N + RC_ATTACK]; break;
                case RF_CLOSER_TO_ENEMY_BASE:
                case RF_CLOSER_TO_ENEMY_UNIT:
                    if (hdr[HX_BASE + 1 - p] >= 0)
                        r = closerDist(hdr[HX_OLDSQ + p]) - closerDist(p == 0 ? newSq0 : newSq1);
                    break;
            }
            if (D.reward) D.reward[ro + (size_t)(slot0 + i) * R + j] = r;
            if (D.done) D.done[ro + (size_t)(slot0 + i) * R + j] = d ? 1 : 0;
        }
        return done0;
    }

    // ------------------------------------------------------------------ observation
    // GameState.getVectorObservation (rts/GameState.java:922-968): 6 planes [C][H][W] int32.
    // Lane = 4 consecutive cells -> one dwordx4 store per plane.
    DEV void obsCell(int c, int player, int v[6]) const {
        const int s = cell[c];
        v[0] = v[1] = v[2] = v[3] = v[4] = 0;
        v[5] = (s == WALL) ? 1 : 0;
        if (s < CAP) {
            const uint32_t cu = uc[s];
            const uint32_t a = ua[s];
            const int pl = uplay(cu);
            v[0] = hp[s];
            v[1] = res[s];
            v[2] = pl >= 0 ? ((pl + player) % 2) + 1 : 0;
            v[3] = utyp(cu) + 1;
            v[4] = (a & UA_PRESENT) ? ua_type(a) : 0;
        }
    }
    // 16x16 full observability with every value below 256 (KDyn.obs_img): the five dynamic planes are
    // rendered as bytes into LDS by one pass over the unit list (lane = unit slot; a live unit owns its
    // cell, the dead are off the cell map, as in the gather below), then each lane's 4 cells x 5 planes
    // come back as zero-extended byte loads (LDS pipe, no VALU) straight into the dwordx4 stores.  The
    // cell-map gather costs the VALU-issue-bound c3 kernel ~150 VALU instructions per game-step more.
    // `snap` is the image (ldsBytes reserves 5 HW bytes there; snapshots exist only in PO games).
    DEV void writeObsFullImg(int slot0, int nslots, int player0) {
        uint8_t* const img = snap;
        const int l = lid();
        uint32_t* const iw = (uint32_t*)img;
#pragma unroll
        for (int i = 0; i < 5; i++) iw[l + 64 * i] = 0u;  // 5 x 256 bytes
        wsync();
        for (int s = l; s < nu; s += 64) {
            const uint32_t cu = uc[s];
            if (!(cu & UC_DEAD)) {
                const int c = uy(cu) * W + ux(cu), pl = uplay(cu);
                const uint32_t a = ua[s];
                img[c] = (uint8_t)hp[s];
                img[HW + c] = (uint8_t)res[s];
                img[2 * HW + c] = (uint8_t)(pl >= 0 ? ((pl + player0) % 2) + 1 : 0);
                img[3 * HW + c] = (uint8_t)(utyp(cu) + 1);
                img[4 * HW + c] = (uint8_t)((a & UA_PRESENT) ? ua_type(a) : 0);
            }
        }
        wsync();
        const int c4 = 4 * l;
        int v[6][4];
#pragma unroll
        for (int q = 0; q < 5; q++)
#pragma unroll
            for (int j = 0; j < 4; j++) v[q][j] = img[q * HW + c4 + j];
        const int npl = firstIt ? 6 : 5;  // the static terrain plane: first write of a launch only
        if (firstIt)
#pragma unroll
            for (int j = 0; j < 4; j++) v[5][j] = cell[c4 + j] == WALL ? 1 : 0;
        else
#pragma unroll
            for (int j = 0; j < 4; j++) v[5][j] = 0;
        int32_t* o0 = D.obs + (size_t)slot0 * D.C * HW;
        const __amdgpu_buffer_rsrc_t rs = bufRsrc(o0, (uint32_t)(nslots * D.C * HW * 4));
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if (i >= nslots) break;
#pragma unroll
            for (int q = 0; q < 6; q++) {
                if (q >= npl) break;
                int w[4];
#pragma unroll
                for (int j = 0; j < 4; j++)  // the other player's owners: 0, 1, 2 -> 0, 2, 1 (bits 2v.. of 0b011000)
                    w[j] = (i && q == 2) ? (int)__builtin_amdgcn_ubfe(24u, 2u * (uint32_t)v[q][j], 2u) : v[q][j];
                const uint32_t off = (uint32_t)((i * D.C + q) * HW + c4);
                if (SC1_OBS) st4sc1(rs, off * 4u, w[0], w[1], w[2], w[3]);
                else st4<WT_OBS>(o0 + off, w[0], w[1], w[2], w[3]);
            }
        }
        if (MRTS_UNLIKELY(D.obs8 != nullptr)) {  // the uint8 transport (mrts_set_exchange_bytes): every plane
            if (!firstIt)
#pragma unroll
                for (int j = 0; j < 4; j++) v[5][j] = cell[c4 + j] == WALL ? 1 : 0;
            uint8_t* b0 = D.obs8 + (size_t)slot0 * D.C * HW;
            for (int i = 0; i < nslots; i++)
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    uint32_t w = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int x = (i && q == 2 && v[q][j]) ? 3 - v[q][j] : v[q][j];  // the other player's owners
                        w |= (uint32_t)x << (8 * j);
                    }
                    *(uint32_t*)(b0 + (size_t)(i * D.C + q) * HW + c4) = w;
                }
        }
        if (MRTS_UNLIKELY(D.obs16 != nullptr)) {  // the int16 transport copy (mrts_set_obs16): every plane
            if (!firstIt)
#pragma unroll
                for (int j = 0; j < 4; j++) v[5][j] = cell[c4 + j] == WALL ? 1 : 0;
            int16_t* h0 = D.obs16 + (size_t)slot0 * D.C * HW;
            for (int i = 0; i < nslots; i++)
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    int4 w4 = make_int4(v[q][0], v[q][1], v[q][2], v[q][3]);
                    if (i && q == 2) {
                        w4.x = w4.x ? 3 - w4.x : 0;
                        w4.y = w4.y ? 3 - w4.y : 0;
                        w4.z = w4.z ? 3 - w4.z : 0;
                        w4.w = w4.w ? 3 - w4.w : 0;
                    }
                    *(uint2*)(h0 + (size_t)(i * D.C + q) * HW + c4) = pk16(w4);
                }
        }
    }
    DEV void writeObsFull(int slot0, int nslots, int player0) {
        if (HW == 256 && !po && D.obs_img && nslots <= 2) {
            writeObsFullImg(slot0, nslots, player0);
            return;
        }
        int32_t* o0 = D.obs + (size_t)slot0 * D.C * HW;
        if (HW <= 64) {
            // small maps (8x8: c2): lane = cell, one LDS round for the cell entry and one for its
            // occupant's fields, one dword store per plane (64 lanes = 256 contiguous bytes) — the
            // 4-cells-per-lane form below would leave 48 of the 64 lanes idle and quadruple each
            // active lane's dependent work
            const int c = lid();
            if (c < HW) {
                const int sc = cell[c];
                const int s = sc < CAP ? sc : 0;
                const uint32_t cu = uc[s], ca = ua[s];
                const int ch = hp[s], cr = res[s];
                const bool occ = sc < CAP;
                const int pl = uplay(cu);
                int v[6];
                v[0] = occ ? ch : 0;
                v[1] = occ ? cr : 0;
                v[2] = (occ && pl >= 0) ? ((pl + player0) % 2) + 1 : 0;
                v[3] = occ ? utyp(cu) + 1 : 0;
                v[4] = (occ && (ca & UA_PRESENT)) ? ua_type(ca) : 0;
                v[5] = sc == WALL ? 1 : 0;
                const __amdgpu_buffer_rsrc_t rs = bufRsrc(o0, (uint32_t)(nslots * D.C * HW * 4));
                const int npl = firstIt ? 6 : 5;  // the static terrain plane: first write of a launch only
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    if (i >= nslots) break;
#pragma unroll
                    for (int q = 0; q < 6; q++) {
                        if (q >= npl) break;
                        // the other player's view differs only in the owner plane
                        const int x = (i && q == 2 && v[2]) ? 3 - v[2] : v[q];
                        const uint32_t off = (uint32_t)((i * D.C + q) * HW + c);
                        if (SC1_OBS) __builtin_amdgcn_raw_buffer_store_b32(x, rs, (int)(off * 4u), 0, 16);
                        else st1<WT_OBS>(o0 + off, x);
                    }
                }
                if (MRTS_UNLIKELY(D.obs16 != nullptr)) {  // the int16 transport copy (mrts_set_obs16)
                    int16_t* h0 = D.obs16 + (size_t)slot0 * D.C * HW;
                    for (int i = 0; i < nslots; i++)
#pragma unroll
                        for (int q = 0; q < 6; q++)
                            h0[(size_t)(i * D.C + q) * HW + c] = (int16_t)((i && q == 2 && v[2]) ? 3 - v[2] : v[q]);
                }
                if (MRTS_UNLIKELY(D.obs8 != nullptr)) {  // the uint8 transport (mrts_set_exchange_bytes)
                    uint8_t* b0 = D.obs8 + (size_t)slot0 * D.C * HW;
                    for (int i = 0; i < nslots; i++)
#pragma unroll
                        for (int q = 0; q < 6; q++)
                            b0[(size_t)(i * D.C + q) * HW + c] = (uint8_t)((i && q == 2 && v[2]) ? 3 - v[2] : v[q]);
                }
            }
        } else if ((HW & 3) == 0) {
            for (int c4 = 4 * lid(); c4 < HW; c4 += 256) {
                // obsCell for 4 cells without branches: the 4 cell entries, then the occupants' 4
                // fields each (an empty cell reads slot 0 and is masked), so the lane waits for two
                // LDS rounds instead of one pair per occupied cell
                int sc[4];
#pragma unroll
                for (int j = 0; j < 4; j++) sc[j] = cell[c4 + j];
                uint32_t cu[4], ca[4];
                int ch[4], cr[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int s = sc[j] < CAP ? sc[j] : 0;
                    cu[j] = uc[s];
                    ca[j] = ua[s];
                    ch[j] = hp[s];
                    cr[j] = res[s];
                }
                int v[4][6];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const bool occ = sc[j] < CAP;
                    const int pl = uplay(cu[j]);
                    v[j][0] = occ ? ch[j] : 0;
                    v[j][1] = occ ? cr[j] : 0;
                    v[j][2] = (occ && pl >= 0) ? ((pl + player0) % 2) + 1 : 0;
                    v[j][3] = occ ? utyp(cu[j]) + 1 : 0;
                    v[j][4] = (occ && (ca[j] & UA_PRESENT)) ? ua_type(ca[j]) : 0;
                    v[j][5] = sc[j] == WALL ? 1 : 0;
                }
                const __amdgpu_buffer_rsrc_t rs = bufRsrc(o0, (uint32_t)(nslots * D.C * HW * 4));
                // the terrain plane (5) is static: within a multi-step launch only its first write stores it
                const int npl = firstIt ? 6 : 5;
#pragma unroll
                for (int pl = 0; pl < 6; pl++) {
                    if (pl >= npl) break;
                    if (SC1_OBS) st4sc1(rs, (uint32_t)(pl * HW + c4) * 4u, v[0][pl], v[1][pl], v[2][pl], v[3][pl]);
                    else st4<WT_OBS>(o0 + (size_t)pl * HW + c4, v[0][pl], v[1][pl], v[2][pl], v[3][pl]);
                }
                if (MRTS_UNLIKELY(D.obs16 != nullptr)) {  // the int16 transport copy (mrts_set_obs16)
                    int16_t* h0 = D.obs16 + (size_t)slot0 * D.C * HW;
#pragma unroll
                    for (int pl = 0; pl < 6; pl++) {
                        int4 w = make_int4(v[0][pl], v[1][pl], v[2][pl], v[3][pl]);
                        *(uint2*)(h0 + (size_t)pl * HW + c4) = pk16(w);
                        if (nslots == 2) {
                            if (pl == 2) {
                                w.x = w.x ? 3 - w.x : 0;
                                w.y = w.y ? 3 - w.y : 0;
                                w.z = w.z ? 3 - w.z : 0;
                                w.w = w.w ? 3 - w.w : 0;
                            }
                            *(uint2*)(h0 + (size_t)(D.C + pl) * HW + c4) = pk16(w);
                        }
                    }
                }
                if (nslots == 2) {  // the other player's view differs only in the owner plane
                    int32_t* o1 = o0 + (size_t)D.C * HW;
#pragma unroll
                    for (int pl = 0; pl < 6; pl++) {
                        if (pl >= npl) break;
                        int4 w = make_int4(v[0][pl], v[1][pl], v[2][pl], v[3][pl]);
                        if (pl == 2) {
                            w.x = w.x ? 3 - w.x : 0;
                            w.y = w.y ? 3 - w.y : 0;
                            w.z = w.z ? 3 - w.z : 0;
                            w.w = w.w ? 3 - w.w : 0;
                        }
                        if (SC1_OBS) st4sc1(rs, (uint32_t)((D.C + pl) * HW + c4) * 4u, w.x, w.y, w.z, w.w);
                        else st4<WT_OBS>(o1 + (size_t)pl * HW + c4, w.x, w.y, w.z, w.w);
                    }
                }
            }
        } else {
            for (int i = 0; i < nslots; i++) {
                int32_t* o = o0 + (size_t)i * D.C * HW;
                for (int c = lid(); c < HW; c += 64) {
                    int v[6];
                    obsCell(c, player0 + i, v);
#pragma unroll
                    for (int pl = 0; pl < 6; pl++) o[(size_t)pl * HW + c] = v[pl];
                    if (D.obs16) {
                        int16_t* h = D.obs16 + (size_t)(slot0 + i) * D.C * HW;
#pragma unroll
                        for (int pl = 0; pl < 6; pl++) h[(size_t)pl * HW + c] = (int16_t)v[pl];
                    }
                }
            }
        }
    }
    // The compact observation record of this game (KDyn.rec_out, mrts_internal.h recWords): the live
    // units in list order, one word each — every field GameState.getVectorObservation reads
    // (rts/GameState.java:922-968: hp, resources, owner, type, the assignment's action type; the
    // terrain plane is the map's).  Both players' observations follow from it (the owner plane is
    // ((owner + p) % 2) + 1), so one record per game replaces 2 x 6 x HW observation values on the
    // wire of the exchange (k_render_records rebuilds them).  More live units than the record holds
    // set E_RECORD (the exchange then reports an error).
    // Partially observable (po): the record holds what PartiallyObservableGameState.getVectorObservation
    // reads for both views (rts/PartiallyObservableGameState.java:82-154, as writeObsPO renders it) — every
    // unit of either view's snapshot in list order with its live fields (a dead one stays until the
    // compaction) and the snapshot byte (membership and seen action per view); walls and sight disks
    // follow on the receiving side from the map and the unit-type table.
    DEV void writeRecord(int it) {
        const int RU = D.rec_units;
        uint32_t* r = D.rec_out + ((size_t)it * D.n_sp_games + g) * (size_t)recWords(RU, po);
        if (po) {
            int n = 0;
            bool bad = false;
            for (int s0 = 0; s0 < nu; s0 += 64) {
                const int s = s0 + lid();
                const bool in = s < nu;  // every LDS read of the lane in one round (no dependent second round)
                const uint32_t sb = in ? (uint32_t)snap[s] : 0u, cu = in ? uc[s] : 0u;
                const int h = in ? hp[s] : 0, rs = in ? res[s] : 0;
                const bool inv = (sb & 3u) != 0;
                const uint64_t m = ballot(inv);
                const int idx = n + lanes_below(m);
                if (inv && idx < RU) {
                    bad |= h < -128 || h > 127 || rs < 0 || rs > 255;
                    r[1 + 2 * idx] = (uint32_t)(uy(cu) * W + ux(cu)) | (((uint32_t)h & 0xFFu) << 16) | ((uint32_t)rs << 24);
                    r[2 + 2 * idx] = (uint32_t)(utyp(cu) + 1) | ((uint32_t)(uplay(cu) + 1) << 4) | ((sb & 0xFFu) << 8);
                }
                n += __popcll(m);
            }
            const bool over = n > RU || ballot(bad) != 0;
            if (lid() == 0) r[0] = (uint32_t)(n < RU ? n : RU) | (over ? 0x80000000u : 0u);
            if (over) addErr(E_RECORD);
            return;
        }
        int n = 0;
        for (int s0 = 0; s0 < nu; s0 += 64) {
            const int s = s0 + lid();
            const bool in = s < nu;  // every LDS read of the lane in one round (no dependent second round)
            const uint32_t cu = in ? uc[s] : UC_DEAD, a = in ? ua[s] : 0u;
            const uint32_t hr = in ? ((uint32_t)hp[s] & 0xFFu) | (((uint32_t)res[s] & 0xFFu) << 8) : 0u;
            const bool live = !(cu & UC_DEAD);
            const uint64_t m = ballot(live);
            const int idx = n + lanes_below(m);
            if (live && idx < RU) {
                const uint32_t act = (a & UA_PRESENT) ? (uint32_t)ua_type(a) : 0u;
                r[1 + idx] = (uint32_t)(uy(cu) * W + ux(cu)) | (hr << 8) | ((uint32_t)(utyp(cu) + 1) << 24) |
                             ((uint32_t)(uplay(cu) + 1) << 27) | (act << 29);
            }
            n += __popcll(m);
        }
        if (lid() == 0) r[0] = (uint32_t)(n < RU ? n : RU) | (n > RU ? 0x80000000u : 0u);
        if (n > RU) addErr(E_RECORD);
    }
    // helper-wave launch: the observation's cells for the helper wave to render (lane = cell, HW <= 64),
    // player 0's view: word 0 = hp | resources << 16, word 1 = owner | type << 4 | action << 8 | wall << 12
    DEV void packObs(uint32_t* buf) const {
        const int c = lid();
        if (c < HW) {
            const int sc = cell[c];
            const int s = sc < CAP ? sc : 0;
            const uint32_t cu = uc[s], ca = ua[s];
            const bool occ = sc < CAP;
            const int pl = uplay(cu);
            const uint32_t v0 = occ ? (uint32_t)(uint16_t)hp[s] : 0u, v1 = occ ? (uint32_t)(uint16_t)res[s] : 0u;
            const uint32_t v2 = (occ && pl >= 0) ? (uint32_t)(pl + 1) : 0u, v3 = occ ? (uint32_t)utyp(cu) + 1 : 0u;
            const uint32_t v4 = (occ && (ca & UA_PRESENT)) ? (uint32_t)ua_type(ca) : 0u, v5 = sc == WALL ? 1u : 0u;
            buf[2 * c] = v0 | (v1 << 16);
            buf[2 * c + 1] = v2 | (v3 << 4) | (v4 << 8) | (v5 << 12);
        }
    }
    // PartiallyObservableGameState.getVectorObservation (rts/PartiallyObservableGameState.java:82-154):
    // the snapshot's units (live fields, possibly dead) in list order, last writer per cell; the
    // snapshot's assignments; walls; own / enemy sight disks of the snapshot units (calculateVisibility, :156-179).
    // delta: the buffer holds this game's view-p render of the previous observation write and the PO
    // record (poVis / poPend / lsnap) describes it.  A cell's planes 0-5 come from the last snapshot
    // unit on it (its current hp, resources, owner, type and snapshot assignment), planes 6-7 from
    // the sight rows; so the cells that can differ are: those of units whose membership in the view
    // or rendered fields changed (before and after — slots keep their index until the compaction),
    // those of rendered units that died last step (gone from the list: poPend), and the exact XOR
    // of old and new sight rows.  Only the 4-cell chunks holding them are rendered and stored.
    // writeObsPO for maps with W % 4 == 0, W <= 32 (one word per sight row), H <= 32, sight <= 15
    // and every unit in one wave (lane = slot).  One unit pass paints the sight disks, marks the
    // chunks of changed units (delta) and of the view's dead units (the next record's pending
    // chunks).  A cell's last snapshot writer (list order) is the later of its live occupant (cell
    // map), when that unit is in the view, and the view's dead units on it (a register list: few),
    // so no per-cell scratch map is built.  Same output as the general form below.
    DEV void writeObsPOFast(int slot, int p, bool delta) {
        const int l = lid(), NCW = poChunkWords(HW), NC = HW >> 2;
        uint32_t* mineRows = vis;
        uint32_t* theirRows = vis + H;
        uint32_t* dirty = poDirty;
        uint32_t* nextPend = poDirty + NCW;
        int32_t* pr = D.po_prev ? D.po_prev + (size_t)g * D.po_words : nullptr;
        const int SW = poSnapWords(CAP);
        const int nu0 = delta ? hget(H_NU) : 0;  // the header holds the loaded unit count until store()
        if (l < 2 * H) vis[l] = 0;
        if (l < NCW) {
            dirty[l] = delta ? poPend[p * NCW + l] : 0u;
            nextPend[l] = 0u;
        }
        const bool live = l < nu;
        uint32_t cu = 0, sb = 0;
        int hv = 0, rv = 0;
        if (live) {
            cu = uc[l];
            sb = snap[l];
            hv = hp[l];
            rv = res[l];
        }
        const bool in = live && snap_in(sb, p);
        const bool dead = in && (cu & UC_DEAD);
        const int cc = uy(cu) * W + ux(cu);
        wsync();
        // visibility planes over the view's units at their current positions (dead ones included:
        // the view's list still holds them): own / other player's sight disks
        const bool painter = in && uplay(cu) >= 0;
#ifdef MRTS_ABLATE
        if (!ab(AB_PO_NOPAINT))
#endif
        if (ballot(painter)) paintDisks(painter, cu, uplay(cu) == p ? mineRows : theirRows);
        const uint64_t deadM = ballot(dead);
        if (pr && dead) atomicOr(&nextPend[cc >> 7], 1u << ((cc >> 2) & 31));
        if (delta && (live || l < nu0)) {
            const bool inP = l < nu0 && ((lsnap >> p) & 1u);
            const int cp = uy(lcu) * W + ux(lcu);
            bool chg = in != inP;
            if (in && inP) {
                const uint32_t key = (uint32_t)(uint16_t)hv | ((uint32_t)(uint16_t)rv << 16);
                chg = cc != cp || key != lkey || snap_act(sb, p) != (int)((lsnap >> (2 + 3 * p)) & 7u);
            }
            if (chg && inP) atomicOr(&dirty[cp >> 7], 1u << ((cp >> 2) & 31));
            if (chg && in) atomicOr(&dirty[cc >> 7], 1u << ((cc >> 2) & 31));
        }
        wsync();
        if (l < 2 * H) {  // sight rows: changed columns -> chunk bits of that row; the record's copy
            const uint32_t row = vis[l];
            if (delta) {
                const uint32_t d = row ^ poVis[p * 2 * H + l];
                if (d) {
                    const int y = l < H ? l : l - H;
                    uint32_t gbits = 0;  // bit j = column group 4j..4j+3 changed
#pragma unroll
                    for (int j = 0; j < 8; j++) gbits |= ((d >> (4 * j)) & 0xFu) ? (1u << j) : 0u;
                    const int k0 = y * (W >> 2);
                    if ((k0 & 31) + (W >> 2) <= 32) {
                        atomicOr(&dirty[k0 >> 5], gbits << (k0 & 31));
                    } else {
                        for (uint32_t gg = gbits; gg; gg &= gg - 1) {
                            const int k = k0 + __builtin_ctz(gg);
                            atomicOr(&dirty[k >> 5], 1u << (k & 31));
                        }
                    }
                }
            }
            if (pr) pr[1 + SW + p * 2 * H + l] = (int32_t)row;
        }
        wsync();
        int n = NC;  // chunks to render: all, or the dirty list
        if (delta) {
            n = 0;
#pragma unroll
            for (int c0 = 0; c0 < 256; c0 += 64) {  // NC <= 256 (H, W <= 32)
                if (c0 < NC) {
                    const int k = c0 + l;
                    const bool dk = k < NC && ((dirty[k >> 5] >> (k & 31)) & 1u);
                    const uint64_t m = ballot(dk);
                    if (dk) poList[n + lanes_below(m)] = (uint16_t)k;
                    n += __popcll(m);
                }
            }
        }
        if (pr && l < NCW) pr[1 + SW + 4 * H + p * NCW + l] = (int32_t)nextPend[l];
        wsync();
        int32_t* out = D.obs + (size_t)slot * D.C * HW;
        for (int it = l; it < n; it += 64) {
            const int c4 = delta ? (int)poList[it] : it;  // lane = 4 consecutive cells of one row
            const int y = (4 * c4) / W, x0 = (4 * c4) % W;
            int cs[4], sl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) cs[j] = cell[4 * c4 + j];
            const uint32_t mr = mineRows[y], tr = theirRows[y];
            uint32_t ocu[4], osb[4];
            int ohp[4], ors[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {  // the live occupant's fields (an empty cell reads slot 0, masked)
                const int s = cs[j] < CAP ? cs[j] : 0;
                ocu[j] = uc[s];
                osb[j] = snap[s];
                ohp[j] = hp[s];
                ors[j] = res[s];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) sl[j] = (cs[j] < CAP && snap_in(osb[j], p)) ? cs[j] : -1;
            for (uint64_t m = deadM; m; m &= m - 1) {  // the view's dead units: a later list position wins
                const int ds = __builtin_ctzll(m);
                // the dead unit's fields from LDS, never by readlane: this loop is divergent (lanes >= n
                // are off), and the compiler may recompute a lane's cu / hp / snapshot byte inside it for
                // the active lanes only, so a readlane of an inactive lane returns a stale register
                // (round 5: the c5 helper's stale-value case)
                const uint32_t dcu = uc[ds];
                const int dcell = uy(dcu) * W + ux(dcu);
                const int dh = hp[ds], dr = res[ds];
                const uint32_t dsb = snap[ds];
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (dcell == 4 * c4 + j && ds > sl[j]) {
                        sl[j] = ds;
                        ocu[j] = dcu;
                        osb[j] = dsb;
                        ohp[j] = dh;
                        ors[j] = dr;
                    }
            }
            int v[4][8];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool occ = sl[j] >= 0;
                const int pl = uplay(ocu[j]);
                const int sa = snap_act(osb[j], p);
                v[j][0] = occ ? ohp[j] : 0;
                v[j][1] = occ ? ors[j] : 0;
                v[j][2] = (occ && pl >= 0) ? ((pl + p) % 2) + 1 : 0;
                v[j][3] = occ ? utyp(ocu[j]) + 1 : 0;
                v[j][4] = (occ && sa) ? sa - 1 : 0;
                v[j][5] = cs[j] == WALL ? 1 : 0;
                v[j][6] = (int)((mr >> (x0 + j)) & 1u);
                v[j][7] = (int)((tr >> (x0 + j)) & 1u);
            }
            if (SC1_POOBS) {
                const __amdgpu_buffer_rsrc_t rs = bufRsrc(out, (uint32_t)(D.C * HW * 4));
#pragma unroll
                for (int k = 0; k < 8; k++) st4sc1(rs, (uint32_t)(k * HW + 4 * c4) * 4u, v[0][k], v[1][k], v[2][k], v[3][k]);
            } else {
#pragma unroll
                for (int k = 0; k < 8; k++) st4<WT_POOBS>(out + k * HW + 4 * c4, v[0][k], v[1][k], v[2][k], v[3][k]);
            }
        }
        wsync();
    }
    // writeObsPOFast for both views of a self-play game in one pass (slot0 + v renders player v's
    // view v): the unit pass reads each unit once and paints its disk into both views' rows, the
    // dirty chunks of both views go into one list, and each render lane takes one (view, chunk)
    // item — half the dependent LDS rounds of two writeObsPOFast calls.  delta: bit v = view v's
    // buffer holds its previous render (writeObsPOFast's delta).  Same output as
    // writeObsPOFast(slot0, 0, delta & 1) followed by writeObsPOFast(slot0 + 1, 1, delta >> 1 & 1).
    DEV void writeObsPOFast2(int slot0, uint32_t delta) {
        const int l = lid(), NCW = poChunkWords(HW), NC = HW >> 2;
        uint32_t* const rowsV0 = vis;   // [mine H][theirs H]
        uint32_t* const rowsV1 = vis2;
        int32_t* pr = D.po_prev ? D.po_prev + (size_t)g * D.po_words : nullptr;
        // the record's global copy is for the next launch: inside a multi-step launch this render keeps
        // the record in LDS (poLds) and the next iteration reads it there, so only the last iteration
        // stores it (the sight rows and pending chunks here, the snapshot bytes in poRecordSnaps)
        int32_t* const prG = (!iter || lastIt) ? pr : nullptr;
        const int SW = poSnapWords(CAP);
        const bool d0 = delta & 1u, d1 = (delta >> 1) & 1u;
        const int nu0 = delta ? hget(H_NU) : 0;  // the header holds the loaded unit count until store()
        if (l < 2 * H) {
            rowsV0[l] = 0;
            rowsV1[l] = 0;
        }
        if (l < NCW) {  // [view][dirty, next pending]
            poDirty[l] = d0 ? poPend[l] : 0u;
            poDirty[NCW + l] = 0u;
            poDirty[2 * NCW + l] = d1 ? poPend[NCW + l] : 0u;
            poDirty[3 * NCW + l] = 0u;
        }
        const bool live = l < nu;
        uint32_t cu = 0, sb = 0;
        int hv = 0, rv = 0;
        if (live) {
            cu = uc[l];
            sb = snap[l];
            hv = hp[l];
            rv = res[l];
        }
        const bool in0 = live && snap_in(sb, 0), in1 = live && snap_in(sb, 1);
        const bool isDead = (cu & UC_DEAD) != 0;
        const bool dead0 = in0 && isDead, dead1 = in1 && isDead;
        const int cc = uy(cu) * W + ux(cu);
        const int own = uplay(cu);
        wsync();
        {
            const bool pt0 = in0 && own >= 0, pt1 = in1 && own >= 0;
#ifdef MRTS_ABLATE
            if (!ab(AB_PO_NOPAINT))
#endif
            if (ballot(pt0 || pt1))
                paintDisks2(pt0, own == 0 ? rowsV0 : rowsV0 + H, pt1, own == 1 ? rowsV1 : rowsV1 + H, cu);
        }
        const uint64_t deadM0 = ballot(dead0), deadM1 = ballot(dead1);
        if (pr && dead0) atomicOr(&poDirty[NCW + (cc >> 7)], 1u << ((cc >> 2) & 31));
        if (pr && dead1) atomicOr(&poDirty[3 * NCW + (cc >> 7)], 1u << ((cc >> 2) & 31));
        if (delta && (live || l < nu0)) {
            const int cp = uy(lcu) * W + ux(lcu);
            const uint32_t key = (uint32_t)(uint16_t)hv | ((uint32_t)(uint16_t)rv << 16);
#pragma unroll
            for (int v = 0; v < 2; v++) {
                if (!(v ? d1 : d0)) continue;
                const bool in = v ? in1 : in0;
                const bool inP = l < nu0 && ((lsnap >> v) & 1u);
                bool chg = in != inP;
                if (in && inP)
                    chg = cc != cp || key != lkey || snap_act(sb, v) != (int)((lsnap >> (2 + 3 * v)) & 7u);
                uint32_t* dirty = poDirty + 2 * v * NCW;
                if (chg && inP) atomicOr(&dirty[cp >> 7], 1u << ((cp >> 2) & 31));
                if (chg && in) atomicOr(&dirty[cc >> 7], 1u << ((cc >> 2) & 31));
            }
        }
        wsync();
        if (l < 2 * H) {  // sight rows: changed columns -> chunk bits of that row; the record's copies
            const int y = l < H ? l : l - H;
            const int k0 = y * (W >> 2);
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const uint32_t row = (v ? rowsV1 : rowsV0)[l];
                if (v ? d1 : d0) {
                    const uint32_t d = row ^ poVis[v * 2 * H + l];
                    poVis[v * 2 * H + l] = row;  // the record's LDS copy (a multi-step launch's next render)
                    if (d) {
                        uint32_t gbits = 0;  // bit j = column group 4j..4j+3 changed
#pragma unroll
                        for (int j = 0; j < 8; j++) gbits |= ((d >> (4 * j)) & 0xFu) ? (1u << j) : 0u;
                        uint32_t* dirty = poDirty + 2 * v * NCW;
                        if ((k0 & 31) + (W >> 2) <= 32) {
                            atomicOr(&dirty[k0 >> 5], gbits << (k0 & 31));
                        } else {
                            for (uint32_t gg = gbits; gg; gg &= gg - 1) {
                                const int k = k0 + __builtin_ctz(gg);
                                atomicOr(&dirty[k >> 5], 1u << (k & 31));
                            }
                        }
                    }
                }
                if (prG) prG[1 + SW + v * 2 * H + l] = (int32_t)row;
                if (!(v ? d1 : d0)) poVis[v * 2 * H + l] = row;
            }
        }
        wsync();
        // one list of (view << 15 | chunk) items: view 0's dirty chunks (all, without delta), then view 1's
        int n = 0;
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const bool dv = v ? d1 : d0;
            const uint32_t* dirty = poDirty + 2 * v * NCW;
#pragma unroll
            for (int c0 = 0; c0 < 256; c0 += 64) {  // NC <= 256 (H, W <= 32)
                if (c0 < NC) {
                    const int k = c0 + l;
                    const bool dk = k < NC && (!dv || ((dirty[k >> 5] >> (k & 31)) & 1u));
                    const uint64_t m = ballot(dk);
                    if (dk) poList[n + lanes_below(m)] = (uint16_t)((v << 15) | k);
                    n += __popcll(m);
                }
            }
        }
        if (pr && l < NCW) {
            if (prG) {
                prG[1 + SW + 4 * H + l] = (int32_t)poDirty[NCW + l];
                prG[1 + SW + 4 * H + NCW + l] = (int32_t)poDirty[3 * NCW + l];
            }
            poPend[l] = poDirty[NCW + l];  // LDS copies, as the sight rows above
            poPend[NCW + l] = poDirty[3 * NCW + l];
        }
        poLds = pr != nullptr;
        wsync();
#ifdef MRTS_ABLATE
        if (ab(AB_COUNT) && l == 0) {  // contended global atomics: only when counting
            atomicAdd(&g_dbg[0], (unsigned long long)n);
            atomicAdd(&g_dbg[1], 1ull);
            if (delta) atomicAdd(&g_dbg[2], 1ull);
        }
        if (ab(AB_PO_NOSTORE)) n = 0;  // no render pass (gather + stores)
#endif
        int32_t* out = D.obs + (size_t)slot0 * D.C * HW;
        const __amdgpu_buffer_rsrc_t rs = bufRsrc(out, (uint32_t)(2 * D.C * HW * 4));
        const uint64_t deadAny = deadM0 | deadM1;
        for (int it = l; it < n; it += 64) {
            const uint32_t e = poList[it];
            const int v = (int)(e >> 15), c4 = (int)(e & 0x7FFFu);  // lane = 4 consecutive cells of one row
            const uint64_t deadM = v ? deadM1 : deadM0;
            const int y = (4 * c4) / W, x0 = (4 * c4) % W;
            const uint32_t* rows = v ? rowsV1 : rowsV0;
            int cs[4], sl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) cs[j] = cell[4 * c4 + j];
            const uint32_t mr = rows[y], tr = rows[H + y];
            uint32_t ocu[4], osb[4];
            int ohp[4], ors[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {  // the live occupant's fields (an empty cell reads slot 0, masked)
                const int s = cs[j] < CAP ? cs[j] : 0;
                ocu[j] = uc[s];
                osb[j] = snap[s];
                ohp[j] = hp[s];
                ors[j] = res[s];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) sl[j] = (cs[j] < CAP && snap_in(osb[j], v)) ? cs[j] : -1;
            for (uint64_t m = deadAny; m; m &= m - 1) {  // the view's dead units: a later list position wins
                const int ds = __builtin_ctzll(m);
                // from LDS, not by readlane of an inactive lane (writeObsPOFast)
                const uint32_t dcu = uc[ds];
                const int dcell = uy(dcu) * W + ux(dcu);
                const int dh = hp[ds], dr = res[ds];
                const uint32_t dsb = snap[ds];
                const bool mine = (deadM >> ds) & 1ull;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (mine && dcell == 4 * c4 + j && ds > sl[j]) {
                        sl[j] = ds;
                        ocu[j] = dcu;
                        osb[j] = dsb;
                        ohp[j] = dh;
                        ors[j] = dr;
                    }
            }
            int vv[4][8];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool occ = sl[j] >= 0;
                const int pl = uplay(ocu[j]);
                const int sa = snap_act(osb[j], v);
                vv[j][0] = occ ? ohp[j] : 0;
                vv[j][1] = occ ? ors[j] : 0;
                vv[j][2] = (occ && pl >= 0) ? ((pl + v) % 2) + 1 : 0;
                vv[j][3] = occ ? utyp(ocu[j]) + 1 : 0;
                vv[j][4] = (occ && sa) ? sa - 1 : 0;
                vv[j][5] = cs[j] == WALL ? 1 : 0;
                vv[j][6] = (int)((mr >> (x0 + j)) & 1u);
                vv[j][7] = (int)((tr >> (x0 + j)) & 1u);
            }
            const uint32_t base = (uint32_t)(v * D.C * HW + 4 * c4) * 4u;
#ifdef MRTS_ABLATE
            if (ab(AB_PO_ZEROSTORE)) {  // pricing: the render's values computed, not stored
                int acc = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) acc += vv[0][k] ^ vv[1][k] ^ vv[2][k] ^ vv[3][k];
                keepv(acc);
                continue;
            }
#endif
            if (SC1_POOBS) {
#pragma unroll
                for (int k = 0; k < 8; k++) st4sc1(rs, base + (uint32_t)(k * HW) * 4u, vv[0][k], vv[1][k], vv[2][k], vv[3][k]);
            } else {
                int32_t* o = out + base / 4;
#pragma unroll
                for (int k = 0; k < 8; k++) st4<WT_POOBS>(o + k * HW, vv[0][k], vv[1][k], vv[2][k], vv[3][k]);
            }
        }
        wsync();
    }
    DEV bool poFast2() const { return (W & 3) == 0 && W <= 32 && H <= 32 && nu <= 64 && U.maxSight <= 15; }
    // the helper's part of a packed step's masks (writeMasksLanes with recOut): each own idle unit's
    // mask record (79 bytes from its 3 bit words) and fused-policy row, and the zero record + zero row
    // of every vacated cell — the same bytes the game wave would have stored.  Lane l = threadIdx.x - 64.
    DEV void storeRecordsHelp(const uint32_t* rb) {
        const int l = (int)threadIdx.x - 64;
        const int total = HW * K, slot0 = 2 * g;
        const uint8_t* mbase = D.masks + (size_t)slot0 * total;
        const __amdgpu_buffer_rsrc_t mrs = bufRsrc((void*)mbase, (uint32_t)(2 * total));
        if (!(uniu(rb[5 * 64]) >> 31)) return;  // the game wave stored this step's masks itself
        const uint32_t e = rb[l];
        if (e != ~0u) {
            const int si = (int)(e >> 16), c = (int)(e & 0xFFFFu), slot = slot0 + si;
            const uint64_t lo = (uint64_t)rb[64 + l] | ((uint64_t)rb[128 + l] << 32);
            const uint32_t w2 = rb[192 + l];
            if (SC1_MASK) storeRecordSc1(mrs, mbase, (uint32_t)(si * total + c * K), lo, w2);
            else storeRecord(D.masks + (size_t)slot * total + (size_t)c * K, lo, w2);
            if (D.pol_actions && D.pol_delta) {
                int32_t a[7];
                unpackFwd(rb[256 + l], a);
                int32_t* dst = D.pol_actions + ((size_t)slot * HW + c) * 7;
                st4u<WT_MASK>(dst, a[0], a[1], a[2], a[3]);
                st3u<WT_MASK>(dst + 4, a[4], a[5], a[6]);
            }
        }
        const int ngone = (int)(uniu(rb[5 * 64]) & 0xFFFFu);
        const uint16_t* gl = (const uint16_t*)(rb + 5 * 64 + 1);
        if (l < ngone) {
            const uint32_t ge = gl[l];
            const int slot = slot0 + (int)(ge >> 15), cz = (int)(ge & 0x7FFFu);
            if (SC1_MASK) storeRecordSc1(mrs, mbase, (uint32_t)((slot - slot0) * total + cz * K), 0ull, 0u);
            else storeRecord(D.masks + (size_t)slot * total + (size_t)cz * K, 0ull, 0u);
            if (D.pol_actions && D.pol_delta) {
                int32_t* dst = D.pol_actions + ((size_t)slot * HW + cz) * 7;
                st4u<WT_MASK>(dst, 0, 0, 0, 0);
                st3u<WT_MASK>(dst + 4, 0, 0, 0);
            }
        }
    }
    // Helper-wave launch, partially observable self-play (k_env HELP && FPO, BASELINE c5): the game
    // wave hands this step's render inputs to the helper wave instead of rendering (writeObsPOFast2's
    // unit pass reads, per unit slot < 64: the unit word, hp | resources, the snapshot byte, and the
    // previous record's position / key / snapshot byte; the assignment type + 1 for the next step's
    // snapshot, snapFromPack), and the helper renders while the game runs its compaction, masks,
    // policy and the next step.  pk = [5][64] words, ph = [4] header words:
    // unit count, the previous record's unit count, flags (bits 0-1 delta per view, `how`: bit 2 =
    // render the pack, bit 3 = render the live state with writeObsPO, the game waiting).
    DEV void packPO(uint32_t* pk, uint32_t* ph, uint32_t delta, uint32_t how) {
        const int l = lid();
        const bool live = l < nu;
        pk[l] = live ? uc[l] : 0u;
        pk[64 + l] = live ? ((uint32_t)(uint16_t)hp[l] | ((uint32_t)(uint16_t)res[l] << 16)) : 0u;
        const uint32_t a = live ? ua[l] : 0u;
        pk[128 + l] = (live ? (uint32_t)snap[l] : 0u) | ((lsnap & 0xFFu) << 8) |
                      ((a & UA_PRESENT) ? (uint32_t)(ua_type(a) + 1) << 16 : 0u);
        pk[192 + l] = lcu;
        pk[256 + l] = lkey;
        if (l == 0) {
            ph[0] = (uint32_t)nu;
            ph[1] = (uint32_t)hget(H_NU);
            ph[2] = (delta & 3u) | how;
        }
        // how = 4: the helper keeps the record's LDS copies, as writeObsPOFast2 does; 8: the general
        // render stores it globally only, and nextStep re-reads it
        poLds = how == 4u && D.po_prev != nullptr;
    }
    // snapshotBoth of the NEXT step, by the helper wave from step k's pack: the state the next step
    // starts from is the packed one after the end-of-step compaction (dead units leave, the rest keep
    // their order and positions, assignments and liveness do not change in between), so each live
    // unit paints its sight disk into its player's rows and takes the membership bits and view 0's
    // assignment bits at its compacted index.  hsnap[slot] = the snapshot byte.
    DEV void snapFromPack(const uint32_t* pk, const uint32_t* ph, uint32_t* rows, uint8_t* hsnap) {
        const int l = (int)threadIdx.x - 64;
        const int nuP = (int)uniu(ph[0]);
        uint32_t* const r0 = rows;
        uint32_t* const r1 = rows + H;
        if (l < 2 * H) rows[l] = 0;
        const uint32_t cu = l < nuP ? pk[l] : UC_DEAD;
        const bool live = !(cu & UC_DEAD);
        const int own = uplay(cu);
        const uint32_t at = (pk[128 + l] >> 16) & 15u;  // assignment type + 1 (0 = none)
        wsync();
        paintDisks2(live && own == 0, r0, live && own == 1, r1, cu);
        wsync();
        const uint64_t m = ballot(live);
        if (live) {
            const int x = ux(cu), y = uy(cu);
            const bool in0 = (r0[y] >> x) & 1u, in1 = (r1[y] >> x) & 1u;
            hsnap[lanes_below(m)] = (uint8_t)((in0 ? 1u : 0u) | (in1 ? 2u : 0u) | (in0 ? at << 2 : 0u));
        }
        wsync();
    }
    // the game wave's side: the helper's snapshot bytes instead of snapshotBoth (same bytes, same header)
    DEV void takeSnap(const uint8_t* hsnap) {
        const int l = lid();
        if (l < nu) snap[l] = hsnap[l];
        hset(HX_SNAP + 0, seq);
        wsync();
    }
    // writeObsPOFast2 as run by the helper wave (lane l = threadIdx.x - 64) from a packed step (packPO):
    // the same passes and stores.  What the game wave's live LDS state gave it comes from the pack:
    // the units' fields, and the live occupant of a cell from hcell (slot, or 0xFF), a per-step map
    // built here from the packed positions (a unit in the list and not dead = the game's cell map);
    // walls from the game's cell map (WALL entries are static: units never stand on walls).  rowsV0 =
    // the helper's own view-0 sight rows (the game wave's snapshots use `vis` meanwhile).  last: the
    // launch's last iteration stores the record's sight rows and pending chunks globally.
    DEV void renderPOPacked(const uint32_t* pk, const uint32_t* ph, uint32_t* rowsV0, uint8_t* hcell, bool last) {
        const int l = (int)threadIdx.x - 64;
        const int NCW = poChunkWords(HW), NC = HW >> 2;
        uint32_t* const rowsV1 = vis2;
        int32_t* pr = D.po_prev ? D.po_prev + (size_t)g * D.po_words : nullptr;
        int32_t* const prG = last ? pr : nullptr;
        const int SW = poSnapWords(CAP);
        const int nuP = (int)ph[0], nu0 = (int)ph[1];
        const uint32_t delta = ph[2] & 3u;
        const bool d0 = delta & 1u, d1 = (delta >> 1) & 1u;
        if (l < 2 * H) {
            rowsV0[l] = 0;
            rowsV1[l] = 0;
        }
        if (l < NCW) {
            poDirty[l] = d0 ? poPend[l] : 0u;
            poDirty[NCW + l] = 0u;
            poDirty[2 * NCW + l] = d1 ? poPend[NCW + l] : 0u;
            poDirty[3 * NCW + l] = 0u;
        }
        for (int i = l; i < HW / 8; i += 64) ((uint2*)hcell)[i] = make_uint2(~0u, ~0u);  // (8-byte aligned)
        const bool live = l < nuP;
        const uint32_t cu = pk[l], kv = pk[64 + l], sw = pk[128 + l];
        const uint32_t lcuP = pk[192 + l], lkeyP = pk[256 + l];
        const uint32_t sb = sw & 0xFFu, lsnapP = (sw >> 8) & 0xFFu;
        const int hv = (int)(int16_t)(kv & 0xFFFFu), rv = (int)(int16_t)(kv >> 16);
        const bool in0 = live && snap_in(sb, 0), in1 = live && snap_in(sb, 1);
        const bool isDead = (cu & UC_DEAD) != 0;
        const bool dead0 = in0 && isDead, dead1 = in1 && isDead;
        const int cc = uy(cu) * W + ux(cu);
        const int own = uplay(cu);
        wsync();
        if (live && !isDead) hcell[cc] = (uint8_t)l;
        {
            const bool pt0 = in0 && own >= 0, pt1 = in1 && own >= 0;
            if (ballot(pt0 || pt1))
                paintDisks2(pt0, own == 0 ? rowsV0 : rowsV0 + H, pt1, own == 1 ? rowsV1 : rowsV1 + H, cu);
        }
        const uint64_t deadM0 = ballot(dead0), deadM1 = ballot(dead1);
        if (pr && dead0) atomicOr(&poDirty[NCW + (cc >> 7)], 1u << ((cc >> 2) & 31));
        if (pr && dead1) atomicOr(&poDirty[3 * NCW + (cc >> 7)], 1u << ((cc >> 2) & 31));
        if (delta && (live || l < nu0)) {
            const int cp = uy(lcuP) * W + ux(lcuP);
            const uint32_t key = (uint32_t)(uint16_t)hv | ((uint32_t)(uint16_t)rv << 16);
#pragma unroll
            for (int v = 0; v < 2; v++) {
                if (!(v ? d1 : d0)) continue;
                const bool in = v ? in1 : in0;
                const bool inP = l < nu0 && ((lsnapP >> v) & 1u);
                bool chg = in != inP;
                if (in && inP)
                    chg = cc != cp || key != lkeyP || snap_act(sb, v) != (int)((lsnapP >> (2 + 3 * v)) & 7u);
                uint32_t* dirty = poDirty + 2 * v * NCW;
                if (chg && inP) atomicOr(&dirty[cp >> 7], 1u << ((cp >> 2) & 31));
                if (chg && in) atomicOr(&dirty[cc >> 7], 1u << ((cc >> 2) & 31));
            }
        }
        wsync();
        if (l < 2 * H) {  // sight rows: changed columns -> chunk bits of that row; the record's copies
            const int y = l < H ? l : l - H;
            const int k0 = y * (W >> 2);
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const uint32_t row = (v ? rowsV1 : rowsV0)[l];
                if (v ? d1 : d0) {
                    const uint32_t d = row ^ poVis[v * 2 * H + l];
                    if (d) {
                        uint32_t gbits = 0;  // bit j = column group 4j..4j+3 changed
#pragma unroll
                        for (int j = 0; j < 8; j++) gbits |= ((d >> (4 * j)) & 0xFu) ? (1u << j) : 0u;
                        uint32_t* dirty = poDirty + 2 * v * NCW;
                        if ((k0 & 31) + (W >> 2) <= 32) {
                            atomicOr(&dirty[k0 >> 5], gbits << (k0 & 31));
                        } else {
                            for (uint32_t gg = gbits; gg; gg &= gg - 1) {
                                const int k = k0 + __builtin_ctz(gg);
                                atomicOr(&dirty[k >> 5], 1u << (k & 31));
                            }
                        }
                    }
                }
                poVis[v * 2 * H + l] = row;  // the record's LDS copy (the next render)
                if (prG) prG[1 + SW + v * 2 * H + l] = (int32_t)row;
            }
        }
        wsync();
        int n = 0;  // (view << 15 | chunk) items: view 0's dirty chunks (all, without delta), then view 1's
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const bool dv = v ? d1 : d0;
            const uint32_t* dirty = poDirty + 2 * v * NCW;
#pragma unroll
            for (int c0 = 0; c0 < 256; c0 += 64) {  // NC <= 256 (H, W <= 32)
                if (c0 < NC) {
                    const int k = c0 + l;
                    const bool dk = k < NC && (!dv || ((dirty[k >> 5] >> (k & 31)) & 1u));
                    const uint64_t m = ballot(dk);
                    if (dk) poList[n + lanes_below(m)] = (uint16_t)((v << 15) | k);
                    n += __popcll(m);
                }
            }
        }
        if (pr && l < NCW) {
            if (prG) {
                prG[1 + SW + 4 * H + l] = (int32_t)poDirty[NCW + l];
                prG[1 + SW + 4 * H + NCW + l] = (int32_t)poDirty[3 * NCW + l];
            }
            poPend[l] = poDirty[NCW + l];
            poPend[NCW + l] = poDirty[3 * NCW + l];
        }
        wsync();
        int32_t* out = D.obs + (size_t)(2 * g) * D.C * HW;
        const __amdgpu_buffer_rsrc_t rs = bufRsrc(out, (uint32_t)(2 * D.C * HW * 4));
        const uint64_t deadAny = deadM0 | deadM1;
#ifdef MRTS_DIAG_HELPER_NORENDER  // diagnostic build only: the helper skips the render items (output wrong)
        n = 0;
#endif
        for (int it = l; it < n; it += 64) {
            const uint32_t e = poList[it];
            const int v = (int)(e >> 15), c4 = (int)(e & 0x7FFFu);  // lane = 4 consecutive cells of one row
            const uint64_t deadM = v ? deadM1 : deadM0;
            const int y = (4 * c4) / W, x0 = (4 * c4) % W;
            const uint32_t* rows = v ? rowsV1 : rowsV0;
            const uint32_t occ4 = ((const uint32_t*)hcell)[c4];
            int cs[4], sl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t o = (occ4 >> (8 * j)) & 0xFFu;
                cs[j] = o != 0xFFu ? (int)o : (cell[4 * c4 + j] == WALL ? (int)WALL : (int)EMPTY);
            }
            const uint32_t mr = rows[y], tr = rows[H + y];
            uint32_t ocu[4], osb[4];
            int ohp[4], ors[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {  // the live occupant's fields (an empty cell reads slot 0, masked)
                const int s = cs[j] < CAP ? cs[j] : 0;
                ocu[j] = pk[s];
                const uint32_t k2 = pk[64 + s];
                osb[j] = pk[128 + s] & 0xFFu;
                ohp[j] = (int)(int16_t)(k2 & 0xFFFFu);
                ors[j] = (int)(int16_t)(k2 >> 16);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) sl[j] = (cs[j] < CAP && snap_in(osb[j], v)) ? cs[j] : -1;
            for (uint64_t m = deadAny; m; m &= m - 1) {  // the view's dead units: a later list position wins
                const int ds = __builtin_ctzll(m);
                // from the pack, not by readlane of an inactive lane (writeObsPOFast): the compiler sank
                // this wave's pack reads (cu, hp | res, snapshot byte) into the divergent item loop, so
                // lane ds's registers held a stale value whenever lane ds had no item (round 4's soak case)
                const uint32_t dcu = pk[ds], dkv = pk[64 + ds];
                const int dcell = uy(dcu) * W + ux(dcu);
                const int dh = (int)(int16_t)(dkv & 0xFFFFu), dr = (int)(int16_t)(dkv >> 16);
                const uint32_t dsb = pk[128 + ds] & 0xFFu;
                const bool mine = (deadM >> ds) & 1ull;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (mine && dcell == 4 * c4 + j && ds > sl[j]) {
                        sl[j] = ds;
                        ocu[j] = dcu;
                        osb[j] = dsb;
                        ohp[j] = dh;
                        ors[j] = dr;
                    }
            }
            int vv[4][8];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool occ = sl[j] >= 0;
                const int pl = uplay(ocu[j]);
                const int sa = snap_act(osb[j], v);
                vv[j][0] = occ ? ohp[j] : 0;
                vv[j][1] = occ ? ors[j] : 0;
                vv[j][2] = (occ && pl >= 0) ? ((pl + v) % 2) + 1 : 0;
                vv[j][3] = occ ? utyp(ocu[j]) + 1 : 0;
                vv[j][4] = (occ && sa) ? sa - 1 : 0;
                vv[j][5] = cs[j] == WALL ? 1 : 0;
                vv[j][6] = (int)((mr >> (x0 + j)) & 1u);
                vv[j][7] = (int)((tr >> (x0 + j)) & 1u);
            }
            const uint32_t base = (uint32_t)(v * D.C * HW + 4 * c4) * 4u;
            if (SC1_POOBS) {
#pragma unroll
                for (int k = 0; k < 8; k++) st4sc1(rs, base + (uint32_t)(k * HW) * 4u, vv[0][k], vv[1][k], vv[2][k], vv[3][k]);
            } else {
                int32_t* o = out + base / 4;
#pragma unroll
                for (int k = 0; k < 8; k++) st4<WT_POOBS>(o + k * HW, vv[0][k], vv[1][k], vv[2][k], vv[3][k]);
            }
        }
        wsync();
    }
    DEV void writeObsPO(int slot, int p, bool delta = false) {
        if ((W & 3) == 0 && W <= 32 && H <= 32 && nu <= 64 && U.maxSight <= 15) {
            writeObsPOFast(slot, p, delta);
            return;
        }
#ifdef MRTS_ABLATE
        if (!ab(AB_PO_NOSCELL))
#endif
        for (int c = lid(); c < HW; c += 64) scell[c] = 0;
        const int NW = H * ((W + 31) >> 5);
        uint32_t* mineRows = vis;
        uint32_t* theirRows = vis + NW;
        for (int i = lid(); i < 2 * NW; i += 64) vis[i] = 0;
        wsync();
        const bool fastPaint = W <= 32 && U.maxSight <= 15;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lid();
            const bool in = o < nu && snap_in(snap[o], p);
            const uint32_t cu = in ? uc[o] : 0u;
            if (in) {
#ifdef MRTS_ABLATE
                if (!ab(AB_PO_NOSCELL))
#endif
                atomicMax(&scell[uy(cu) * W + ux(cu)], (uint32_t)(o + 1));
            }
            // visibility planes over the view's units at their current positions (dead ones
            // included: the view's list still holds them): own / other player's sight disks
#ifdef MRTS_ABLATE
            if (!ab(AB_PO_NOPAINT))
#endif
            {
                const bool painter = in && uplay(cu) >= 0;
                if (fastPaint) {
                    if (ballot(painter)) paintDisks(painter, cu, uplay(cu) == p ? mineRows : theirRows);
                } else if (painter) {
                    paintDisk(uplay(cu) == p ? mineRows : theirRows, cu);
                }
            }
        }
        wsync();
        const int NC = (HW + 3) >> 2, NCW = poChunkWords(HW);
        int n = NC;  // chunks to render: all, or the dirty list (delta maps have HW % 4 == 0)
        if (delta) {
            const int l = lid();
            if (l < NCW) poDirty[l] = poPend[p * NCW + l];
            wsync();
            const int nu0 = hget(H_NU);  // the header holds the loaded unit count until store()
            if (l < nu || l < nu0) {
                const uint32_t cu = l < nu ? uc[l] : 0u;
                const uint32_t sb = l < nu ? (uint32_t)snap[l] : 0u;
                const bool inC = l < nu && snap_in(sb, p), inP = l < nu0 && ((lsnap >> p) & 1u);
                const int cc = uy(cu) * W + ux(cu), cp = uy(lcu) * W + ux(lcu);
                bool chg = inC != inP;
                if (inC && inP) {
                    const uint32_t key = (uint32_t)(uint16_t)hp[l] | ((uint32_t)(uint16_t)res[l] << 16);
                    chg = cc != cp || key != lkey || snap_act(sb, p) != (int)((lsnap >> (2 + 3 * p)) & 7u);
                }
                if (chg && inP) atomicOr(&poDirty[cp >> 7], 1u << ((cp >> 2) & 31));
                if (chg && inC) atomicOr(&poDirty[cc >> 7], 1u << ((cc >> 2) & 31));
            }
            // sight rows (W <= 32: one word per row): changed columns -> chunk bits of that row
            for (int i = l; i < 2 * H; i += 64) {
                const uint32_t d = vis[i] ^ poVis[p * 2 * H + i];
                if (d) {
                    const int y = i < H ? i : i - H;
                    uint32_t g = 0;  // bit j = column group 4j..4j+3 changed
#pragma unroll
                    for (int j = 0; j < 8; j++) g |= ((d >> (4 * j)) & 0xFu) ? (1u << j) : 0u;
                    const int k0 = y * (W >> 2);  // first chunk of row y (W/4 chunks per row, <= 8)
                    if ((k0 & 31) + (W >> 2) <= 32) {
                        atomicOr(&poDirty[k0 >> 5], g << (k0 & 31));
                    } else {
                        for (uint32_t gg = g; gg; gg &= gg - 1) {
                            const int k = k0 + __builtin_ctz(gg);
                            atomicOr(&poDirty[k >> 5], 1u << (k & 31));
                        }
                    }
                }
            }
            wsync();
            n = 0;
            for (int c0 = 0; c0 < NC; c0 += 64) {
                const int k = c0 + l;
                const bool dk = k < NC && ((poDirty[k >> 5] >> (k & 31)) & 1u);
                const uint64_t m = ballot(dk);
                if (dk) poList[n + lanes_below(m)] = (uint16_t)k;
                n += __popcll(m);
            }
            wsync();
        }
        int32_t* out = D.obs + (size_t)slot * D.C * HW;
        for (int it = lid(); it < n; it += 64) {
            const int c4 = delta ? (int)poList[it] : it;  // lane = 4 consecutive cells, dwordx4 per plane
            int sc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) sc[j] = 4 * c4 + j < HW ? (int)scell[4 * c4 + j] - 1 : -1;
            uint32_t cu[4];
            int ch[4], cr[4], ca[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {  // branch-free: an empty cell reads slot 0 and is masked
                const int s = sc[j] >= 0 ? sc[j] : 0;
                cu[j] = uc[s];
                ch[j] = hp[s];
                cr[j] = res[s];
                ca[j] = snap_act(snap[s], p);
            }
            const int cy = (4 * c4) / W, cx0 = (4 * c4) % W;  // W % 4 == 0 here, or one cell per lane below
            int v[4][8];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool occ = sc[j] >= 0;
                const int pl = uplay(cu[j]);
                v[j][0] = occ ? ch[j] : 0;
                v[j][1] = occ ? cr[j] : 0;
                v[j][2] = (occ && pl >= 0) ? ((pl + p) % 2) + 1 : 0;
                v[j][3] = occ ? utyp(cu[j]) + 1 : 0;
                v[j][4] = (occ && ca[j]) ? ca[j] - 1 : 0;
                const bool in = 4 * c4 + j < HW;
                v[j][5] = in && cell[4 * c4 + j] == WALL ? 1 : 0;
                const int x = (W & 3) == 0 ? cx0 + j : (4 * c4 + j) % W, y = (W & 3) == 0 ? cy : (4 * c4 + j) / W;
                v[j][6] = in && seen(mineRows, x, y) ? 1 : 0;
                v[j][7] = in && seen(theirRows, x, y) ? 1 : 0;
            }
            if ((HW & 3) == 0) {
#pragma unroll
                for (int k = 0; k < 8; k++) st4<WT_POOBS>(out + k * HW + 4 * c4, v[0][k], v[1][k], v[2][k], v[3][k]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (4 * c4 + j < HW)
#pragma unroll
                        for (int k = 0; k < 8; k++) out[k * HW + 4 * c4 + j] = v[j][k];
            }
        }
#ifdef MRTS_ABLATE
        if (!ab(AB_PO_NORECORD))
#endif
        if (D.po_prev && poDeltaShape(H, W)) poRecord(p);
    }
    // the PO record of view p for the next write: this render's sight rows and the chunks of its units
    // that died (the compaction removes them before the next render)
    DEV void poRecord(int p) {
        const int l = lid(), NCW = poChunkWords(HW), SW = poSnapWords(CAP);
        int32_t* pr = D.po_prev + (size_t)g * D.po_words;
        for (int i = l; i < 2 * H; i += 64) pr[1 + SW + p * 2 * H + i] = (int32_t)vis[i];
        if (l < NCW) poDirty[l] = 0;
        wsync();
        for (int o = l; o < nu; o += 64) {
            const uint32_t cu = uc[o];
            if ((cu & UC_DEAD) && snap_in(snap[o], p)) {
                const int c = uy(cu) * W + ux(cu);
                atomicOr(&poDirty[c >> 7], 1u << ((c >> 2) & 31));
            }
        }
        wsync();
        if (l < NCW) pr[1 + SW + 4 * H + p * NCW + l] = (int32_t)poDirty[l];
        wsync();
    }
    // after the compaction: the snapshot bytes of the final slots and the views this launch rendered
    DEV void poRecordSnaps(uint32_t views) {
        int32_t* pr = D.po_prev + (size_t)g * D.po_words;
        // a render that kept its record in LDS (poLds) is followed, inside a multi-step launch, by an
        // iteration that reads the LDS copies: the global record is then stored at the last iteration only
        const bool glob = !iter || lastIt || !poLds;
        const uint32_t* sw = (const uint32_t*)snap;
        if (glob)
            for (int w = lid(); w < (nu + 3) / 4; w += 64) pr[1 + w] = (int32_t)sw[w];
        if (lid() == 0) {
            if (glob) pr[0] = (int32_t)views;
            hdr[HX_POVALID] = (int32_t)views;  // the record's LDS copy (multi-step launch)
        }
    }

    // ------------------------------------------------------------------ legal-action masks
    // JNIGridnetClient.getMasks (tests/JNIGridnetClient.java:210-223) + UnitAction.getValidActionArray
    // (rts/UnitAction.java:711-751) over Unit.getUnitActions(gs, 10) (rts/units/Unit.java:382-522).
    // farFromLanes: the range > 1 attack bits are left to farAttackBits (the caller's whole wave)
    DEV void unitMask(int s, uint32_t& w0, uint32_t& w1, uint32_t& w2, bool farFromLanes = false) const {
        uint64_t lo = 0;
        uint32_t hi = 0;
        auto setb = [&](int k) {
            if (k < 64) lo |= 1ull << k;
            else hi |= 1u << (k - 64);
        };
        const uint32_t cu = uc[s];
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const uint32_t fl = U.flags[typ];
        const int nt = NT, ctr = R / 2;
        const int atkBase = 1 + 6 + 16 + nt;
        setb(0);
        setb(1 + T_NONE);
        const bool canProduce = false;
        (void)canProduce;
        bool afford[MAX_PRODUCES];
#pragma unroll
        for (int i = 0; i < MAX_PRODUCES; i++) afford[i] = i < U.nprod[typ] && pres(pl) >= U.cost[U.prod[typ][i]];
        const int carried = res[s];
        const int r = U.range[typ];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int nx = x + dxo(d), ny = y + dyo(d);
            const int n = inb(nx, ny) ? cell[ny * W + nx] : WALL;
            if (n < CAP) {
                const uint32_t oc = uc[n];
                const int op = uplay(oc);
                const uint32_t ofl = U.flags[utyp(oc)];
                if ((fl & F_ATTACK) && r == 1 && op >= 0 && op != pl) {
                    setb(1 + T_ATTACK);
                    setb(atkBase + (ctr + dyo(d)) * R + (ctr + dxo(d)));
                }
                if (fl & F_HARVEST) {
                    if (carried == 0 && (ofl & F_RESOURCE)) {
                        setb(1 + T_HARVEST);
                        setb(1 + 6 + 4 + d);
                    }
                    if (carried > 0 && (ofl & F_STOCKPILE) && op == pl) {
                        setb(1 + T_RETURN);
                        setb(1 + 6 + 8 + d);
                    }
                }
            } else if (n == EMPTY) {
#pragma unroll
                for (int i = 0; i < MAX_PRODUCES; i++)
                    if (afford[i]) {
                        setb(1 + T_PRODUCE);
                        setb(1 + 6 + 12 + d);
                        setb(1 + 6 + 16 + U.prod[typ][i]);
                    }
                if (fl & F_MOVE) {
                    setb(1 + T_MOVE);
                    setb(1 + 6 + d);
                }
            }
        }
        if (!farFromLanes && (fl & F_ATTACK) && r > 1) {
            for (int dy = -r; dy <= r; dy++)
                for (int dx = -r; dx <= r; dx++) {
                    if (dx * dx + dy * dy > r * r || !inb(x + dx, y + dy)) continue;
                    const int n = cell[(y + dy) * W + x + dx];
                    if (n < CAP) {
                        const int op = uplay(uc[n]);
                        if (op >= 0 && op != pl) {
                            setb(1 + T_ATTACK);
                            setb(atkBase + (ctr + dy) * R + (ctr + dx));
                        }
                    }
                }
        }
        w0 = (uint32_t)lo;
        w1 = (uint32_t)(lo >> 32);
        w2 = hi;
    }
    // Wave-uniform per-type bit sets for maskBitsFast (bit t = unit type t has the property), the
    // produce lists as 8-bit type sets (type t's set in bits 8t..8t+7; mask bits ignore list order)
    // and, per player, the types whose cost the player's current resources cover.
    struct MaskTables {
        uint32_t attack1, attackFar, harvest, move, resource, stockpile, aff0, aff1;
        uint64_t prod;
    };
    DEV MaskTables maskTables() const {
        // the constant sets come with the unit-type table (host-computed, DevUtt::mt*); only the
        // affordability sets depend on the step (the players' resources now)
        const int t = lid();
        const bool ok = t < NT;
        const int cost = ok ? U.cost[t] : 0;
        MaskTables T;
        T.attack1 = uniu(U.mtAttack1);
        T.attackFar = uniu(U.mtAttackFar);
        T.harvest = uniu(U.mtHarvest);
        T.move = uniu(U.mtMove);
        T.resource = uniu(U.mtResource);
        T.stockpile = uniu(U.mtStockpile);
        T.prod = (uint64_t)uniu(U.mtProdLo) | ((uint64_t)uniu(U.mtProdHi) << 32);
        T.aff0 = (uint32_t)ballot(ok && pres0 >= cost);
        T.aff1 = (uint32_t)ballot(ok && pres1 >= cost);
        return T;
    }
    // unitMask's bits for range <= 1 units (the range > 1 attack window: farAttackBits) from the
    // tables: two LDS rounds (the 4 neighbour cells, then the units on them) instead of a dependent
    // read chain per neighbour and produce-list entry.  cu = the unit's core word, carried = its
    // resources.  Same bits as unitMask(s, ..., true).
    DEV void maskBitsFast(const MaskTables& T, uint32_t cu, int carried, uint32_t& w0, uint32_t& w1, uint32_t& w2) const {
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const int ctr = R / 2, atkBase = 1 + 6 + 16 + NT;
        int n[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int nx = x + dxo(d), ny = y + dyo(d);
            n[d] = inb(nx, ny) ? cell[ny * W + nx] : WALL;
        }
        uint32_t oc[4];
#pragma unroll
        for (int d = 0; d < 4; d++) oc[d] = n[d] < CAP ? uc[n[d]] : 0u;
        const bool atk = (T.attack1 >> typ) & 1u, harv = (T.harvest >> typ) & 1u, mov = (T.move >> typ) & 1u;
        const uint32_t canProd = (uint32_t)(T.prod >> (8 * typ)) & 0xFFu & (pl == 0 ? T.aff0 : T.aff1);
        uint64_t lo = 1ull | (1ull << (1 + T_NONE));
        uint32_t hi = 0;
        auto setb = [&](int k) {
            if (k < 64) lo |= 1ull << k;
            else hi |= 1u << (k - 64);
        };
#pragma unroll
        for (int d = 0; d < 4; d++) {
            if (n[d] < CAP) {
                const int op = uplay(oc[d]), ot = utyp(oc[d]);
                if (atk && op >= 0 && op != pl) {
                    setb(1 + T_ATTACK);
                    setb(atkBase + (ctr + dyo(d)) * R + (ctr + dxo(d)));
                }
                if (harv && carried == 0 && ((T.resource >> ot) & 1u)) {
                    setb(1 + T_HARVEST);
                    setb(1 + 6 + 4 + d);
                }
                if (harv && carried > 0 && ((T.stockpile >> ot) & 1u) && op == pl) {
                    setb(1 + T_RETURN);
                    setb(1 + 6 + 8 + d);
                }
            } else if (n[d] == EMPTY) {
                if (canProd) {
                    setb(1 + T_PRODUCE);
                    setb(1 + 6 + 12 + d);
                }
                if (mov) {
                    setb(1 + T_MOVE);
                    setb(1 + 6 + d);
                }
            }
        }
        // produce-type bits 23 + ut (below 64 for any table with <= 8 types)
        if (canProd && (n[0] == EMPTY || n[1] == EMPTY || n[2] == EMPTY || n[3] == EMPTY)) lo |= (uint64_t)canProd << (1 + 6 + 16);
        w0 = (uint32_t)lo;
        w1 = (uint32_t)(lo >> 32);
        w2 = hi;
    }
    // maskBitsFast's bits of ONE direction d (the lane of a quad that computes d; VERDICT r5 #4: the per-idle-unit
    // phases spread over lanes so that their instruction count falls): the unit-type and NONE bits, and what the
    // neighbour cell d holds — an enemy (range-1 attack), a resource (harvest), an own stockpile (return), an empty
    // cell (produce direction, move).  The quad's OR of its four results is maskBitsFast's, but for the produce-type
    // bits, which the caller adds once the OR shows a free cell (they need any of the four).  Every bit below the
    // attack window is in w0 (slot 1 + 6 + 12 + 3 = 22 < 32).
    DEV void maskBitsDir(const MaskTables& T, uint32_t cu, int carried, int d, uint32_t& w0, uint32_t& w1,
                         uint32_t& w2) const {
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const int ctr = R / 2, atkBase = 1 + 6 + 16 + NT;
        const int ddx = dxo(d), ddy = dyo(d), nx = x + ddx, ny = y + ddy;
        const int n = inb(nx, ny) ? cell[ny * W + nx] : WALL;
        const uint32_t oc = n < CAP ? uc[n] : 0u;
        const bool atk = (T.attack1 >> typ) & 1u, harv = (T.harvest >> typ) & 1u, mov = (T.move >> typ) & 1u;
        const uint32_t canProd = (uint32_t)(T.prod >> (8 * typ)) & 0xFFu & (pl == 0 ? T.aff0 : T.aff1);
        uint32_t lo = 1u | (1u << (1 + T_NONE)), mid = 0, hi = 0;
        if (n < CAP) {
            const int op = uplay(oc), ot = utyp(oc);
            if (atk && op >= 0 && op != pl) {
                lo |= 1u << (1 + T_ATTACK);
                const int k = atkBase + (ctr + ddy) * R + (ctr + ddx);
                if (k < 32) lo |= 1u << k;
                else if (k < 64) mid |= 1u << (k - 32);
                else hi |= 1u << (k - 64);
            }
            if (harv && carried == 0 && ((T.resource >> ot) & 1u)) lo |= (1u << (1 + T_HARVEST)) | (1u << (1 + 6 + 4 + d));
            if (harv && carried > 0 && ((T.stockpile >> ot) & 1u) && op == pl) lo |= (1u << (1 + T_RETURN)) | (1u << (1 + 6 + 8 + d));
        } else if (n == EMPTY) {
            if (canProd) lo |= (1u << (1 + T_PRODUCE)) | (1u << (1 + 6 + 12 + d));
            if (mov) lo |= (1u << (1 + T_MOVE)) | (1u << (1 + 6 + d));
        }
        w0 = lo;
        w1 = mid;
        w2 = hi;
    }
    // farAttackRows for the quad lane of direction d: its rows dy = d - ctr and d - ctr + 4 of the 2 ctr + 1 <= 7
    // (attack range <= 3: K <= 80), the same bits; the whole wave calls it
    DEV void farAttackRowsDir(bool far, uint32_t cu, int d, const uint32_t* rows, uint32_t& w0, uint32_t& w1,
                              uint32_t& w2) const {
        if (!ballot(far)) return;
        const int x = ux(cu), y = uy(cu), pl = uplay(cu);
        const int r = far ? U.range[utyp(cu)] : 0, ctr = R / 2, atkBase = 1 + 6 + 16 + NT;
        const uint32_t* er = rows + (far ? (1 - pl) * H : 0);
        uint64_t lo = 0;
        uint32_t hi = 0;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int dy = d - ctr + 4 * j, yy = y + dy;
            if (!far || dy > ctr || dy < -r || dy > r || yy < 0 || yy >= H) continue;
            const uint64_t word = er[yy];
            uint64_t win = x >= r ? (word >> (x - r)) : (word << (r - x));  // bit j = column x - r + j
            // the disk's columns of row dy: |dx| <= half, half^2 + dy^2 <= r^2
            int half = 0;
            while (half < r && (half + 1) * (half + 1) + dy * dy <= r * r) half++;
            win &= ((2ull << (2 * half)) - 1ull) << (r - half);
            if (!win) continue;
            const int base = atkBase + (ctr + dy) * R + (ctr - r);
            if (base < 64) {
                lo |= win << base;
                if (base > 0) hi |= (uint32_t)(win >> (64 - base));
            } else {
                hi |= (uint32_t)(win << (base - 64));
            }
            lo |= 1ull << (1 + T_ATTACK);
        }
        w0 |= (uint32_t)lo;
        w1 |= (uint32_t)(lo >> 32);
        w2 |= hi;
    }
    static DEV uint32_t quadOr(uint32_t v) {  // OR over the lane's quad (DPP quad_perm; whole wave)
        LANE_AUDIT_WAVE(2);
        v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        return v;
    }
    // maskBitsFast + farAttackRows of every idle unit (si >= 0), four lanes per unit: the units' words go to LDS
    // in rank order (16 per pass), lane 4 q + d computes direction d (and rows d - ctr, d - ctr + 4 of the
    // ranged window) of unit q, the quad ORs its words, and the unit's own lane reads them back — the same bits
    // as one lane per unit, in about a quarter of the instructions.  rows complete (wsync'd);
    // rseq words 16..63 are scratch here.  Whole wave.
    DEV void maskBitsQuads(const MaskTables& T, int si, uint32_t cu, int carried, const uint32_t* rows, uint32_t& w0,
                           uint32_t& w1, uint32_t& w2, uint32_t* qb /* [16][3] scratch words */) {
        const int l = lid();
        const uint64_t m = ballot(si >= 0);
        const int RI = __popcll(m), r = lanes_below(m);
        const int q = l >> 2, d = l & 3;
        for (int p0 = 0; p0 < RI; p0 += 16) {
            const bool mine = si >= 0 && r >= p0 && r < p0 + 16;
            if (mine) {
                qb[3 * (r - p0)] = cu;
                qb[3 * (r - p0) + 1] = (uint32_t)carried;
            }
            wsync();
            const bool qa = p0 + q < RI;
            uint32_t qcu = 0, v0 = 0, v1 = 0, v2 = 0;
            if (qa) {
                qcu = qb[3 * q];
                maskBitsDir(T, qcu, (int)qb[3 * q + 1], d, v0, v1, v2);
            }
            farAttackRowsDir(qa && ((T.attackFar >> utyp(qcu)) & 1u), qcu, d, rows, v0, v1, v2);
            v0 = quadOr(v0);
            v1 = quadOr(v1);
            v2 = quadOr(v2);
            // produce-type bits 23 + ut, when a direction of the quad found a free cell (produce direction bits)
            const uint32_t canProd =
                (uint32_t)(T.prod >> (8 * utyp(qcu))) & 0xFFu & (uplay(qcu) == 0 ? T.aff0 : T.aff1);
            if (((v0 >> (1 + 6 + 12)) & 0xFu) != 0u) v0 |= canProd << (1 + 6 + 16);
            wsync();  // every lane of a quad has read its entry
            if (qa && d == 0) {
                qb[3 * q] = v0;
                qb[3 * q + 1] = v1;
                qb[3 * q + 2] = v2;
            }
            wsync();
            if (mine) {
                w0 = qb[3 * (r - p0)];
                w1 = qb[3 * (r - p0) + 1];
                w2 = qb[3 * (r - p0) + 2];
            }
            wsync();  // read before the next pass rewrites the entries
        }
    }
    // The range > 1 attack bits of unitMask (Unit.java:424-434: every enemy unit within the disk) for
    // lanes with far = true, from the unit list held one unit per lane (cuLane = unit core word of
    // lane j, all units in one wave, none dead): one pass over the live owned units instead of a
    // (2r+1)^2 cell scan per ranged unit — the same set, as a cell holds at most one unit.  Whole wave.
    DEV void farAttackBits(bool far, uint32_t cu, uint32_t cuLane, uint64_t owned, uint32_t& w0, uint32_t& w1,
                           uint32_t& w2) const {
        if (!ballot(far)) return;
        const int x = ux(cu), y = uy(cu), pl = uplay(cu);
        const int r = far ? U.range[utyp(cu)] : 0, ctr = R / 2, atkBase = 1 + 6 + 16 + NT;
        uint64_t lo = 0;
        uint32_t hi = 0;
        for (uint64_t m = owned; m; m &= m - 1) {
            const uint32_t cj = uniu((uint32_t)rl((int)cuLane, __builtin_ctzll(m)));
            const int dx = ux(cj) - x, dy = uy(cj) - y;
            if (far && uplay(cj) != pl && dx * dx + dy * dy <= r * r) {
                const int k = atkBase + (ctr + dy) * R + (ctr + dx);
                if (k < 64) lo |= 1ull << k;
                else hi |= 1u << (k - 64);
                lo |= 1ull << (1 + T_ATTACK);
            }
        }
        w0 |= (uint32_t)lo;
        w1 |= (uint32_t)(lo >> 32);
        w2 |= hi;
    }
    // farAttackBits from per-player unit row bitmaps (rows[p * H + y] bit x = a unit of player p at
    // (x, y); W <= 32): each far lane reads the 2r + 1 enemy rows around it and keeps the bits inside
    // the disk.  Whole wave; rows complete (after a wsync).
    DEV void farAttackRows(bool far, uint32_t cu, const uint32_t* rows, uint32_t& w0, uint32_t& w1, uint32_t& w2) const {
        if (!ballot(far)) return;
        const int x = ux(cu), y = uy(cu), pl = uplay(cu);
        const int r = far ? U.range[utyp(cu)] : 0, ctr = R / 2, atkBase = 1 + 6 + 16 + NT;
        const uint32_t* er = rows + (far ? (1 - pl) * H : 0);
        uint64_t lo = 0;
        uint32_t hi = 0;
#pragma unroll
        for (int dy = -ctr; dy <= ctr; dy++) {
            const int yy = y + dy;
            if (!far || dy < -r || dy > r || yy < 0 || yy >= H) continue;
            const uint64_t word = er[yy];
            uint64_t win = x >= r ? (word >> (x - r)) : (word << (r - x));  // bit j = column x - r + j
            uint64_t disk = 0;
#pragma unroll
            for (int j = 0; j <= 2 * ctr; j++)
                if (j <= 2 * r && (j - r) * (j - r) + dy * dy <= r * r) disk |= 1ull << j;
            win &= disk;
            if (!win) continue;
            const int base = atkBase + (ctr + dy) * R + (ctr - r);
            if (base < 64) {
                lo |= win << base;
                if (base > 0) hi |= (uint32_t)(win >> (64 - base));
            } else {
                hi |= (uint32_t)(win << (base - 64));
            }
            lo |= 1ull << (1 + T_ATTACK);
        }
        w0 |= (uint32_t)lo;
        w1 |= (uint32_t)(lo >> 32);
        w2 |= hi;
    }
    // Park each idle unit's 79-bit mask in its unused assignment words (at/as/ua low bits).
    // pset: bit p = park the masks of player p's idle units (both players in one pass for self-play)
    DEV void stashMasks(int pset) {
        for (int o = lid(); o < nu; o += 64) {
            const uint32_t c = uc[o];
            const int op = uplay(c);
            if ((c & UC_DEAD) || op < 0 || !((pset >> op) & 1) || (ua[o] & UA_PRESENT)) continue;
            uint32_t w0, w1, w2;
            unitMask(o, w0, w1, w2);
            at[o] = (int32_t)w0;
            as[o] = (int32_t)w1;
            ua[o] = w2 & 0xFFFFu;
        }
    }
    DEV void cellMaskBits(int c, int p, uint64_t& lo, uint32_t& hi) const {
        lo = 0;
        hi = 0;
        if (c >= HW) return;
        const int s = cell[c];
        if (s < CAP && uplay(uc[s]) == p && !(ua[s] & UA_PRESENT)) {
            lo = (uint64_t)(uint32_t)at[s] | ((uint64_t)(uint32_t)as[s] << 32);
            hi = ua[s] & 0xFFFFu;
        }
    }
    static DEV uint32_t bits16(uint64_t lo, uint32_t hi, int k) {  // bits k..k+15 of a 96-bit vector
        uint64_t v;
        if (k == 0) v = lo;
        else if (k < 64) v = (lo >> k) | ((uint64_t)hi << (64 - k));
        else v = (uint64_t)hi >> (k - 64);
        return (uint32_t)v & 0xFFFFu;
    }
    static DEV uint32_t expand4(uint32_t b) { return ((b & 0xFu) * 0x00204081u) & 0x01010101u; }
    // one 16-byte chunk j of the [HW][K] byte mask of player p, from the parked per-unit bits
    DEV uint4 maskChunk(int j, int p) const {
        const int o0 = 16 * j;
        const int cA = o0 / K, kA = o0 - cA * K;
        uint64_t lo;
        uint32_t hi;
        cellMaskBits(cA, p, lo, hi);
        uint32_t b = bits16(lo, hi, kA);
        const int nA = K - kA;
        if (nA < 16) {
            b &= (1u << nA) - 1u;
            cellMaskBits(cA + 1, p, lo, hi);
            b |= (bits16(lo, hi, 0) << nA) & 0xFFFFu;
        }
        uint4 v;
        v.x = expand4(b);
        v.y = expand4(b >> 4);
        v.z = expand4(b >> 8);
        v.w = expand4(b >> 12);
        return v;
    }
    DEV bool ownIdleAt(int c, int p) const {
        const int s = c < HW ? cell[c] : EMPTY;
        return s < CAP && uplay(uc[s]) == p && !(ua[s] & UA_PRESENT);
    }
    // The mask rows of the game's external slots (slot0 + i is player pl[i]'s view).  Full mode writes
    // all H*W*K bytes per slot; delta mode (the buffer holds this handle's previous masks) rewrites
    // only the 16-byte chunks overlapping a cell that has, or had at the previous write, an own idle
    // unit — the buffer ends up identical.  The dirty cells of both slots are gathered into one list
    // and their chunks are spread over the lanes, so a typical step is a single parallel pass.
    DEV void writeMasks(int slot0, int nslots, int pl0, int pl1) {
        const int total = HW * K;
        const int MW = maskWords(HW);
        const bool delta = D.mask_delta && (total & 15) == 0;
        uint32_t* pg = prevG();
        const int l = lid();
        if (delta && nu <= 64 && nslots * MW <= 64 && writeMasksUnits(slot0, nslots, pl0, pl1)) return;
        int nlist = 0;
        for (int i = 0; i < nslots; i++) {
            const int p = i ? pl1 : pl0;
            const int slot = slot0 + i;
            for (int c0 = 0; c0 < HW; c0 += 64) {
                const uint64_t m = ballot(ownIdleAt(c0 + l, p));
                const int w = c0 >> 5;
                const uint32_t mine = l == 0 ? (uint32_t)m : (uint32_t)(m >> 32);
                if (l < 2 && w + l < MW) {
                    if (D.source) D.source[(size_t)slot * MW + w + l] = mine;
                    if (lastIt) pg[p * MW + w + l] = mine;
                }
                if (delta) {
                    const uint64_t old = (uint64_t)mprev[p * MW + w] | (w + 1 < MW ? (uint64_t)mprev[p * MW + w + 1] << 32 : 0ull);
                    const uint64_t dirty = old | m;
                    const int n = __popcll(dirty);
                    if (n) {
                        if (nlist + n > 64) {
                            flushDirty(nlist, slot0, pl0, pl1);
                            nlist = 0;
                        }
                        if ((dirty >> l) & 1ull) rslot[nlist + lanes_below(dirty)] = (uint16_t)((i << 15) | (c0 + l));
                        nlist += n;
                    }
                }
                if (l < 2 && w + l < MW) mprev[p * MW + w + l] = mine;  // after the read: a multi-step launch's next base
            }
        }
        MPHASE(11);
        if (delta) {
            if (nlist) flushDirty(nlist, slot0, pl0, pl1);
            return;
        }
        for (int i = 0; i < nslots; i++) {
            const int p = i ? pl1 : pl0;
            uint8_t* out = D.masks + (size_t)(slot0 + i) * total;
            if ((total & 15) == 0) {
                for (int j = l; j < total / 16; j += 64) {
                    const uint4 v = maskChunk(j, p);
                    st4<WT_FULLMASK>(out + 16 * j, (int)v.x, (int)v.y, (int)v.z, (int)v.w);
                }
            } else {
                for (int o = l; o < total; o += 64) {
                    const int c = o / K, k = o - c * K;
                    uint64_t lo;
                    uint32_t hi;
                    cellMaskBits(c, p, lo, hi);
                    out[o] = (uint8_t)(k < 64 ? ((lo >> k) & 1u) : ((hi >> (k - 64)) & 1u));
                }
            }
        }
    }
    // Delta form with all units in one wave: the new row sets come from the units (one atomicOr per
    // idle unit), old|new per bit word gives the dirty cells, and a wave prefix sum lists them.
    // Returns false (nothing written) when the list would exceed 64 cells.
    DEV bool writeMasksUnits(int slot0, int nslots, int pl0, int pl1) {
        const int MW = maskWords(HW), NW = nslots * MW;
        const int l = lid();
        uint32_t* nb = (uint32_t*)rseq;  // cycle() scratch, free here: [slot i][MW] new bits
        if (l < NW) nb[l] = 0;
        wsync();
        if (l < nu) {
            const uint32_t cu = uc[l];
            if (!(cu & UC_DEAD) && !(ua[l] & UA_PRESENT)) {
                const int op = uplay(cu), c = uy(cu) * W + ux(cu);
                if (op >= 0 && op == pl0) atomicOr(&nb[c >> 5], 1u << (c & 31));
                if (nslots > 1 && op >= 0 && op == pl1) atomicOr(&nb[MW + (c >> 5)], 1u << (c & 31));
            }
        }
        wsync();
        uint32_t cur = 0, old = 0;
        int i = 0, w = 0;
        if (l < NW) {
            i = l >= MW;
            w = l - i * MW;
            cur = nb[l];
            old = mprev[(i ? pl1 : pl0) * MW + w];
        }
        const uint32_t dirty = cur | old;
        const int n = __popc(dirty);
        const int incl = wave_incl_sum(n);
        const int total = rl(incl, 63);
        if (total > 64) return false;
        if (l < NW) {
            if (D.source) D.source[(size_t)(slot0 + i) * MW + w] = cur;
            if (lastIt) prevG()[(i ? pl1 : pl0) * MW + w] = cur;  // the next launch's copy
            mprev[(i ? pl1 : pl0) * MW + w] = cur;
        }
        if (total == 0) return true;
        int k = incl - n;
        for (uint32_t d = dirty; d; d &= d - 1) rslot[k++] = (uint16_t)((i << 15) | (32 * w + __builtin_ctz(d)));
        flushDirty(total, slot0, pl0, pl1);
        return true;
    }
    // One cell's K-byte mask record (byte k = bit k of lo:hi) at dst, byte-exact: up to 3 head bytes to
    // reach dword alignment, whole dwords (dwordx4 / dwordx3 stores, 4-byte aligned), then the tail
    // bytes — neighbouring records written by other lanes are never touched.
    // storeRecord as write-through (`sc1`) buffer stores (SC1_MASK): byte offset `off` into the raw
    // buffer `r` whose base address is `base`
    DEV void storeRecordSc1(__amdgpu_buffer_rsrc_t r, const uint8_t* base, uint32_t off, uint64_t lo, uint32_t hi) const {
        const int head = (int)((4u - (((uint32_t)(uintptr_t)base + off) & 3u)) & 3u);
#pragma unroll
        for (int i = 0; i < 3; i++)
            if (i < head) __builtin_amdgcn_raw_buffer_store_b8((char)((lo >> i) & 1u), r, (int)(off + i), 0, 16);
        const uint64_t sl = (lo >> head) | (head ? ((uint64_t)hi << (64 - head)) : 0ull);
        const uint32_t sh = hi >> head;
        const uint32_t v[3] = {(uint32_t)sl, (uint32_t)(sl >> 32), sh};
        const int nd = (K - head) >> 2;
        const uint32_t dwo = off + (uint32_t)head;
        auto nib = [&](int k) -> int { return (int)expand4(v[k >> 3] >> (4 * (k & 7))); };
        if (K == 79) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const i32x4v w = {nib(4 * q), nib(4 * q + 1), nib(4 * q + 2), nib(4 * q + 3)};
                __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(dwo + 16 * q), 0, 16);
            }
            typedef int32_t i32x3v __attribute__((ext_vector_type(3)));
            const i32x3v w3 = {nib(16), nib(17), nib(18)};
            __builtin_amdgcn_raw_buffer_store_b96(w3, r, (int)(dwo + 64), 0, 16);
        } else {
            for (int k = 0; k < nd; k++) __builtin_amdgcn_raw_buffer_store_b32(nib(k), r, (int)(dwo + 4 * k), 0, 16);
        }
        const int t0 = head + 4 * nd;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int b = t0 + i;
            if (b < K)
                __builtin_amdgcn_raw_buffer_store_b8((char)((b < 64 ? (lo >> b) : (uint64_t)(hi >> (b - 64))) & 1u), r,
                                                     (int)(off + b), 0, 16);
        }
    }
    DEV void storeRecord(uint8_t* dst, uint64_t lo, uint32_t hi) const {
        const int head = (int)((4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u);
#pragma unroll
        for (int i = 0; i < 3; i++)
            if (i < head) dst[i] = (uint8_t)((lo >> i) & 1u);
        // bits head.. as a 96-bit value v0:v1:v2
        const uint64_t sl = (lo >> head) | (head ? ((uint64_t)hi << (64 - head)) : 0ull);
        const uint32_t sh = hi >> head;
        const uint32_t v[3] = {(uint32_t)sl, (uint32_t)(sl >> 32), sh};
        const int nd = (K - head) >> 2;  // whole dwords
        uint32_t* dw = (uint32_t*)(dst + head);
        auto nib = [&](int k) -> uint32_t { return expand4(v[k >> 3] >> (4 * (k & 7))); };
        if (K == 79) {  // nd == 19 for every head
#pragma unroll
            for (int q = 0; q < 4; q++) {
                st4u<WT_MASK>(dw + 4 * q, (int)nib(4 * q), (int)nib(4 * q + 1), (int)nib(4 * q + 2), (int)nib(4 * q + 3));
            }
            st3u<WT_MASK>(dw + 16, (int)nib(16), (int)nib(17), (int)nib(18));
        } else {
            for (int k = 0; k < nd; k++) dw[k] = nib(k);
        }
        const int t0 = head + 4 * nd;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int b = t0 + i;
            if (b < K) dst[b] = (uint8_t)((b < 64 ? (lo >> b) : (uint64_t)(hi >> (b - 64))) & 1u);
        }
    }
    // The K = 79 mask records of the lanes with si >= 0 (slot index si, cell c, mask bits w0:w1:w2) stored
    // lane-parallel: the records are listed in LDS (rseq words 16..63, 12 records of 4 words), then five lanes
    // store each record — lanes 0..3 of it 16 bytes each, lane 4 the last 12 — from the record's 16-bit
    // field at their offset (byte k = bit k, expand4), and lanes 0..2 one of its 3 head / tail bytes each.
    // The record's bytes are storeRecord's; a lane storing its own record (storeRecord) spent ~85 VALU
    // instructions on it, all of which the other lanes waited through (round 5: ~35 for 12 records).
    // `mrs` covers the game's records from `mbase`; the caller's rseq words 0..15 are not touched.
    DEV void storeRecordsLanes(int si, int c, uint32_t w0, uint32_t w1, uint32_t w2, __amdgpu_buffer_rsrc_t mrs,
                               const uint8_t* mbase, int total) const {
        const uint64_t m = ballot(si >= 0);
        const int R = __popcll(m);
        if (R == 0) return;
        const int l = lid();
        const int r = lanes_below(m);
        uint32_t* rb = (uint32_t*)rseq + 16;
        const int tr = (l * 13) >> 6, q = l - 5 * tr;  // record tr of a pass, its part q (lanes 0..59)
        const int sel = q >> 1;                         // words sel, sel + 1 hold the part's bits
        const uint32_t mbLo = (uint32_t)(uintptr_t)mbase;
        for (int p0 = 0; p0 < R; p0 += 12) {
            if (si >= 0 && r >= p0 && r < p0 + 12) {
                uint32_t* e = rb + 4 * (r - p0);
                e[0] = w0;
                e[1] = w1;
                e[2] = w2;
                e[3] = ((uint32_t)si << 16) | (uint32_t)c;
            }
            wsync();
            if (l < 60 && p0 + tr < R) {
                const uint32_t* e = rb + 4 * tr;
                const uint32_t lo = e[sel], hi = e[sel + 1], meta = e[3];
                const uint32_t s = (meta >> 16) * (uint32_t)total + (meta & 0xFFFFu) * 79u;
                const uint32_t h = (0u - (mbLo + s)) & 3u;  // head bytes before the first aligned dword
                // bits h + 16 q .. + 15 of the record: the low half of the funnel shift of (hi:lo)
                const uint32_t x = __builtin_amdgcn_alignbit(hi, lo, h + 16u * (uint32_t)(q & 1));
                const int d0 = (int)expand4(x), d1 = (int)expand4(x >> 4), d2 = (int)expand4(x >> 8),
                          d3 = (int)expand4(x >> 12);
                const int off = (int)(s + h) + 16 * q;
                if (q < 4) {
                    const i32x4v v = {d0, d1, d2, d3};
                    __builtin_amdgcn_raw_buffer_store_b128(v, mrs, off, 0, SC1_MASK ? 16 : 0);
                } else {
                    typedef int32_t i32x3v __attribute__((ext_vector_type(3)));
                    const i32x3v v = {d0, d1, d2};
                    __builtin_amdgcn_raw_buffer_store_b96(v, mrs, off, 0, SC1_MASK ? 16 : 0);
                }
                if (q < 3) {  // byte q of the 3 outside the 19 dwords: head byte q, else tail byte 76 + q
                    const bool head = (uint32_t)q < h;
                    const uint32_t b = head ? (uint32_t)q : 76u + (uint32_t)q;
                    const uint32_t v = ((head ? e[0] : (e[2] >> 12)) >> q) & 1u;
                    __builtin_amdgcn_raw_buffer_store_b8((char)v, mrs, (int)(s + b), 0, SC1_MASK ? 16 : 0);
                }
            }
            wsync();
        }
    }
    // Delta mask writes with every unit in one wave (nu <= 64, K <= 96): each own idle unit's lane
    // computes its Unit.getUnitActions mask bits in registers and stores its whole record (and, fused
    // policy, its action row) itself; cells that held an idle unit at the previous write and hold none
    // now get a zero record (and a zero row).  Same buffer contents as stashMasks + writeMasks.
    DEV void writeMasksLanes(int slot0, int nslots, int pl0, int pl1) {
        const int MW = maskWords(HW), NW = nslots * MW;
        const int l = lid();
        const int total = HW * K;
        uint32_t* nb = (uint32_t*)rseq;  // cycle() scratch, free here: [slot i][MW] new bits
        if (l < NW) nb[l] = 0;
        // per-player unit row bitmaps for the range > 1 attack bits (rslot scratch, free here)
        // (partially observable games on maps of 16 to 32 columns: in the tail of `scell`, free during the masks —
        // the general render's scratch map is done with, and a helper wave's packs and cell map end at word 896 of
        // 32x32's 1,024 (round 6: c5's ranged units had taken farAttackBits' walk over every live unit))
        const bool rowS = W <= 32 && 2 * H <= 32;
        const bool rowP = MRTS_PO_ROWS && !rowS && po && W <= 32 && W >= 16 && 2 * H <= 64;
        uint32_t* rows = rowS ? (uint32_t*)rslot : rowP ? scell + (HW - 2 * H) : nullptr;
        const bool rowB = rowS || rowP;
        if (rowB && l < 2 * H) rows[l] = 0;
        int si = -1;  // slot index of this lane's unit record, -1 = none
        uint32_t cu = 0;
        if (l < nu) {
            cu = uc[l];
            if (!(cu & UC_DEAD) && !(ua[l] & UA_PRESENT)) {
                const int op = uplay(cu);
                if (op >= 0 && op == pl0) si = 0;
                else if (nslots > 1 && op >= 0 && op == pl1) si = 1;
            }
        }
        const int c = uy(cu) * W + ux(cu);
        wsync();
        if (si >= 0) atomicOr(&nb[si * MW + (c >> 5)], 1u << (c & 31));
        if (rowB && l < nu && !(cu & UC_DEAD) && uplay(cu) >= 0) atomicOr(&rows[uplay(cu) * H + uy(cu)], 1u << ux(cu));
        uint32_t w0 = 0, w1 = 0, w2 = 0;
        {
            MPHASE(16);
            const MaskTables T = maskTables();
#ifdef MRTS_ABLATE
            if (ab(AB_TABLES)) {
                const MaskTables T2 = maskTables();
                keepv(T2.attack1 ^ T2.attackFar ^ T2.harvest ^ T2.move ^ T2.resource ^ T2.stockpile ^ T2.aff0 ^ T2.aff1 ^
                      (uint32_t)T2.prod);
            }
#endif
            MPHASE(17);
            const int carried = l < nu ? res[l] : 0;
            // four lanes per idle unit wherever the row bitmaps exist: its 48 scratch words are rseq words 16..63
            // while the new row sets nb take <= 16 words, else (32x32 views) the 48 words of scell's tail below
            // the rows (past a helper wave's packs and cell map, which end at word 896 of 1,024)
            uint32_t* const qb = NW <= 16 ? (uint32_t*)rseq + 16 : (rowP && HW - 2 * H - 48 >= 896) ? rows - 48 : nullptr;
            if (MRTS_MASK_QUADS && rowB && qb && (MRTS_QUADS_PO || !po)) {
                wsync();
                maskBitsQuads(T, si, cu, carried, rows, w0, w1, w2, qb);
            } else {
            if (si >= 0) maskBitsFast(T, cu, carried, w0, w1, w2);
            MPHASE(18);
            const bool far = si >= 0 && ((T.attackFar >> utyp(cu)) & 1u);
            if (rowB) {
                wsync();
                farAttackRows(far, cu, rows, w0, w1, w2);
            } else {
                farAttackBits(far, cu, cu, ballot(l < nu && !(cu & UC_DEAD) && uplay(cu) >= 0), w0, w1, w2);
            }
            }
#ifdef MRTS_ABLATE
            if (ab(AB_MASKBITS) && rowB) {  // a second copy of whichever form ran above
                uint32_t v0 = 0, v1 = 0, v2 = 0;
                const uint32_t cu2 = launder(cu);
                if (MRTS_MASK_QUADS && qb && (MRTS_QUADS_PO || !po)) {
                    wsync();
                    maskBitsQuads(T, launder(si), cu2, launder(carried), rows, v0, v1, v2, qb);
                } else {
                    if (si >= 0) maskBitsFast(T, cu2, launder(carried), v0, v1, v2);
                    farAttackRows(si >= 0 && ((T.attackFar >> utyp(cu2)) & 1u), cu2, rows, v0, v1, v2);
                }
                keepv(v0 ^ v1 ^ v2);
            }
#endif
            MPHASE(19);
        }
        wsync();
        MPHASE(12);
        uint32_t cur = 0, old = 0;
        int i = 0, w = 0;
        if (l < NW) {
            i = l >= MW;
            w = l - i * MW;
            cur = nb[l];
            old = mprev[(i ? pl1 : pl0) * MW + w];
            if (D.source) D.source[(size_t)(slot0 + i) * MW + w] = cur;
            if (lastIt) prevG()[(i ? pl1 : pl0) * MW + w] = cur;  // the next launch's copy
            mprev[(i ? pl1 : pl0) * MW + w] = cur;  // the next iteration's base (multi-step launch)
        }
        const bool pol = D.pol_actions && D.pol_delta;
        // forward the sampled rows of a self-play game (read by selfPlayFast next launch); K - 23 - NT
        // attack slots fit packFwd's 7-bit field
        const bool fwdW = pol && nslots == 2 && K - 23 - NT <= 126;
        const uint8_t* mbase = D.masks + (size_t)slot0 * total;  // this game's records (SC1_MASK buffer)
        const __amdgpu_buffer_rsrc_t mrs = bufRsrc((void*)mbase, (uint32_t)(nslots * total));
        // the kernel's full policy pass (writePolicyAll, no delta base) reads the parked bits
        if (si >= 0 && D.pol_actions && !(D.pol_delta && D.mask_delta && (total & 15) == 0)) {
            at[l] = (int32_t)w0;
            as[l] = (int32_t)w1;
            ua[l] = w2 & 0xFFFFu;
        }
        if (recOut && si < 0) recOut[l] = ~0u;  // (no record from this lane)
        // the records stored lane-parallel (storeRecordsLanes) rather than each by its own lane
        const bool lanePar = MRTS_REC_LANES && !recOut && K == 79 && NW <= 16;
        if (lanePar) {
#ifdef MRTS_ABLATE
            if (!ab(AB_SKIP_RECORD))
#endif
            storeRecordsLanes(si, c, w0, w1, w2, mrs, mbase, total);
#ifdef MRTS_ABLATE
            if (ab(AB_RECORD)) storeRecordsLanes(launder(si), launder(c), launder(w0), launder(w1), launder(w2), mrs, mbase, total);
#endif
        }
        if (si >= 0) {
            const int slot = slot0 + si;
            const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32);
            if (recOut) {  // the helper expands and stores it (storeRecordsHelp)
                recOut[l] = ((uint32_t)si << 16) | (uint32_t)c;
                recOut[64 + l] = w0;
                recOut[128 + l] = w1;
                recOut[192 + l] = w2;
            } else if (lanePar) {
            } else
#ifdef MRTS_ABLATE
            if (!ab(AB_SKIP_RECORD))
#endif
            if (SC1_MASK) storeRecordSc1(mrs, mbase, (uint32_t)(si * total + c * K), lo, w2);
            else storeRecord(D.masks + (size_t)slot * total + (size_t)c * K, lo, w2);
#ifdef MRTS_ABLATE
            if (ab(AB_RECORD)) storeRecord(D.masks + (size_t)slot * total + (size_t)c * K, launder(lo), launder(w2));
#endif
            MPHASE(13);
            if (pol) {
                int32_t a[7];
#ifdef MRTS_ABLATE
                if (ab(AB_POLICY)) {
                    int32_t a2[7];
                    sampleBitsRaw(D.pol_seed, polStep, D.pol_slot_base + (uint32_t)launder(slot), NT, K,
                                  launder((lo >> 1) | ((uint64_t)w2 << 63)), launder((uint64_t)(w2 >> 1)), launder(c), a2);
                    keepv(a2[0] + a2[1] + a2[2] + a2[3] + a2[4] + a2[5] + a2[6]);
                }
#endif
                uint32_t pk;
                sampleBitsRaw(D.pol_seed, polStep, D.pol_slot_base + (uint32_t)slot, NT, K, (lo >> 1) | ((uint64_t)w2 << 63),
                              (uint64_t)(w2 >> 1), c, a, &pk);
                if (recOut) {
                    recOut[256 + l] = pk;
                } else {
                    int32_t* dst = D.pol_actions + ((size_t)slot * HW + c) * 7;
                    st4u<WT_MASK>(dst, a[0], a[1], a[2], a[3]);
                    st3u<WT_MASK>(dst + 4, a[4], a[5], a[6]);
                }
                if (fwdW) {
                    lfwd = pk;  // packFwd(a): the next iteration of a multi-step launch decodes from it
                    if (lastIt) st1<WT_STATE>(st() + stateFwdOff(CAP, HW) + l, (int32_t)lfwd);  // the next launch's
                }
            }
        }
        fwdWritten = fwdW;
        MPHASE(14);
        // cells whose idle unit is gone: zero record + zero row
        const uint32_t gone = old & ~cur;
        const int n = __popc(gone);
        const int incl = wave_incl_sum(n);
        const int ngone = rl(incl, 63);
        if (recOut) {  // the vacated cells go to the helper too (up to 64 of them; more: stored here below)
            uint16_t* gl = (uint16_t*)(recOut + 5 * 64 + 1);
            if (ngone <= 64) {
                int k = incl - n;
                for (uint32_t d = gone; d; d &= d - 1, k++) gl[k] = (uint16_t)((i << 15) | (32 * w + __builtin_ctz(d)));
            }
            if (l == 0) recOut[5 * 64] = (1u << 31) | (uint32_t)(ngone <= 64 ? ngone : 0);  // (bit 31: records valid)
            if (ngone <= 64) {
                wsync();
                return;
            }
        }
        if (ngone == 0) {
            wsync();
            return;
        }
#ifdef MRTS_ABLATE
        for (int rep_ = 0; rep_ < (ab(AB_GONE) ? 2 : 1); rep_++)
#endif
        for (int b0 = 0; b0 < ngone; b0 += 64) {  // rslot holds 64 list entries at a time
            wsync();
            int k = incl - n;
            for (uint32_t d = gone; d; d &= d - 1, k++)
                if (k >= b0 && k < b0 + 64) rslot[k - b0] = (uint16_t)((i << 15) | (32 * w + __builtin_ctz(d)));
            wsync();
            if (b0 + l < ngone) {
                const uint32_t e = rslot[l];
                const int slot = slot0 + (int)(e >> 15), cz = (int)(e & 0x7FFFu);
                if (SC1_MASK) storeRecordSc1(mrs, mbase, (uint32_t)((slot - slot0) * total + cz * K), 0ull, 0u);
                else storeRecord(D.masks + (size_t)slot * total + (size_t)cz * K, 0ull, 0u);
                if (pol) {
                    int32_t* dst = D.pol_actions + ((size_t)slot * HW + cz) * 7;
                    st4u<WT_MASK>(dst, 0, 0, 0, 0);
                    st3u<WT_MASK>(dst + 4, 0, 0, 0);
                }
            }
        }
        wsync();
    }
    // the fused random policy's action row of cell c of slot (slot0 + i): masked-uniform sample from
    // the parked mask bits (bit k = mask slot k) of an own idle unit, else a zero row
    DEV void policyRow(int slot, int c, int p) const {
        uint64_t lo;
        uint32_t hi;
        cellMaskBits(c, p, lo, hi);
        int32_t a[7];
        if (lo & 1ull) {
            sampleBitsRaw(D.pol_seed, polStep, D.pol_slot_base + (uint32_t)slot, NT, K, (lo >> 1) | ((uint64_t)hi << 63),
                          (uint64_t)(hi >> 1), c, a);
        } else {
#pragma unroll
            for (int q = 0; q < 7; q++) a[q] = 0;
        }
        int32_t* dst = D.pol_actions + ((size_t)slot * HW + c) * 7;
#pragma unroll
        for (int q = 0; q < 7; q++) dst[q] = a[q];
    }
    DEV void writePolicyAll(int slot0, int nslots, int pl0, int pl1) const {
        for (int i = 0; i < nslots; i++)
            for (int c = lid(); c < HW; c += 64) policyRow(slot0 + i, c, i ? pl1 : pl0);
    }
    // rewrite the chunks of the listed dirty cells (rslot[0..n): slot index << 15 | cell)
    DEV void flushDirty(int n, int slot0, int pl0, int pl1) {
        wsync();
        const int total = HW * K;
        const int NCH = (K + 14) / 16 + 1;  // chunks a K-byte record can touch
        for (int base = 0; base < NCH * n; base += 64) {
            const int item = base + lid();
            if (item < NCH * n) {
                const int k = item / NCH, t = item - k * NCH;
                const uint32_t e = rslot[k];
                const int i = (int)(e >> 15), c = (int)(e & 0x7FFFu);
                const int j = ((c * K) >> 4) + t;
                if (j <= ((c * K + K - 1) >> 4))
                    *(uint4*)(D.masks + (size_t)(slot0 + i) * total + 16 * j) = maskChunk(j, i ? pl1 : pl0);
                if (t == 0 && D.pol_actions && D.pol_delta) policyRow(slot0 + i, c, i ? pl1 : pl0);
            }
        }
        wsync();
    }
#undef D
};

// PassiveAI.getAction = fillWithNones(gs, p, 10) (ai/PassiveAI.java:41-45): nothing to park, the
// list-order fill in issuePlayer does it; RandomBiasedAI parks its actions.
DEV void aiGetAction(Game& G, int kind, int p) {
    if (kind == GK_RANDOM_BIASED) G.randomBiased(p);
}

// Specialisations (FIX = map width, square maps): batches of self-play games with grid actions and a
// built-in unit-type table (K = 79, 7 types, attack window 7), the map size, unit slots FCAP and
// observability compile-time constants, so LDS offsets fold into immediates and the bot / Java-row
// code vanishes — c3 (16x16, 320 slots), c2 (8x8, 128), c5 (32x32 PO, 320 slots = max_units 256).
// FIX = 0: anything (launchEnv picks).
// The helper wave of a HELP launch (8x8 fused uniform multi-step rollouts, BASELINE c2: one game per
// SIMD, so the SIMD idles while the game's wave runs its dependent chain).  Work with no input from the
// game's state moves to a second wave of the workgroup: the unmasked uniform rows (a pure function of
// slot, step and cell) of the NEXT step — to the action tensor, and packed into LDS for the game wave's
// decode — and the observation planes of the PREVIOUS step from the cells the game wave packed.  One
// workgroup barrier per step (A_k: rows(k) ready, obs cells of step k - 1 packed); each LDS buffer is
// double-buffered by step parity, so a buffer is rewritten only after the other wave passed the
// barrier that ends its use.  Output: every buffer ends exactly as after the same steps in one wave.
DEV void helperLoop(const KDyn& D, uint8_t* smem, int g, int niter) {
    constexpr int HW = 64, NT = 7, K = 79;
    const int l = (int)threadIdx.x - 64;
    uint32_t* rowbuf = (uint32_t*)(smem + D.help_off);  // [parity][player slot][cell]
    uint32_t* obsbuf = rowbuf + 2 * 2 * HW;             // [parity][cell][2]
    const int slot0 = 2 * g;
    auto rowsOf = [&](int k) {
        for (int i = 0; i < 2; i++) {
            int32_t a[7];
            uniformRow(D.uni_seed, D.uni_step + (uint32_t)k, D.uni_slot_base + (uint32_t)(slot0 + i), l, NT, K - 23 - NT, a);
            int32_t* dst = D.uni_actions + ((size_t)(slot0 + i) * HW + l) * 7;
            st4u<false>(dst, a[0], a[1], a[2], a[3]);
            st3u<false>(dst + 4, a[4], a[5], a[6]);
            rowbuf[(k & 1) * 2 * HW + i * HW + l] = packFwd(a);
        }
    };
    auto render = [&](int k) {
        if (!D.obs) return;
        const uint32_t w0 = obsbuf[(k & 1) * 2 * HW + 2 * l], w1 = obsbuf[(k & 1) * 2 * HW + 2 * l + 1];
        int v[6];
        v[0] = (int)(int16_t)(w0 & 0xFFFFu);
        v[1] = (int)(int16_t)(w0 >> 16);  // resources, signed as writeObsFull stores them
        v[3] = (int)((w1 >> 4) & 15u);
        v[4] = (int)((w1 >> 8) & 15u);
        v[5] = (int)((w1 >> 12) & 1u);
        const int own = (int)(w1 & 15u);  // player + 1, 0 = none
        int32_t* o0 = D.obs + (size_t)slot0 * D.C * HW;
        const __amdgpu_buffer_rsrc_t rs = bufRsrc(o0, (uint32_t)(2 * D.C * HW * 4));
        const int npl = k == 0 ? 6 : 5;  // the static terrain plane: first write of the launch only
#pragma unroll
        for (int i = 0; i < 2; i++) {
            v[2] = own ? ((own - 1 + i) % 2) + 1 : 0;  // ((owner + player) % 2) + 1 (GameState.java:947-949)
#pragma unroll
            for (int q = 0; q < 6; q++) {
                if (q >= npl) break;
                const uint32_t off = (uint32_t)((i * D.C + q) * HW + l);
                if (SC1_OBS) __builtin_amdgcn_raw_buffer_store_b32(v[q], rs, (int)(off * 4u), 0, 16);
                else st1<WT_OBS>(o0 + off, v[q]);
            }
            if (MRTS_UNLIKELY(D.obs16 != nullptr)) {
                int16_t* h0 = D.obs16 + (size_t)(slot0 + i) * D.C * HW;
#pragma unroll
                for (int q = 0; q < 6; q++) h0[(size_t)q * HW + l] = (int16_t)v[q];
            }
            if (MRTS_UNLIKELY(D.obs8 != nullptr)) {  // the uint8 transport: every plane, every step
                uint8_t* b0 = D.obs8 + (size_t)(slot0 + i) * D.C * HW;
#pragma unroll
                for (int q = 0; q < 6; q++) b0[(size_t)q * HW + l] = (uint8_t)v[q];
            }
        }
    };
    rowsOf(0);
    __syncthreads();  // A_0
    for (int k = 0; k < niter; k++) {
        if (k + 1 < niter) rowsOf(k + 1);
        __syncthreads();  // A_{k+1}: the game wave packed step k's cells; rows(k + 1) are in LDS
        render(k);
    }
}

// Issue priority by rank among the waves that share a SIMD (multi-step launches, KDyn.prio_tab).  A
// launch ends with its slowest SIMD, and a SIMD with its last game: the four games of a SIMD finish
// far apart (round 3 span build: 1.6-2.9 ms in a 200-step c3 launch), while the heaviest game alone
// needs ~2.2 ms and the SIMD's whole issue work ~2.0 ms.  So the game with the most remaining work
// (longest processing time first) should issue first, the next one second, and so on — a ranking
// the absolute unit-count thresholds only approximate.  Each wave posts, once per step, its game's
// remaining-work estimate (units + own idle units, times the steps left in the launch) with the
// launch stamp into its SIMD's row of the table (key from HW_ID / XCC_ID, slot = wave id), reads the
// row back, and at its next step sets s_setprio 3 - rank.  The reads may be a step old or see a
// neighbour's entry mid-update: priority never changes what a game computes, only when it issues.
struct SimdRank {
    uint32_t* row;  // this SIMD's 16 entries (stamp << 24 | estimate; 0 = free)
    int me;         // this wave's slot in the row
    uint32_t tag;   // this launch's stamp byte, never 0
    uint32_t seen;  // lane l < 16: entry l as last read
};
DEV SimdRank simdRankInit(uint32_t* tab, uint32_t stamp) {
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));        // HW_ID
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 7u;  // XCC_ID
    const uint32_t simd = (hw >> 4) & 3u, cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
    const uint32_t key = (((xcc * 8u + se) * 2u + sh) * 16u + cu) * 4u + simd;
    SimdRank r;
    r.row = tab + (size_t)key * 16;
    r.me = (int)(hw & 15u);
    r.tag = (stamp & 0x7Fu) | 0x80u;
    r.seen = 0;
    return r;
}
// rank of estimate `est` among the entries read last time (ties: lower slot first), then post `est`
// and read the row again for the next call
DEV int simdRankStep(SimdRank& r, uint32_t est) {
    const int l = lane_id();
    est = est > 0xFFFFFFu ? 0xFFFFFFu : est;
    const uint32_t e = r.seen, ee = e & 0xFFFFFFu;
    const bool higher = l < 16 && l != r.me && (e >> 24) == r.tag && (ee > est || (ee == est && l < r.me));
    const int rank = __popcll(ballot(higher));
    if (l == 0) r.row[r.me] = (r.tag << 24) | est;
    r.seen = l < 16 ? __builtin_nontemporal_load(r.row + l) : 0u;
    return rank;
}

// Balanced game placement (multi-step c3 and c5 launches, KDyn.bal).  With the rank priority above the four
// games of a SIMD finish together, and a launch ends with its slowest SIMD: round 3 span data, a SIMD's
// end time correlates 0.86-0.96 with its games' total unit count and the slowest SIMD ends 8 % after the
// mean.  The dispatcher places blocks b, b + n/4, b + 2n/4, b + 3n/4 on one SIMD (one dispatch round of
// four waves per SIMD; identical in every launch and process measured; c5's 128-thread blocks: the game waves
// of b and b + n/2), so a permutation of games over blocks that gives each such group a heavy-to-light mix
// balances the SIMDs.  Each game posts its cost (units + own idle units, MRTS_BAL_COST_IDLE) at the end of a launch; the last wave of each XCD class counting-sorts that class's posted
// counts and writes its part of the permutation for the next launches — snake order over the groups,
// so a group gets one game from each quarter of the order, heavy paired with light — and the stamp.  A launch whose predecessor on the
// handle left a permutation uses it (block b runs game perm[b]), else identity.  The permutation is
// sticky: only launches of at least MRTS_BAL_MIN_ITER steps post costs and write a new one, shorter
// ones reuse the last (a game that changes CU pays cold TLB misses for its output pages: moving games
// at every launch cost a 20-step launch ~12 us, round 3 span data).  Which block runs a
// game never changes what the game computes: correctness needs only that perm is a permutation
// (a counting sort's output is one), and a missing or stale posted cost leaves the old stamp in place.
DEV int balancedGame(const KDyn& D) {
    const int n = (int)gridDim.x;
    const int32_t hdr1 = __builtin_nontemporal_load(D.bal + 1);
    const int32_t pg = __builtin_nontemporal_load(D.bal + BAL_COST + n + (int)blockIdx.x);
    return hdr1 != 0 ? pg : (int)blockIdx.x;
}
DEV void balancePerm(const KDyn& D, uint32_t* hist, int c, int GS) {
    // games stay on their XCD: block b runs on XCD b % 8 and the four blocks of a SIMD group share b % 8,
    // so the permutation only moves games between blocks of the same residue class c (the state a game
    // left in that XCD's L2 stays near; round 6: one permutation over all games, balancing the XCDs' loads
    // too, was 1.2 % slower on c3 and -0.5 % on c5), and each class's LAST wave sorts that class alone: n / 8
    // games, n / 32 SIMD groups, the snake order as above (1/8 of the work on the launch's tail)
    // GS: games per SIMD group (c3: four game waves per SIMD; c5: MRTS_BAL_PO_GS), blocks n / GS apart
    const int n = (int)gridDim.x, l = lane_id(), Q = (int)((uint32_t)n / (8u * (uint32_t)GS)), per = n >> 9;  // per: games per lane
    int32_t* const cost = D.bal + BAL_COST;
    int32_t* const perm = cost + n;
    const uint32_t tag = D.fwd_stamp & 0xFFFFu;
#pragma unroll
    for (int j = 0; j < 4; j++) hist[l + 64 * j] = 0;
    // this lane's games c + 8 * (l * per + i): all loads in flight at once, system scope (the costs
    // came through other XCDs' L2s)
    const __amdgpu_buffer_rsrc_t rs = bufRsrc(cost, (uint32_t)(n * 4));
    uint32_t cv[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (i < per) cv[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)((c + 8 * (l * per + i)) * 4), 0, 17);
    wsync();
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (i < per) {
            ok = ok && (cv[i] >> 16) == tag;
            atomicAdd(&hist[255u - (cv[i] & 255u)], 1u);  // heaviest first
        }
    if (ballot(!ok)) return;  // a game has not posted (cannot happen: every wave posts before it counts): keep the old
    wsync();
    uint32_t v[4], sum = 0;  // exclusive prefix over the 256 bins: 4 per lane, then a wave scan
#pragma unroll
    for (int j = 0; j < 4; j++) {
        v[j] = hist[4 * l + j];
        sum += v[j];
    }
    const uint32_t incl = (uint32_t)wave_incl_sum((int)sum);
    uint32_t run = incl - sum;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        hist[4 * l + j] = run;
        run += v[j];
    }
    wsync();
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (i < per) {
            const int r = (int)atomicAdd(&hist[255u - (cv[i] & 255u)], 1u);  // rank in the class
            const int q = r / Q, j = r - q * Q;
            perm[c + 8 * (q * Q + ((q & 1) ? Q - 1 - j : j))] = c + 8 * (l * per + i);
        }
    if (l == 0) D.bal[1] = (int32_t)D.fwd_stamp;  // (every class writes the same) the next launches take it
}

// Workgroup barrier for an LDS handoff: the release / acquire fences cover LDS only, so a wave does
// not drain its outstanding global stores at every step (a __syncthreads fence would).
DEV void ldsBarrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
DEV void drainStores() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // s_waitcnt vmcnt(0): this wave's stores done

// The helper wave of a partially observable HELP launch (32x32 self-play multi-step rollouts, BASELINE
// c5: two games per SIMD, the SIMD's vector issue half idle while the games run their dependent
// chains).  The render of both views (writeObsPOFast2, a third of the step's instructions) reads the
// state after the cycle and writes only the observation and the render record, so it moves to the
// helper: at step k the game wave packs the render inputs (packPO, double-buffered by step parity)
// and passes barrier B_k; the helper renders step k (renderPOPacked) while the game compacts, writes
// masks and the next rows and runs step k + 1, and is back at B_{k+1} before the game packs over
// the buffer it read.  The render record (sight rows, pending chunks) stays with the helper between
// steps; the game keeps the per-slot part (poRecordSnaps, the lane registers) as before.  A step the
// fast render cannot take (more than 64 units, sight > 15) the helper renders with the general
// writeObsPO straight from the game's live state while the game waits at a second barrier B'_k
// (the helper's stores, the global render record included, complete before it: the game re-reads
// that record in nextStep).  Only the helper ever writes the observation buffer, in step order; the
// game wave carries no render code.  The next step's snapshotBoth comes from the same pack: after
// B_k the helper first computes it (snapFromPack) and passes S_k, where the game, back from its
// compaction, masks and policy, takes the bytes (takeSnap), then renders step k.  Header flags: bit 2
// = packed render, bit 3 = general render from the live state.  Layout: hdr [2][4] words, the
// helper's view-0 sight rows [2][H] (the snapshot's rows before the render) and the snapshot bytes
// [64] at KDyn.help_off; the packs [2][5][64] words and the per-step occupant map (u8 per cell) in the
// game's `scell` area, which only the general render uses.
// After the snapshot bytes, at PO_HELP_REC words: the game's mask records of a packed step
// (writeMasksLanes with recOut: [5][64] words + a count word + 64 u16 vacated cells), stored by the
// helper after S_k (S_last after the last step), so the game wave issues none of those stores.
constexpr int PO_HELP_REC = 8 + 2 * 32 + 16, PO_HELP_REC_WORDS = 5 * 64 + 1 + 32;
DEV void helperLoopPO(Game& G, uint32_t* hdr, int niter) {
    uint32_t* const rows0 = hdr + 8;
    uint8_t* const hsnap = (uint8_t*)(rows0 + 2 * G.H);
    uint8_t* const hcell = (uint8_t*)(G.scell + 2 * 5 * 64);
    uint32_t* const recs = hdr + PO_HELP_REC;
    G.helperLane();
    const int l = G.lid();
    if (MRTS_HELPER_PRIO) __builtin_amdgcn_s_setprio(3);  // the games wait for it at the handoff barriers
    for (int k = 0; k < niter; k++) {
        ldsBarrier();  // B_k
        const uint32_t* ph = hdr + (k & 1) * 4;
        const uint32_t f = uniu(ph[2]);
        const uint32_t* pk = G.scell + (k & 1) * 5 * 64;
        if (f & 4u) {
            if (k + 1 < niter) {
                G.snapFromPack(pk, ph, rows0, hsnap);
                ldsBarrier();  // S_k: the next step's snapshot bytes are ready
            }
            G.renderPOPacked(pk, ph, rows0, hcell, k == niter - 1);
            if (k + 1 == niter) ldsBarrier();  // S_last: the game's masks of the last step are out
#ifndef MRTS_DIAG_HELPER_NORECORDS  // diagnostic build only: the helper skips the record stores (output wrong)
            G.storeRecordsHelp(recs);  // step k's mask records and policy rows (written before S_k)
#endif
        } else if (f & 8u) {
            // the game's live state, as its own writeObsPO call would see it (the general render
            // overwrites `scell`, so the pack's record words are taken first)
            G.nu = (int)uniu(ph[0]);
            G.lcu = pk[192 + l];
            G.lkey = pk[256 + l];
            G.lsnap = (pk[128 + l] >> 8) & 0xFFu;
            for (int p = 0; p < 2; p++) G.writeObsPO(2 * G.g + p, p, ((f >> p) & 1u) != 0);
            drainStores();
            ldsBarrier();  // B'_k: the game continues (compaction)
        }
    }
}

template <int MODE, int FIX, int FCAP = 0, bool FPO = false, bool MULTI = false, bool HELP = false>
// stateArg and PS lead the argument list so that kernarg preloading (-amdgpu-kernarg-preload-count,
// Makefile) hands them over in SGPRs: the first memory round (state block, unit-type table) issues
// without waiting for a scalar load of the kernel arguments.  The 16x16 instances (c3: four games per
// SIMD, at the 128-VGPR edge) and the helper instances are held to 4 waves per SIMD: one VGPR more
// silently halves nothing but drops a quarter of the games into a second dispatch round (1.7x slower).
__global__ __launch_bounds__(HELP ? 128 : 64, (HELP || FIX == 16) ? 4 : 1) void k_env(int32_t* __restrict__ stateArg, const KStatic* __restrict__ PS, KDyn D) {
    extern __shared__ __align__(16) uint8_t smem[];
    if (HELP && !FPO && threadIdx.x >= 64) {
        helperLoop(D, smem, (int)blockIdx.x, D.n_iter);
        return;
    }
    const KStatic& P = *PS;
    // balanced placement (c3's and c5's multi-step kernels): this block's game from the previous launch's permutation
    // (balancePerm: a multiple of 512 games, at most 8 per lane and class)
    const bool balanced = MULTI && MRTS_BALANCE && ((FIX == 16 && !FPO) || (MRTS_BALANCE_PO && FIX == 32 && FPO && HELP)) &&
                          D.bal != nullptr && (gridDim.x & 511) == 0 &&
                          gridDim.x <= 4096;
    const bool rebalance = balanced && D.n_iter >= MRTS_BAL_MIN_ITER;  // this launch writes the next permutation
    const int game = balanced ? balancedGame(D) : -1;
    Game G(P, D, stateArg, FIX ? stateWords(FCAP, FIX * FIX) : D.state_words, smem, FIX ? FIX : D.H, FIX ? FIX : D.W, FIX ? FIX * FIX : D.HW, FIX ? FCAP : D.CAP,
           FIX ? FPO : P.partial_obs != 0, FIX ? 79 : P.utt.K, FIX ? 7 : P.utt.ntypes, FIX ? 7 : P.utt.maxAttackRadius, MULTI, game,
           MRTS_INDEX_WALK && (FIX == 16 || (MRTS_WALK32 && FIX == 32)));
    // the partially observable helper wave: one packed render per step (helperLoopPO)
    uint32_t* const poHelpHdr = (HELP && FPO) ? (uint32_t*)(smem + D.help_off) : nullptr;
    if (HELP && FPO && threadIdx.x >= 64) {
        helperLoopPO(G, poHelpHdr, D.n_iter);
        return;
    }
#ifdef MRTS_ABLATE
    G.G_AB = g_ablate;
#endif
    // games [0, n_sp_games) are self-play (mrts_create's layout): no load needed to place the slots
    const bool selfplay = FIX ? true : G.g < D.n_sp_games;
    const int slot0 = selfplay ? 2 * G.g : 2 * D.n_sp_games + (G.g - D.n_sp_games);
    const int nslots = selfplay ? 2 : 1;
    // agent-vs-bot: the agent's side; bot-vs-bot: the side ai1 plays (JNIBotClient.gameStep(player))
    const int side = selfplay ? 0 : (D.players ? uni(D.players[slot0]) : 0);
    bool freshObs = true;  // observation comes from the current (post-step or fresh) state
#ifdef MRTS_PHASE_TIMING
#ifndef MRTS_SPAN_ONLY
    for (int i = 0; i < NPH; i++) G.phAcc[i] = 0;
#endif
    G.tph_ = __builtin_amdgcn_s_memtime();
    const uint64_t rt0_ = __builtin_amdgcn_s_memrealtime();
#endif

    if (MODE == MODE_RESET) {
        G.copyUtt();
        G.loadHeader(G.st());
        G.hset(H_KIND, P.game_kind[G.g]);
        G.hset(H_ERR, 0);
        G.initCells();
        G.storeTerrain();
        G.resetFromTemplate();
        if (D.mask_delta && D.masks) G.loadPrev();
        // JNIGridnetClientSelfPlay.reset zeroes reward/done slots j < rewards.length == 2 only
        // (tests/JNIGridnetClientSelfPlay.java:103-104,235-238): slots >= 2 keep the caller buffer's
        // previous values; JNIGridnetClient / JNIBotClient.reset zero every slot
        // (JNIGridnetClient.java:248-251, JNIBotClient.java:159-162)
        for (int k = lane_id(); k < nslots * D.n_rewards; k += 64) {
            if (selfplay && k % D.n_rewards >= 2) continue;
            if (D.reward) D.reward[(size_t)slot0 * D.n_rewards + k] = 0.0;
            if (D.done) D.done[(size_t)slot0 * D.n_rewards + k] = 0;
        }
    } else {
        G.load(D.mask_delta && D.masks);
#ifdef MRTS_ABLATE
        if (G.ab(AB_LOAD)) G.load(D.mask_delta && D.masks);
#endif
    }
    // Multi-step launch (MULTI instances: mrts_rollout_fused_dev on the specialised full-observability
    // self-play shapes): the game runs D.n_iter consecutive fused steps with its state in LDS — each
    // iteration is one whole step (decode, issue, cycle, rewards, auto-reset, observation, masks, next
    // rows, all written to their buffers) — and stores the state once at the end.  A separate
    // instance: the loop changes register allocation (values live across iterations), and the
    // single-step kernels must not pay for it.
    const int kind = FIX ? GT_SELFPLAY : G.hget(H_KIND);
    const int gtype = kind & 15, ai1 = (kind >> 4) & 15, ai2 = (kind >> 8) & 15;
    const bool external = gtype != GT_BOT_VS_BOT;  // bot-only clients return no observation / masks
    const int niter = MULTI ? D.n_iter : 1;
#ifdef MRTS_PHASE_TIMING
    int nu0_ = 0;
#endif
    uint32_t* const helpBuf = (HELP && !FPO) ? (uint32_t*)(smem + D.help_off) : nullptr;  // helperLoop's layout
    bool poPacked = false;  // HELP && FPO: the previous iteration handed its render to the helper (packPO, flag 4)
    // c3 (four games per SIMD) and c5 (two games + their helper waves, which keep priority 0)
    const bool ranked = MULTI && MRTS_SIMD_RANK && (FIX == 16 || (FIX == 32 && FPO && MRTS_SIMD_RANK_PO)) &&
                        D.prio_tab != nullptr && niter > 1;
    SimdRank srank;
    if (ranked) srank = simdRankInit(D.prio_tab, D.fwd_stamp);
    if (HELP && !FPO) __syncthreads();  // A_0: the helper drew step 0's rows
    for (int it = 0; it < niter; it++) {
    if (it > 0) {
        G.nextStep();
        freshObs = true;
    }
#if MRTS_BODY_LAUNDER
    // the step body reads the kernel argument through the Game's per-iteration opaque pointer too (as its
    // methods do, freshLane): the by-value argument's fields and the conditions derived from them were
    // loaded once before the loop and held across it in spilled SGPRs — a v_readlane per use, every step
    auto& D = *G.Dp;
#endif
    if (HELP && !FPO) G.helpRows = helpBuf + (it & 1) * 2 * 64;
    G.lastIt = it == niter - 1;
    G.firstIt = it == 0;
    bool snapTaken = false;
    if (MODE != MODE_RESET && !(MULTI && MRTS_MULTI_NOPRIO)) {
        // Issue priority by game size: a SIMD runs several games at once and the kernel ends with its
        // slowest one, so the games with the most units (the longest serial chains) issue first.
        int q;
        if (MRTS_PRIO_IDLE && FIX == 16) {
            // the c3 shape (four games per SIMD): units + own idle units (the step's decode / issue /
            // mask / policy work grows with the idle ones)
            const int wq = G.nu + (int)__popcll(ballot(G.lid() < G.nu && !(G.lua & UA_PRESENT) && uplay(G.lcu) >= 0));
            q = wq >= MRTS_PRIO_T3 ? 3 : wq >= MRTS_PRIO_T2 ? 2 : wq >= MRTS_PRIO_T1 ? 1 : 0;
            if (ranked) {  // from the second step on: the rank among the SIMD's waves by remaining work
                const int rk = simdRankStep(srank, (uint32_t)(wq + MRTS_RANK_C) * (uint32_t)(niter - it));
                if (it > 0) q = 3 - (rk < 3 ? rk : 3);
            }
        } else {  // units (the idle count's ballot costs the latency-bound one-game-per-SIMD c2 4.5 %)
            // (c5, two games + their helper waves per SIMD: without any priority -9 %, the games all at 3 or all
            // above the helpers' 0 +-0.5 % — what counts is the games issuing before the helpers, round 6)
            q = G.nu >= 36 ? 3 : G.nu >= 30 ? 2 : G.nu >= 24 ? 1 : 0;
            if (ranked) {
                const int wq = G.nu + (int)__popcll(ballot(G.lid() < G.nu && !(G.lua & UA_PRESENT) && uplay(G.lcu) >= 0));
                const int rk = simdRankStep(srank, (uint32_t)(wq + MRTS_RANK_C) * (uint32_t)(niter - it));
                if (it > 0) q = 3 - (rk < 3 ? rk : 3);
            }
        }
        if (HELP && !FPO && MRTS_GAME_OVER_HELPER) q = q < 1 ? 1 : q;
        if (q == 0) {
            if (it > 0) __builtin_amdgcn_s_setprio(0);
        } else if (q == 1) __builtin_amdgcn_s_setprio(1);
        else if (q == 2) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(3);
    }
#ifdef MRTS_PHASE_TIMING
    if (it == 0) nu0_ = G.nu;
#endif
    if (G.po) G.clearSnap();
    if (HELP && FPO && poPacked) {  // S_{it-1}: the helper's snapshot of this step (snapFromPack)
        ldsBarrier();
#ifndef MRTS_PO_HELPER_NOSNAP  // diagnostic build: the game wave takes its own snapshot
        G.takeSnap((const uint8_t*)(poHelpHdr + 8 + 2 * G.H));
        snapTaken = true;
#endif
    }
    PHASE(0);

    if (MODE == MODE_PLAYOUT) {
        // NaiveMCTS.simulate (ai/mcts/naivemcts/NaiveMCTS.java:297-308, the same loop as
        // ai/AALL/mcts/ModelledEvaluationMCTS.java:313-324): do { if (isComplete()) gameover = cycle();
        // else { issue(policy.getAction(0)); issue(policy.getAction(1)); } } while (!gameover &&
        // time < until).  The policies give every idle unit an action, so after an issue pass the
        // state is complete: one pass below = [issue pass if incomplete] + cycle.  The state stays in
        // LDS for the whole playout; time grows by one per pass, so every wave reaches the exit.
        const int until = G.time + D.horizon;
        bool first = true;
        for (;;) {
            if (!G.complete()) {
                aiGetAction(G, ai1, 0);
                G.issuePlayer(0, 10, true);
                aiGetAction(G, ai2, 1);
                G.issuePlayer(1, 10, true);
                if (first && G.time >= until) break;  // the do-while's first test follows the issue pass
            }
            first = false;
            G.cycle();
            bool over;
            int winner;
            G.outcome(over, winner);
            if (G.deaths) {
                G.compact();
                G.deaths = 0;
            }
            if (over || G.time >= until) break;
        }
        wsync();
        G.store();
        return;
    }

    if (MODE == MODE_TRACE) {
        // TestTracesIntegrity.testTrace (test/microrts/TestTracesIntegrity.java:72-127), one entry per
        // launch: issueSafe(p0's pairs), issueSafe(p1's pairs) (:119-120), then GameState.cycle() until
        // the next entry's time (:83-86).  The Java asserts that no cycle follows a cycle that ended the
        // game; cycle() returns gameover() of the state it leaves, which is this state again before the
        // next cycle (issuing moves no unit) — so a game over before any further cycle is that failure.
        uint32_t flags = 0;
        const int32_t* rows = D.rows + (size_t)G.g * D.n_rows * 8;
        const bool i0 = G.traceIssue(0, rows, D.n_rows, flags);
        const bool i1 = G.traceIssue(1, rows, D.n_rows, flags);
        if (i0 || i1) flags |= TR_ISSUED;
        const int until = uni(D.trace_until[G.g]);
        while (G.time < until) {
            if (G.time > 0) {
                bool over;
                int winner;
                G.outcome(over, winner);
                if (over) {
                    flags |= TR_GAMEOVER;
                    break;
                }
            }
            G.cycle();
            if (G.deaths) {
                G.compact();
                G.deaths = 0;
            }
        }
        wsync();
        G.store();
        if (lane_id() == 0) D.trace_out[G.g] = (int32_t)flags;
        return;
    }

    if (MODE == MODE_STEP) {
        const size_t rowStride = (size_t)G.HW * 7;
        // fused uniform policy: this step's rows go out first (fire-and-forget stores, nothing in the
        // launch reads them back: fetchRow draws the idle units' rows again)
        if (D.uni_actions && !(HELP && !FPO)) G.writeUniformRows(slot0, nslots);
        if (MRTS_UNLIKELY(D.reward_need & RN_COUNTS))
            if (lane_id() < 2 * RC_N) G.rwc[lane_id()] = 0;
        if (MRTS_UNLIKELY(D.reward_need & RN_CLOSER)) G.closerBefore();
        const bool rowsMode = FIX ? false : D.rows != nullptr;
        if (rowsMode && gtype == GT_SELFPLAY) {
            for (int p = 0; p < 2; p++) {
                if (G.po) G.snapshot(p);
                const int np = G.rowsDecode(p, D.rows + (size_t)(slot0 + p) * D.n_rows * 8);
                G.rowsIssue(p, np, 1);
            }
        } else if (rowsMode && gtype == GT_AGENT_VS_BOT) {
            if (G.po) {
                G.snapshot(side);
                G.snapshot(1 - side);
            }
            const int np = G.rowsDecode(side, D.rows + (size_t)slot0 * D.n_rows * 8);
            aiGetAction(G, ai2, 1 - side);
            G.rowsIssue(side, np, 1);
            G.issuePlayer(1 - side, 10, true);
        } else if (gtype == GT_SELFPLAY) {
            // JNIGridnetClientSelfPlay.gameStep (tests/JNIGridnetClientSelfPlay.java:159-189)
            if (MRTS_LIKELY(G.nu <= 64 && (!G.po || (MRTS_PO_FAST && G.snapBothOk())))) {
                G.selfPlayFast(D.actions + (size_t)slot0 * rowStride, D.actions + (size_t)(slot0 + 1) * rowStride, slot0,
                               snapTaken);
            } else {
            G.predecode(D.actions + (size_t)slot0 * rowStride, D.actions + (size_t)(slot0 + 1) * rowStride, -1, slot0, slot0 + 1);
            PHASE(1);
            const bool snapBoth = G.po && G.snapBothOk();
            for (int p = 0; p < 2; p++) {
                if (snapBoth) {
                    if (p == 0 && !snapTaken) G.snapshotBoth();
                    else G.snapshotActions(1);
                } else if (G.po) {
                    G.snapshot(p);
                }
                if (G.nu <= 64) {
                    G.decode(p, true);
                } else {
                    G.decode(p);
                    PHASE(2);
                    G.issuePlayer(p, 1, false);
                }
                PHASE(3);
            }
            }
        } else if (gtype == GT_AGENT_VS_BOT) {
            // JNIGridnetClient.gameStep (tests/JNIGridnetClient.java:163-203): both views are taken and
            // both actions computed before either issueSafe
            const int32_t* rows = D.actions + (size_t)slot0 * rowStride;
            G.predecode(rows, rows, side, slot0, slot0);
            if (G.po) {
                G.snapshot(side);
                G.snapshot(1 - side);
            }
            G.decode(side);
            aiGetAction(G, ai2, 1 - side);
            G.issuePlayer(side, 1, false);
            G.issuePlayer(1 - side, 10, true);
        } else {
            // JNIBotClient.gameStep (tests/JNIBotClient.java:108-135): both AIs on the full state
            aiGetAction(G, ai1, side);
            aiGetAction(G, ai2, 1 - side);
            G.issuePlayer(side, 10, true);
            G.issuePlayer(1 - side, 10, true);
        }
        G.cycle();
        PHASE(4);
        bool gameover;
        int winner;
#ifdef MRTS_ABLATE
        if (G.ab(AB_OUTCOME)) {
            G.outcome(gameover, winner);
            G.writeRewards(slot0, nslots, selfplay ? 0 : side, selfplay ? 1 : side, gameover, winner);
        }
#endif
        G.outcome(gameover, winner);
        // reward functions + VecClient auto-reset on done[0] or max steps, keeping the terminal
        // reward/done and forcing done[0] (tests/JNIGridnetVecClient.java:214-287)
        const int steps = G.hget(H_STEPS) + 1;
        G.hset(H_STEPS, steps);
        const bool done0 = G.writeRewards(slot0, nslots, selfplay ? 0 : side, selfplay ? 1 : side, gameover, winner, it);
        const bool reset = done0 || steps >= D.max_steps;
        if (reset && D.done && lane_id() < nslots)
            D.done[(MRTS_RESP_RING ? (size_t)((uint32_t)it * (uint32_t)D.resp_stride) : 0) + (size_t)(slot0 + lane_id()) * D.n_rewards] = 1;
        if (MRTS_UNLIKELY(reset)) {
            G.hset(H_STEPS, 0);  // envSteps[i] = 0 (JNIGridnetVecClient.java:229,264-265,285)
            G.resetFromTemplate();
            if (G.po) G.clearSnap();
        } else {
            freshObs = false;
        }
        PHASE(5);
    }

    uint32_t poHelpFlags = 0;  // HELP && FPO: bit 2 = the helper renders this step, bit 3 = the game does
    if (MODE != MODE_MASKS && D.obs && external) {
        if (G.po) {
            // persistent buffer: the views the previous write rendered for this game can be updated
            // in place (writeObsPO's delta)
            const bool canDelta = MODE == MODE_STEP && !freshObs && D.obs_delta && D.po_prev && poDeltaShape(G.H, G.W) &&
                                  G.nu <= 64 && G.hget(H_NU) <= 64;
            const uint32_t valid = canDelta ? (uint32_t)G.hget(Game::HX_POVALID) : 0u;
            if (selfplay && G.poFast2()) {
                if (freshObs) {  // PO views of the reset state (snapshot(p) touches only view p's bits)
                    if (G.snapBothOk()) {
                        G.snapshotBoth();
                        G.snapshotActions(1);
                    } else {
                        G.snapshot(0);
                        G.snapshot(1);
                    }
                }
                if (HELP && FPO) {
                    G.packPO(G.scell + (it & 1) * 5 * 64, poHelpHdr + (it & 1) * 4, valid & 3u, 4u);
                    poHelpFlags = 4u;
                } else
#ifdef MRTS_ABLATE
                if (!G.ab(AB_SKIP_OBS))
#endif
                G.writeObsPOFast2(slot0, valid & 3u);
            } else if (HELP && FPO) {
                // the helper renders from the live state while this wave waits at B'_it (below)
                if (freshObs) {
                    G.snapshot(0);
                    G.snapshot(1);
                }
                G.packPO(G.scell + (it & 1) * 5 * 64, poHelpHdr + (it & 1) * 4, valid & 3u, 8u);
                poHelpFlags = 8u;
            } else
            for (int i = 0; i < nslots; i++) {
                const int p = selfplay ? i : side;
                if (freshObs) G.snapshot(p);  // PO view of the reset state
#ifdef MRTS_ABLATE
                if (!G.ab(AB_SKIP_OBS))
#endif
                G.writeObsPO(slot0 + i, p, ((valid >> p) & 1u) != 0);
            }
        } else if (HELP) {
            G.packObs(helpBuf + 2 * 2 * 64 + (it & 1) * 2 * 64);  // the helper wave renders it
        } else {
#ifdef MRTS_ABLATE
            if (!G.ab(AB_SKIP_OBS))
#endif
            G.writeObsFull(slot0, nslots, side);
#ifdef MRTS_ABLATE
            if (G.ab(AB_OBS)) G.writeObsFull(slot0, nslots, side);
#endif
        }
    }
    if (MODE == MODE_STEP && MRTS_UNLIKELY(D.rec_out != nullptr) && external) G.writeRecord(it);
    if (HELP && !FPO) __syncthreads();  // A_{it+1}: step it's cells packed; the helper's rows of step it + 1 ready
    if (HELP && FPO) {
        if (poHelpFlags == 0u && G.lid() == 0) poHelpHdr[(it & 1) * 4 + 2] = 0u;
        ldsBarrier();  // B_it: the helper takes step it's pack (helperLoopPO)
        if (poHelpFlags == 8u) ldsBarrier();  // B'_it: the helper rendered from this wave's live state
        poPacked = poHelpFlags == 4u;
    }
    PHASE(6);
    if (MODE == MODE_STEP && !freshObs && G.deaths) G.compact();
    PHASE(7);
    if (HELP && FPO) {  // a packed step's mask records go to the helper (storeRecordsHelp)
        G.recOut = poHelpFlags == 4u ? poHelpHdr + PO_HELP_REC : nullptr;
        if (poHelpFlags == 4u && G.lid() == 0) G.recOut[5 * 64] = 0u;  // none, unless writeMasksLanes hands them over
    }
    if (D.masks && external) {
        const int nsl = selfplay ? 2 : 1;
        if (MRTS_LIKELY(D.mask_delta && G.nu <= 64 && nsl * maskWords(G.HW) <= 64 && G.K <= 96)) {
            PHASE(8);
            if (selfplay) G.writeMasksLanes(slot0, 2, 0, 1);
            else G.writeMasksLanes(slot0, 1, D.mask_player, D.mask_player);
        } else {
        wsync();
        G.stashMasks(selfplay ? 3 : (1 << D.mask_player));
        wsync();
        PHASE(8);
        if (selfplay) G.writeMasks(slot0, 2, 0, 1);
        else G.writeMasks(slot0, 1, D.mask_player, D.mask_player);
        }
        if (D.pol_actions && !(D.pol_delta && D.mask_delta && ((G.HW * G.K) & 15) == 0)) {  // no dirty-row pass ran
            wsync();
            if (selfplay) G.writePolicyAll(slot0, 2, 0, 1);
            else G.writePolicyAll(slot0, 1, D.mask_player, D.mask_player);
        }
        PHASE(9);
    }
    if (MODE != MODE_MASKS && G.po && D.obs && external && D.po_prev && poDeltaShape(G.H, G.W)) {
        wsync();
        G.poRecordSnaps(selfplay ? 3u : (1u << side));
    }
    if (HELP && FPO && poPacked && it == niter - 1) ldsBarrier();  // S_last (helperLoopPO)
    }  // iterations
    if (ranked && lane_id() == 0) srank.row[srank.me] = 0u;  // this game no longer competes on its SIMD
    if (MODE != MODE_MASKS) {
        wsync();
        G.store();
#ifdef MRTS_ABLATE
        if (G.ab(AB_STORE)) G.store();
#endif
    }
    if (rebalance) {  // post this game's final unit count; the launch's LAST wave writes the next placement
        const uint32_t tag = D.fwd_stamp & 0xFFFFu;
        uint32_t last = 0;
        const int cost = MRTS_BAL_COST_IDLE ? G.nu + (int)__popcll(ballot(G.lid() < G.nu && !(G.lua & UA_PRESENT) && uplay(G.lcu) >= 0))
                                            : G.nu;
        if (lane_id() == 0) {
            // agent scope, written through: the last wave may sit on another XCD (another L2)
            __hip_atomic_store(D.bal + BAL_COST + G.g, (int32_t)((tag << 16) | (uint32_t)(cost < 255 ? cost : 255)),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            drainStores();  // the cost is in memory before this wave counts itself
            // waves of this block's class (b % 8) finished in this launch, wrapping to 0 at the last
            // (atomicInc): no reset needed, and no compare-and-swap retries (4096 contending CAS loops
            // at device scope took milliseconds)
            const uint32_t old = atomicInc((uint32_t*)D.bal + 2 + (blockIdx.x & 7u), gridDim.x / 8u - 1u);
            last = old == gridDim.x / 8u - 1u ? 1u : 0u;
        }
        if (uniu(last)) {
            wsync();
            balancePerm(D, (uint32_t*)smem, (int)(blockIdx.x & 7u), FIX == 16 ? 4 : MRTS_BAL_PO_GS);
        }
    }
    PHASE(10);
#ifdef MRTS_PHASE_TIMING
    if (lane_id() == 0 && G.g < PH_GAMES) {
#ifndef MRTS_SPAN_ONLY
        for (int i = 0; i < NPH; i++) g_phase[i * PH_GAMES + G.g] += G.phAcc[i];
#endif
#ifdef MRTS_NO_MILESTONES
        // odd launch stamps go to blocks 3 / 4 (free without milestones): two back-to-back launches
        // can be compared (tools/launch_gap.py)
        const int sb_ = (D.fwd_stamp & 1u) ? 3 : 0;
#else
        const int sb_ = 0;
#endif
        g_span[sb_ * PH_GAMES + G.g] = rt0_;
        g_span[(sb_ + 1) * PH_GAMES + G.g] = __builtin_amdgcn_s_memrealtime();
        g_span[2 * PH_GAMES + G.g] = (unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                                     ((unsigned long long)(__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 15) << 32) |
                                     ((unsigned long long)(nu0_ & 255) << 40) | ((unsigned long long)(G.nu & 255) << 48);
    }
#endif
}

// ---------------------------------------------------------------- random policy (bench / rollouts)
DEV void sampleBits(const PolicyParams& Q, uint64_t lo, uint64_t hi, int slot, int c, int32_t a[7]) {
    sampleBitsRaw(Q.seed, Q.step, Q.slot_id_base + (uint32_t)slot, Q.ntypes, Q.K, lo, hi, c, a);
}
DEV void sampleCell(const PolicyParams& Q, const uint8_t* m, int slot, int c, int32_t a[7]) {
    for (int k = 0; k < 7; k++) a[k] = 0;
    if (!m[0]) return;
    uint64_t lo = 0, hi = 0;
    for (int i = 1; i < Q.K; i++) {
        const uint64_t b = m[i] ? 1ull : 0ull;
        if (i - 1 < 64) lo |= b << (i - 1);
        else hi |= b << (i - 1 - 64);
    }
    sampleBits(Q, lo, hi, slot, c, a);
}
// 16 mask bytes (0 / non-zero) -> 16 bits, byte k -> bit k
DEV uint32_t nz4(uint32_t w) {
    uint32_t t = w | (w >> 4);
    t |= t >> 2;
    t |= t >> 1;
    return ((t & 0x01010101u) * 0x01020408u) >> 24;
}
DEV uint32_t pack16(uint4 v) { return nz4(v.x) | (nz4(v.y) << 4) | (nz4(v.z) << 8) | (nz4(v.w) << 12); }

// Tiled form: one wave = 64 cells of one slot.  The 64 mask records (64*K bytes, 16-B aligned when
// HW*K and 64*K are multiples of 16) stream in with dwordx4 loads and are packed to bits in
// registers on arrival (LDS holds 1 bit per mask byte); the 64 action rows (1792 B) stream out of
// LDS with dwordx4 stores.
__global__ __launch_bounds__(64) void k_policy_tiled(PolicyParams Q) {
    __shared__ uint16_t tb[64 * 96 / 16 + 8];
    __shared__ __align__(16) int32_t sa[64 * 7];
    const int lane = (int)threadIdx.x, slot = (int)blockIdx.y;
    const int c0 = (int)blockIdx.x * 64;
    const int ncell = min(64, Q.HW - c0);
    const uint8_t* src = Q.masks + ((size_t)slot * Q.HW + c0) * Q.K;
    const int nbytes = ncell * Q.K, n16 = nbytes >> 4;
    for (int i = lane; i < n16; i += 64) tb[i] = (uint16_t)pack16(((const uint4*)src)[i]);
    if (lane == 0 && (nbytes & 15)) {
        uint32_t b = 0;
        for (int i = 16 * n16; i < nbytes; i++) b |= (src[i] ? 1u : 0u) << (i - 16 * n16);
        tb[n16] = (uint16_t)b;
    }
    __syncthreads();
    int32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
    if (lane < ncell) {
        const int b0 = lane * Q.K;
        if ((tb[b0 >> 4] >> (b0 & 15)) & 1) {
            // bits b0+1 .. b0+K-1 -> lo/hi
            const int s = b0 + 1, w0 = s >> 4, sh = s & 15;
            uint64_t x0 = 0, x1 = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) x0 |= (uint64_t)tb[w0 + j] << (16 * j);
#pragma unroll
            for (int j = 0; j < 3; j++) x1 |= (uint64_t)tb[w0 + 4 + j] << (16 * j);
            uint64_t lo = sh ? ((x0 >> sh) | (x1 << (64 - sh))) : x0;
            uint64_t hi = x1 >> sh;
            const int nb = Q.K - 1;  // valid bits
            if (nb < 64) {
                lo &= (1ull << nb) - 1;
                hi = 0;
            } else if (nb < 128) {
                hi &= (1ull << (nb - 64)) - 1;
            }
            sampleBits(Q, lo, hi, slot, c0 + lane, a);
        }
    }
#pragma unroll
    for (int k = 0; k < 7; k++) sa[lane * 7 + k] = a[k];
    __syncthreads();
    int32_t* dst = Q.actions + ((size_t)slot * Q.HW + c0) * 7;
    const int nw = ncell * 7, nw4 = nw >> 2;
    for (int i = lane; i < nw4; i += 64) ((int4*)dst)[i] = ((const int4*)sa)[i];
    for (int i = 4 * nw4 + lane; i < nw; i += 64) dst[i] = sa[i];
}

// one candidate cell's action from its K-byte mask record: record bits 0..K-1 gathered from the
// covering aligned 16-B chunks (chunk q's byte 0 sits at record bit pos = 16q - b0)
DEV void sampleRecord(const PolicyParams& Q, const uint8_t* mrec, int slot, int c, int32_t row[7]) {
    const int b0 = c * Q.K, j0 = b0 >> 4, j1 = (b0 + Q.K - 1) >> 4;
    uint64_t r0 = 0, r1 = 0;
    for (int q = j0; q <= j1; q++) {
        const uint64_t b16 = pack16(((const uint4*)mrec)[q]);
        const int pos = 16 * q - b0;
        if (pos < 0) {
            r0 |= b16 >> (-pos);
        } else if (pos < 64) {
            r0 |= b16 << pos;
            if (pos > 48) r1 |= b16 >> (64 - pos);
        } else {
            r1 |= b16 << (pos - 64);
        }
    }
    // record bits 1..K-1 -> lo/hi (bit i -> bit i-1)
    uint64_t lo = (r0 >> 1) | (r1 << 63), hi = r1 >> 1;
    const int nb = Q.K - 1;
    if (nb < 64) {
        lo &= (1ull << nb) - 1;
        hi = 0;
    } else {
        hi &= (1ull << (nb - 64)) - 1;
    }
    sampleBits(Q, lo, hi, slot, c, row);
}

// Source-bit form: one wave = one slot.  Candidate cells come from the env's source bits; only their
// mask records are read (the <= 6 aligned 16-B chunks covering each).  Rows are composed in LDS,
// 256 cells (7 KB) at a time, and leave with coalesced dwordx4 stores.
__global__ __launch_bounds__(64) void k_policy_src(PolicyParams Q) {
    __shared__ __align__(16) int32_t sa[256 * 7];
    const int lane = (int)threadIdx.x, slot = (int)blockIdx.x;
    const int MW = (Q.HW + 31) / 32;
    const uint32_t* src = Q.source + (size_t)slot * MW;
    const uint8_t* mrec = Q.masks + (size_t)slot * Q.HW * Q.K;
    int32_t* dst = Q.actions + (size_t)slot * Q.HW * 7;
    for (int c0 = 0; c0 < Q.HW; c0 += 256) {
        const int ncell = min(256, Q.HW - c0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int c = c0 + 64 * j + lane;
            int32_t row[7] = {0, 0, 0, 0, 0, 0, 0};
            if (c < Q.HW && ((src[c >> 5] >> (c & 31)) & 1u)) sampleRecord(Q, mrec, slot, c, row);
            const int r = 64 * j + lane;  // stride-7 words: conflict-free LDS writes
#pragma unroll
            for (int k = 0; k < 7; k++) sa[r * 7 + k] = row[k];
        }
        __syncthreads();
        int32_t* d = dst + (size_t)c0 * 7;
        const int nw = ncell * 7, nw4 = nw >> 2;
        for (int i = lane; i < nw4; i += 64) ((int4*)d)[i] = ((const int4*)sa)[i];
        for (int i = 4 * nw4 + lane; i < nw; i += 64) d[i] = sa[i];
        __syncthreads();
    }
    if (Q.prev_out)
        for (int w = lane; w < MW; w += 64) Q.prev_out[(size_t)slot * MW + w] = src[w];
}

// Delta form (actions holds this policy's previous output, whose candidate set is prev): only rows
// in prev | source change — candidates get a fresh action, former candidates a zero row.  A wave
// takes 64 (slot, 32-cell bit word) items in one load round, compacts their dirty cells into an LDS
// list (wave prefix sum), and spreads the list over its lanes, so each dirty row costs one record
// round trip in parallel with the others.  The candidate set is double-buffered (prev -> prev_out).
__global__ __launch_bounds__(64) void k_policy_delta(PolicyParams Q) {
    __shared__ uint32_t list[64 * 32];
    const int lane = (int)threadIdx.x;
    const uint32_t MW = (uint32_t)(Q.HW + 31) / 32;
    const uint32_t nitems = (uint32_t)Q.n_slots * MW;
    const uint32_t item = blockIdx.x * 64u + (uint32_t)lane;
    const bool valid = item < nitems;
    const uint32_t cur = valid ? Q.source[item] : 0u, old = valid ? Q.prev[item] : 0u;
    if (valid) Q.prev_out[item] = cur;
    const uint32_t dirty = cur | old;
    const int n = __popc(dirty);
    const int incl = wave_incl_sum(n);  // inclusive prefix sum over lanes
    const int total = rl(incl, 63);
    if (total == 0) return;
    const uint32_t slot = item / MW, w = item - slot * MW;
    int k = incl - n;
    for (uint32_t d = dirty; d; d &= d - 1) {
        const int b = __builtin_ctz(d);
        // row index slot*HW + cell (< 2^31 by the host's size checks), bit 31 = candidate
        list[k++] = (slot * (uint32_t)Q.HW + 32u * w + (uint32_t)b) | (((cur >> b) & 1u) << 31);
    }
    __syncthreads();
    for (int i = lane; i < total; i += 64) {
        const uint32_t e = list[i], r = e & 0x7FFFFFFFu;
        const int sl = (int)(r / (uint32_t)Q.HW), c = (int)(r - (uint32_t)sl * Q.HW);
        int32_t row[7] = {0, 0, 0, 0, 0, 0, 0};
        if (e >> 31) sampleRecord(Q, Q.masks + (size_t)sl * Q.HW * Q.K, sl, c, row);
        int32_t* dst = Q.actions + (size_t)r * 7;
#pragma unroll
        for (int q = 0; q < 7; q++) dst[q] = row[q];
    }
}

__global__ __launch_bounds__(64) void k_policy(PolicyParams Q) {
    const int c = (int)(blockIdx.x * 64 + threadIdx.x);
    const int slot = (int)blockIdx.y;
    if (c >= Q.HW) return;
    int32_t a[7];
    sampleCell(Q, Q.masks + ((size_t)slot * Q.HW + c) * Q.K, slot, c, a);
    int32_t* out = Q.actions + ((size_t)slot * Q.HW + c) * 7;
#pragma unroll
    for (int k = 0; k < 7; k++) out[k] = a[k];
}

#ifdef MRTS_LANE_AUDIT
// the audit's negative control: a readlane of lane 40 from a branch only lanes 0..31 take
__global__ __launch_bounds__(64) void k_lane_audit_probe(int32_t* out) {
    int v = 0;
    if (threadIdx.x < 32) v = rl((int)threadIdx.x * 3, 40);
    out[threadIdx.x] = v;
}
#endif
}  // namespace

namespace mrts {
#ifdef MRTS_LANE_AUDIT
hipError_t laneAuditProbe(int32_t* scratch) {
    hipLaunchKernelGGL(k_lane_audit_probe, dim3(1), dim3(64), 0, 0, scratch);
    return hipGetLastError();
}
// out[256]: per thread slot the last violation (source line | kind << 24: 1 readlane, 2 DPP, 3 ballot), 0 = none
hipError_t laneAudit(int32_t* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_laneAudit), sizeof(int32_t) * 256);
    if (e == hipSuccess && reset) {
        int32_t z[256] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_laneAudit), z, sizeof(z));
    }
    return e;
}
#endif
#ifdef MRTS_ABLATE
hipError_t setAblate(uint32_t v) { return hipMemcpyToSymbol(HIP_SYMBOL(g_ablate), &v, sizeof(v)); }
hipError_t getDbg(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(unsigned long long) * 4);
    if (e == hipSuccess && reset) {
        unsigned long long z[4] = {0, 0, 0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z));
    }
    return e;
}
#endif
#ifdef MRTS_PHASE_TIMING
// out[16]: per-phase sums over games (and the max over games in out[16..31] when given 32 slots)
hipError_t phaseTimes(unsigned long long* out, int reset) {
    std::vector<unsigned long long> h((size_t)NPH * PH_GAMES);
    hipError_t e = hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_phase), h.size() * sizeof(h[0]));
    if (e != hipSuccess) return e;
    for (int i = 0; i < NPH; i++) {
        unsigned long long sum = 0, mx = 0;
        for (int g = 0; g < PH_GAMES; g++) {
            sum += h[(size_t)i * PH_GAMES + g];
            mx = h[(size_t)i * PH_GAMES + g] > mx ? h[(size_t)i * PH_GAMES + g] : mx;
        }
        out[i] = sum;
        out[NPH + i] = mx;
    }
    if (reset) {
        std::fill(h.begin(), h.end(), 0ull);
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), h.data(), h.size() * sizeof(h[0]));
    }
    return e;
}
hipError_t phaseSpans(unsigned long long* out, int n) {  // [11][n]: starts, ends, placements, milestones of the last launch
    std::vector<unsigned long long> h((size_t)11 * PH_GAMES);
    hipError_t e = hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_span), h.size() * sizeof(h[0]));
    if (e != hipSuccess) return e;
    for (int b = 0; b < 11; b++)  // starts, ends, placements, then the span build's 8 milestones
        for (int i = 0; i < n && i < PH_GAMES; i++) out[(size_t)b * n + i] = h[(size_t)b * PH_GAMES + i];
    return e;
}
#endif
size_t ldsBytes(int HW, int W, int CAP, int po) {
    return (size_t)UTT_LDS + (size_t)16 * CAP + 4 * (size_t)((HW + 2 * W + 31) / 32) + 4 * 64 + 8 * (size_t)maskWords(HW) + 64 + 128 +
           (po ? 4 * (size_t)HW + 8 * (size_t)(HW / W) * (size_t)((W + 31) / 32) : 0) +
           (po && poDeltaShape(HW / W, W) ? 4 * (6 * (size_t)(HW / W) + 6 * (size_t)poChunkWords(HW)) + 4 * (size_t)((HW / 4 + 1) & ~1) : 0) +
           6 * (size_t)CAP + 2 * (size_t)HW + 2 * 64 +
           // the snapshot bytes (PO) — or, full observability on 16x16, the observation byte image (writeObsFullImg)
           std::max((((size_t)CAP + 3) & ~(size_t)3), (!po && HW == 256) ? 5 * (size_t)HW : (size_t)0);
}
// MicroRTS-Py GridnetVecEnv observation encoding (gym_microrts `_encode_obs`: clip each plane to
// [0, n_k - 1], one-hot, channels-last): int32 obs [S][C][H][W] -> uint8 [S][H][W][F] with plane sizes
// n = {5 hp, 5 resources, 3 owner, ntypes + 1 type, 6 action, 2 terrain, 2 per PO visibility plane}.
// One thread per cell over the flattened (slot, cell) index; a block's 256 cells x F bytes are
// composed in LDS and leave as aligned 16-byte stores (256 * F is a multiple of 16 for any F).
struct OneHotParams {
    const int32_t* obs;
    uint8_t* out;
    int32_t n_cells, HW, C, F;
    int32_t sizes[8], offs[8];
};
__global__ __launch_bounds__(256) void k_onehot(OneHotParams Q) {
    __shared__ __align__(16) uint8_t buf[256 * 40];
    const int t = (int)threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.x * 256, i = i0 + t;
    const int F = Q.F;
    for (int k = t; k < 256 * F / 4; k += 256) ((uint32_t*)buf)[k] = 0u;
    __syncthreads();
    if (i < Q.n_cells) {
        const int64_t slot = i / Q.HW;
        const int c = (int)(i - slot * Q.HW);
        const int32_t* o = Q.obs + slot * Q.C * Q.HW + c;
        for (int p = 0; p < Q.C; p++) {
            const int v = min(max(o[(int64_t)p * Q.HW], 0), Q.sizes[p] - 1);
            buf[t * F + Q.offs[p] + v] = 1;
        }
    }
    __syncthreads();
    const int64_t ncell = min((int64_t)256, (int64_t)Q.n_cells - i0);
    const int64_t nbytes = ncell * F, n16 = nbytes / 16;
    uint8_t* dst = Q.out + i0 * F;
    for (int64_t k = t; k < n16; k += 256) ((uint4*)dst)[k] = ((const uint4*)buf)[k];
    for (int64_t k = 16 * n16 + t; k < nbytes; k += 256) dst[k] = buf[k];
}
hipError_t launchOneHot(const int32_t* obs, uint8_t* out, int n_slots, int HW, int C, int ntypes, hipStream_t stream) {
    OneHotParams Q;
    Q.obs = obs;
    Q.out = out;
    Q.n_cells = n_slots * HW;
    Q.HW = HW;
    Q.C = C;
    const int base[6] = {5, 5, 3, ntypes + 1, 6, 2};
    int f = 0;
    for (int p = 0; p < 8; p++) {
        Q.sizes[p] = p < 6 ? base[p] : 2;
        Q.offs[p] = f;
        if (p < C) f += Q.sizes[p];
    }
    Q.F = f;
    if (C > 8 || f > 40 || ((uintptr_t)out & 15)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_onehot, dim3((unsigned)((Q.n_cells + 255) / 256)), dim3(256), 0, stream, Q);
    return hipGetLastError();
}

// int32 copy of a uint8 mask buffer (the Java int[][][][] layout), 16 mask bytes per thread
__global__ __launch_bounds__(256) void k_widen(const uint8_t* __restrict__ in, int32_t* __restrict__ out, size_t n) {
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (i + 16 <= n) {
        const uint4 v = *(const uint4*)(in + i);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++)
            *(int4*)(out + i + 4 * q) = make_int4((int)(w[q] & 0xFF), (int)((w[q] >> 8) & 0xFF), (int)((w[q] >> 16) & 0xFF),
                                                  (int)(w[q] >> 24));
    } else {
        for (size_t k = i; k < n; k++) out[k] = in[k];
    }
}
hipError_t launchWiden(const uint8_t* in, int32_t* out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (((uintptr_t)in & 15) || ((uintptr_t)out & 15)) return hipErrorInvalidValue;
    const size_t threads = (n + 15) / 16;
    hipLaunchKernelGGL(k_widen, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, in, out, n);
    return hipGetLastError();
}
// ---------------------------------------------------------------- forward model
// GameState.clone() (rts/GameState.java:591-610) of pairs (dst game, src game): units, players,
// time, the cancel counter and the assignments (LinkedHashMap order = the sequence numbers) travel;
// the dst game keeps its own random streams (Sampler.generator / GameState.r / UnitAction.r are
// JVM-global, not part of a GameState), its kind (playout policies), and its mask row sets (they
// describe the dst handle's mask buffer).  One block of 256 threads per pair.
// Receiver side of the compact observation exchange: the records of n_ranks x n_games games (rank r's
// game g at rec + r * rank_stride + g * recWords(units) words) back into both player slots'
// observation planes — GameState.getVectorObservation (rts/GameState.java:922-968), the owner plane
// per viewing player (:947-949), the terrain plane from the local handle's map of game g (every rank
// holds the same maps per game index).  out = [n_ranks][2 * n_games][C][HW] as uint8 (out_bytes 1)
// or int32 (4).  One wave per game: the units paint a byte image in LDS, then each lane stores 4 cells
// per plane.  HW <= 256, HW % 4 == 0 (the host checks).
// A record whose overflow bit is set (its game had more units than the record holds) renders without
// the missing units: the kernel then sets *err (mrts_render_status reports it).
__global__ __launch_bounds__(64) void k_render_records(const KStatic* __restrict__ PS, const uint32_t* __restrict__ rec,
                                                       int units, int64_t rank_stride, void* __restrict__ out, int out_bytes,
                                                       int32_t* __restrict__ err) {
    __shared__ uint32_t imgw[5 * 256 / 4];
    uint8_t* img = (uint8_t*)imgw;
    const KStatic& P = *PS;
    const int g = (int)blockIdx.x, r = (int)blockIdx.y, l = (int)threadIdx.x, HW = P.HW, C = P.C, G = P.n_games;
    const uint32_t* rc = rec + (size_t)r * (size_t)rank_stride + (size_t)g * recWords(units, false);
    for (int i = l; i < 5 * HW / 4; i += 64) imgw[i] = 0u;
    const uint32_t hdr = rc[0];
    if (l == 0 && (hdr >> 31)) *err = 1;  // a vector store from one lane (rare)
    __syncthreads();
    const int n = min((int)(hdr & 0xFFFFu), units);
    for (int i = l; i < n; i += 64) {
        const uint32_t w = rc[1 + i];
        const int c = (int)(w & 0xFFu);
        if (c >= HW) continue;  // (a foreign buffer: no LDS write out of range)
        img[c] = (uint8_t)(w >> 8);
        img[HW + c] = (uint8_t)(w >> 16);
        img[2 * HW + c] = (uint8_t)((w >> 27) & 3u);
        img[3 * HW + c] = (uint8_t)((w >> 24) & 7u);
        img[4 * HW + c] = (uint8_t)(w >> 29);
    }
    __syncthreads();
    const uint32_t* terr = (const uint32_t*)(P.tmpl + P.tmpl_off[g] + T_TERR);
    const size_t slot0 = (size_t)r * 2 * G + 2 * (size_t)g;
    for (int c4 = 4 * l; c4 < HW; c4 += 256) {
        uint32_t pw[6];
#pragma unroll
        for (int q = 0; q < 5; q++) pw[q] = imgw[(q * HW + c4) >> 2];
        const uint32_t t = terr[c4 >> 2];  // walls: non-zero terrain bytes
        uint32_t tw = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) tw |= (((t >> (8 * j)) & 0xFFu) ? 1u : 0u) << (8 * j);
        pw[5] = tw;
#pragma unroll
        for (int i = 0; i < 2; i++) {
#pragma unroll
            for (int q = 0; q < 6; q++) {
                uint32_t w = pw[q];
                if (i == 1 && q == 2) {  // the other player's owners: 1 <-> 2, 0 stays
                    uint32_t x = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t b = (w >> (8 * j)) & 0xFFu;
                        x |= (b ? 3u - b : 0u) << (8 * j);
                    }
                    w = x;
                }
                const size_t off = ((slot0 + i) * C + q) * (size_t)HW + c4;
                if (out_bytes == 1) {
                    *(uint32_t*)((uint8_t*)out + off) = w;
                } else {
                    st4<true>((int32_t*)out + off, (int)(w & 0xFFu), (int)((w >> 8) & 0xFFu), (int)((w >> 16) & 0xFFu),
                              (int)(w >> 24));
                }
            }
        }
    }
}
// The same for partially observable handles (PartiallyObservableGameState.getVectorObservation,
// rts/PartiallyObservableGameState.java:82-154, as Game::writeObsPO renders it): per view p, the last
// unit of p's snapshot on each cell (list order) gives planes 0-4 — its live hp, resources, owner
// relative to p, type, and the action type p's snapshot saw — plane 5 the map's walls, planes 6 / 7
// whether a sight disk of one of the view's units owned by p / by the other player covers the cell.
// out = [n_ranks][2 * n_games][8][HW] as int8 (out_bytes 1: a dead unit's hp can be negative) or int32.
// One block of 256 threads per game and rank; LDS: the per-view cell owners (2 x HW words), sight rows
// (2 views x 2 x H x (W + 31) / 32 words) and the record itself (the per-cell lookups stay on chip).
// HW % 4 == 0 (the host checks).
__global__ __launch_bounds__(256) void k_render_records_po(const KStatic* __restrict__ PS, const uint32_t* __restrict__ rec,
                                                           int units, int64_t rank_stride, void* __restrict__ out, int out_bytes,
                                                           int32_t* __restrict__ err) {
    extern __shared__ __align__(16) uint32_t lds[];
    const KStatic& P = *PS;
    const int g = (int)blockIdx.x, r = (int)blockIdx.y, t = (int)threadIdx.x;
    const int H = P.H, W = P.W, HW = P.HW, C = P.C, G = P.n_games, NR = H * ((W + 31) >> 5);
    uint32_t* const sc = lds;             // [view][cell]: index + 1 of the view's last unit on the cell, 0 = none
    uint32_t* const rows = lds + 2 * HW;  // [view][own, other][NR]
    uint32_t* const rc = rows + 4 * NR;   // the record (1 + 2 x units words)
    const uint32_t* rg = rec + (size_t)r * (size_t)rank_stride + (size_t)g * recWords(units, true);
    const int n = min((int)(rg[0] & 0xFFFFu), units);
    if (t == 0 && (rg[0] >> 31)) *err = 1;  // overflow: units or an hp / resource value missing
    for (int i = t; i < 2 * HW + 4 * NR; i += 256) lds[i] = 0u;
    for (int i = t; i < 1 + 2 * n; i += 256) rc[i] = rg[i];
    __syncthreads();
    const int SM = P.utt.maxSight;
    const bool rowPaint = W <= 32 && SM <= 15;  // one word per sight row, table half-widths
    for (int i = t; i < n; i += 256) {  // the views' last unit per cell; and the sight disks (general maps)
        const uint32_t w0 = rc[1 + 2 * i], w1 = rc[2 + 2 * i];
        const int c = (int)(w0 & 0xFFFFu), ty = (int)(w1 & 15u) - 1, pl = (int)((w1 >> 4) & 3u) - 1;
        const uint32_t sb = (c < HW && ty >= 0 && ty < MAX_TYPES) ? (w1 >> 8) & 0xFFu : 0u;  // (a foreign buffer: no LDS write out of range)
        const int x = c % W, y = c / W;
        for (int p = 0; p < 2; p++) {
            if (!((sb >> p) & 1u)) continue;
            atomicMax(&sc[p * HW + c], (uint32_t)(i + 1));
#ifdef MRTS_RENDER_NOPAINT  // diagnostic build: the render without its sight disks
            if (false)
#else
            if (pl >= 0 && !rowPaint)
#endif
                paintDiskRows(rows + (2 * p + (pl == p ? 0 : 1)) * NR, H, W, x, y, P.utt.sight[ty], P.utt.diskLo[ty],
                              P.utt.diskHi[ty]);
        }
    }
#ifndef MRTS_RENDER_NOPAINT
    if (rowPaint) {
        // every (unit, row offset) pair on its own thread: 8 units x 32 row offsets per pass (2 SM + 1 <= 31),
        // one atomicOr per view the unit is in — not one thread looping over a unit's rows
        const int dy = (t & 31) - SM;
        for (int i = t >> 5; i < n; i += 8) {
            const uint32_t w0 = rc[1 + 2 * i], w1 = rc[2 + 2 * i];
            const int c = (int)(w0 & 0xFFFFu), ty = (int)(w1 & 15u) - 1, pl = (int)((w1 >> 4) & 3u) - 1;
            const uint32_t sb = (c < HW && ty >= 0 && ty < MAX_TYPES && pl >= 0) ? (w1 >> 8) & 3u : 0u;
            const int ady = dy < 0 ? -dy : dy, sr = sb ? P.utt.sight[ty] : -1;
            const int x = c % W, yy = c / W + dy;
            if (ady <= sr && yy >= 0 && yy < H) {
                const uint32_t half = ((ady < 8 ? P.utt.diskLo[ty] : P.utt.diskHi[ty]) >> (4 * (ady & 7))) & 0xFu;
                const int x0 = max(0, x - (int)half), x1 = min(W - 1, x + (int)half);
                const uint32_t b = ((2u << (x1 - x0)) - 1u) << x0;  // columns x0..x1 (x1 - x0 = 31: 2u << 31 wraps to 0)
                if (sb & 1u) atomicOr(&rows[(pl == 0 ? 0 : 1) * NR + yy], b);
                if (sb & 2u) atomicOr(&rows[(2 + (pl == 1 ? 0 : 1)) * NR + yy], b);
            }
        }
    }
#endif
    __syncthreads();
    const uint32_t* terr = (const uint32_t*)(P.tmpl + P.tmpl_off[g] + T_TERR);
    const int WPR = (W + 31) >> 5;
    for (int c4 = 4 * t; c4 < HW; c4 += 4 * 256) {
        const uint32_t tw = terr[c4 >> 2];  // walls: non-zero terrain bytes
        for (int p = 0; p < 2; p++) {
            int v[8][4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int c = c4 + j, x = c % W, y = c / W;
                const uint32_t s = sc[p * HW + c];
                const uint32_t w0 = s ? rc[2 * s - 1] : 0u, w1 = s ? rc[2 * s] : 0u;
                const int pl = (int)((w1 >> 4) & 3u) - 1, ca = (int)((w1 >> (10 + 3 * p)) & 7u);
                v[0][j] = s ? (int)(int8_t)(uint8_t)(w0 >> 16) : 0;
                v[1][j] = s ? (int)(w0 >> 24) : 0;
                v[2][j] = (s && pl >= 0) ? ((pl + p) % 2) + 1 : 0;
                v[3][j] = s ? (int)(w1 & 15u) : 0;
                v[4][j] = (s && ca) ? ca - 1 : 0;
                v[5][j] = ((tw >> (8 * j)) & 0xFFu) ? 1 : 0;
                v[6][j] = (int)((rows[(2 * p) * NR + y * WPR + (x >> 5)] >> (x & 31)) & 1u);
                v[7][j] = (int)((rows[(2 * p + 1) * NR + y * WPR + (x >> 5)] >> (x & 31)) & 1u);
            }
            const size_t slot = (size_t)r * 2 * G + 2 * (size_t)g + p;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const size_t off = (slot * C + q) * (size_t)HW + c4;
                if (out_bytes == 1)
                    *(uint32_t*)((uint8_t*)out + off) = (uint32_t)(v[q][0] & 0xFF) | ((uint32_t)(v[q][1] & 0xFF) << 8) |
                                                         ((uint32_t)(v[q][2] & 0xFF) << 16) | ((uint32_t)(v[q][3] & 0xFF) << 24);
                else
                    st4<true>((int32_t*)out + off, v[q][0], v[q][1], v[q][2], v[q][3]);
            }
        }
    }
}
// A learner's batch straight from the exchanged records, in the layout it consumes: the
// MicroRTS-Py encoding of the observation (gym_microrts `_encode_obs`, as k_onehot: clip each plane, one-hot,
// channels last) of n_sel samples: sample i is slot sel[i] (global index r * n_slots + slot over every rank's
// slots) of the step whose rank-0 records start at rec + step_off[2i] with rank stride step_off[2i + 1] (the
// rollout's step_offsets row; null: rec and rank_stride) — a minibatch of (step, slot) pairs from a whole
// rollout window in one launch, with no int32 / uint8 planes of all ranks in between.  Full observability.  One 256-thread block per selected
// slot: its game's record paints the 5 dynamic planes as bytes in LDS (as k_render_records), each cell's
// F one-hot bytes are composed in LDS, and the slot's H x W x F bytes leave as aligned 16-byte stores.
// out = [n_sel][H][W][F] uint8 (HW * F % 16 == 0, the host checks).
__global__ __launch_bounds__(256) void k_render_records_onehot(const KStatic* __restrict__ PS, const uint32_t* __restrict__ rec,
                                                               int units, int64_t rank_stride, const int32_t* __restrict__ sel,
                                                               const int64_t* __restrict__ step_off, uint8_t* __restrict__ out,
                                                               OneHotParams Q, int32_t* __restrict__ err, int64_t rec_words,
                                                               int n_ranks) {
    __shared__ uint32_t imgw[5 * 256 / 4];
    __shared__ __align__(16) uint8_t buf[256 * 40];
    uint8_t* img = (uint8_t*)imgw;
    const KStatic& P = *PS;
    const int t = (int)threadIdx.x, HW = P.HW, S = 2 * P.n_games, F = Q.F;
    const int gs = sel[blockIdx.x];
    const int r = gs / S, slot = gs - r * S, g = slot >> 1, p = slot & 1;
    const int64_t o = step_off ? step_off[2 * blockIdx.x] : 0, rs = step_off ? step_off[2 * blockIdx.x + 1] : rank_stride;
    // a sample outside the buffer (a bad sel index or step_off row): a zero image and the render flag
    // (mrts_render_status), never a read past the receive buffer.  Block-uniform: the whole block returns.
    const int64_t at = o + (int64_t)r * rs + (int64_t)g * recWords(units, false);
    if (gs < 0 || r >= n_ranks || o < 0 || rs < 0 || at + recWords(units, false) > rec_words) {
        if (t == 0) *err = 1;
        uint4* dz = (uint4*)(out + (size_t)blockIdx.x * HW * F);
        for (int k = t; k < HW * F / 16; k += 256) dz[k] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const uint32_t* rc = rec + at;
    for (int i = t; i < 5 * HW / 4; i += 256) imgw[i] = 0u;
    for (int k = t; k < HW * F / 4; k += 256) ((uint32_t*)buf)[k] = 0u;
    const uint32_t hdr = rc[0];
    if (t == 0 && (hdr >> 31)) *err = 1;  // overflow (mrts_render_status)
    __syncthreads();
    const int n = min((int)(hdr & 0xFFFFu), units);
    for (int i = t; i < n; i += 256) {
        const uint32_t w = rc[1 + i];
        const int c = (int)(w & 0xFFu);
        if (c >= HW) continue;
        img[c] = (uint8_t)(w >> 8);
        img[HW + c] = (uint8_t)(w >> 16);
        img[2 * HW + c] = (uint8_t)((w >> 27) & 3u);  // player + 1 (0 = none)
        img[3 * HW + c] = (uint8_t)((w >> 24) & 7u);
        img[4 * HW + c] = (uint8_t)(w >> 29);
    }
    __syncthreads();
    const uint8_t* terr = (const uint8_t*)(P.tmpl + P.tmpl_off[g] + T_TERR);
    for (int c = t; c < HW; c += 256) {
        const int pl1 = img[2 * HW + c];  // owner plane of slot p: ((player + p) % 2) + 1
        const int v[6] = {img[c], img[HW + c], pl1 ? ((pl1 - 1 + p) & 1) + 1 : 0, img[3 * HW + c], img[4 * HW + c],
                          terr[c] ? 1 : 0};
#pragma unroll
        for (int q = 0; q < 6; q++) buf[c * F + Q.offs[q] + min(max(v[q], 0), Q.sizes[q] - 1)] = 1;
    }
    __syncthreads();
    uint4* dst = (uint4*)(out + (size_t)blockIdx.x * HW * F);
    for (int k = t; k < HW * F / 16; k += 256) dst[k] = ((const uint4*)buf)[k];
}
hipError_t launchRenderRecordsOneHot(const KStatic& hs, const KStatic* ds, const uint32_t* rec, int64_t rec_words, int n_ranks,
                                     int units, int64_t rank_stride, const int32_t* sel, const int64_t* step_off, int n_sel,
                                     uint8_t* out, int32_t* err, hipStream_t stream) {
    OneHotParams Q{};
    const int base[6] = {5, 5, 3, hs.utt.ntypes + 1, 6, 2};
    int f = 0;
    for (int q = 0; q < 6; q++) {
        Q.sizes[q] = base[q];
        Q.offs[q] = f;
        f += base[q];
    }
    Q.F = f;
    if (hs.partial_obs || hs.HW > 256 || f > 40 || ((size_t)hs.HW * f) % 16 || ((uintptr_t)out & 15)) return hipErrorInvalidValue;
    if (n_sel <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_render_records_onehot, dim3((unsigned)n_sel), dim3(256), 0, stream, ds, rec, units, rank_stride, sel,
                       step_off, out, Q, err, rec_words, n_ranks);
    return hipGetLastError();
}
hipError_t launchRenderRecords(const KStatic& hs, const KStatic* ds, const uint32_t* rec, int units, int n_ranks,
                               int64_t rank_stride, void* out, int out_bytes, int32_t* err, hipStream_t stream) {
    if (hs.partial_obs) {
        const size_t lds = 4 * (size_t)(2 * hs.HW + 4 * hs.H * ((hs.W + 31) / 32) + recWords(units, true));
        hipLaunchKernelGGL(k_render_records_po, dim3((unsigned)hs.n_games, (unsigned)n_ranks), dim3(256), lds, stream, ds, rec,
                           units, rank_stride, out, out_bytes, err);
    } else {
        hipLaunchKernelGGL(k_render_records, dim3((unsigned)hs.n_games, (unsigned)n_ranks), dim3(64), 0, stream, ds, rec, units,
                           rank_stride, out, out_bytes, err);
    }
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_copy_games(int32_t* __restrict__ dst, const int32_t* __restrict__ src,
                                                    const int32_t* __restrict__ pairs, int n_dst, int n_src,
                                                    int words, int maskLo, int maskHi) {
    const int d = pairs[2 * blockIdx.x], s = pairs[2 * blockIdx.x + 1];
    if (d < 0 || d >= n_dst || s < 0 || s >= n_src) return;
    int32_t* o = dst + (size_t)d * words;
    const int32_t* i = src + (size_t)s * words;
    for (int w = threadIdx.x; w < words; w += 256) {
        const bool keep = (w >= H_RNG_CANCEL && w <= H_KIND) || (w >= maskLo && w < maskHi);
        if (!keep) o[w] = w == H_STEPS ? 0 : i[w];
    }
}
hipError_t launchCopyGames(int32_t* dst, const int32_t* src, const int32_t* pairs, int n, int n_dst, int n_src,
                           int CAP, int HW, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int lo = H_WORDS + N_ARRAYS * CAP;
    hipLaunchKernelGGL(k_copy_games, dim3((unsigned)n), dim3(256), 0, stream, dst, src, pairs, n_dst, n_src,
                       stateWords(CAP, HW), lo, lo + 2 * maskWords(HW));
    return hipGetLastError();
}

// SimpleSqrtEvaluationFunction3.evaluate(maxplayer, 1 - maxplayer, gs)
// (ai/evaluation/SimpleSqrtEvaluationFunction3.java:24-44), Java float semantics: the unit loop runs
// in list order, `score += res * 10f` is a float add, `score += 40f * cost * Math.sqrt(hp / maxHp)`
// (integer division) is a double add rounded back to float; no contraction into FMAs.  One wave per
// game: lanes load 64 units at a time, every lane runs the same ordered sum over readlane values.
__global__ __launch_bounds__(64) void k_evaluate(const KStatic* __restrict__ PS, const int32_t* __restrict__ state,
                                                 int words, int CAP, int maxplayer, float* __restrict__ out) {
#pragma clang fp contract(off)
    const KStatic& P = *PS;
    const int32_t* s = state + (size_t)blockIdx.x * words;
    const int nu = uni(s[H_NU]);
    const int l = lane_id();
    float score[2];
    bool any[2] = {false, false};
    score[0] = __fmul_rn((float)uni(s[H_RES0]), 20.0f);
    score[1] = __fmul_rn((float)uni(s[H_RES1]), 20.0f);
    for (int o0 = 0; o0 < nu; o0 += 64) {
        const int o = o0 + l;
        uint32_t c = UC_DEAD;
        int hpv = 0, rv = 0;
        if (o < nu) {
            c = (uint32_t)s[H_WORDS + A_UC * CAP + o];
            hpv = s[H_WORDS + A_HP * CAP + o];
            rv = s[H_WORDS + A_RES * CAP + o];
        }
        const int n = min(64, nu - o0);
        for (int k = 0; k < n; k++) {
            const uint32_t ck = (uint32_t)rl((int)c, k);
            if (ck & UC_DEAD) continue;
            const int p = uplay(ck);
            if (p != 0 && p != 1) continue;
            const int typ = utyp(ck);
            const int h = rl(hpv, k), r = rl(rv, k);
            float sc = score[p];
            sc = __fadd_rn(sc, __fmul_rn((float)r, 10.0f));
            const double bonus = __dmul_rn((double)__fmul_rn(40.0f, (float)P.utt.cost[typ]),
                                           __builtin_sqrt((double)(h / P.utt.hp[typ])));
            sc = (float)__dadd_rn((double)sc, bonus);
            score[p] = sc;
            any[p] = true;
        }
    }
    const float s1 = any[maxplayer] ? score[maxplayer] : 0.0f;
    const float s2 = any[1 - maxplayer] ? score[1 - maxplayer] : 0.0f;
    const float tot = __fadd_rn(s1, s2);
    const float v = tot == 0.0f ? 0.5f : __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, s1), tot), 1.0f);
    if (l == 0) out[blockIdx.x] = v;
}
hipError_t launchEvaluate(const KStatic& hs, const KStatic* ds, int maxplayer, float* out, hipStream_t stream) {
    hipLaunchKernelGGL(k_evaluate, dim3((unsigned)hs.n_games), dim3(64), 0, stream, ds, hs.state,
                       stateWords(hs.CAP, hs.HW), hs.CAP, maxplayer, out);
    return hipGetLastError();
}

// e0 / e1 (may be null): timing events the launch records itself (hipExtLaunchKernelGGL: the kernel
// dispatch's own start / end timestamps — no separate marker packets around it; mrts_set_rollout_events)
hipError_t launchEnv(int mode, const KStatic& hs, const KStatic* ds, const KDyn& D, hipStream_t stream, hipEvent_t e0, hipEvent_t e1) {
    const size_t lds = ldsBytes(hs.HW, hs.W, hs.CAP, hs.partial_obs);
    dim3 grid((unsigned)hs.n_games), block(64);
    const bool fixable = hs.n_sp_games == hs.n_games && D.rows == nullptr && hs.utt.K == 79 && hs.utt.ntypes == 7 &&
                         hs.utt.maxAttackRadius == 7 && hs.H == hs.W;
    auto is = [&](int w, int cap, bool po) { return fixable && hs.W == w && hs.CAP == cap && (hs.partial_obs != 0) == po; };
#if MRTS_EXT_EVENTS
#define LAUNCH(kern, g_, b_, l_, s_, ...) hipExtLaunchKernelGGL(kern, g_, b_, (uint32_t)(l_), s_, e0, e1, 0, __VA_ARGS__)
#else  // events as separate records around the launch (A/B builds)
#define LAUNCH(kern, g_, b_, l_, s_, ...)                                 \
    do {                                                                  \
        if (e0) (void)hipEventRecord(e0, s_);                             \
        hipLaunchKernelGGL(kern, g_, b_, (uint32_t)(l_), s_, __VA_ARGS__); \
        if (e1) (void)hipEventRecord(e1, s_);                             \
    } while (0)
#endif
    switch (mode) {
        case MODE_STEP:
            if (D.n_iter > 1 && is(16, 320, false)) LAUNCH((k_env<MODE_STEP, 16, 320, false, true>), grid, block, lds, stream, D.state, ds, D);
            else if (D.n_iter > 1 && is(8, 128, false) && D.uni_actions && !D.masks) {
                // c2's fused uniform rollout: a helper wave per game (helperLoop)
                KDyn D2 = D;
                D2.help_off = (int32_t)((lds + 15) & ~(size_t)15);
                LAUNCH((k_env<MODE_STEP, 8, 128, false, true, true>), grid, dim3(128), (size_t)D2.help_off + 2048, stream,
                                   D.state, ds, D2);
            } else if (D.n_iter > 1 && is(8, 128, false)) LAUNCH((k_env<MODE_STEP, 8, 128, false, true>), grid, block, lds, stream, D.state, ds, D);
            else if (D.n_iter > 1 && is(32, 320, true) && D.obs && !MRTS_NO_PO_HELPER) {
                // c5's partially observable rollout: a helper wave per game renders the views (helperLoopPO)
                KDyn D2 = D;
                D2.help_off = (int32_t)((lds + 15) & ~(size_t)15);
                LAUNCH((k_env<MODE_STEP, 32, 320, true, true, true>), grid, dim3(128), (size_t)D2.help_off + 4 * (PO_HELP_REC + PO_HELP_REC_WORDS),
                                   stream, D.state, ds, D2);
            } else if (D.n_iter > 1 && is(32, 320, true)) LAUNCH((k_env<MODE_STEP, 32, 320, true, true>), grid, block, lds, stream, D.state, ds, D);
            else if (is(16, 320, false)) LAUNCH((k_env<MODE_STEP, 16, 320, false>), grid, block, lds, stream, D.state, ds, D);
            else if (is(8, 128, false)) LAUNCH((k_env<MODE_STEP, 8, 128, false>), grid, block, lds, stream, D.state, ds, D);
            else if (is(32, 320, true)) LAUNCH((k_env<MODE_STEP, 32, 320, true>), grid, block, lds, stream, D.state, ds, D);
            else LAUNCH((k_env<MODE_STEP, 0>), grid, block, lds, stream, D.state, ds, D);
            break;
        case MODE_RESET: LAUNCH((k_env<MODE_RESET, 0>), grid, block, lds, stream, D.state, ds, D); break;
        case MODE_PLAYOUT: LAUNCH((k_env<MODE_PLAYOUT, 0>), grid, block, lds, stream, D.state, ds, D); break;
        case MODE_TRACE: {
            // the specialised 16x16 / 8x8 step instances' dimensions (their games' code with constant
            // sizes), else the generic kernel
            const bool fix = !D.trace_generic && hs.utt.K == 79 && hs.utt.ntypes == 7 && hs.utt.maxAttackRadius == 7 &&
                             hs.H == hs.W && !hs.partial_obs;
            if (fix && hs.W == 16 && hs.CAP == 320) LAUNCH((k_env<MODE_TRACE, 16, 320>), grid, block, lds, stream, D.state, ds, D);
            else if (fix && hs.W == 8 && hs.CAP == 128) LAUNCH((k_env<MODE_TRACE, 8, 128>), grid, block, lds, stream, D.state, ds, D);
            else LAUNCH((k_env<MODE_TRACE, 0>), grid, block, lds, stream, D.state, ds, D);
        } break;
        default:LAUNCH((k_env<MODE_MASKS, 0>), grid, block, lds, stream, D.state, ds, D); break;
    }
#undef LAUNCH
    return hipGetLastError();
}
// launchEnv(MODE_STEP) would run a specialised self-play kernel (16x16 / 8x8 full observability,
// 32x32 partially observable), the ones whose games can iterate several steps in one launch
// (KDyn.n_iter, MULTI instances)
bool envIterable(const KStatic& hs) {
    const bool fixable = hs.n_sp_games == hs.n_games && hs.utt.K == 79 && hs.utt.ntypes == 7 && hs.utt.maxAttackRadius == 7 &&
                         hs.H == hs.W;
    return fixable && ((hs.W == 16 && hs.CAP == 320 && !hs.partial_obs) || (hs.W == 8 && hs.CAP == 128 && !hs.partial_obs) ||
                       (hs.W == 32 && hs.CAP == 320 && hs.partial_obs));
}
hipError_t prepareLds(size_t bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_env<MODE_STEP, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_RESET, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_MASKS, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_PLAYOUT, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_TRACE, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    return e;
}
// Unmasked uniform random policy (BASELINE config c2), uniformRow for every cell of
// every slot.  One thread per (slot, cell): the whole action tensor, dwordx4 + dwordx3 per row.
__global__ __launch_bounds__(64) void k_policy_uniform(int32_t* __restrict__ actions, int HW, int ntypes, int natt,
                                                        uint64_t seed, uint32_t step, uint32_t slot_base) {
    const int slot = (int)blockIdx.y, c = (int)(blockIdx.x * 64 + threadIdx.x);
    if (c >= HW) return;
    int32_t a[7];
    uniformRow(seed, step, slot_base + (uint32_t)slot, c, ntypes, natt, a);
    int32_t* dst = actions + ((size_t)slot * HW + c) * 7;
    st4u<false>(dst, a[0], a[1], a[2], a[3]);
    st3u<false>(dst + 4, a[4], a[5], a[6]);
}
hipError_t launchPolicyUniform(int32_t* actions, int n_slots, int HW, int ntypes, int natt, uint64_t seed, uint32_t step,
                               uint32_t slot_base, hipStream_t stream) {
    if (n_slots <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_policy_uniform, dim3((unsigned)((HW + 63) / 64), (unsigned)n_slots), dim3(64), 0, stream, actions, HW,
                       ntypes, natt, seed, step, slot_base);
    return hipGetLastError();
}

// *prevWritten: the launch recorded its candidate set in Q.prev (a later call may use the delta form)
hipError_t launchPolicy(const PolicyParams& Q, hipStream_t stream, bool* prevWritten) {
    dim3 grid((unsigned)((Q.HW + 63) / 64), (unsigned)Q.n_slots), block(64);
    const bool srcOk = Q.source && ((size_t)Q.HW * Q.K) % 16 == 0 && Q.HW % 4 == 0 && Q.K <= 96 && Q.K >= 65;
    *prevWritten = srcOk && Q.prev_out;
    if (srcOk && Q.delta && Q.prev)
        hipLaunchKernelGGL(k_policy_delta, dim3((unsigned)(((size_t)Q.n_slots * ((Q.HW + 31) / 32) + 63) / 64)), block,
                           0, stream, Q);
    else if (srcOk)
        hipLaunchKernelGGL(k_policy_src, dim3((unsigned)Q.n_slots), block, 0, stream, Q);
    else if (((size_t)Q.HW * Q.K) % 16 == 0 && (64 * Q.K) % 16 == 0 && Q.HW % 4 == 0 && Q.K <= 96)
        hipLaunchKernelGGL(k_policy_tiled, grid, block, 0, stream, Q);
    else
        hipLaunchKernelGGL(k_policy, grid, block, 0, stream, Q);
    return hipGetLastError();
}
}  // namespace mrts
