// mrts_kernels.hip — gfx950 kernels for the vectorised microRTS env step.
//
// One 64-lane wavefront (= one workgroup) owns one game.  The game's units live in LDS as
// struct-of-arrays in PhysicalGameState list order (slot order == LinkedList order), with a
// cell -> slot occupancy map (one live unit per cell is an engine invariant:
// PhysicalGameState.addUnit, reference src/rts/PhysicalGameState.java:189-201).  The Java
// semantics are order-dependent (rows in cell order, fillWithNones in list order, conflict scans
// and cycle() execution in LinkedHashMap insertion order), so every ORDERED decision runs
// wave-uniformly (all lanes agree, scalar branches), while every order-free sub-problem
// (candidate search, row decode, legality, conflict flags, ready flags, death compaction,
// observation planes, legal-action masks) runs lane-parallel with ballots/reductions.
// No MFMA: integer/indexing work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrts_internal.h"

using namespace mrts;

#define DEV __device__ __forceinline__

namespace {

constexpr uint16_t EMPTY = 0xFFFF, WALL = 0xFFFE;
enum { T_NONE = 0, T_MOVE = 1, T_HARVEST = 2, T_RETURN = 3, T_PRODUCE = 4, T_ATTACK = 5 };
enum { MODE_STEP = 0, MODE_RESET = 1, MODE_MASKS = 2 };
enum : uint32_t {
    E_CAPACITY = 1u << 0, E_ADDUNIT = 1u << 1, E_PRODUCE_TYPE = 1u << 2, E_OLDER = 1u << 3,
    E_NEG_RES = 1u << 4, E_COLLISION = 1u << 5
};

DEV int lane_id() { return (int)threadIdx.x; }
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

DEV int rl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
DEV int wave_min(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return uni(v);
}
DEV int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return uni(v);
}
DEV uint64_t ballot(bool p) { return __ballot(p); }
DEV void wsync() { __syncthreads(); }  // one wave per workgroup: s_barrier is nearly free

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
};

struct Game {
    const KParams& P;
    const DevUtt& U;
    int g, H, W, HW, CAP;
    uint32_t* uc;   // unit core: x | y<<8 | type<<16 | (player+1)<<20 | dead<<31
    uint32_t* ua;   // assignment: type | utype<<4 | tx<<8 | ty<<16 | PRESENT/READY/PA flags
    int32_t* at;    // assignment issue time (UnitActionAssignment.time)
    int32_t* as;    // assignment insertion sequence number
    int16_t* hp;
    int16_t* res;
    int16_t* par;   // UnitAction.parameter (direction / NONE duration)
    uint16_t* cell; // cell -> slot, EMPTY or WALL
    uint32_t* bits; // running ResourceUsage positions, indices [-W, HW+W)
    // wave-uniform scalars (only ever modified in uniform control flow)
    int time, nu, pres0, pres1, seq, steps, ccnt, deaths;
    uint32_t err;
    JRand rngCancel, rngDamage, rngSampler;

    DEV Game(const KParams& p, uint8_t* smem)
        : P(p), U(p.utt), g((int)blockIdx.x), H(p.H), W(p.W), HW(p.HW), CAP(p.CAP) {
        uint8_t* q = smem;
        uc = (uint32_t*)q; q += 4 * CAP;
        ua = (uint32_t*)q; q += 4 * CAP;
        at = (int32_t*)q; q += 4 * CAP;
        as = (int32_t*)q; q += 4 * CAP;
        bits = (uint32_t*)q; q += 4 * ((HW + 2 * W + 31) / 32);
        hp = (int16_t*)q; q += 2 * CAP;
        res = (int16_t*)q; q += 2 * CAP;
        par = (int16_t*)q; q += 2 * CAP;
        cell = (uint16_t*)q;
    }
    DEV int pres(int p) const { return p == 0 ? pres0 : pres1; }
    DEV void addPres(int p, int v) {
        if (p == 0) pres0 += v;
        else pres1 += v;
    }
    DEV bool inb(int x, int y) const { return x >= 0 && x < W && y >= 0 && y < H; }
    DEV const int32_t* tmpl() const { return P.tmpl + P.tmpl_off[g]; }
    DEV int32_t* st() const { return P.state + (size_t)g * stateWords(CAP); }

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
    DEV int etaSlot(int s) const {
        uint32_t a = ua[s];
        return eta(ua_type(a), par[s], ua_ut(a), utyp(uc[s]));
    }

    // ------------------------------------------------------------------ state load / store
    DEV void initCells() {  // terrain walls from the map template, units on top
        const int32_t* t = tmpl();
        const int nu_t = t[T_NU];
        const uint8_t* terr = (const uint8_t*)(t + T_UNITS + 3 * nu_t);
        for (int c = lane_id(); c < HW; c += 64) cell[c] = terr[c] ? WALL : EMPTY;
        wsync();
    }
    DEV void placeUnits() {
        for (int i = lane_id(); i < nu; i += 64) {
            uint32_t c = uc[i];
            if (!(c & UC_DEAD)) cell[uy(c) * W + ux(c)] = (uint16_t)i;
        }
        wsync();
    }
    DEV void load() {
        const int32_t* s = st();
        int hv = lane_id() < H_WORDS ? s[lane_id()] : 0;
        time = rl(hv, H_TIME);
        nu = rl(hv, H_NU);
        pres0 = rl(hv, H_RES0);
        pres1 = rl(hv, H_RES1);
        seq = rl(hv, H_SEQ);
        steps = rl(hv, H_STEPS);
        err = (uint32_t)rl(hv, H_ERR);
        ccnt = rl(hv, H_CANCEL_CNT);
        rngCancel.s = (uint64_t)(uint32_t)rl(hv, H_RNG_CANCEL) | ((uint64_t)(uint32_t)rl(hv, H_RNG_CANCEL + 1) << 32);
        rngDamage.s = (uint64_t)(uint32_t)rl(hv, H_RNG_DAMAGE) | ((uint64_t)(uint32_t)rl(hv, H_RNG_DAMAGE + 1) << 32);
        rngSampler.s = (uint64_t)(uint32_t)rl(hv, H_RNG_SAMPLER) | ((uint64_t)(uint32_t)rl(hv, H_RNG_SAMPLER + 1) << 32);
        deaths = 0;
        const int32_t* arr = s + H_WORDS;
        for (int i = lane_id(); i < nu; i += 64) {
            uc[i] = (uint32_t)arr[A_UC * CAP + i];
            hp[i] = (int16_t)arr[A_HP * CAP + i];
            res[i] = (int16_t)arr[A_RES * CAP + i];
            ua[i] = (uint32_t)arr[A_UA * CAP + i];
            par[i] = (int16_t)arr[A_PAR * CAP + i];
            at[i] = arr[A_AT * CAP + i];
            as[i] = arr[A_AS * CAP + i];
        }
        initCells();
        placeUnits();
    }
    DEV void store() {
        int32_t* s = st();
        int l = lane_id();
        int hv = 0;
        switch (l) {
            case H_TIME: hv = time; break;
            case H_NU: hv = nu; break;
            case H_RES0: hv = pres0; break;
            case H_RES1: hv = pres1; break;
            case H_SEQ: hv = seq; break;
            case H_STEPS: hv = steps; break;
            case H_ERR: hv = (int)err; break;
            case H_CANCEL_CNT: hv = ccnt; break;
            case H_RNG_CANCEL: hv = (int)(uint32_t)rngCancel.s; break;
            case H_RNG_CANCEL + 1: hv = (int)(uint32_t)(rngCancel.s >> 32); break;
            case H_RNG_DAMAGE: hv = (int)(uint32_t)rngDamage.s; break;
            case H_RNG_DAMAGE + 1: hv = (int)(uint32_t)(rngDamage.s >> 32); break;
            case H_RNG_SAMPLER: hv = (int)(uint32_t)rngSampler.s; break;
            case H_RNG_SAMPLER + 1: hv = (int)(uint32_t)(rngSampler.s >> 32); break;
        }
        if (l < H_WORDS) s[l] = hv;
        int32_t* arr = s + H_WORDS;
        for (int i = l; i < nu; i += 64) {
            arr[A_UC * CAP + i] = (int32_t)uc[i];
            arr[A_HP * CAP + i] = hp[i];
            arr[A_RES * CAP + i] = res[i];
            arr[A_UA * CAP + i] = (int32_t)ua[i];
            arr[A_PAR * CAP + i] = par[i];
            arr[A_AT * CAP + i] = at[i];
            arr[A_AS * CAP + i] = as[i];
        }
    }
    // new GameState(PhysicalGameState.load(map)) — JNIGridnetClient.reset (tests/JNIGridnetClient.java:239-241)
    DEV void resetFromTemplate() {
        const int32_t* t = tmpl();
        const int nu_t = t[T_NU];
        time = 0;
        seq = 0;
        steps = 0;
        deaths = 0;
        pres0 = t[T_RES0];
        pres1 = t[T_RES1];
        nu = nu_t;
        for (int i = lane_id(); i < nu_t; i += 64) {
            uc[i] = (uint32_t)t[T_UNITS + i];
            hp[i] = (int16_t)t[T_UNITS + nu_t + i];
            res[i] = (int16_t)t[T_UNITS + 2 * nu_t + i];
            ua[i] = 0;
            par[i] = -1;
            at[i] = 0;
            as[i] = 0;
        }
        wsync();
        for (int c = lane_id(); c < HW; c += 64)
            if (cell[c] != WALL) cell[c] = EMPTY;
        wsync();
        placeUnits();
    }

    // ------------------------------------------------------------------ decode (fromVectorAction)
    // Base reservations of every current assignment (PlayerAction.java:497-505, the merge at
    // ResourceUsage.java:92-97); returns their per-player resource sums.
    DEV void baseReservations(int& r0, int& r1) {
        const int NB = (HW + 2 * W + 31) / 32;
        for (int i = lane_id(); i < NB; i += 64) bits[i] = 0;
        wsync();
        int s0 = 0, s1 = 0;
        for (int o = lane_id(); o < nu; o += 64) {
            uint32_t a = ua[o];
            if (a & UA_PRESENT) {
                int t = ua_type(a);
                if (t == T_MOVE || t == T_PRODUCE) {
                    uint32_t c = uc[o];
                    int d = par[o];
                    int pos = (uy(c) + dyo(d)) * W + ux(c) + dxo(d) + W;
                    atomicOr(&bits[pos >> 5], 1u << (pos & 31));
                    if (t == T_PRODUCE) {
                        if (uplay(c) == 0) s0 += U.cost[ua_ut(a)];
                        else s1 += U.cost[ua_ut(a)];
                    }
                }
            }
        }
        r0 = wave_sum(s0);
        r1 = wave_sum(s1);
        wsync();
    }

    // PlayerAction.fromVectorAction (rts/PlayerAction.java:495-528) + UnitAction.fromVectorAction
    // (rts/UnitAction.java:675-709): rows in ascending cell order; a row is decoded iff the unit at
    // its cell is owned by p and has no assignment; accepted iff ua.ru.consistentWith(running ru)
    // (rts/ResourceUsage.java:31-50).  Accepted actions are parked in the unit's (empty) assignment
    // fields with the UA_PA flag.
    DEV void decode(int p, const int32_t* rows) {
        int run0, run1;
        baseReservations(run0, run1);
        const int R = U.maxAttackRadius, ctr = R / 2;
        for (int c0 = 0; c0 < HW; c0 += 64) {
            const int c = c0 + lane_id();
            const int s = c < HW ? cell[c] : EMPTY;
            const uint32_t cu = s < CAP ? uc[s] : 0u;
            const bool cand = s < CAP && uplay(cu) == p && !(ua[s] & UA_PRESENT);
            uint64_t m = ballot(cand);
            if (m == 0) continue;
            int t = 0, pr = -1, ut = 0, tx = 0, ty = 0, tpos = 0, cost = 0;
            bool usesPos = false, bad = false;
            if (cand) {
                const int32_t* r = rows + (size_t)c * 7;
                const int a0 = r[0], a1 = r[1], a2 = r[2], a3 = r[3], a4 = r[4], a5 = r[5], a6 = r[6];
                const int x = ux(cu), y = uy(cu);
                t = (a0 >= 0 && a0 <= 5) ? a0 : ACT_INVALID;
                switch (t) {
                    case T_MOVE: pr = clampdir(a1); break;
                    case T_HARVEST: pr = clampdir(a2); break;
                    case T_RETURN: pr = clampdir(a3); break;
                    case T_PRODUCE:
                        pr = clampdir(a4);
                        if (a5 < 0 || a5 >= U.ntypes) bad = true;  // utt.getUnitType(int) throws
                        else ut = a5;
                        break;
                    case T_ATTACK: {
                        const int ax = x + (a6 % R - ctr), ay = y + (a6 / R - ctr);
                        if (inb(ax, ay)) {
                            tx = ax;
                            ty = ay;
                        } else {
                            tx = ty = 255;  // off-map target: never legal
                        }
                    } break;
                }
                usesPos = (t == T_MOVE || t == T_PRODUCE);
                tpos = c + dyo(pr) * W + dxo(pr);  // ResourceUsage position (UnitAction.java:254-291)
                cost = (t == T_PRODUCE && !bad) ? U.cost[ut] : 0;
            }
            if (ballot(bad)) err |= E_PRODUCE_TYPE;
            uint64_t acc = 0;
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                if (rl(bad, k)) continue;
                const bool up = rl(usesPos, k);
                const int tp = rl(tpos, k), cst = rl(cost, k);
                bool ok = true;
                const int bi = tp + W;
                if (up) ok = !((bits[bi >> 5] >> (bi & 31)) & 1u);
                if (run0 != 0) {
                    const int sum = (p == 0 ? cst : 0) + run0;
                    if (sum > 0 && sum > pres0) ok = false;
                }
                if (run1 != 0) {
                    const int sum = (p == 1 ? cst : 0) + run1;
                    if (sum > 0 && sum > pres1) ok = false;
                }
                if (ok) {
                    if (up && lane_id() == 0) bits[bi >> 5] |= 1u << (bi & 31);
                    if (p == 0) run0 += cst;
                    else run1 += cst;
                    acc |= 1ull << k;
                }
            }
            if ((acc >> lane_id()) & 1ull) {
                ua[s] = pack_ua(t, ut, tx, ty) | UA_PA;
                par[s] = (int16_t)pr;
            }
            wsync();
        }
    }

    // ------------------------------------------------------------------ issueSafe / issue
    // Unit.canExecuteAction (rts/units/Unit.java:531-534) = membership in getUnitActions
    // (:382-522) under UnitAction.equals (rts/UnitAction.java:191-208); an illegal action becomes
    // NONE(ETA(original)) (rts/GameState.java:347-354).  Lane-local.
    DEV void legality(int s, int& t, int& prm, int& tx, int& ty, int& ut) const {
        const uint32_t cu = uc[s];
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

    // GameState.issue for one pair (rts/GameState.java:252-326), wave-uniform arguments.
    DEV void issueOne(int s, int t, int prm, int tx, int ty, int ut) {
        if (t == T_MOVE || t == T_PRODUCE) {
            const uint32_t cu = uc[s];
            const int pl = uplay(cu), typ = utyp(cu);
            const int ntgt = (uy(cu) + dyo(prm)) * W + ux(cu) + dxo(prm);
            const bool nProduce = (t == T_PRODUCE);
            const int ncost = nProduce ? U.cost[ut] : 0;
            int lastSeq = -1;
            while (true) {
                // next conflicting assignment in insertion order (consistentWith against the
                // ORIGINAL ru of the new action; the old action as it is now)
                int best = 0x7FFFFFFF;
                for (int o = lane_id(); o < nu; o += 64) {
                    const uint32_t a = ua[o];
                    if (!(a & UA_PRESENT) || as[o] <= lastSeq) continue;
                    const int ot = ua_type(a);
                    if (ot != T_MOVE && ot != T_PRODUCE) continue;
                    const uint32_t oc = uc[o];
                    const int od = par[o];
                    bool conf = ((uy(oc) + dyo(od)) * W + ux(oc) + dxo(od)) == ntgt;
                    if (nProduce) {
                        const int ores = (ot == T_PRODUCE && uplay(oc) == pl) ? U.cost[ua_ut(a)] : 0;
                        const int sum = ores + ncost;
                        if (sum > 0 && sum > pres(pl)) conf = true;
                    }
                    if (conf) best = min(best, as[o]);
                }
                best = wave_min(best);
                if (best == 0x7FFFFFFF) break;
                int os = -1;
                for (int o = lane_id(); o < nu; o += 64)
                    if ((ua[o] & UA_PRESENT) && as[o] == best) os = o;
                os = wave_min(os < 0 ? 0x7FFFFFFF : os);
                lastSeq = best;
                if (at[os] == time) {  // same-cycle conflict: policy (GameState.java:266-297)
                    bool cold = false, cnew = false;
                    if (U.crs == 2) {
                        if (rngCancel.nextInt(2) == 0) cnew = true;
                        else cold = true;
                    } else if (U.crs == 3) {
                        if ((ccnt % 2) == 0) cnew = true;
                        else cold = true;
                        ccnt++;
                    } else {
                        cold = cnew = true;
                    }
                    const int d1 = etaSlot(os);
                    const int d2 = eta(t, prm, ut, typ);
                    const int md = min(d1, d2);
                    if (cold && lane_id() == 0) {
                        ua[os] = pack_ua(T_NONE, 0, 0, 0) | UA_PRESENT;
                        par[os] = (int16_t)md;
                    }
                    if (cnew) {
                        t = T_NONE;
                        prm = md;
                        tx = ty = ut = 0;
                    }
                    wsync();
                } else {  // older assignment: only the new one is cancelled (:298-317)
                    err |= E_OLDER;
                    t = T_NONE;
                    prm = -1;
                    tx = ty = ut = 0;
                }
            }
        }
        if (lane_id() == 0) {
            ua[s] = pack_ua(t, ut, tx, ty) | UA_PRESENT;
            par[s] = (int16_t)prm;
            at[s] = time;
            as[s] = seq;
        }
        seq++;
        wsync();
    }

    // GameState.issueSafe(pa) (rts/GameState.java:338-408) for pa = [accepted rows in cell order]
    // + PlayerAction.fillWithNones(gs, p, fillDur) (rts/PlayerAction.java:328-346) in list order.
    DEV void issuePlayer(int p, int fillDur) {
        for (int c0 = 0; c0 < HW; c0 += 64) {
            const int c = c0 + lane_id();
            const int s = c < HW ? cell[c] : EMPTY;
            const bool isPA = s < CAP && uplay(uc[s]) == p && (ua[s] & UA_PA);
            uint64_t m = ballot(isPA);
            if (m == 0) continue;
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
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                issueOne(rl(s, k), rl(t, k), rl(prm, k), rl(tx, k), rl(ty, k), rl(ut, k));
            }
        }
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lane_id();
            bool fill = false;
            if (o < nu) {
                const uint32_t c = uc[o];
                fill = !(c & UC_DEAD) && uplay(c) == p && !(ua[o] & (UA_PRESENT | UA_PA));
            }
            uint64_t m = ballot(fill);
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                issueOne(o0 + k, T_NONE, fillDur, 0, 0, 0);
            }
        }
    }

    // ------------------------------------------------------------------ cycle
    DEV void kill(int k) {  // GameState.removeUnit (rts/GameState.java:79-82)
        if (lane_id() == 0) {
            const uint32_t c = uc[k];
            uc[k] = c | UC_DEAD;
            cell[uy(c) * W + ux(c)] = EMPTY;
            ua[k] &= ~UA_PRESENT;  // stays READY if it is in this cycle's snapshot
        }
        deaths++;
        wsync();
    }
    // UnitAction.execute (rts/UnitAction.java:338-465) — also for units killed earlier in the loop
    DEV void execute(int s) {
        const uint32_t cu = uc[s];
        const bool dead = cu & UC_DEAD;
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const uint32_t a = ua[s];
        const int t = ua_type(a);
        const int prm = par[s];
        switch (t) {
            case T_MOVE: {
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (!dead) {
                    if (cell[ny * W + nx] != EMPTY) err |= E_COLLISION;
                    if (lane_id() == 0) {
                        cell[y * W + x] = EMPTY;
                        cell[ny * W + nx] = (uint16_t)s;
                    }
                }
                if (lane_id() == 0) uc[s] = (cu & ~0xFFFFu) | (uint32_t)nx | ((uint32_t)ny << 8);
                wsync();
            } break;
            case T_ATTACK: {
                const int n = cell[ua_ty(a) * W + ua_tx(a)];
                if (n < CAP) {
                    int dmg = U.minD[typ];
                    if (U.minD[typ] != U.maxD[typ]) dmg = U.minD[typ] + rngDamage.nextInt(1 + (U.maxD[typ] - U.minD[typ]));
                    const int nhp = hp[n] - dmg;
                    if (lane_id() == 0) hp[n] = (int16_t)nhp;
                    wsync();
                    if (nhp <= 0) kill(n);
                }
            } break;
            case T_HARVEST: {
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (inb(nx, ny)) {
                    const int n = cell[ny * W + nx];
                    if (n < CAP && (U.flags[utyp(uc[n])] & F_RESOURCE) && (U.flags[typ] & F_HARVEST) && res[s] == 0) {
                        const int nr = res[n] - U.harvestAmt[typ];
                        if (lane_id() == 0) {
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
                    const int n = cell[ny * W + nx];
                    const int carried = res[s];
                    if (n < CAP && (U.flags[utyp(uc[n])] & F_STOCKPILE) && carried > 0) {
                        addPres(pl, carried);
                        if (lane_id() == 0) res[s] = 0;
                        wsync();
                    }
                }
            } break;
            case T_PRODUCE: {
                const int ut = ua_ut(a);
                const int nx = x + dxo(prm), ny = y + dyo(prm);
                if (pres(pl) - U.cost[ut] >= 0) {
                    if (cell[ny * W + nx] != EMPTY) {
                        err |= E_ADDUNIT;  // PhysicalGameState.addUnit throws (:190-195)
                    } else if (nu >= CAP) {
                        err |= E_CAPACITY;
                    } else {
                        if (lane_id() == 0) {
                            uc[nu] = pack_uc(nx, ny, ut, pl);
                            hp[nu] = (int16_t)U.hp[ut];
                            res[nu] = 0;
                            ua[nu] = 0;
                            par[nu] = -1;
                            cell[ny * W + nx] = (uint16_t)nu;
                        }
                        nu++;
                        addPres(pl, -U.cost[ut]);
                        wsync();
                    }
                } else {
                    err |= E_NEG_RES;
                }
            } break;
            default: break;
        }
    }
    // GameState.cycle (rts/GameState.java:553-571); returns gameover()
    DEV void cycle() {
        time++;
        for (int o = lane_id(); o < nu; o += 64) {
            const uint32_t a = ua[o];
            if ((a & UA_PRESENT) && etaSlot(o) + at[o] <= time) ua[o] = a | UA_READY;
        }
        wsync();
        while (true) {
            int best = 0x7FFFFFFF;
            for (int o = lane_id(); o < nu; o += 64)
                if (ua[o] & UA_READY) best = min(best, as[o]);
            best = wave_min(best);
            if (best == 0x7FFFFFFF) break;
            int os = 0x7FFFFFFF;
            for (int o = lane_id(); o < nu; o += 64)
                if ((ua[o] & UA_READY) && as[o] == best) os = o;
            os = wave_min(os);
            if (lane_id() == 0) ua[os] &= ~(UA_READY | UA_PRESENT);
            wsync();
            execute(os);
        }
    }
    // PhysicalGameState.gameover/winner (rts/PhysicalGameState.java:334-387)
    DEV void outcome(bool& gameover, int& winner) {
        int c0 = 0, c1 = 0;
        for (int o = lane_id(); o < nu; o += 64) {
            const uint32_t c = uc[o];
            if (!(c & UC_DEAD)) {
                const int p = uplay(c);
                c0 += (p == 0);
                c1 += (p == 1);
            }
        }
        c0 = wave_sum(c0);
        c1 = wave_sum(c1);
        gameover = (c0 + c1 == 0) || ((c0 > 0) != (c1 > 0));
        winner = (c0 > 0 && c1 == 0) ? 0 : ((c1 > 0 && c0 == 0) ? 1 : -1);
    }
    // order-preserving removal of dead slots (LinkedList.remove, PhysicalGameState.java:208-210)
    DEV void compact() {
        int base = 0;
        for (int o0 = 0; o0 < nu; o0 += 64) {
            const int o = o0 + lane_id();
            const bool alive = o < nu && !(uc[o] & UC_DEAD);
            const uint64_t m = ballot(alive);
            const int idx = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            uint32_t c = 0, a = 0;
            int32_t t0 = 0, t1 = 0;
            int16_t h = 0, r = 0, pr = 0;
            if (alive) {
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
        for (int c = lane_id(); c < HW; c += 64)
            if (cell[c] != WALL) cell[c] = EMPTY;
        wsync();
        placeUnits();
    }

    // ------------------------------------------------------------------ observation
    // GameState.getVectorObservation (rts/GameState.java:922-968): 6 planes [C][H][W] int32
    DEV void writeObs(int slot, int player) {
        int32_t* o = P.obs + (size_t)slot * P.C * HW;
        for (int c = lane_id(); c < HW; c += 64) {
            const int s = cell[c];
            int v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
            if (s < CAP) {
                const uint32_t cu = uc[s];
                const uint32_t a = ua[s];
                const int pl = uplay(cu);
                v0 = hp[s];
                v1 = res[s];
                v2 = pl >= 0 ? ((pl + player) % 2) + 1 : 0;
                v3 = utyp(cu) + 1;
                v4 = (a & UA_PRESENT) ? ua_type(a) : 0;
            }
            o[c] = v0;
            o[HW + c] = v1;
            o[2 * HW + c] = v2;
            o[3 * HW + c] = v3;
            o[4 * HW + c] = v4;
            o[5 * HW + c] = (s == WALL) ? 1 : 0;
        }
    }

    // ------------------------------------------------------------------ legal-action masks
    // JNIGridnetClient.getMasks (tests/JNIGridnetClient.java:210-223) + UnitAction.getValidActionArray
    // (rts/UnitAction.java:711-751) over Unit.getUnitActions(gs, 10) (rts/units/Unit.java:382-522).
    DEV void unitMask(int s, uint32_t& w0, uint32_t& w1, uint32_t& w2) const {
        w0 = w1 = w2 = 0;
        auto setb = [&](int k) {
            if (k < 32) w0 |= 1u << k;
            else if (k < 64) w1 |= 1u << (k - 32);
            else w2 |= 1u << (k - 64);
        };
        const uint32_t cu = uc[s];
        const int x = ux(cu), y = uy(cu), typ = utyp(cu), pl = uplay(cu);
        const uint32_t fl = U.flags[typ];
        const int nt = U.ntypes, R = U.maxAttackRadius, ctr = R / 2;
        const int atkBase = 1 + 6 + 16 + nt;
        int nc[4];
        bool nin[4];
        for (int d = 0; d < 4; d++) {
            const int nx = x + dxo(d), ny = y + dyo(d);
            nin[d] = inb(nx, ny);
            nc[d] = nin[d] ? cell[ny * W + nx] : WALL;
        }
        setb(0);
        setb(1 + T_NONE);
        if (fl & F_ATTACK) {
            const int r = U.range[typ];
            if (r == 1) {
                for (int d = 0; d < 4; d++) {
                    if (nc[d] < CAP) {
                        const int op = uplay(uc[nc[d]]);
                        if (op >= 0 && op != pl) {
                            setb(1 + T_ATTACK);
                            setb(atkBase + (ctr + dyo(d)) * R + (ctr + dxo(d)));
                        }
                    }
                }
            } else {
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
        }
        if (fl & F_HARVEST) {
            const int carried = res[s];
            for (int d = 0; d < 4; d++) {
                if (nc[d] >= CAP) continue;
                const uint32_t oc = uc[nc[d]];
                const uint32_t ofl = U.flags[utyp(oc)];
                if (carried == 0 && (ofl & F_RESOURCE)) {
                    setb(1 + T_HARVEST);
                    setb(1 + 6 + 4 + d);
                }
                if (carried > 0 && (ofl & F_STOCKPILE) && uplay(oc) == pl) {
                    setb(1 + T_RETURN);
                    setb(1 + 6 + 8 + d);
                }
            }
        }
        for (int i = 0; i < U.nprod[typ]; i++) {
            const int ut = U.prod[typ][i];
            if (pres(pl) >= U.cost[ut]) {
                for (int d = 0; d < 4; d++)
                    if (nc[d] == EMPTY) {
                        setb(1 + T_PRODUCE);
                        setb(1 + 6 + 12 + d);
                        setb(1 + 6 + 16 + ut);
                    }
            }
        }
        if (fl & F_MOVE) {
            for (int d = 0; d < 4; d++)
                if (nc[d] == EMPTY) {
                    setb(1 + T_MOVE);
                    setb(1 + 6 + d);
                }
        }
    }
    // Park each idle unit's 79-bit mask in its unused assignment words (at/as/ua low bits).
    DEV void stashMasks(int p) {
        for (int o = lane_id(); o < nu; o += 64) {
            const uint32_t c = uc[o];
            if ((c & UC_DEAD) || uplay(c) != p || (ua[o] & UA_PRESENT)) continue;
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
    DEV void writeMasks(int slot, int p) {
        const int K = U.K;
        uint8_t* out = P.masks + (size_t)slot * HW * K;
        const int total = HW * K;
        if ((total & 15) == 0) {
            for (int j = lane_id(); j < total / 16; j += 64) {
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
                *(uint4*)(out + o0) = v;
            }
        } else {
            for (int o = lane_id(); o < total; o += 64) {
                const int c = o / K, k = o - c * K;
                uint64_t lo;
                uint32_t hi;
                cellMaskBits(c, p, lo, hi);
                out[o] = (uint8_t)(k < 64 ? ((lo >> k) & 1u) : ((hi >> (k - 64)) & 1u));
            }
        }
    }
};

template <int MODE>
__global__ __launch_bounds__(64) void k_env(KParams P) {
    extern __shared__ __align__(16) uint8_t smem[];
    Game G(P, smem);
    const bool selfplay = G.g < P.n_sp_games;
    const int slot0 = selfplay ? 2 * G.g : 2 * P.n_sp_games + (G.g - P.n_sp_games);
    const int nslots = selfplay ? 2 : 1;

    if (MODE == MODE_RESET) {
        const int32_t* s = G.st();
        int hv = lane_id() < H_WORDS ? s[lane_id()] : 0;
        G.err = 0;
        G.ccnt = rl(hv, H_CANCEL_CNT);
        G.rngCancel.s = (uint64_t)(uint32_t)rl(hv, H_RNG_CANCEL) | ((uint64_t)(uint32_t)rl(hv, H_RNG_CANCEL + 1) << 32);
        G.rngDamage.s = (uint64_t)(uint32_t)rl(hv, H_RNG_DAMAGE) | ((uint64_t)(uint32_t)rl(hv, H_RNG_DAMAGE + 1) << 32);
        G.rngSampler.s = (uint64_t)(uint32_t)rl(hv, H_RNG_SAMPLER) | ((uint64_t)(uint32_t)rl(hv, H_RNG_SAMPLER + 1) << 32);
        G.initCells();
        G.resetFromTemplate();
        if (lane_id() < nslots) {
            if (P.reward) P.reward[slot0 + lane_id()] = 0.0;
            if (P.done) P.done[slot0 + lane_id()] = 0;
        }
    } else {
        G.load();
    }

    if (MODE == MODE_STEP) {
        const size_t rowStride = (size_t)G.HW * 7;
        if (selfplay) {
            // JNIGridnetClientSelfPlay.gameStep (tests/JNIGridnetClientSelfPlay.java:159-189)
            for (int p = 0; p < 2; p++) {
                G.decode(p, P.actions + (size_t)(slot0 + p) * rowStride);
                G.issuePlayer(p, 1);
            }
        } else {
            // JNIGridnetClient.gameStep (tests/JNIGridnetClient.java:163-203), PassiveAI opponent
            const int player = P.players ? uni(P.players[slot0]) : 0;
            G.decode(player, P.actions + (size_t)slot0 * rowStride);
            G.issuePlayer(player, 1);
            G.issuePlayer(1 - player, 10);  // PassiveAI.getAction = fillWithNones(gs, p, 10)
        }
        G.cycle();
        bool gameover;
        int winner;
        G.outcome(gameover, winner);
        // WinLossRewardFunction (ai/reward/WinLossRewardFunction.java:16-24) + VecClient auto-reset
        // keeping the terminal reward/done (tests/JNIGridnetVecClient.java:241-287)
        G.steps++;
        const bool reset = gameover || G.steps >= P.max_steps;
        if (lane_id() < nslots) {
            const int slot = slot0 + lane_id();
            const int maxp = selfplay ? lane_id() : (P.players ? P.players[slot] : 0);
            if (P.reward) P.reward[slot] = gameover ? (winner == maxp ? 1.0 : -1.0) : 0.0;
            if (P.done) P.done[slot] = (gameover || reset) ? 1 : 0;
        }
        if (reset) G.resetFromTemplate();
        else if (G.deaths) G.compact();
    }

    if (MODE != MODE_MASKS && P.obs) {
        for (int i = 0; i < nslots; i++) {
            const int player = selfplay ? i : (P.players ? P.players[slot0] : 0);
            G.writeObs(slot0 + i, player);
        }
    }
    if (P.masks) {
        wsync();
        for (int i = 0; i < nslots; i++) G.stashMasks(selfplay ? i : P.mask_player);
        wsync();
        for (int i = 0; i < nslots; i++) G.writeMasks(slot0 + i, selfplay ? i : P.mask_player);
    }
    if (MODE != MODE_MASKS) {
        wsync();
        G.store();
    }
}

// ---------------------------------------------------------------- random policy (bench / rollouts)
DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
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

__global__ __launch_bounds__(64) void k_policy(PolicyParams Q) {
    const int c = (int)(blockIdx.x * 64 + threadIdx.x);
    const int slot = (int)blockIdx.y;
    if (c >= Q.HW) return;
    const uint8_t* m = Q.masks + ((size_t)slot * Q.HW + c) * Q.K;
    int32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
    if (m[0]) {
        uint64_t lo = 0, hi = 0;  // mask bits 1..K-1 → bit i-1
        for (int i = 1; i < Q.K; i++) {
            const uint64_t b = m[i] ? 1ull : 0ull;
            if (i - 1 < 64) lo |= b << (i - 1);
            else hi |= b << (i - 1 - 64);
        }
        uint32_t ctr[4] = {Q.slot_id_base + (uint32_t)slot, Q.step, (uint32_t)c, 0u};
        philox(ctr, (uint32_t)Q.seed, (uint32_t)(Q.seed >> 32));
        auto field = [&](int off, int n) -> uint64_t {  // mask slots [off, off+n) (off >= 1)
            const int b = off - 1;
            uint64_t v;
            if (b >= 64) v = hi >> (b - 64);
            else v = (lo >> b) | (b ? (hi << (64 - b)) : 0ull);
            return n >= 64 ? v : (v & ((1ull << n) - 1));
        };
        const int t = pickBit(ctr[0], field(1, 6), 6);
        if (t >= 0) {
            a[0] = t;
            switch (t) {
                case 1: a[1] = pickBit(ctr[1], field(7, 4), 4); break;
                case 2: a[2] = pickBit(ctr[1], field(11, 4), 4); break;
                case 3: a[3] = pickBit(ctr[1], field(15, 4), 4); break;
                case 4:
                    a[4] = pickBit(ctr[1], field(19, 4), 4);
                    a[5] = pickBit(ctr[2], field(23, Q.ntypes), Q.ntypes);
                    break;
                case 5: {
                    const int off = 23 + Q.ntypes, n = Q.K - off;
                    a[6] = pickBit(ctr[1], field(off, n), n);
                } break;
            }
        }
    }
    int32_t* out = Q.actions + ((size_t)slot * Q.HW + c) * 7;
#pragma unroll
    for (int k = 0; k < 7; k++) out[k] = a[k];
}

}  // namespace

namespace mrts {
size_t ldsBytes(int HW, int W, int CAP) {
    return (size_t)16 * CAP + 4 * (size_t)((HW + 2 * W + 31) / 32) + 6 * (size_t)CAP + 2 * (size_t)HW;
}
hipError_t launchEnv(int mode, const KParams& P, hipStream_t stream) {
    const size_t lds = ldsBytes(P.HW, P.W, P.CAP);
    dim3 grid((unsigned)P.n_games), block(64);
    switch (mode) {
        case MODE_STEP: hipLaunchKernelGGL(k_env<MODE_STEP>, grid, block, lds, stream, P); break;
        case MODE_RESET: hipLaunchKernelGGL(k_env<MODE_RESET>, grid, block, lds, stream, P); break;
        default: hipLaunchKernelGGL(k_env<MODE_MASKS>, grid, block, lds, stream, P); break;
    }
    return hipGetLastError();
}
hipError_t prepareLds(size_t bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_env<MODE_STEP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_RESET>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_env<MODE_MASKS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    return e;
}
hipError_t launchPolicy(const PolicyParams& Q, hipStream_t stream) {
    dim3 grid((unsigned)((Q.HW + 63) / 64), (unsigned)Q.n_slots), block(64);
    hipLaunchKernelGGL(k_policy, grid, block, 0, stream, Q);
    return hipGetLastError();
}
}  // namespace mrts
