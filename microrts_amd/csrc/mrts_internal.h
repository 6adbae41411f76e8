// Internal layouts shared by the HIP kernels (mrts_kernels.hip) and the host runtime (mrts_host.cpp).
#pragma once
#include <stdint.h>

namespace mrts {

constexpr int MAX_TYPES = 8;
constexpr int MAX_PRODUCES = 4;
constexpr int MAX_REWARDS = 8;
// reward functions (src/ai/reward/*.java), ids = include/mrts.h MRTS_RF_*
enum { RF_WINLOSS = 0, RF_RESOURCE_GATHER = 1, RF_PRODUCE_WORKER = 2, RF_PRODUCE_BUILDING = 3, RF_ATTACK = 4,
       RF_PRODUCE_COMBAT_UNIT = 5, RF_CLOSER_TO_ENEMY_BASE = 6, RF_CLOSER_TO_ENEMY_UNIT = 7, RF_COUNT = 8 };

// UnitTypeTable constants (reference src/rts/units/UnitTypeTable.java:104-289), passed by value as
// kernel arguments so that handles with different tables never share device globals.
struct DevUtt {
    int32_t ntypes;
    int32_t cost[MAX_TYPES], hp[MAX_TYPES], minD[MAX_TYPES], maxD[MAX_TYPES], range[MAX_TYPES];
    int32_t produceT[MAX_TYPES], moveT[MAX_TYPES], attackT[MAX_TYPES], harvestT[MAX_TYPES], harvestAmt[MAX_TYPES];
    int32_t sight[MAX_TYPES];
    uint32_t flags[MAX_TYPES];  // F_* below
    int32_t nprod[MAX_TYPES];
    int32_t prod[MAX_TYPES][MAX_PRODUCES];  // type.produces, list order
    int32_t crs;                // move-conflict resolution strategy 1/2/3
    int32_t maxAttackRadius;    // 2 * max attack range + 1 (JNIGridnetClient.java:125)
    int32_t K;                  // mask slots per cell (JNIGridnetClient.java:138)
    // sight disk half-widths floor(sqrt(r^2 - dy^2)) for r = sight[t] <= 15, 4 bits per |dy|:
    // dy 0..7 in diskLo, 8..15 in diskHi (PartiallyObservableGameState visibility, painted per row)
    uint32_t diskLo[MAX_TYPES], diskHi[MAX_TYPES];
    int32_t maxSight;           // max sight[t] over the types
    // per-type bit sets of the mask tables (bit t = type t has the property; host-computed) and the
    // produce lists as 8-bit type sets (type t's set in bits 8t..8t+7 of mtProd)
    uint32_t mtAttack1, mtAttackFar, mtHarvest, mtMove, mtResource, mtStockpile;
    uint32_t mtProdLo, mtProdHi;
};
enum : uint32_t { F_RESOURCE = 1, F_STOCKPILE = 2, F_HARVEST = 4, F_MOVE = 8, F_ATTACK = 16,
                  // the type-name tests of the reward functions (src/ai/reward/*.java), set from the names
                  N_RESOURCE = 1u << 8,   // "Resource"
                  N_BASE = 1u << 9,       // "Base"
                  N_WORKER = 1u << 10,    // "Worker"
                  N_BUILDING = 1u << 11,  // "Base" or "Barracks"
                  N_COMBAT = 1u << 12 };  // "Light", "Heavy" or "Ranged"

// ---- per-game state block in HBM (int32 words) -------------------------------------------------
// header
enum {
    H_TIME = 0,       // GameState.time
    H_NU = 1,         // unit slots in use (== live units between steps; list order == slot order)
    H_RES0 = 2,       // Player 0 resources
    H_RES1 = 3,       // Player 1 resources
    H_SEQ = 4,        // next assignment sequence number (LinkedHashMap insertion order)
    H_STEPS = 5,      // VecClient envSteps
    H_ERR = 6,        // MRTS_ERR_* flags (sticky until reset by the host)
    H_CANCEL_CNT = 7, // GameState.unitCancelationCounter
    H_RNG_CANCEL = 8, // 2 words: java.util.Random for CANCEL_RANDOM (GameState.r)
    H_RNG_DAMAGE = 10,// 2 words: java.util.Random for non-deterministic damage (UnitAction.r)
    H_RNG_SAMPLER = 12,// 2 words: java.util.Random for RandomBiasedAI (Sampler.generator)
    H_KIND = 14,      // game kind (KStatic.game_kind), copied here so a step needs no dependent load
    H_FWD = 15,       // launch stamp of the fused policy's forwarded action rows (0 = none; see stateFwdOff)
    H_WORDS = 16
};
// followed by 7 SoA arrays of CAP int32: UC, HP, RES, UA, PAR, AT, AS (see mrts_kernels.hip)
enum { A_UC = 0, A_HP = 1, A_RES = 2, A_UA = 3, A_PAR = 4, A_AT = 5, A_AS = 6, N_ARRAYS = 7 };
// followed by 2 x maskWords(HW): per player, the cells whose mask rows were non-zero in the mask buffer
// written last (delta mask writes, mrts_config.mask_delta)
constexpr int maskWords(int hw) { return (hw + 31) / 32; }
// after the arrays: the previous mask row sets (2 x maskWords), then the map's terrain bytes (copied
// from the template at reset, so a step's first memory round needs nothing but the state block)
constexpr int stateTerrOff(int cap, int hw) { return H_WORDS + N_ARRAYS * cap + 2 * maskWords(hw); }
// then FWD_WORDS words: the fused random policy's action rows of the idle units in slots 0..63, one
// packed word per slot (packFwd in mrts_kernels.hip), written by the launch whose stamp is in H_FWD.
// The next launch of a self-play game reads them in its first memory round instead of fetching the
// rows from the action tensor the same launch wrote them to (KDyn.fwd_read), which removes the
// step's second dependent global round trip.
constexpr int FWD_WORDS = 64;
constexpr int stateFwdOff(int cap, int hw) { return stateTerrOff(cap, hw) + (hw + 3) / 4; }
constexpr int stateWords(int cap, int hw) { return stateFwdOff(cap, hw) + FWD_WORDS; }  // host + device

// unit core word
constexpr uint32_t UC_DEAD = 1u << 31;
// assignment word
constexpr uint32_t UA_PRESENT = 1u << 24, UA_READY = 1u << 25, UA_PA = 1u << 26, UA_DEC = 1u << 27, UA_BAD = 1u << 28;
constexpr int ACT_INVALID = 7;  // action type / direction outside the Java ranges

// ---- map templates (one per distinct map), int32 words --------------------------------------------
// [0] H [1] W [2] res0 [3] res1 [4] nu [5..5+nu) uc [..+nu) hp [..+nu) res [..+ceil(HW/4)) terrain (u8 x4)
// map template: header, terrain bytes ((HW+3)/4 words, fixed offset so it loads with the state), units
enum { T_H = 0, T_W = 1, T_RES0 = 2, T_RES1 = 3, T_NU = 4, T_TERR = 5 };
constexpr int tmplUnits(int hw) { return T_TERR + (hw + 3) / 4; }  // host + device

// Static per-handle parameters live in a device buffer (uploaded once at mrts_create): the kernels
// read them through a pointer, so the unit-type tables can be indexed per lane without the
// compiler copying a by-value kernel argument into scratch memory.
struct KStatic {
    DevUtt utt;
    int32_t H, W, HW, CAP;
    int32_t n_games, n_sp_games;   // games [0, n_sp_games) are self-play, the rest agent-vs-bot
    int32_t max_steps, C;
    int32_t partial_obs;           // PartiallyObservableGameState views (8 planes)
    int32_t* state;                // [n_games][stateWords(CAP, HW)]
    const int32_t* tmpl;           // template blob
    const int32_t* tmpl_off;       // [n_games] word offset of each game's template
    const int32_t* game_kind;      // [n_games]: type | ai1 << 4 | ai2 << 8 (see mrts_kernels.hip)
    int32_t n_rewards;             // reward functions per slot (a_rfs), 1..MAX_REWARDS
    int32_t reward_kinds[MAX_REWARDS];  // MRTS_RF_* in a_rfs order; reward / done are [n_slots][n_rewards]
    uint32_t reward_need;          // RN_* bits: which per-step bookkeeping the kinds need
};
enum : uint32_t { RN_COUNTS = 1, RN_CLOSER = 2, RN_RESOURCES = 4 };
// Per-call buffers (kernel arguments by value)
struct KDyn {
    const int32_t* actions;        // [n_slots][HW][7]
    const int32_t* players;        // [n_slots] or null
    int32_t* obs;                  // [n_slots][C][HW] or null
    double* reward;                // [n_slots][n_rewards] or null
    uint8_t* done;                 // [n_slots][n_rewards] or null
    uint8_t* masks;                // [n_slots][HW][K] or null
    uint32_t* source;              // [n_slots][maskWords(HW)] mask slot 0 as bits, or null
    int32_t mask_player;           // player whose masks bot-env slots receive
    int32_t mask_delta;            // 1: `masks` holds the previous masks of this handle -> rewrite changed rows only
    // copies of KStatic fields the first memory round needs (kernel arguments: no dependent load)
    int32_t* state;
    int32_t state_words, H, W, HW, CAP, n_sp_games;
    const int32_t* rows;           // Java row layout [n_slots][n_rows][8] (replaces `actions`) or null
    int32_t n_rows;
    uint32_t* pairs;               // rows mode: per game [n_rows][2] accepted-pair scratch
    int32_t horizon;               // playout mode: NaiveMCTS.simulate(gs, gs.getTime() + horizon)
    // fused random policy (mrts_step_fused_dev): the next step's action rows, sampled from the masks
    // this launch writes, go to pol_actions (the buffer the launch consumed); null = off
    int32_t* pol_actions;
    uint64_t pol_seed;
    uint32_t pol_step, pol_slot_base;
    int32_t pol_delta;             // 1: pol_actions holds the policy rows of the previous mask write's candidates
    // forwarded action rows: fwd_read = 1 when `actions` is the buffer the previous launch on this
    // handle wrote as pol_actions and nothing has written it since (the host's fusedActions); a game
    // uses its forwarded words iff its H_FWD == fwd_stamp - 1 (this launch's stamp minus one, i.e.
    // the previous launch wrote them).  Every launch that stores a state writes H_FWD.
    int32_t fwd_read;
    uint32_t fwd_stamp;
    // copies of the KStatic fields the step reads after its first memory round (kernel arguments sit
    // in SGPRs from the kernel's start; a KStatic load there is a dependent round trip on the chain)
    int32_t n_rewards, max_steps, C;
    uint32_t reward_need;
    uint32_t reward_kinds4;        // reward_kinds[j] in bits 4j..4j+3
    // persistent-buffer partially observable observations (mrts_set_obs_delta): obs_delta = 1 when
    // `obs` holds this handle's last observation write; po_prev = per game [po_words] the previous
    // render's record (poPrevWords), rewritten by every observation write
    int32_t obs_delta;
    int32_t po_words;
    int32_t* po_prev;
    // fused unmasked uniform policy (mrts_step_uniform_dev, BASELINE config c2): this launch draws
    // its own rows (the values k_policy_uniform would write for uni_step) for the idle units it
    // decodes and writes every row of its slots to uni_actions; null = off (rows come from `actions`)
    int32_t* uni_actions;
    uint64_t uni_seed;
    uint32_t uni_step, uni_slot_base;
    // full observability: the observation planes also as int16 [n_slots][C][HW] (the compact transport
    // of the observation exchange, mrts_set_obs16); null = off
    int16_t* obs16;
    // the uint8 form of that transport (mrts_set_exchange_bytes(env, 1)): written only by the 16x16
    // byte-image render (writeObsFullImg) and the one-cell-per-lane render of maps of <= 64 cells,
    // every value < 256; null = off
    uint8_t* obs8;
    // multi-step launch (mrts_rollout_fused_dev): > 1 = this launch runs n_iter consecutive fused steps
    // per game (pol_step, pol_step + 1, ...), the state kept in LDS in between (specialised
    // full-observability self-play kernels; the host issues it only in the steady fused state:
    // pol_delta = fwd_read = mask_delta = 1)
    int32_t n_iter;
    // helper-wave multi-step launches (8x8 fused uniform rollouts, BASELINE c2): byte offset of the
    // LDS handoff area (rows of the next step, packed observation cells) after the game's own LDS
    int32_t help_off;
    // multi-step launches: per-SIMD issue-rank table [PRIO_KEYS][16] (mrts_kernels.hip, simdRank):
    // each wave posts its game's remaining-work estimate and takes its s_setprio from its rank among
    // the waves sharing its SIMD; null = the unit-count thresholds only
    uint32_t* prio_tab;
    // multi-step launches: balanced game placement (mrts_kernels.hip, balancePerm): [1] the stamp of the launch that wrote perm, [2 + c] finished waves of block class c (b % 8), [BAL_COST + g] game g's cost as posted by the
    // launch (stamp << 16 | units), [BAL_COST + n + b] the game block b of the NEXT launch runs; null = off
    int32_t* bal;
    // 1: every value a full-observability plane shows fits a byte (hp, resources of the maps' units and
    // the unit-type table, mrts_create), so 16x16 observations render through the byte image
    // (writeObsFullImg)
    int32_t obs_img;
    // trace replay (MODE_TRACE, mrts_trace_step): `rows` holds per game [n_rows] issue rows [player, x, y,
    // type, parameter, target x, target y, unit type]; each game then cycles until its time reaches
    // trace_until[g] and reports TR_* bits in trace_out[g]; trace_generic = 1 runs the generic kernel
    // even where a specialised instance exists
    const int32_t* trace_until;
    int32_t* trace_out;
    int32_t trace_generic;
    // compact observation records (mrts_rollout_*_records_dev): after each step's observation write, game
    // g of iteration it writes its record at rec_out + (it * n_sp_games + g) * recWords(rec_units, po)
    // words (writeRecord in mrts_kernels.hip); null = off
    uint32_t* rec_out;
    int32_t rec_units;
    // every step's Responses (mrts_set_step_responses): `reward` / `done` then point at this launch's first
    // step in the call's ring and iteration it writes its reward / done [n_slots][n_rewards] at
    // + it * resp_stride (= n_slots * n_rewards); 0 = every iteration writes the same buffers
    int32_t resp_stride;
};
// compact observation record of one game, word 0 = units n (<= rec_units) | overflow << 31, then per unit
// in list order:
// * full observability (maps of <= 256 cells, every plane value < 256), the live units, one word each:
//   cell | hp << 8 | resources << 16 | (type + 1) << 24 | (player + 1) << 27 | action type << 29;
// * partial observability, the units either player's view holds (dead ones included: a view keeps the
//   units of its snapshot), two words each: cell | (hp as int8) << 16 | resources << 24, and
//   (type + 1) | (player + 1) << 4 | snapshot byte << 8 (bit p: in view p; bits 2+3p..4+3p: the action
//   type + 1 view p saw, 0 = none) — hp of a dead unit may be negative, a value outside int8 / uint8
//   sets the overflow bit
constexpr int recWords(int units, bool po) { return 1 + (po ? 2 : 1) * units; }
constexpr int BAL_COST = 16;
constexpr int PRIO_KEYS = 8 * 8 * 2 * 16 * 4;  // XCC x SE x SH x CU x SIMD (HW_ID / XCC_ID fields)
// PO render record per game (int32 words): [0] views rendered by the last observation write (bit p);
// snapshot bytes of the unit slots (after the end-of-step compaction); per view p the sight rows
// (own, other) the render used; per view the 4-cell chunks of rendered units that died (they leave
// the list before the next render).  Delta rendering needs W % 4 == 0, W <= 32, H <= 32.
constexpr int poSnapWords(int cap) { return (cap + 3) / 4; }
constexpr int poChunkWords(int hw) { return (hw / 4 + 31) / 32; }
constexpr int poPrevWords(int cap, int h, int hw) { return 1 + poSnapWords(cap) + 4 * h + 2 * poChunkWords(hw); }
constexpr bool poDeltaShape(int h, int w) { return (w & 3) == 0 && w <= 32 && h <= 32; }

struct PolicyParams {
    int32_t HW, K, ntypes, n_slots;
    uint32_t slot_id_base, step;
    uint64_t seed;
    const uint8_t* masks;
    const uint32_t* source;        // optional [n_slots][maskWords(HW)]
    int32_t* actions;
    const uint32_t* prev;          // delta: candidate set of the previous write to actions
    uint32_t* prev_out;            // optional (with source): where this write records its candidate set
    int32_t delta;                 // 1: actions holds the previous output; rewrite only prev|source rows
};

}  // namespace mrts
