/*
 * mrts.h — C ABI of libmrts.so, the MI355X (gfx950) vectorised microRTS env step.
 *
 * Drop-in boundary for tests.JNIGridnetVecClient (reference src/tests/JNIGridnetVecClient.java:17-335).
 * Every entry point names the Java member it replaces.  Plain C: no C++ types, no exceptions,
 * no torch types.  A handle lives on ONE HIP device and owns ONE HIP stream; it is not thread-safe
 * (the Java client is single-threaded too, JNIGridnetVecClient.java:11-13).
 *
 * Slot layout (JNIGridnetVecClient.java:106-142): slots [0, n_selfplay_slots) belong to self-play
 * games (game i = slots 2i, 2i+1 = players 0, 1; map = map_paths[2i], :119), then one slot per
 * agent-vs-bot env (map = map_paths[n_selfplay_slots + j], :123).
 *
 * Actions (gameStep's int[][][] action, :213): int32 [n_slots][H*W][7], row r = the unit at cell r
 * (x = r % W, y = r / W); components [type, move dir, harvest dir, return dir, produce dir,
 * produce type, attack index] (rts/UnitAction.java:663-664,675-709).  This is exactly the Java row
 * [pos, ...] with pos = r, in ascending cell order — the MicroRTS-Py gridnet contract.
 *
 * Errors: 0 on success, a negative errno on failure; mrts_last_error() (thread-local) says why.
 * Java exceptions of the reference become errors: an out-of-range produce type in a decoded row
 * (UnitAction.java:697) → -EINVAL after the step; unit-capacity overflow or an addUnit collision
 * (PhysicalGameState.java:189-201) → -ENOSPC / -EFAULT.  Per-game detail in mrts_error_flags().
 */
#ifndef MRTS_H
#define MRTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mrts_env mrts_env;

enum { MRTS_BOT_PASSIVE = 0, MRTS_BOT_RANDOM_BIASED = 1 };

/* reward functions, a_rfs (:106): the classes of src/ai/reward */
enum {
    MRTS_RF_WIN_LOSS = 0,            /* WinLossRewardFunction: +1 / -1 at gameover, done = gameover */
    MRTS_RF_RESOURCE_GATHER = 1,     /* ResourceGatherRewardFunction: +1 per HARVEST / RETURN issued; done = no resources */
    MRTS_RF_PRODUCE_WORKER = 2,      /* ProduceWorkerRewardFunction */
    MRTS_RF_PRODUCE_BUILDING = 3,    /* ProduceBuildingRewardFunction (Base, Barracks) */
    MRTS_RF_ATTACK = 4,              /* AttackRewardFunction */
    MRTS_RF_PRODUCE_COMBAT_UNIT = 5, /* ProduceCombatUnitRewardFunction (Light, Heavy, Ranged) */
    MRTS_RF_CLOSER_TO_ENEMY_BASE = 6,/* CloserToEnemyBaseRewardFunction: fp64 sqrt distances */
    MRTS_RF_CLOSER_TO_ENEMY_UNIT = 7 /* CloserToEnemyUnitRewardFunction (the reference's text is identical to 6) */
};

/* per-game error flag bits (mrts_error_flags) */
enum {
    MRTS_ERR_CAPACITY = 1u << 0,      /* unit slots exhausted (no Java equivalent; env must be reset) */
    MRTS_ERR_ADDUNIT = 1u << 1,       /* produce into an occupied cell: Java throws (PhysicalGameState.java:192) */
    MRTS_ERR_PRODUCE_TYPE = 1u << 2,  /* decoded produce type out of range: Java throws (UnitAction.java:697) */
    MRTS_ERR_OLDER_CONFLICT = 1u << 3,/* issue() older-conflict branch: Java prints (GameState.java:298-317) */
    MRTS_ERR_NEG_RESOURCES = 1u << 4, /* produce skipped at execution: Java prints (UnitAction.java:457-461) */
    MRTS_ERR_MOVE_COLLISION = 1u << 5,/* internal invariant (one unit per cell) violated */
    MRTS_ERR_RECORD = 1u << 6         /* more live units than an observation record holds (mrts_set_records) */
};

typedef struct {
    int32_t n_selfplay_slots;   /* a_num_selfplayenvs (:106), even */
    int32_t n_bot_envs;         /* a_num_envs (:106) */
    int32_t max_steps;          /* a_max_steps (:106) */
    int32_t partial_obs;        /* partial_obs (:107) — 8 observation planes when set */
    int32_t utt_version;        /* new UnitTypeTable(version, crs): 1 ORIGINAL, 2 FINETUNED, 3 NON_DETERMINISTIC */
    int32_t conflict_policy;    /* 1 CANCEL_BOTH, 2 CANCEL_RANDOM, 3 CANCEL_ALTERNATING (UnitTypeTable.java:46-57) */
    const int32_t* bot_kinds;   /* a_ai2s (:107): per bot env, MRTS_BOT_* ; NULL = all passive */
    const int32_t* ai1_kinds;   /* non-NULL selects the bot-only client (:157-177, JNIBotClient): per env the
                                   MRTS_BOT_* of a_ai1s (bot_kinds = a_ai2s); n_selfplay_slots must be 0;
                                   observations and masks are not produced (Java returns null) */
    const char* const* map_paths; /* a_mapPaths (:106): one per slot */
    int32_t device;             /* HIP device ordinal */
    uint64_t seed;              /* seeds the per-game java.util.Random streams */
    int32_t slot_id_base;       /* global id of this handle's slot 0 (multi-GPU: disjoint RNG streams) */
    int32_t mask_delta;         /* 1: when a *_dev call gets the same mask buffer (and mask_player) as this
                                   handle's previous mask write, only rows that changed are rewritten; the
                                   buffer must not be modified by the caller in between (the Java client
                                   owns and reuses its mask array the same way, JNIGridnetClient.java:211) */
    const int32_t* reward_kinds;/* a_rfs (:106): MRTS_RF_* in order, n_rewards of them; NULL/0 = {WIN_LOSS}.
                                   reward / done become [n_slots][n_rewards]; the auto-reset follows done
                                   of the FIRST function (rs.done[0], :247,272) */
    int32_t n_rewards;          /* 0..8 */
    int32_t forward_model;      /* 1 (with ai1_kinds): a batched forward model for search AIs instead of the
                                   bot-only client: games advance only through mrts_playout*, never
                                   auto-reset; ai1_kinds / bot_kinds are players 0 / 1's playout policies */
    const char* utt_json;       /* non-NULL: UnitTypeTable.fromJSON(utt_json) (UnitTypeTable.java:414-433)
                                   replaces utt_version / conflict_policy (the JSON names its own policy) */
    int32_t max_units;          /* 0 = H*W (exact for any game).  A smaller bound on live units per game
                                   shrinks the per-game LDS footprint (more games resident per CU on
                                   large maps); a game that runs out of unit slots (max_units plus the
                                   births-in-a-step slack) gets MRTS_ERR_CAPACITY */
} mrts_config;

typedef struct {               /* ai/jni/Responses.java:12-30 */
    const int32_t* obs;        /* [n_slots][C][H][W] */
    const double* reward;      /* [n_slots][n_rewards] */
    const uint8_t* done;       /* [n_slots][n_rewards] */
} mrts_responses;

/* new JNIGridnetVecClient(...) (:106-142).  Parses the XML maps (PhysicalGameState.java:700-726). */
int mrts_create(const mrts_config* cfg, mrts_env** out);
/* storage sizes (:127-133): slots, map H/W, observation planes C (6 or 8), mask slots K (79) */
int mrts_dims(const mrts_env* env, int32_t* n_slots, int32_t* H, int32_t* W, int32_t* C, int32_t* K);

/* Host-pointer API (mirrors the Java reuse semantics: returned arrays are library-owned and valid
 * until the next call on the handle, GameState.java:923-925 / JNIGridnetClient.java:211-215). */
/* reset(int[]) :179-211.  Reward / done after a reset follow the Java clients: an agent-vs-bot or
 * bot-only env zeroes every slot (JNIGridnetClient.java:248-251, JNIBotClient.java:159-162); a
 * self-play game zeroes only reward functions 0 and 1 — its loop runs to rewards.length == 2 players,
 * not to rfs.length (JNIGridnetClientSelfPlay.java:103-104,235-238) — so functions >= 2 keep the
 * values the buffer held (the previous step's; zeros before any step).  With ONE reward function
 * Java's self-play reset throws ArrayIndexOutOfBounds (rewards[i][1]); here the one slot is zeroed
 * (DESIGN.md §8).  The auto-reset inside a step returns the terminal values of every slot (:248-263). */
int mrts_reset(mrts_env* env, const int32_t* players, mrts_responses* out);
int mrts_step(mrts_env* env, const int32_t* actions, const int32_t* players, mrts_responses* out); /* gameStep :213-297 */
int mrts_get_masks(mrts_env* env, int32_t player, uint8_t* out /* [n_slots][H][W][K] */);          /* getMasks :307-316 */
/* gameStep with the Java layout, int[][][] action (:213), as flat int32 [n_slots][n_rows][8]: row =
 * [pos, type, move dir, harvest dir, return dir, produce dir, produce type, attack index], any order,
 * any count, a unit may be named twice — exactly PlayerAction.fromVectorAction's list semantics
 * (rts/PlayerAction.java:384-417) followed by issueSafe (rts/GameState.java:338-408). */
int mrts_step_rows(mrts_env* env, const int32_t* rows, int32_t n_rows, const int32_t* players, mrts_responses* out);
/* getMasks in the Java element type: int32 [n_slots][H][W][K] (int[][][][], :307-316) */
int mrts_get_masks_i32(mrts_env* env, int32_t player, int32_t* out);
/* getMasks into a library-owned pinned host array, *out valid until the next call on the handle
 * (the Java client reuses its mask array the same way, JNIGridnetClient.java:211-215); the copy runs
 * at pinned rate instead of staging through a pageable caller buffer */
int mrts_get_masks_host(mrts_env* env, int32_t player, const uint8_t** out);
int mrts_get_masks_i32_host(mrts_env* env, int32_t player, const int32_t** out);

/* Device-pointer API: same semantics, caller-owned HBM buffers, stream-ordered on `stream`
 * (a hipStream_t; NULL = HIP's default stream, as everywhere in HIP; mrts_stream() gives the handle's
 * own stream), no host synchronisation. d_players may be NULL
 * (all zeros).  d_masks may be NULL; when given, the masks getMasks(mask_player) would return after
 * this call are written too (fused, saves a launch). */
int mrts_reset_dev(mrts_env* env, const int32_t* d_players, int32_t* d_obs, double* d_reward, uint8_t* d_done,
                   uint8_t* d_masks, int32_t mask_player, void* stream);
int mrts_step_dev(mrts_env* env, const int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                  uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, void* stream);
int mrts_get_masks_dev(mrts_env* env, int32_t player, uint8_t* d_out, void* stream);
/* device forms of mrts_step_rows / mrts_get_masks_i32 (d_out 16-byte aligned) */
int mrts_step_rows_dev(mrts_env* env, const int32_t* d_rows, int32_t n_rows, const int32_t* d_players, int32_t* d_obs,
                       double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, void* stream);
int mrts_get_masks_i32_dev(mrts_env* env, int32_t player, int32_t* d_out, void* stream);

/* Synthetic masked-uniform random policy (bench / rollouts): per own idle cell a uniform action
 * type among the mask's set type bits, then a uniform parameter among that type's set bits
 * (Philox4x32-10, key = seed, counter = (slot_id_base + slot, step, cell, 0)).  d_masks as written
 * by the calls above (d_source: their source bits, or NULL); d_actions = [n_slots][H*W][7].
 * With mask_delta and d_source, a call into the same d_actions as the previous call rewrites only
 * the rows whose candidate status changed or is set (the result is identical to a full write);
 * call mrts_policy_invalidate() after writing d_actions yourself. */
int mrts_policy_dev(mrts_env* env, const uint8_t* d_masks, const uint32_t* d_source, uint64_t seed, uint32_t step,
                    int32_t* d_actions, void* stream);
/* mrts_step_dev fused with the policy above: consumes d_actions, writes obs / reward / done / masks
 * (d_masks required), then overwrites d_actions with the policy's actions for step `next_step`
 * sampled from the masks just written — identical to mrts_policy_dev(env, d_masks, ..., seed,
 * next_step, d_actions) afterwards, without the second launch and its full pass.  Consecutive fused
 * calls on the same buffers rewrite only changed rows (mask_delta).
 * IMPORTANT: the rows a fused call samples are also kept in the handle's state and the next fused
 * call on the same d_actions decodes from that copy, not from d_actions.  Any write to d_actions
 * between fused calls (e.g. overriding some units' rows) MUST be followed by mrts_policy_invalidate(),
 * otherwise the written rows are ignored.  The same holds for mrts_rollout_fused_dev. */
int mrts_step_fused_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                        uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t next_step,
                        void* stream);
/* n_steps consecutive mrts_step_fused_dev calls (next_step = first_next_step, first_next_step + 1,
 * ...) enqueued from native code, without a host language's per-call overhead between them (a
 * random-policy rollout; the outputs of the last step remain in the buffers).  n_steps >= 0.
 * Multi-step launches (default on, mrts_set_multi_step): on self-play handles of the specialised
 * shapes (16x16 / 8x8 full observability, 32x32 partially observable with the default unit capacity
 * of max_units 256; the built-in unit-type tables), once the handle is in the
 * steady fused state (the previous launch was a fused step on these buffers), one launch runs up to
 * MRTS_MAX_ITER of the steps: each game's wave keeps its state in LDS between steps and performs
 * every step in full (decode, issue, cycle, rewards, auto-reset, observation, masks and the next
 * action rows, all written to the buffers).  Results are bit-identical to one launch per step. */
int mrts_rollout_fused_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                           uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t first_next_step,
                           int32_t n_steps, void* stream);
#define MRTS_MAX_ITER 1024
/* Native observation exchange over RCCL (BASELINE configs[3] "RCCL obs all-gather"; no
 * Java counterpart — MicroRTS-Py gathers the envs' Responses.observation arrays in one process,
 * Responses.java:12-30).  One process per GPU; every rank's handle joins one RCCL communicator:
 * rank 0 calls mrts_rccl_unique_id, the id (128 bytes) travels to every rank by the caller's own
 * means (torch.distributed), and each rank calls mrts_exchange_init with its rank.  rccl_path names
 * the RCCL library the process already loaded (NULL or "" = "librccl.so"); its entry points are taken
 * with dlopen / dlsym, so libmrts has no link-time dependency on RCCL. */
int mrts_rccl_unique_id(const char* rccl_path, void* out);
int mrts_exchange_init(mrts_env* env, const char* rccl_path, int32_t nranks, int32_t rank, const void* unique_id);
/* Test transport (no RCCL, one GPU): the exchange calls behave as on rank `rank` of `nranks`, and each
 * all-gather copies this rank's bytes into every rank's place — as if the nranks - 1 peers had produced
 * the same data — so the multi-rank layout (rank offsets, strides, chunk bases, the render of every
 * rank) is checkable where RCCL cannot place two ranks on one device. */
int mrts_exchange_init_loopback(mrts_env* env, int32_t nranks, int32_t rank);
/* n_steps fused steps (mrts_rollout_fused_dev's, but one launch per step: every step's observation is
 * exchanged) each followed by an all-gather of that step's observation as int16 [n_slots][C][H][W]
 * (the step kernel writes it into d_send0 / d_send1 alternately, mrts_set_obs16's transport) from every
 * rank into d_recv [nranks][n_slots][C][H][W], on the handle's own communication stream: the collective
 * of step k overlaps step k + 1, and a send buffer is rewritten only after the collective that read it
 * two steps earlier finished.  All collectives of the call are complete when `stream` reaches the end
 * of the call's work.  Full observability only (-ENOTSUP otherwise). */
int mrts_rollout_fused_exchange_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                    double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed,
                                    uint32_t first_next_step, int32_t n_steps, int16_t* d_send0, int16_t* d_send1,
                                    int16_t* d_recv, void* stream);
/* Bytes per exchanged observation value: 2 (int16, the default) or 1 (uint8: the send / recv buffers
 * of the two calls above and below then hold uint8 [..][n_slots][C][H][W], half the all-gather's bytes).
 * uint8 needs a handle whose every observation value fits a byte — full observability on 16x16 maps or
 * maps of at most 64 cells, with the maps' hp / resources and the unit-type table checked at
 * mrts_create — else -ENOTSUP. */
int mrts_set_exchange_bytes(mrts_env* env, int32_t bytes_per_value);
/* The same for BASELINE config c2's unmasked uniform rollout (mrts_rollout_uniform_dev, fused form). */
int mrts_rollout_uniform_exchange_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                      double* d_reward, uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps,
                                      int16_t* d_send0, int16_t* d_send1, int16_t* d_recv, void* stream);
/* Compact observation exchange (the payload of BASELINE configs[3]'s all-gather).  The
 * observation GameState.getVectorObservation returns (rts/GameState.java:922-968) is a pure function of
 * the unit list (position, hp, resources, owner, type, the assignment's action type) and the map's
 * terrain, so the exchange all-gathers that: one record per game and step = 1 + units_per_record
 * 32-bit words (live units in list order; layout in microrts_amd/csrc/mrts_internal.h recWords), and
 * the receiver rebuilds any rank's observations with mrts_render_records_dev.  c3: ~0.26 KB per game
 * instead of 3 KB of uint8 planes for its two slots.  Partially observable handles
 * (PartiallyObservableGameState.getVectorObservation, rts/PartiallyObservableGameState.java:82-154):
 * 1 + 2 * units_per_record words — the units of either view's snapshot with the snapshot's membership
 * and seen action per view; the receiver paints the sight disks from the unit-type table.  c5: ~0.5 KB
 * per game instead of 16 KB of byte planes.
 * mrts_set_records: units per record (0 = off) and steps per launch of a records rollout (0 = up to
 * MRTS_MAX_ITER); self-play handles on maps whose cell count is a multiple of 4 — full observability:
 * <= 256 cells, every observation value fits a byte; partial observability: <= 15 unit types — else
 * -ENOTSUP.  A game with more units than a record holds (or, partially observable, an hp outside int8 /
 * resources outside uint8) sets MRTS_ERR_RECORD.
 * mrts_record_words: 32-bit words per game record as set (0 = records off).
 * mrts_rollout_{fused,uniform}_records_dev: mrts_rollout_{fused,uniform}_dev's steps (multi-step
 * launches where possible), each launch's records written at this rank's place of its chunk of d_recv
 * and all-gathered in place on the handle's RCCL communicator (mrts_exchange_init) while the next launch
 * runs; all collectives are complete when `stream` reaches the end of the call.  d_recv (16-byte aligned)
 * holds n_steps * nranks * n_games * mrts_record_words words; step_offsets (may be NULL) receives,
 * per step, int64 [2]: the word offset in d_recv of rank 0's records of that step and the stride between
 * consecutive ranks' records of it.
 * mrts_render_records_dev: records of n_ranks x n_games games (rank r's game g at d_rec + r * rank_stride
 * + g * mrts_record_words words; the terrain of game g from this handle's map of game g) into
 * d_out [n_ranks][2 * n_games][C][H][W] as uint8 (out_bytes 1; int8 for partially observable handles,
 * whose dead units' hp may be negative) or int32 (out_bytes 4, 16-byte aligned).  rec_words: the words of
 * d_rec from d_rec on; every rank's records must lie inside them (else -EINVAL). */
int mrts_set_records(mrts_env* env, int32_t units_per_record, int32_t steps_per_launch);
int mrts_rollout_fused_records_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                   double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed,
                                   uint32_t first_next_step, int32_t n_steps, uint32_t* d_recv, int64_t* step_offsets,
                                   void* stream);
int mrts_rollout_uniform_records_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                     double* d_reward, uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps,
                                     uint32_t* d_recv, int64_t* step_offsets, void* stream);
int32_t mrts_record_words(const mrts_env* env);
int mrts_render_records_dev(mrts_env* env, const uint32_t* d_rec, int64_t rec_words, int32_t n_ranks, int64_t rank_stride,
                            void* d_out, int32_t out_bytes, void* stream);
/* A learner's minibatch straight from the records (no Java counterpart: MicroRTS-Py's GridnetVecEnv
 * encoding, gym_microrts `_encode_obs` — clip each plane to its size, one-hot, channels last;
 * mrts_onehot_dev's layout), in ONE launch: sample i is slot d_sel[i] (int32, global index r * n_slots + slot
 * over the ranks whose records hold that step) of the step whose rank-0 records start at d_rec +
 * d_step_off[2i] words with rank stride d_step_off[2i + 1] (int64 pairs: the records rollout's step_offsets
 * row of that step; d_step_off NULL: every sample at d_rec with rank_stride) — e.g. random (step, slot) pairs
 * of a whole records rollout.  Out: d_out
 * [n_sel][H][W][F] uint8 (F = mrts_onehot_features, 16-byte aligned).  Full observability (else -ENOTSUP);
 * the render flag of mrts_render_status applies.  rec_words: the words of d_rec from d_rec on, n_ranks: the
 * ranks it holds — a sample whose index is outside [0, n_ranks x n_slots) or whose record lies outside the
 * rec_words renders as zeros and raises the render flag (never a read past the buffer). */
int mrts_render_records_onehot_dev(mrts_env* env, const uint32_t* d_rec, int64_t rec_words, int32_t n_ranks, int64_t rank_stride,
                                   const int32_t* d_sel, const int64_t* d_step_off, int32_t n_sel, uint8_t* d_out, void* stream);
/* 1 if a record rendered by this handle since the last call had its overflow bit set (its game held more
 * units than the record, or a value outside the record's range: the rendered observation lacks them —
 * the sender's handle flagged MRTS_ERR_RECORD), else 0; resets the flag.  Synchronises the device. */
int mrts_render_status(mrts_env* env);
/* Every step's Responses from a rollout call (JNIGridnetVecClient.gameStep returns observation, reward
 * and done on EVERY call, src/tests/JNIGridnetVecClient.java:213-297, src/ai/jni/Responses.java:12-30;
 * a multi-step launch otherwise leaves only the last step's in d_reward / d_done).  After this call,
 * every mrts_rollout_{fused,uniform}[_records|_exchange]_dev call also writes the reward / done of its
 * k-th step ([n_slots][n_rewards], as d_reward / d_done; done[.][0] = 1 when the step auto-reset the
 * game) at d_rewards / d_dones + k * n_slots * n_rewards, k = 0 .. n_steps - 1 — inside multi-step
 * launches too — INSTEAD of d_reward / d_done, which such calls leave untouched (the last step's values
 * are ring step n_steps - 1).  With a records rollout, step k's observation is its records rendered
 * (mrts_render_records_dev at step_offsets[k]): the full per-step Responses without one launch per step.
 * A rollout call of more than max_steps steps returns -EINVAL.  NULL, NULL turns it off. */
int mrts_set_step_responses(mrts_env* env, double* d_rewards, uint8_t* d_dones, int32_t max_steps);
/* Graph form of a handle's calls (no Java counterpart): everything this handle enqueues on `stream`
 * between mrts_capture_begin and mrts_capture_end (stream capture, thread-local mode; the exchange
 * stream of an exchange rollout is joined inside the call) is instantiated as one graph, which
 * mrts_replay launches on any stream with no host work per step.  A replay repeats the captured calls
 * verbatim — the same step indices, seeds and buffers; the handle's bookkeeping advanced at capture
 * time, as if the calls had run then.  Used to time the per-step exchange without host overhead. */
int mrts_capture_begin(mrts_env* env, void* stream);
int mrts_capture_end(mrts_env* env, void* stream);
int mrts_replay(mrts_env* env, void* stream);
/* Timing hook (no Java counterpart): the NEXT mrts_rollout_fused_dev / mrts_rollout_uniform_dev call
 * records `start` (a hipEvent_t) with its first kernel launch and `end` with its last — as the kernel
 * dispatches' own start / end timestamps (hipExtLaunchKernelGGL), so a benchmark's events bracket
 * exactly the rollout's kernels with no extra host call or marker packet in its timed window (the
 * exchange rollouts record them on their stream around the call's work).  One shot: the handle forgets
 * both events when that call begins.  Either may be NULL. */
int mrts_set_rollout_events(mrts_env* env, void* start, void* end);
/* Every later observation write of this handle (any step / reset call with an observation buffer)
 * also writes the planes as int16 into d_obs16 [n_slots][C][H][W] (every value fits: hp, unit
 * types, action types, 0..2 owner, terrain, resources <= 32767 by map validation) — the compact
 * transport of the observation exchange, written by the step kernel instead of a
 * separate narrowing pass.  NULL turns it off.  Full observability only; 8-byte aligned. */
int mrts_set_obs16(mrts_env* env, int16_t* d_obs16);
/* on = 0: mrts_rollout_fused_dev issues one launch per step (for comparison / debugging). */
int mrts_set_multi_step(mrts_env* env, int32_t on);
/* 1 when this handle's kernel shape and the switch allow multi-step launches, else 0.  Then
 * mrts_rollout_uniform_dev uses them; mrts_rollout_fused_dev uses them only on a handle created with
 * mask_delta = 1 (its steady fused state needs delta masks) — otherwise one launch per step. */
int mrts_multi_step_capable(const mrts_env* env);
/* Unmasked uniform random policy (BASELINE config c2): every row of d_actions
 * [n_slots][H*W][7] gets type in [0,6), the four directions in [0,4), produce type in [0,ntypes)
 * and attack index in [0, K-23-ntypes) — no masks needed; illegal rows become NONE in issueSafe
 * like Java's (Philox4x32-10, key = seed, counter = (slot_id_base + slot, step, cell, 0x554E4946)). */
int mrts_policy_uniform_dev(mrts_env* env, uint64_t seed, uint32_t step, int32_t* d_actions, void* stream);
/* mrts_policy_uniform_dev(seed, step, d_actions) followed by mrts_step_dev(d_actions, ...) in ONE
 * launch: the step kernel writes every row of d_actions (the same values) and draws the rows of the
 * idle units it decodes itself instead of reading them back.  Bit-identical to the two calls; one
 * kernel launch (and one launch gap) per step instead of two. */
int mrts_step_uniform_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                          uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t step,
                          void* stream);
/* n_steps x (mrts_policy_uniform_dev(step = first_step + k) then mrts_step_dev without masks),
 * enqueued from native code: the c2 random-policy rollout.  fused != 0: each step as one
 * mrts_step_uniform_dev launch, or — on the multi-step shapes of mrts_rollout_fused_dev, unless
 * mrts_set_multi_step(env, 0) — up to MRTS_MAX_ITER steps per launch (same results).  n_steps >= 0. */
int mrts_rollout_uniform_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                             uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps, int32_t fused,
                             void* stream);
/* Persistent-buffer observations (default off; always on for the library-owned buffer of the
 * host-pointer API).  When a call writes observations into the same buffer as this handle's previous
 * call did, partially observable views re-render only the 4-cell chunks whose cells can have changed
 * (maps with W % 4 == 0, W <= 32, H <= 32; every unit in one wave) — the buffer ends byte-identical
 * to a full rewrite, provided nothing else wrote to it in between (Java's clients also hand out
 * internal arrays that the next call refills or replaces: GameState.java:923-925).
 * A call without an observation buffer, a restore / state injection / copy, or mrts_obs_invalidate
 * makes the next write a full one. */
int mrts_set_obs_delta(mrts_env* env, int32_t on);
int mrts_obs_invalidate(mrts_env* env);
/* the next mrts_policy_dev call writes every row, and the next fused step decodes the rows of
 * d_actions (not the copy the previous fused call kept): call it after writing d_actions yourself */
int mrts_policy_invalidate(mrts_env* env);
/* Optional compact output of every mask write: mask slot 0 ("own unit without an action here") as
 * bits, uint32 [n_slots][ceil(H*W/32)] (sticky; NULL disables).  mrts_policy_dev uses it, when
 * given, to read only the candidate cells' mask rows. */
int mrts_set_source_output(mrts_env* env, uint32_t* d_source);

/* MicroRTS-Py observation encoding (gym_microrts GridnetVecEnv `_encode_obs`, external to the
 * reference: clip each plane to [0, n-1] and one-hot it, channels last) of an observation tensor as
 * written above: uint8 [n_slots][H][W][F], plane sizes {5 hp, 5 resources, 3 owner, types+1, 6 action,
 * 2 terrain} (+ 2 per partial-observability plane); F = mrts_onehot_features(env) (29 / 33).
 * d_out 16-byte aligned. */
int mrts_onehot_features(const mrts_env* env);
int mrts_onehot_dev(mrts_env* env, const int32_t* d_obs, uint8_t* d_out, void* stream);

/* Batched forward model for search AIs: GameState.clone() + playouts + evaluation,
 * as NaiveMCTS / ModelledEvaluationMCTS use the engine.  Games of a forward-model handle are its slots
 * (one per game); a self-play handle's game g holds its slots 2g and 2g+1. */
#define MRTS_MAX_HORIZON 65536
/* GameState.clone() (rts/GameState.java:591-610) for pairs [n][2] = (dst game, src game): dst games of
 * the forward-model handle `dst`, src games of `src` (any handle with the same map size and unit-type
 * table on the same device; NULL = dst).  A dst game keeps its own random streams and playout
 * policies.  No game may be both a source and a destination, nor a destination twice (the host form
 * checks; the device form skips out-of-range pairs and is stream-ordered on `stream` only). */
int mrts_copy_games(mrts_env* dst, const mrts_env* src, const int32_t* pairs, int32_t n);
int mrts_copy_games_dev(mrts_env* dst, const mrts_env* src, const int32_t* d_pairs, int32_t n, void* stream);
/* NaiveMCTS.simulate(gs, gs.getTime() + horizon) (ai/mcts/naivemcts/NaiveMCTS.java:297-308) on every
 * game of a forward-model handle, each with its own policies; |horizon| <= MRTS_MAX_HORIZON. */
int mrts_playout(mrts_env* env, int32_t horizon);
int mrts_playout_dev(mrts_env* env, int32_t horizon, void* stream);
/* SimpleSqrtEvaluationFunction3.evaluate(maxplayer, 1 - maxplayer, gs)
 * (ai/evaluation/SimpleSqrtEvaluationFunction3.java:24-44) of every game: float [n_games] */
int mrts_evaluate(mrts_env* env, int32_t maxplayer, float* out);
int mrts_evaluate_dev(mrts_env* env, int32_t maxplayer, float* d_out, void* stream);

/* Trace replay (test-facing; the replay rule of test/microrts/TestTracesIntegrity.java:72-127, which
 * checks the engine against the reference's recorded games under data/traces): on every game of a
 * forward-model handle (games never auto-reset), issueSafe of player 0's rows, then issueSafe of
 * player 1's rows (:119-120; rts/GameState.java:338-408, each action judged on the unit at (x, y) and
 * issued to it, :356-382), then GameState.cycle() until the game's time reaches until[g] (:83-86).
 * pairs = int32 [n_games][n_pairs][8]: [player (-1 = padding), x, y, UnitAction type, parameter,
 * target x, target y, unit type] (the fields of a trace action, rts/UnitAction.java:110-130), a
 * player's rows in the entry's order.  out[g] (may be NULL) = MRTS_TRACE_* bits.  generic = 1 runs the
 * generic kernel even on the 16x16 / 8x8 shapes that have specialised instances.  Synchronous. */
enum {
    MRTS_TRACE_ISSUED = 1,   /* issueSafe returned true for a player (TestTracesIntegrity.java:119-124) */
    MRTS_TRACE_GAMEOVER = 2, /* a cycle was due after one that ended the game (the Java assertFalse, :84) */
    MRTS_TRACE_NO_UNIT = 4   /* no unit at a pair's (x, y): Java prints "Inconsistent order" (:371-375) */
};
int mrts_trace_step(mrts_env* env, const int32_t* pairs, int32_t n_pairs, const int32_t* until, int32_t* out,
                    int32_t generic);

/* Canonical state dump of the game behind `slot` (same format as the CPU oracle's dumpState):
 * [time, 2, res0, res1, n_units, (type, player, x, y, hp, resources)*, n_assignments,
 *  (unit index, action type, parameter, x, y, unit type or -1, issue time)*] — units in
 * PhysicalGameState list order, assignments in LinkedHashMap insertion order.  Synchronous.
 * Returns the number of int32 written, or -(needed) when cap is too small. */
int mrts_get_state(mrts_env* env, int32_t slot, int32_t* buf, int32_t cap);
/* The unit-type table a config names (utt_json, else utt_version + conflict_policy) as
 * UnitTypeTable.toJSON writes it (UnitTypeTable.java:372-383) — what the clients' sendUTT() returns
 * (JNIGridnetClient.java:225-233).  NUL-terminated; returns the length, or -(length + 1) when cap
 * is too small, or a negative errno for an invalid table. */
int mrts_utt_json(int32_t utt_version, int32_t conflict_policy, const char* utt_json, char* buf, int32_t cap);
/* per-game error flags (MRTS_ERR_*), one uint32 per slot; synchronous */
int mrts_error_flags(mrts_env* env, uint32_t* flags);
/* per-slot envSteps (JNIGridnetVecClient.envSteps, :27); synchronous */
int mrts_env_steps(mrts_env* env, int32_t* out);
/* GameState.toJSON (rts/GameState.java:819-837; includeConstants, raw terrain) of the game behind
 * `slot`; unit IDs are list positions (Java's come from a JVM-global counter).  NUL-terminated;
 * returns the length, or -(length + 1) when cap is too small.  Synchronous. */
int mrts_get_state_json(mrts_env* env, int32_t slot, char* buf, int32_t cap);
/* GameState.fromJSON (rts/GameState.java:897-915) into the game behind `slot` (both slots of a
 * self-play game): time, players, units, terrain and assignments from the JSON; envSteps and the
 * cancel counter restart at 0; the game's random streams are kept.  The next mask / policy write of
 * the handle is a full one.  Synchronous. */
int mrts_set_state_json(mrts_env* env, int32_t slot, const char* json);
/* Whole-handle checkpoint / resume: every game's state block (including the random streams, envSteps
 * and error flags) behind a small header.  mrts_restore accepts only a checkpoint of an identically
 * configured handle (map size, games, unit-type table).  Synchronous. */
int64_t mrts_checkpoint_size(const mrts_env* env);
int mrts_checkpoint(mrts_env* env, void* buf, int64_t cap);
int mrts_restore(mrts_env* env, const void* buf, int64_t size);
/* the handle's hipStream_t */
void* mrts_stream(mrts_env* env);
/* close() (:318-334) + free */
void mrts_destroy(mrts_env* env);
const char* mrts_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MRTS_H */
