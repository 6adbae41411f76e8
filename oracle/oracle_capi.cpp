// ref_cpu — CPU ORACLE (TEST INFRASTRUCTURE ONLY). See ref_cpu.hpp header.
// Clients (tests/JNIGridnetVecClient.java, JNIGridnetClient.java,
// JNIGridnetClientSelfPlay.java, JNIBotClient.java), the WinLoss reward
// (ai/reward/WinLossRewardFunction.java:16-24), the strict trace replay
// (test/microrts/TestTracesIntegrity.java:72-127) and the Philox random policy
// used by bench.py, behind a small C API consumed by ctypes from tests/.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "ref_cpu.hpp"

using namespace oref;

static thread_local std::string g_err;

namespace {

enum BotKind { BOT_PASSIVE = 0, BOT_RANDOM_BIASED = 1 };

// ---------------------------------------------------------------- reward functions (src/ai/reward/*.java)
// ids shared with include/mrts.h MRTS_RF_*
enum RewardKind {
    RF_WINLOSS = 0, RF_RESOURCE_GATHER = 1, RF_PRODUCE_WORKER = 2, RF_PRODUCE_BUILDING = 3, RF_ATTACK = 4,
    RF_PRODUCE_COMBAT_UNIT = 5, RF_CLOSER_TO_ENEMY_BASE = 6, RF_CLOSER_TO_ENEMY_UNIT = 7, RF_COUNT = 8
};

// rts/TraceEntry.java:18-63: a pgs clone + the issued pairs (PlayerAction.clone, PlayerAction.java:264-272:
// new Pair objects holding the same unit and action objects)
struct TraceEntry {
    PGSP pgs;
    int time;
    std::vector<PairP> actions;
    explicit TraceEntry(const GameState& gs) : pgs(gs.pgs->clone()), time(gs.time) {}
    void addPlayerAction(const PlayerAction& pa) {
        for (auto& p : pa.actions) actions.push_back(std::make_shared<Pair>(Pair{p->m_a, p->m_b}));
    }
};

static bool named(const Unit& u, const char* n) { return u.type->name == n; }
static bool mobile(const Unit& u) {  // the "Light" / "Heavy" / "Ranged" / "Worker" name tests
    return named(u, "Light") || named(u, "Heavy") || named(u, "Ranged") || named(u, "Worker");
}

// RewardFunctionInterface.computeReward(maxplayer, minplayer, te, afterGs) for each kind
static void computeReward(int kind, int maxplayer, int minplayer, const TraceEntry& te, const GameState& after,
                          double& reward, uint8_t& done) {
    reward = 0.0;
    done = 0;
    switch (kind) {
        case RF_WINLOSS:  // WinLossRewardFunction.java:16-24
            if (after.gameover()) {
                done = 1;
                reward = after.winner() == maxplayer ? 1.0 : -1.0;
            }
            break;
        case RF_RESOURCE_GATHER: {  // ResourceGatherRewardFunction.java:22-42 (float constants 1)
            for (auto& p : te.actions) {
                if (p->m_a->player == maxplayer && p->m_b->type == UnitAction::TYPE_HARVEST) reward += 1.0f;
                else if (p->m_a->player == maxplayer && p->m_b->type == UnitAction::TYPE_RETURN) reward += 1.0f;
            }
            done = 1;
            for (auto& u : after.pgs->units)
                if (named(*u, "Resource") && u->resources > 0) {
                    done = 0;
                    break;
                }
        } break;
        case RF_PRODUCE_WORKER:       // ProduceWorkerRewardFunction.java:20-30
        case RF_PRODUCE_BUILDING:     // ProduceBuildingRewardFunction.java:20-30
        case RF_PRODUCE_COMBAT_UNIT:  // ProduceCombatUnitRewardFunction.java:20-30
            for (auto& p : te.actions) {
                if (p->m_a->player != maxplayer || p->m_b->type != UnitAction::TYPE_PRODUCE || !p->m_b->unitType) continue;
                const std::string& n = p->m_b->unitType->name;
                bool hit = kind == RF_PRODUCE_WORKER ? n == "Worker"
                         : kind == RF_PRODUCE_BUILDING ? (n == "Barracks" || n == "Base")
                                                       : (n == "Light" || n == "Heavy" || n == "Ranged");
                if (hit) reward += 1.0f;
            }
            break;
        case RF_ATTACK:  // AttackRewardFunction.java:20-36
            for (auto& p : te.actions) {
                if (p->m_a->player == maxplayer && p->m_b->type == UnitAction::TYPE_ATTACK_LOCATION) {
                    const Unit* other = te.pgs->getUnitAt(p->m_b->x, p->m_b->y);
                    if (other) {
                        if (other->player == minplayer) reward += 1.0f;
                        else if (other->player == maxplayer) reward -= 1.0f;
                    }
                }
            }
            break;
        case RF_CLOSER_TO_ENEMY_BASE:    // CloserToEnemyBaseRewardFunction.java:16-60
        case RF_CLOSER_TO_ENEMY_UNIT: {  // CloserToEnemyUnitRewardFunction.java:16-60 (same text: enemy *Base*)
            int baseX = 0, baseY = 0;
            bool baseExists = false;
            for (auto& t : te.pgs->units)
                if (t->player == minplayer && named(*t, "Base")) {
                    baseExists = true;
                    baseX = t->x;
                    baseY = t->y;
                    break;
                }
            if (!baseExists) return;
            double oldMin = 2000000000;
            for (auto& t : te.pgs->units)
                if (t->player == maxplayer && mobile(*t)) {
                    double d = std::sqrt(std::pow((double)(baseX - t->x), 2.0) + std::pow((double)(baseY - t->y), 2.0));
                    if (d < oldMin) oldMin = d;
                }
            double newMin = 2000000000;
            for (auto& t : after.pgs->units)
                if (t->player == maxplayer && mobile(*t)) {
                    double d = std::sqrt(std::pow((double)(baseX - t->x), 2.0) + std::pow((double)(baseY - t->y), 2.0));
                    if (d < newMin) newMin = d;
                }
            reward = oldMin - newMin;
        } break;
        default: throw std::runtime_error("unknown reward function");
    }
}

struct Resp {  // ai/jni/Response.java:12-30: per reward function
    std::vector<int32_t> obs;
    std::vector<double> reward;
    std::vector<uint8_t> done;
};

struct Env;

struct World {
    UnitTypeTable utt;
    int maxAttackRadius, K;
    int H = 0, W = 0, C = 6;
    bool partialObs = false;
    uint64_t seed = 0;
    std::vector<int> rfs{RF_WINLOSS};  // a_rfs (JNIGridnetVecClient.java:106)
    World(int ver, int crs, const char* uttJson = nullptr)
        : utt(uttJson ? UnitTypeTable::fromJSON(uttJson) : UnitTypeTable(ver, crs)) {
        maxAttackRadius = utt.getMaxAttackRange() * 2 + 1;
        K = maskSlotsPerCell(utt);
    }
};

// One game (self-play: 2 external players; bot: 1 external + 1 AI)
struct Env {
    World* w;
    MapTemplate map;
    bool selfplay;
    BotKind botKind = BOT_PASSIVE;
    GSP gs;
    GSP playergs[2];
    JavaRandom samplerGen, cancelGen, damageGen;
    std::unique_ptr<AI> ai2;
    Resp resp[2];

    Env(World* wd, const MapTemplate& m, bool sp, BotKind bk, uint64_t envSeed)
        : w(wd), map(m), selfplay(sp), botKind(bk), samplerGen((int64_t)envSeed),
          cancelGen((int64_t)(envSeed ^ 0x9E3779B97F4A7C15ULL)), damageGen((int64_t)(envSeed ^ 0xC2B2AE3D27D4EB4FULL)) {
        if (!sp) {
            if (bk == BOT_PASSIVE) ai2.reset(new PassiveAI());
            else ai2.reset(new RandomBiasedAI(&samplerGen));
        }
        for (auto& r : resp) {
            r.obs.assign((size_t)w->C * w->H * w->W, 0);
            r.reward.assign(w->rfs.size(), 0.0);
            r.done.assign(w->rfs.size(), 0);
        }
    }
    void rewards(Resp& r, int maxplayer, const TraceEntry& te) {
        for (size_t j = 0; j < w->rfs.size(); j++) computeReward(w->rfs[j], maxplayer, 1 - maxplayer, te, *gs, r.reward[j], r.done[j]);
    }
    // JNIGridnetClient.reset zeroes every slot (tests/JNIGridnetClient.java:248-251); the self-play
    // client's loop is bounded by rewards.length == numPlayers == 2, not by rfs.length
    // (tests/JNIGridnetClientSelfPlay.java:103-104,235-238): slots >= 2 keep the previous step's
    // values.  (With one reward function Java throws there; here the single slot is zeroed —
    // DESIGN.md §8.)
    void clearRewards(Resp& r) {
        const size_t n = selfplay ? std::min<size_t>(2, r.reward.size()) : r.reward.size();
        std::fill(r.reward.begin(), r.reward.begin() + n, 0.0);
        std::fill(r.done.begin(), r.done.begin() + n, 0);
    }
    GSP makeView(int player) {
        if (w->partialObs) return std::make_shared<PartiallyObservableGameState>(*gs, player);
        return gs;
    }
    void newGame() {
        gs = std::make_shared<GameState>(instantiate(map, w->utt), &w->utt);
        gs->cancelRandom = &cancelGen;
        gs->damageRandom = &damageGen;
    }
    // JNIGridnetClientSelfPlay.reset (tests/JNIGridnetClientSelfPlay.java:221-247)
    // JNIGridnetClient.reset (tests/JNIGridnetClient.java:235-258)
    void reset(int player) {
        newGame();
        if (selfplay) {
            for (int i = 0; i < 2; i++) {
                playergs[i] = makeView(i);
                clearRewards(resp[i]);
                playergs[i]->getVectorObservation(i, resp[i].obs.data());
            }
        } else {
            playergs[0] = makeView(player);
            clearRewards(resp[0]);
            playergs[0]->getVectorObservation(player, resp[0].obs.data());
        }
    }
    std::vector<int> rowsFromGrid(const int32_t* a) const {  // [HW][7] → Java rows [pos, 7 comps]
        const int HW = w->H * w->W;
        std::vector<int> rows((size_t)HW * 8);
        for (int c = 0; c < HW; c++) {
            rows[(size_t)c * 8] = c;
            for (int k = 0; k < 7; k++) rows[(size_t)c * 8 + 1 + k] = a[(size_t)c * 7 + k];
        }
        return rows;
    }
    // JNIAI.getAction (ai/jni/JNIAI.java:51-55)
    PlayerAction jniGetAction(int player, const GameState& g, const std::vector<int>& rows) const {
        int n = (int)(rows.size() / 8);
        PlayerAction pa = PlayerAction::fromVectorAction(rows, n, g, w->utt, player, w->maxAttackRadius);
        pa.fillWithNones(g, player, 1);
        return pa;
    }
    // JNIGridnetClientSelfPlay.gameStep (tests/JNIGridnetClientSelfPlay.java:159-189)
    void stepSelfPlay(const std::vector<int>& rows0, const std::vector<int>& rows1) {
        const std::vector<int>* rows[2] = {&rows0, &rows1};
        TraceEntry te(*gs);  // before either issue (JNIGridnetClientSelfPlay.java:160)
        for (int i = 0; i < 2; i++) {
            playergs[i] = makeView(i);
            PlayerAction pa = jniGetAction(i, *playergs[i], *rows[i]);
            gs->issueSafe(pa);
            te.addPlayerAction(pa);
        }
        gs->cycle();
        for (int i = 0; i < 2; i++) {
            rewards(resp[i], i, te);
            playergs[i]->getVectorObservation(i, resp[i].obs.data());
        }
    }
    // JNIGridnetClient.gameStep (tests/JNIGridnetClient.java:163-203)
    void stepBot(const std::vector<int>& rows, int player) {
        GSP p1 = makeView(player);
        GSP p2 = makeView(1 - player);
        playergs[0] = p1;
        PlayerAction pa1 = jniGetAction(player, *p1, rows);
        PlayerAction pa2 = ai2->getAction(1 - player, *p2);
        gs->issueSafe(pa1);
        gs->issueSafe(pa2);
        TraceEntry te(*gs);  // after both issues (JNIGridnetClient.java:182-184)
        te.addPlayerAction(pa1);
        te.addPlayerAction(pa2);
        gs->cycle();
        rewards(resp[0], player, te);
        p1->getVectorObservation(player, resp[0].obs.data());
    }
};

// tests/JNIGridnetVecClient.java:17-335
struct VecClient {
    std::unique_ptr<World> world;
    std::vector<std::unique_ptr<Env>> selfPlay;  // one per pair of slots
    std::vector<std::unique_ptr<Env>> bots;
    std::vector<int> envSteps;
    int maxSteps = 2000;
    int nSlots() const { return (int)(selfPlay.size() * 2 + bots.size()); }
    Env* slotEnv(int s, int* player) {
        int nsp = (int)selfPlay.size() * 2;
        if (s < nsp) {
            *player = s & 1;
            return selfPlay[(size_t)s / 2].get();
        }
        *player = 0;
        return bots[(size_t)(s - nsp)].get();
    }
    void collect(int32_t* obs, double* reward, uint8_t* done) {  // reward / done: [slots][R]
        const size_t osz = (size_t)world->C * world->H * world->W;
        const size_t R = world->rfs.size();
        for (int s = 0; s < nSlots(); s++) {
            int p;
            Env* e = slotEnv(s, &p);
            Resp& r = e->resp[e->selfplay ? p : 0];
            if (obs) std::memcpy(obs + (size_t)s * osz, r.obs.data(), osz * sizeof(int32_t));
            for (size_t j = 0; j < R; j++) {
                if (reward) reward[(size_t)s * R + j] = r.reward[j];
                if (done) done[(size_t)s * R + j] = r.done[j];
            }
        }
    }
    // reset (:179-211)
    void reset(const int32_t* players) {
        for (auto& e : selfPlay) e->reset(0);
        int nsp = (int)selfPlay.size() * 2;
        for (size_t j = 0; j < bots.size(); j++) bots[j]->reset(players ? players[nsp + (int)j] : 0);
        // envSteps[] is left alone: reset() never touches it (JNIGridnetVecClient.java:179-211); it is
        // zeroed only by the constructor (:116) and the auto-reset path (:229,264-265,285)
    }
    // gameStep (:213-297) with the grid layout [slot][HW][7] (row r = cell r, ascending)
    void step(const int32_t* actions, const int32_t* players) {
        const size_t asz = (size_t)world->H * world->W * 7;
        stepWith([&](Env& e, int s) { return e.rowsFromGrid(actions + (size_t)s * asz); }, players);
    }
    // gameStep with the Java layout: action[slot] = n_rows rows [pos, 7 comps], any order, duplicates
    void stepRows(const int32_t* rows, int nrows, const int32_t* players) {
        stepWith([&](Env&, int s) {
            const int32_t* r = rows + (size_t)s * nrows * 8;
            return std::vector<int>(r, r + (size_t)nrows * 8);
        }, players);
    }
    template <class RowsOf>
    void stepWith(RowsOf rowsOf, const int32_t* players) {
        for (size_t i = 0; i < selfPlay.size(); i++) {
            Env& e = *selfPlay[i];
            e.stepSelfPlay(rowsOf(e, (int)(2 * i)), rowsOf(e, (int)(2 * i + 1)));
            envSteps[2 * i] += 1;
            envSteps[2 * i + 1] += 1;
            if (e.resp[0].done[0] || envSteps[2 * i] >= maxSteps) {  // done[0]: the first reward function's
                std::vector<double> tr0 = e.resp[0].reward, tr1 = e.resp[1].reward;
                std::vector<uint8_t> td0 = e.resp[0].done, td1 = e.resp[1].done;
                e.reset(0);
                e.resp[0].reward = tr0;
                e.resp[0].done = td0;
                e.resp[1].reward = tr1;
                e.resp[1].done = td1;
                e.resp[0].done[0] = 1;
                e.resp[1].done[0] = 1;
                envSteps[2 * i] = 0;
                envSteps[2 * i + 1] = 0;
            }
        }
        int nsp = (int)selfPlay.size() * 2;
        for (size_t j = 0; j < bots.size(); j++) {
            int s = nsp + (int)j;
            Env& e = *bots[j];
            int pl = players ? players[s] : 0;
            envSteps[(size_t)s] += 1;
            e.stepBot(rowsOf(e, s), pl);
            if (e.resp[0].done[0] || envSteps[(size_t)s] >= maxSteps) {
                std::vector<double> tr = e.resp[0].reward;
                std::vector<uint8_t> td = e.resp[0].done;
                e.reset(pl);
                e.resp[0].reward = tr;
                e.resp[0].done = td;
                e.resp[0].done[0] = 1;
                envSteps[(size_t)s] = 0;
            }
        }
    }
    // getMasks (:307-316) → JNIGridnetClient(SelfPlay).getMasks
    void masks(int player, uint8_t* out) {
        const size_t msz = (size_t)world->H * world->W * world->K;
        int nsp = (int)selfPlay.size() * 2;
        for (size_t i = 0; i < selfPlay.size(); i++) {
            computeMasks(*selfPlay[i]->gs, world->utt, 0, out + (2 * i) * msz);
            computeMasks(*selfPlay[i]->gs, world->utt, 1, out + (2 * i + 1) * msz);
        }
        for (size_t j = 0; j < bots.size(); j++) computeMasks(*bots[j]->gs, world->utt, player, out + (size_t)(nsp + (int)j) * msz);
    }
};

// ---------------------------------------------------------------- Philox4x32-10 random policy
struct Philox {
    static inline uint32_t mulhi(uint32_t a, uint32_t b, uint32_t* lo) {
        uint64_t p = (uint64_t)a * b;
        *lo = (uint32_t)p;
        return (uint32_t)(p >> 32);
    }
    static void gen(uint32_t c[4], uint32_t k0, uint32_t k1) {
        for (int r = 0; r < 10; r++) {
            uint32_t lo0, lo1;
            uint32_t hi0 = mulhi(0xD2511F53u, c[0], &lo0);
            uint32_t hi1 = mulhi(0xCD9E8D57u, c[2], &lo1);
            uint32_t n0 = hi1 ^ c[1] ^ k0, n1 = lo1, n2 = hi0 ^ c[3] ^ k1, n3 = lo0;
            c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
    }
};
static inline int pickBit(uint32_t r, const uint8_t* bits, int n) {  // uniform among set bits (multiply-shift)
    int cnt = 0;
    for (int i = 0; i < n; i++) cnt += bits[i] ? 1 : 0;
    if (cnt == 0) return -1;
    int k = (int)(((uint64_t)r * (uint32_t)cnt) >> 32);
    for (int i = 0; i < n; i++)
        if (bits[i]) {
            if (k == 0) return i;
            k--;
        }
    return -1;
}

}  // namespace

// Masked uniform random policy shared bit-for-bit with the GPU kernel
// (microrts_amd/csrc/mrts_kernels.hip: policy_kernel).  mask = u8[HW][K], out = int32[HW][7].
extern "C" void oref_policy(const uint8_t* mask, int HW, int K, int n_types, uint64_t seed, uint32_t env_id,
                            uint32_t step, uint32_t player, int32_t* out) {
    for (int c = 0; c < HW; c++) {
        const uint8_t* m = mask + (size_t)c * K;
        int32_t* a = out + (size_t)c * 7;
        for (int k = 0; k < 7; k++) a[k] = 0;
        if (!m[0]) continue;
        uint32_t ctr[4] = {env_id, step, (uint32_t)c, player};
        Philox::gen(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        int t = pickBit(ctr[0], m + 1, 6);
        if (t < 0) continue;
        a[0] = t;
        switch (t) {
            case 1: a[1] = pickBit(ctr[1], m + 7, 4); break;
            case 2: a[2] = pickBit(ctr[1], m + 11, 4); break;
            case 3: a[3] = pickBit(ctr[1], m + 15, 4); break;
            case 4:
                a[4] = pickBit(ctr[1], m + 19, 4);
                a[5] = pickBit(ctr[2], m + 23, n_types);
                break;
            case 5: a[6] = pickBit(ctr[1], m + 23 + n_types, K - 23 - n_types); break;
        }
    }
}

// Unmasked uniform random policy (BASELINE config c2; include/mrts.h
// mrts_policy_uniform_dev): per cell, Philox4x32-10 with counter (slot id, step, cell, "UNIF"),
// type = 6 * w0 >> 32, directions = 2-bit fields of w1, produce type = ntypes * w2 >> 32, attack
// index = natt * w3 >> 32 (natt = K - 23 - ntypes).
extern "C" void oref_policy_uniform(int HW, int K, int n_types, uint64_t seed, uint32_t slot_id, uint32_t step, int32_t* out) {
    const int natt = K - 23 - n_types;
    for (int c = 0; c < HW; c++) {
        uint32_t ctr[4] = {slot_id, step, (uint32_t)c, 0x554E4946u};
        Philox::gen(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        int32_t* a = out + (size_t)c * 7;
        a[0] = (int32_t)(((uint64_t)ctr[0] * 6u) >> 32);
        a[1] = (int32_t)(ctr[1] & 3u);
        a[2] = (int32_t)((ctr[1] >> 2) & 3u);
        a[3] = (int32_t)((ctr[1] >> 4) & 3u);
        a[4] = (int32_t)((ctr[1] >> 6) & 3u);
        a[5] = (int32_t)(((uint64_t)ctr[2] * (uint32_t)n_types) >> 32);
        a[6] = (int32_t)(((uint64_t)ctr[3] * (uint32_t)natt) >> 32);
    }
}

extern "C" {

const char* oref_last_error() { return g_err.c_str(); }

// map_paths: one per slot (self-play games use map_paths[2i], like :119); bot_kinds: per bot env
void* oref_create(int n_selfplay_slots, int n_bot_envs, const int32_t* bot_kinds, int max_steps, int partial_obs,
                  int utt_version, int crs, const char** map_paths, uint64_t seed, const char* utt_json) {
    try {
        if (n_selfplay_slots % 2) throw std::runtime_error("n_selfplay_slots must be even");
        auto v = new VecClient();
        v->world.reset(new World(utt_version, crs, utt_json));
        v->world->partialObs = partial_obs != 0;
        v->world->C = partial_obs ? 8 : 6;
        v->world->seed = seed;
        v->maxSteps = max_steps;
        int nslots = n_selfplay_slots + n_bot_envs;
        std::vector<MapTemplate> maps;
        for (int s = 0; s < nslots; s++) maps.push_back(loadMapFile(map_paths[s]));
        v->world->H = maps[0].height;
        v->world->W = maps[0].width;
        for (auto& m : maps)
            if (m.height != v->world->H || m.width != v->world->W) throw std::runtime_error("all maps must share env 0's size");
        for (int i = 0; i < n_selfplay_slots / 2; i++)
            v->selfPlay.emplace_back(new Env(v->world.get(), maps[(size_t)(2 * i)], true, BOT_PASSIVE, seed + (uint64_t)(2 * i)));
        for (int j = 0; j < n_bot_envs; j++)
            v->bots.emplace_back(new Env(v->world.get(), maps[(size_t)(n_selfplay_slots + j)], false,
                                         (BotKind)(bot_kinds ? bot_kinds[j] : 0), seed + (uint64_t)(n_selfplay_slots + j)));
        v->envSteps.assign((size_t)nslots, 0);
        return v;
    } catch (std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

void oref_destroy(void* h) { delete (VecClient*)h; }

int oref_dims(void* h, int32_t* slots, int32_t* H, int32_t* W, int32_t* C, int32_t* K) {
    auto v = (VecClient*)h;
    *slots = v->nSlots();
    *H = v->world->H;
    *W = v->world->W;
    *C = v->world->C;
    *K = v->world->K;
    return 0;
}

int oref_reset(void* h, const int32_t* players, int32_t* obs, double* reward, uint8_t* done) {
    try {
        auto v = (VecClient*)h;
        v->reset(players);
        v->collect(obs, reward, done);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}

int oref_step(void* h, const int32_t* actions, const int32_t* players, int32_t* obs, double* reward, uint8_t* done) {
    try {
        auto v = (VecClient*)h;
        v->step(actions, players);
        v->collect(obs, reward, done);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}

// a_rfs (JNIGridnetVecClient.java:106): the reward functions (RewardKind ids), in order; call before
// reset.  reward / done of reset / step are then [slots][n].
int oref_set_rewards(void* h, const int32_t* kinds, int n) {
    auto v = (VecClient*)h;
    if (n < 1 || n > RF_COUNT) return -22;
    for (int i = 0; i < n; i++)
        if (kinds[i] < 0 || kinds[i] >= RF_COUNT) return -22;
    v->world->rfs.assign(kinds, kinds + n);
    auto fix = [&](Env& e) {
        for (auto& r : e.resp) {
            r.reward.assign((size_t)n, 0.0);
            r.done.assign((size_t)n, 0);
        }
    };
    for (auto& e : v->selfPlay) fix(*e);
    for (auto& e : v->bots) fix(*e);
    return 0;
}

// gameStep(int[][][] action, players) with Java rows: rows = [slots][n_rows][8]
int oref_step_rows(void* h, const int32_t* rows, int n_rows, const int32_t* players, int32_t* obs, double* reward,
                   uint8_t* done) {
    try {
        auto v = (VecClient*)h;
        v->stepRows(rows, n_rows, players);
        v->collect(obs, reward, done);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}

int oref_get_masks(void* h, int player, uint8_t* out) {
    try {
        ((VecClient*)h)->masks(player, out);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}

// Canonical dump of the game behind slot s (ref_cpu.hpp dumpState)
int oref_dump_state(void* h, int slot, int32_t* buf, int cap) {
    auto v = (VecClient*)h;
    int p;
    Env* e = v->slotEnv(slot, &p);
    auto d = dumpState(*e->gs);
    if ((int)d.size() > cap) return -(int)d.size();
    std::memcpy(buf, d.data(), d.size() * sizeof(int32_t));
    return (int)d.size();
}

int oref_env_steps(void* h, int slot) { return ((VecClient*)h)->envSteps[(size_t)slot]; }
// GameState.toJSON of the game behind `slot`; returns the length or -(length + 1)
int oref_state_json(void* h, int slot, char* buf, int cap) {
    int p;
    const std::string j = gameStateToJSON(*((VecClient*)h)->slotEnv(slot, &p)->gs);
    if (!buf || cap < (int)j.size() + 1) return -((int)j.size() + 1);
    std::memcpy(buf, j.c_str(), j.size() + 1);
    return (int)j.size();
}
// GameState.fromJSON into the game behind `slot` (its random streams kept, envSteps restarts at 0)
int oref_set_state_json(void* h, int slot, const char* json) {
    try {
        auto v = (VecClient*)h;
        int p;
        Env* e = v->slotEnv(slot, &p);
        e->gs = gameStateFromJSON(json, v->world->utt);
        e->gs->cancelRandom = &e->cancelGen;
        e->gs->damageRandom = &e->damageGen;
        const int nsp = (int)v->selfPlay.size() * 2;
        if (slot < nsp) {
            v->envSteps[(size_t)(slot & ~1)] = 0;
            v->envSteps[(size_t)(slot | 1)] = 0;
        } else {
            v->envSteps[(size_t)slot] = 0;
        }
        return 0;
    } catch (std::exception& ex) {
        g_err = ex.what();
        return -22;
    }
}
int oref_errors(void* h, int slot) {
    int p;
    return ((VecClient*)h)->slotEnv(slot, &p)->gs->errors;
}

// ------------------------------------------------ bot-vs-bot client (config 1; tests/JNIBotClient.java)
struct BotVec {
    std::unique_ptr<World> world;
    MapTemplate map;
    GSP gs;
    JavaRandom gen;  // util/Sampler.java:17 — one JVM-global generator shared by both AIs
    JavaRandom cancelGen, damageGen;
    void newGame() {
        gs = std::make_shared<GameState>(instantiate(map, world->utt), &world->utt);
        gs->cancelRandom = &cancelGen;
        gs->damageRandom = &damageGen;
    }
    std::unique_ptr<AI> ai1, ai2;
    int envSteps = 0, maxSteps = 2000;
    std::vector<int> rfs{RF_WINLOSS};
};

void* oref_botclient_create(const char* map_path, int ai1, int ai2, int max_steps, int utt_version, int crs, int64_t seed,
                            const char* utt_json) {
    try {
        auto b = new BotVec();
        b->world.reset(new World(utt_version, crs, utt_json));
        b->map = loadMapFile(map_path);
        b->world->H = b->map.height;
        b->world->W = b->map.width;
        b->gen.setSeed(seed);
        b->cancelGen.setSeed((int64_t)((uint64_t)seed ^ 0x9E3779B97F4A7C15ULL));
        b->damageGen.setSeed((int64_t)((uint64_t)seed ^ 0xC2B2AE3D27D4EB4FULL));
        b->maxSteps = max_steps;
        auto mk = [&](int k) -> AI* { return k == BOT_PASSIVE ? (AI*)new PassiveAI() : (AI*)new RandomBiasedAI(&b->gen); };
        b->ai1.reset(mk(ai1));
        b->ai2.reset(mk(ai2));
        b->newGame();
        return b;
    } catch (std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}
void oref_botclient_destroy(void* h) { delete (BotVec*)h; }
// a_rfs: the reward functions (RewardKind ids), in order; reward/done of oref_botclient_step get n values
int oref_botclient_set_rewards(void* h, const int32_t* kinds, int n) {
    auto b = (BotVec*)h;
    if (n < 1 || n > RF_COUNT) return -22;
    b->rfs.assign(kinds, kinds + n);
    return 0;
}
// JNIBotClient.gameStep (:108-135) + VecClient bot-only auto-reset (JNIGridnetVecClient.java:214-238); returns 0
int oref_botclient_step(void* h, int player, double* reward, uint8_t* done) {
    try {
        auto b = (BotVec*)h;
        PlayerAction pa1 = b->ai1->getAction(player, *b->gs);
        PlayerAction pa2 = b->ai2->getAction(1 - player, *b->gs);
        b->gs->issueSafe(pa1);
        b->gs->issueSafe(pa2);
        TraceEntry te(*b->gs);  // JNIBotClient.java:114-116
        te.addPlayerAction(pa1);
        te.addPlayerAction(pa2);
        b->gs->cycle();
        const size_t R = b->rfs.size();
        for (size_t j = 0; j < R; j++) computeReward(b->rfs[j], player, 1 - player, te, *b->gs, reward[j], done[j]);
        b->envSteps++;
        if (done[0] || b->envSteps >= b->maxSteps) {  // rs[i].done[0] (JNIGridnetVecClient.java:218-230)
            b->newGame();
            done[0] = 1;
            b->envSteps = 0;
        }
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}
int oref_botclient_dump(void* h, int32_t* buf, int cap) {
    auto d = dumpState(*((BotVec*)h)->gs);
    if ((int)d.size() > cap) return -(int)d.size();
    std::memcpy(buf, d.data(), d.size() * sizeof(int32_t));
    return (int)d.size();
}

// ------------------------------------------------ batched forward model
// GameState.clone() (rts/GameState.java:591-610) + NaiveMCTS.simulate (ai/mcts/naivemcts/
// NaiveMCTS.java:297-308) + SimpleSqrtEvaluationFunction3, one GameState per game.  Game j's random
// streams are seeded like bot env j of oref_create (seed + j): one JVM running that playout with
// Sampler.generator (shared by both policies), GameState.r and UnitAction.r seeded so.
struct FwdModel {
    std::unique_ptr<World> world;
    MapTemplate map;
    struct Game {
        GSP gs;
        JavaRandom gen, cancelGen, damageGen;
        std::unique_ptr<AI> ai[2];
    };
    std::vector<std::unique_ptr<Game>> games;
    void attach(Game& g) {
        g.gs->cancelRandom = &g.cancelGen;
        g.gs->damageRandom = &g.damageGen;
    }
};

void* oref_fm_create(const char* map_path, int n, const int32_t* ai1, const int32_t* ai2, int utt_version, int crs,
                     int64_t seed, const char* utt_json) {
    try {
        auto f = new FwdModel();
        f->world.reset(new World(utt_version, crs, utt_json));
        f->map = loadMapFile(map_path);
        f->world->H = f->map.height;
        f->world->W = f->map.width;
        for (int j = 0; j < n; j++) {
            auto g = std::make_unique<FwdModel::Game>();
            const int64_t es = seed + j;
            g->gen.setSeed(es);
            g->cancelGen.setSeed((int64_t)((uint64_t)es ^ 0x9E3779B97F4A7C15ULL));
            g->damageGen.setSeed((int64_t)((uint64_t)es ^ 0xC2B2AE3D27D4EB4FULL));
            const int k[2] = {ai1[j], ai2[j]};
            for (int p = 0; p < 2; p++)
                g->ai[p].reset(k[p] == BOT_PASSIVE ? (AI*)new PassiveAI() : (AI*)new RandomBiasedAI(&g->gen));
            g->gs = std::make_shared<GameState>(instantiate(f->map, f->world->utt), &f->world->utt);
            f->attach(*g);
            f->games.push_back(std::move(g));
        }
        return f;
    } catch (std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}
void oref_fm_destroy(void* h) { delete (FwdModel*)h; }
// gs[dst] = gs[src].clone()
int oref_fm_copy(void* h, int dst, int src) {
    auto f = (FwdModel*)h;
    auto& g = *f->games.at((size_t)dst);
    g.gs = f->games.at((size_t)src)->gs->clone();
    f->attach(g);
    return 0;
}
// gs[dst] = (the game behind slot `slot` of VecClient `vec`).clone()
int oref_fm_copy_from_vec(void* h, int dst, void* vec, int slot) {
    auto f = (FwdModel*)h;
    int p;
    auto& g = *f->games.at((size_t)dst);
    g.gs = ((VecClient*)vec)->slotEnv(slot, &p)->gs->clone();
    f->attach(g);
    return 0;
}
// NaiveMCTS.simulate(gs, gs.getTime() + horizon) (NaiveMCTS.java:297-308)
int oref_fm_playout(void* h, int game, int horizon) {
    try {
        auto& g = *((FwdModel*)h)->games.at((size_t)game);
        GameState& gs = *g.gs;
        const int time = gs.time + horizon;
        bool gameover = false;
        do {
            if (gs.isComplete()) {
                gameover = gs.cycle();
            } else {
                PlayerAction pa0 = g.ai[0]->getAction(0, gs);
                gs.issue(pa0);
                PlayerAction pa1 = g.ai[1]->getAction(1, gs);
                gs.issue(pa1);
            }
        } while (!gameover && gs.time < time);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}
float oref_fm_evaluate(void* h, int game, int maxplayer) {
    return simpleSqrtEvaluation3(maxplayer, 1 - maxplayer, *((FwdModel*)h)->games.at((size_t)game)->gs);
}
int oref_fm_dump(void* h, int game, int32_t* buf, int cap) {
    auto d = dumpState(*((FwdModel*)h)->games.at((size_t)game)->gs);
    if ((int)d.size() > cap) return -(int)d.size();
    std::memcpy(buf, d.data(), d.size() * sizeof(int32_t));
    return (int)d.size();
}
int oref_fm_errors(void* h, int game) { return ((FwdModel*)h)->games.at((size_t)game)->gs->errors; }

// ------------------------------------------------ strict trace replay
// Fixture text (tests/golden/make_trace_fixtures.py): see that script's docstring.
// Replays like TestTracesIntegrity.testTrace and additionally compares the full
// PhysicalGameState with each entry's snapshot.  Returns #entries checked (>=0)
// or -1 with a message.  onEntry(e, gs) runs after the replay caught up with entry e (the state the
// strict check just compared); onIssued(e, issued) after entry e's actions were issued.
}  // extern "C"
namespace {
template <class OnEntry, class OnIssued>
int replayTrace(const char* map_path, const char* fixture, char* msg, int msglen, OnEntry onEntry, OnIssued onIssued) {
    auto fail = [&](const std::string& s) {
        std::snprintf(msg, (size_t)msglen, "%s", s.c_str());
        return -1;
    };
    try {
        UnitTypeTable utt(1, 1);
        MapTemplate m = loadMapFile(map_path);
        GameState gs(instantiate(m, utt), &utt);
        std::istringstream in(fixture);
        std::string tok;
        int nentries;
        in >> tok >> nentries;
        if (tok != "TRACE") return fail("bad fixture header");
        bool gameOver = false;
        int checked = 0;
        for (int e = 0; e < nentries; e++) {
            int time, r0, r1, nu;
            in >> tok >> time;
            if (tok != "E") return fail("bad entry");
            in >> tok >> r0 >> r1;
            in >> tok >> nu;
            auto tp = std::make_shared<PhysicalGameState>();
            tp->width = m.width;
            tp->height = m.height;
            tp->terrain = gs.pgs->terrain;
            tp->players.push_back(std::make_shared<Player>(Player{0, r0}));
            tp->players.push_back(std::make_shared<Player>(Player{1, r1}));
            for (int i = 0; i < nu; i++) {
                auto u = std::make_shared<Unit>();
                int t;
                in >> tok >> t >> u->ID >> u->player >> u->x >> u->y >> u->resources >> u->hitpoints;
                u->type = utt.getUnitType(t);
                tp->units.push_back(u);
            }
            int na;
            in >> tok >> na;
            struct TA { int64_t id; int type, param, x, y, ut; };
            std::vector<TA> tas((size_t)na);
            for (auto& a : tas) in >> tok >> a.id >> a.type >> a.param >> a.x >> a.y >> a.ut;
            // TestTracesIntegrity.java:83-86
            while (gs.time < time) {
                if (gameOver) return fail("game over before entry time " + std::to_string(time));
                gameOver = gs.cycle();
            }
            // STRICT: full pgs equality (stronger than the reference's own test)
            const PhysicalGameState& p = *gs.pgs;
            std::ostringstream why;
            if (p.players[0]->resources != r0 || p.players[1]->resources != r1)
                why << "player resources " << p.players[0]->resources << "," << p.players[1]->resources << " vs " << r0 << "," << r1;
            else if ((int)p.units.size() != nu)
                why << "unit count " << p.units.size() << " vs " << nu;
            else
                for (int i = 0; i < nu; i++) {
                    const Unit& a = *p.units[(size_t)i];
                    const Unit& b = *tp->units[(size_t)i];
                    if (a.type->ID != b.type->ID || a.player != b.player || a.x != b.x || a.y != b.y || a.hitpoints != b.hitpoints ||
                        a.resources != b.resources) {
                        why << "unit " << i << " (" << a.type->name << " p" << a.player << " @" << a.x << "," << a.y << " hp" << a.hitpoints
                            << " r" << a.resources << ") vs (" << b.type->name << " p" << b.player << " @" << b.x << "," << b.y << " hp"
                            << b.hitpoints << " r" << b.resources << ")";
                        break;
                    }
                }
            if (!why.str().empty()) return fail("time " + std::to_string(time) + ": " + why.str());
            onEntry(e, gs);
            checked++;
            bool issued = false;
            if (!tas.empty()) {  // :101-125
                bool containsRealActions = false;
                PlayerAction p1, p2;
                for (auto& a : tas) {
                    UnitP tu;
                    for (auto& u : tp->units)
                        if (u->ID == a.id) { tu = u; break; }
                    if (!tu) return fail("undefined unit ID in trace action");
                    auto ua = std::make_shared<UnitAction>(a.type, a.param);
                    ua->x = a.x;
                    ua->y = a.y;
                    ua->unitType = a.ut >= 0 ? utt.getUnitType(a.ut) : nullptr;
                    if (tu->player == 0) p1.addUnitAction(tu, ua);
                    else if (tu->player == 1) p2.addUnitAction(tu, ua);
                    else return fail("action for a non-player unit");
                    containsRealActions = containsRealActions || ua->type != UnitAction::TYPE_NONE;
                }
                issued = gs.issueSafe(p1);
                issued = gs.issueSafe(p2) || issued;
                if (containsRealActions != issued) return fail("containsRealActions != issuedActions at time " + std::to_string(time));
            }
            onIssued(e, issued);
        }
        return checked;
    } catch (std::exception& e) {
        return fail(std::string("exception: ") + e.what());
    }
}
}  // namespace
extern "C" {

int oref_trace_replay(const char* map_path, const char* fixture, char* msg, int msglen) {
    return replayTrace(map_path, fixture, msg, msglen, [](int, const GameState&) {}, [](int, bool) {});
}

// The same replay, keeping the canonical dump (dumpState: units in list order, assignments in
// LinkedHashMap order) of the state at every entry — what the GPU replay (tests/test_gpu_traces.py)
// compares against beyond the trace's own snapshot — into buf (offsets[e] .. offsets[e + 1]), and
// issueSafe's combined return value per entry into issued[e].  Returns #entries, -1 with a message,
// or -2 when cap / max_entries is too small.
int oref_trace_dumps(const char* map_path, const char* fixture, int32_t* buf, int64_t cap, int32_t* offsets, int32_t* issued,
                     int32_t max_entries, char* msg, int msglen) {
    int64_t used = 0;
    bool overflow = false;
    offsets[0] = 0;
    const int n = replayTrace(
        map_path, fixture, msg, msglen,
        [&](int e, const GameState& gs) {
            if (e >= max_entries) {
                overflow = true;
                return;
            }
            const auto d = dumpState(gs);
            if (used + (int64_t)d.size() > cap) {
                overflow = true;
            } else {
                std::memcpy(buf + used, d.data(), d.size() * 4);
                used += (int64_t)d.size();
            }
            offsets[e + 1] = (int32_t)used;
        },
        [&](int e, bool is) {
            if (e < max_entries) issued[e] = is ? 1 : 0;
        });
    if (n >= 0 && overflow) {
        std::snprintf(msg, (size_t)msglen, "buffer too small");
        return -2;
    }
    return n;
}

// n_steps of the benchmark's rollout on every slot of handle h, in native code (the full-size parity
// tests run one handle per shard of games on its own Python thread: ctypes drops the GIL here).
// Step t = step0 + k: uniform = 0 — getMasks(0) (JNIGridnetVecClient.java:307-316), then each slot's
// masked-uniform row from its own masks (oref_policy, env id slot_base + s, player 0: the GPU's fused
// policy); uniform = 1 — oref_policy_uniform rows (slot id slot_base + s); then gameStep (:213-297).
// The last step's responses go to obs / reward / done (each may be null).
int oref_rollout_policy(void* h, int n_steps, int uniform, int n_types, uint64_t seed, uint32_t slot_base, uint32_t step0,
                        int32_t* obs, double* reward, uint8_t* done) {
    try {
        auto v = (VecClient*)h;
        const int S = v->nSlots(), HW = v->world->H * v->world->W, K = v->world->K;
        std::vector<uint8_t> masks(uniform ? 0 : (size_t)S * HW * K);
        std::vector<int32_t> acts((size_t)S * HW * 7);
        for (int k = 0; k < n_steps; k++) {
            const uint32_t t = step0 + (uint32_t)k;
            if (!uniform) v->masks(0, masks.data());
            for (int s = 0; s < S; s++) {
                int32_t* a = acts.data() + (size_t)s * HW * 7;
                if (uniform) oref_policy_uniform(HW, K, n_types, seed, slot_base + (uint32_t)s, t, a);
                else oref_policy(masks.data() + (size_t)s * HW * K, HW, K, n_types, seed, slot_base + (uint32_t)s, t, 0, a);
            }
            v->step(acts.data(), nullptr);
        }
        v->collect(obs, reward, done);
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -22;
    }
}

// ------------------------------------------------ CPU baseline: VecClient + random policy,
// `threads` std::threads each stepping a disjoint shard of games (cores = threads).
// Returns env-steps executed; *seconds = wall time of the timed region.
double oref_bench2(const char* map_path, int n_games, int steps, int threads, uint64_t seed, int burnin, int uniform);
double oref_bench(const char* map_path, int n_games, int steps, int threads, uint64_t seed, int burnin) {
    return oref_bench2(map_path, n_games, steps, threads, seed, burnin, 0);
}
double oref_bench3(const char* map_path, int n_games, int steps, int threads, uint64_t seed, int burnin, int flags);
// uniform = 1: the c2 workload (unmasked uniform rows, no masks) instead of masks + masked policy
double oref_bench2(const char* map_path, int n_games, int steps, int threads, uint64_t seed, int burnin, int uniform) {
    return oref_bench3(map_path, n_games, steps, threads, seed, burnin, uniform ? 1 : 0);
}
// flags bit 0: uniform rows (c2); bit 1: partially observable views (c5, PartiallyObservableGameState);
// bits 2-3: the UnitTypeTable version (0 = 1, VERSION_ORIGINAL; 2 = VERSION_ORIGINAL_FINETUNED)
double oref_bench3(const char* map_path, int n_games, int steps, int threads, uint64_t seed, int burnin, int flags) {
    const int uniform = flags & 1, po = (flags >> 1) & 1, uttv = ((flags >> 2) & 3) ? ((flags >> 2) & 3) : 1;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    std::chrono::steady_clock::time_point t0;
    std::vector<void*> hs((size_t)threads);
    std::vector<int> per((size_t)threads);
    for (int t = 0; t < threads; t++) {
        per[(size_t)t] = n_games / threads + (t < n_games % threads ? 1 : 0);
        std::vector<const char*> paths((size_t)per[(size_t)t] * 2, map_path);
        hs[(size_t)t] = oref_create(per[(size_t)t] * 2, 0, nullptr, 2000, po, uttv, 1, paths.data(), seed + (uint64_t)t * 1000003ULL, nullptr);
        oref_reset(hs[(size_t)t], nullptr, nullptr, nullptr, nullptr);
    }
    auto worker = [&](int t) {
        void* h = hs[(size_t)t];
        int32_t S, H, W, C, K;
        oref_dims(h, &S, &H, &W, &C, &K);
        std::vector<uint8_t> masks((size_t)S * H * W * K);
        std::vector<int32_t> acts((size_t)S * H * W * 7), obs((size_t)S * C * H * W);
        std::vector<double> rew((size_t)S);
        std::vector<uint8_t> done((size_t)S);
        for (int k = -burnin; k < steps; k++) {
            if (k == 0) {  // end of the untimed burn-in: rendezvous, then the timed region starts
                std::unique_lock<std::mutex> lk(mu);
                if (++arrived == threads) {
                    t0 = std::chrono::steady_clock::now();
                    cv.notify_all();
                } else {
                    cv.wait(lk, [&] { return arrived == threads; });
                }
            }
            if (uniform) {
                for (int s = 0; s < S; s++)
                    oref_policy_uniform(H * W, K, 7, seed, (uint32_t)(t * 100000 + s), (uint32_t)(k + burnin),
                                        acts.data() + (size_t)s * H * W * 7);
                oref_step(h, acts.data(), nullptr, obs.data(), rew.data(), done.data());
                continue;
            }
            oref_get_masks(h, 0, masks.data());
            for (int s = 0; s < S; s++)
                oref_policy(masks.data() + (size_t)s * H * W * K, H * W, K, 7, seed, (uint32_t)(t * 100000 + s / 2), (uint32_t)(k + burnin),
                            (uint32_t)(s & 1), acts.data() + (size_t)s * H * W * 7);
            oref_step(h, acts.data(), nullptr, obs.data(), rew.data(), done.data());
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    for (auto h : hs) oref_destroy(h);
    return std::chrono::duration<double>(t1 - t0).count();
}

// BASELINE config c1: JNIBotClient (tests/JNIBotClient.java:108-135) with two RandomBiasedAI sharing
// one seeded java.util.Random (Sampler.generator is a JVM static, util/Sampler.java:17), one env,
// bot-only VecClient auto-reset; `steps` timed gameSteps after `burnin` untimed ones.  Seconds.
double oref_bench_bots(const char* map_path, int steps, int64_t seed, int burnin) {
    void* h = oref_botclient_create(map_path, BOT_RANDOM_BIASED, BOT_RANDOM_BIASED, 2000, 1, 1, seed, nullptr);
    if (!h) return -1.0;
    double rew[RF_COUNT];
    uint8_t done[RF_COUNT];
    for (int k = 0; k < burnin; k++) oref_botclient_step(h, 0, rew, done);
    auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < steps; k++) oref_botclient_step(h, 0, rew, done);
    auto t1 = std::chrono::steady_clock::now();
    oref_botclient_destroy(h);
    return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
