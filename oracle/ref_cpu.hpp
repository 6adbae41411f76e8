// ============================================================================
// ref_cpu — CPU ORACLE (TEST INFRASTRUCTURE ONLY, NOT PRODUCT CODE)
//
// An object-per-unit, list-ordered, line-by-line restatement of the Java
// microRTS engine (ConnAALL/MicroRTS, snapshot 2025-02-26) for the vectorised
// env-step hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it, and only as the checker / reported baseline.
// The product (microrts_amd/libmrts.so) never links or calls it.
//
// Parity pin: the reference's own golden vectors, data/traces/**/trace_0.zip
// (280 LightRush/PortfolioAI games, UTT VERSION_ORIGINAL), replayed with the
// rule of test/microrts/TestTracesIntegrity.java:72-127 but STRICTER: the full
// PhysicalGameState is compared at every trace entry (tests/test_oracle_traces.py).
// The Java reference itself cannot run here (no JDK/JRE in the image), so there
// is no oracle/_ref build; see DESIGN.md §Oracle.
//
// Every function cites the Java file:line it restates (paths relative to the
// reference's src/).
// ============================================================================
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oref {

// java.util.Random (JDK 8 spec, 48-bit LCG).  Used for Sampler.generator
// (util/Sampler.java:17), UnitAction.r (rts/UnitAction.java:24) and
// GameState.r (rts/GameState.java:37).  The Java statics are unseeded; the
// oracle (and the GPU build) seed them per env — documented divergence.
struct JavaRandom {
    uint64_t seed = 0;
    explicit JavaRandom(int64_t s = 0) { setSeed(s); }
    void setSeed(int64_t s) { seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
    int32_t next(int bits) {
        seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int32_t)(uint32_t)(seed >> (48 - bits));
    }
    int32_t nextInt(int32_t bound) {
        if (bound <= 0) throw std::invalid_argument("bound must be positive");
        if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)next(31)) >> 31);
        int32_t bits, val;
        do {
            bits = next(31);
            val = bits % bound;
        } while ((int32_t)((uint32_t)bits - (uint32_t)val + (uint32_t)(bound - 1)) < 0);
        return val;
    }
    double nextDouble() { return (double)(((int64_t)next(26) << 27) + next(27)) * (1.0 / 9007199254740992.0); }
};

// rts/units/UnitType.java:18-110 (defaults at :23-100)
struct UnitType {
    int ID = 0;
    std::string name;
    int cost = 1, hp = 1, minDamage = 1, maxDamage = 1, attackRange = 1;
    int produceTime = 10, moveTime = 10, attackTime = 10, harvestTime = 10, returnTime = 10;
    int harvestAmount = 1, sightRadius = 4;
    bool isResource = false, isStockpile = false, canHarvest = false, canMove = true, canAttack = true;
    std::vector<UnitType*> produces;
};

// rts/units/UnitTypeTable.java:22-349
struct UnitTypeTable {
    std::vector<std::unique_ptr<UnitType>> unitTypes;
    int moveConflictResolutionStrategy = 1;
    int version = 1;
    UnitTypeTable(int version = 1, int crs = 1);
    static UnitTypeTable fromJSON(const std::string& json);  // :414-433
    UnitType* getUnitType(int ID) const;  // ArrayList.get: throws on bad index (:305-307)
    UnitType* getUnitType(const std::string& name) const;  // :314-319
    int getMaxAttackRange() const;  // :341-349
};

struct Player {  // rts/Player.java:13-56
    int ID = 0;
    int resources = 0;
};

struct Unit {  // rts/units/Unit.java:23-59
    UnitType* type = nullptr;
    int64_t ID = 0;
    int player = 0, x = 0, y = 0, resources = 0, hitpoints = 0;
};
using UnitP = std::shared_ptr<Unit>;
using PlayerP = std::shared_ptr<Player>;

struct PhysicalGameState;
struct GameState;

// rts/ResourceUsage.java:10-111
struct ResourceUsage {
    std::vector<int> positionsUsed;
    int resourcesUsed[2] = {0, 0};
    bool consistentWith(const ResourceUsage& anotherUsage, const GameState& gs) const;
    void merge(const ResourceUsage& other);
};

// rts/UnitAction.java:22-752
struct UnitAction {
    enum { TYPE_NONE = 0, TYPE_MOVE = 1, TYPE_HARVEST = 2, TYPE_RETURN = 3, TYPE_PRODUCE = 4,
           TYPE_ATTACK_LOCATION = 5, NUMBER_OF_ACTION_TYPES = 6 };
    enum { DIRECTION_NONE = -1, DIRECTION_UP = 0, DIRECTION_RIGHT = 1, DIRECTION_DOWN = 2, DIRECTION_LEFT = 3 };
    int type = TYPE_NONE;
    int parameter = DIRECTION_NONE;
    int x = 0, y = 0;
    UnitType* unitType = nullptr;
    std::unique_ptr<ResourceUsage> r_cache;

    UnitAction(int t) : type(t) {}
    UnitAction(int t, int p) : type(t), parameter(p) {}
    UnitAction(int t, int p, UnitType* ut) : type(t), parameter(p), unitType(ut) {}
    static std::shared_ptr<UnitAction> attack(int ax, int ay) {
        auto a = std::make_shared<UnitAction>(TYPE_ATTACK_LOCATION);
        a->x = ax;
        a->y = ay;
        return a;
    }
    bool equals(const UnitAction& a) const;
    const ResourceUsage& resourceUsage(const Unit& u, const PhysicalGameState& pgs);
    int ETA(const Unit& u) const;
    void execute(const UnitP& u, GameState& s);
};
using UnitActionP = std::shared_ptr<UnitAction>;

struct UnitActionAssignment {  // rts/UnitActionAssignment.java:9-21
    UnitP unit;
    UnitActionP action;
    int time;
};
using UAAP = std::shared_ptr<UnitActionAssignment>;

// The LinkedHashMap<Unit,UnitActionAssignment> of rts/GameState.java:42:
// identity keys (Unit has no equals override), insertion-ordered values,
// put() on an existing key keeps the entry's position.
struct UAMap {
    std::vector<UAAP> order;
    UAAP get(const Unit* u) const {
        for (auto& a : order)
            if (a->unit.get() == u) return a;
        return nullptr;
    }
    void put(const UnitP& u, const UAAP& a) {
        for (auto& e : order)
            if (e->unit.get() == u.get()) {
                e = a;
                return;
            }
        order.push_back(a);
    }
    void remove(const Unit* u) {
        for (size_t i = 0; i < order.size(); i++)
            if (order[i]->unit.get() == u) {
                order.erase(order.begin() + i);
                return;
            }
    }
};

// rts/PhysicalGameState.java:31-787
struct PhysicalGameState {
    int width = 8, height = 8;
    std::shared_ptr<std::vector<int>> terrain;
    std::vector<PlayerP> players;
    std::vector<UnitP> units;  // LinkedList order

    int getTerrain(int x, int y) const { return (*terrain).at((size_t)(x + y * width)); }
    Unit* getUnitAt(int x, int y) const;         // :263-270
    UnitP getUnitAtP(int x, int y) const;
    void addUnit(const UnitP& u);                // :189-201
    void removeUnit(const Unit* u);              // :208-210
    Player& getPlayer(int id) const { return *players.at((size_t)id); }
    int winner() const;                          // :334-353
    bool gameover() const;                       // :361-387
    std::shared_ptr<PhysicalGameState> clone() const;              // :392-401
    std::shared_ptr<PhysicalGameState> cloneKeepingUnits() const;  // :409-414
};
using PGSP = std::shared_ptr<PhysicalGameState>;

struct Pair {  // util/Pair — mutable fields, identity semantics
    UnitP m_a;
    UnitActionP m_b;
};
using PairP = std::shared_ptr<Pair>;

// rts/PlayerAction.java:23-419
struct PlayerAction {
    std::vector<PairP> actions;
    ResourceUsage r;
    void addUnitAction(const UnitP& u, const UnitActionP& a) { actions.push_back(std::make_shared<Pair>(Pair{u, a})); }
    bool isEmpty() const { return actions.empty(); }
    void fillWithNones(const GameState& s, int pID, int duration);  // :217-235
    bool integrityCheck() const;                                    // :244-259
    static PlayerAction fromVectorAction(const std::vector<int>& rows, int nrows, const GameState& gs,
                                         const UnitTypeTable& utt, int currentPlayer, int maxAttackRadius);
};

// rts/GameState.java:34-970
struct GameState {
    int unitCancelationCounter = 0;
    int time = 0;
    PGSP pgs;
    UAMap unitActions;
    const UnitTypeTable* utt;
    JavaRandom* cancelRandom = nullptr;  // GameState.r (:37), per-env seeded here
    JavaRandom* damageRandom = nullptr;  // UnitAction.r (UnitAction.java:24), per-env seeded here
    int errors = 0;                      // Java exceptions / prints we record instead of throwing

    GameState(PGSP p, const UnitTypeTable* u) : pgs(std::move(p)), utt(u) {}
    virtual ~GameState() = default;
    void removeUnit(const Unit* u) {  // :79-82
        pgs->removeUnit(u);
        unitActions.remove(u);
    }
    Player& getPlayer(int id) const { return pgs->getPlayer(id); }
    UAAP getActionAssignment(const Unit* u) const { return unitActions.get(u); }
    virtual bool observable(int, int) const { return true; }  // :239-241
    bool issue(PlayerAction& pa);      // :249-328
    bool issueSafe(PlayerAction& pa);  // :338-408
    bool canExecuteAnyAction(int pID) const;  // :416-423
    bool isComplete() const;           // :148-157
    std::shared_ptr<GameState> clone() const;  // :591-610 (random-stream pointers are the caller's)
    bool cycle();                      // :553-571
    bool integrityCheck() const;       // :703-719
    bool gameover() const { return pgs->gameover(); }
    int winner() const { return pgs->winner(); }
    // GameState.java:922-968; out = int32[C][H][W]
    virtual void getVectorObservation(int player, int32_t* out) const;
    virtual int numObservationPlanes() const { return 6; }
};
using GSP = std::shared_ptr<GameState>;

// rts/PartiallyObservableGameState.java:15-180
struct PartiallyObservableGameState : GameState {
    int observer;
    PartiallyObservableGameState(const GameState& gs, int a_player);  // :35-54
    bool observable(int x, int y) const override;                      // :61-71
    void getVectorObservation(int player, int32_t* out) const override;  // :82-154
    int numObservationPlanes() const override { return 8; }
};

// rts/units/Unit.java:382-522 and :531-534
std::vector<UnitActionP> getUnitActions(const Unit& u, const GameState& s, int noneDuration = 10);
bool canExecuteAction(const Unit& u, const UnitAction& ua, const GameState& gs);
// rts/UnitAction.java:675-709
UnitActionP actionFromVector(const int* action, const UnitTypeTable& utt, const Unit& u, int maxAttackRange);
// rts/UnitAction.java:711-751 — mask is the 79 (K) slots of one cell, offset 1
void getValidActionArray(const Unit& u, const GameState& gs, const UnitTypeTable& utt, uint8_t* mask,
                         int maxAttackRange, int idxOffset);
int maskSlotsPerCell(const UnitTypeTable& utt);

// Map loading (rts/PhysicalGameState.java:700-726, :765-777; rts/units/Unit.java:597-620)
struct MapTemplate {
    int width = 0, height = 0;
    std::vector<int> terrain;
    std::vector<int> playerResources;
    struct U { std::string type; int64_t id; int player, x, y, resources, hitpoints; };
    std::vector<U> units;
};
MapTemplate parseMapXML(const std::string& xml);
MapTemplate loadMapFile(const std::string& path);
PGSP instantiate(const MapTemplate& t, const UnitTypeTable& utt);

// AIs
struct AI {
    virtual ~AI() = default;
    virtual PlayerAction getAction(int player, GameState& gs) = 0;
    virtual void reset() {}
};
struct PassiveAI : AI {  // ai/PassiveAI.java:41-45
    PlayerAction getAction(int player, GameState& gs) override;
};
struct RandomBiasedAI : AI {  // ai/RandomBiasedAI.java:51-107 + util/Sampler.java:116-135
    JavaRandom* generator;
    explicit RandomBiasedAI(JavaRandom* g) : generator(g) {}
    PlayerAction getAction(int player, GameState& gs) override;
};

// ai/evaluation/SimpleSqrtEvaluationFunction3.java:24-44 (Java float / double arithmetic)
float simpleSqrtEvaluation3(int maxplayer, int minplayer, const GameState& gs);

// masks: JNIGridnetClient.getMasks (tests/JNIGridnetClient.java:210-223); out = u8[H][W][K]
void computeMasks(const GameState& gs, const UnitTypeTable& utt, int player, uint8_t* out);

// Canonical state dump shared with the GPU build (see DESIGN.md §State dump)
std::vector<int32_t> dumpState(const GameState& gs);

// rts/GameState.java:819-837 toJSON(w, true, false) and :889-915 fromJSON (Java's own unit IDs)
std::string gameStateToJSON(const GameState& gs);
GSP gameStateFromJSON(const std::string& json, const UnitTypeTable& utt);

}  // namespace oref
