// mrts_host.cpp — host runtime behind include/mrts.h: map parsing, unit-type tables, per-game
// state allocation in HBM, kernel launches, the Java-compatible host-pointer API and the
// canonical state dump.  Compiled by hipcc into microrts_amd/libmrts.so.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the entry points are taken from the RCCL library the process loaded

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/mrts.h"
#include "mrts_internal.h"
#include "mrts_json.hpp"

using namespace mrts;

namespace mrts {
size_t ldsBytes(int HW, int W, int CAP, int po);
hipError_t launchEnv(int mode, const KStatic& hs, const KStatic* ds, const KDyn& D, hipStream_t stream, hipEvent_t e0 = nullptr,
                     hipEvent_t e1 = nullptr);
bool envIterable(const KStatic& hs);
hipError_t launchPolicyUniform(int32_t* actions, int n_slots, int HW, int ntypes, int natt, uint64_t seed, uint32_t step,
                               uint32_t slot_base, hipStream_t stream);
#ifdef MRTS_LANE_AUDIT
hipError_t laneAudit(int32_t* out, int reset);
hipError_t laneAuditProbe(int32_t* scratch);
#endif
#ifdef MRTS_ABLATE
hipError_t setAblate(uint32_t v);
hipError_t getDbg(unsigned long long* out, int reset);
#endif
#ifdef MRTS_PHASE_TIMING
hipError_t phaseTimes(unsigned long long* out, int reset);
hipError_t phaseSpans(unsigned long long* out, int n);
#endif
hipError_t launchPolicy(const PolicyParams& Q, hipStream_t stream, bool* prevWritten);
hipError_t launchWiden(const uint8_t* in, int32_t* out, size_t n, hipStream_t stream);
hipError_t launchOneHot(const int32_t* obs, uint8_t* out, int n_slots, int HW, int C, int ntypes, hipStream_t stream);
hipError_t prepareLds(size_t bytes);
hipError_t launchCopyGames(int32_t* dst, const int32_t* src, const int32_t* pairs, int n, int n_dst, int n_src,
                           int CAP, int HW, hipStream_t stream);
hipError_t launchEvaluate(const KStatic& hs, const KStatic* ds, int maxplayer, float* out, hipStream_t stream);
hipError_t launchRenderRecords(const KStatic& hs, const KStatic* ds, const uint32_t* rec, int units, int n_ranks,
                               int64_t rank_stride, void* out, int out_bytes, int32_t* err, hipStream_t stream);
hipError_t launchRenderRecordsOneHot(const KStatic& hs, const KStatic* ds, const uint32_t* rec, int64_t rec_words, int n_ranks,
                                     int units, int64_t rank_stride, const int32_t* sel, const int64_t* step_off, int n_sel,
                                     uint8_t* out, int32_t* err, hipStream_t stream);
}  // namespace mrts

static thread_local std::string g_err;

namespace {

struct Fail {
    int code;
    std::string msg;
};
#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) throw Fail{-EIO, std::string(#x) + ": " + hipGetErrorString(e_)}; \
    } while (0)

// ------------------------------------------------------------------ unit type tables
// The device table (DevUtt) plus what only the host needs: names (map loading, toJSON),
// returnTime and producedBy (toJSON only; RETURN lasts moveTime, UnitAction.java:321-322).
struct UttInfo {
    DevUtt dev;
    std::vector<std::string> names;
    std::vector<int> returnT;
    std::vector<std::vector<int>> producedBy;
    int typeOf(const std::string& n) const {
        for (size_t t = 0; t < names.size(); t++)
            if (names[t] == n) return (int)t;
        return -1;
    }
};

static const char* kTypeNames[7] = {"Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"};

// the reward functions' type-name tests as flag bits; K and the attack radius from the table
static void finishUtt(UttInfo& I) {
    DevUtt& u = I.dev;
    for (int t = 0; t < u.ntypes; t++) {
        const std::string& n = I.names[(size_t)t];
        if (n == "Resource") u.flags[t] |= N_RESOURCE;
        if (n == "Base") u.flags[t] |= N_BASE | N_BUILDING;
        if (n == "Barracks") u.flags[t] |= N_BUILDING;
        if (n == "Worker") u.flags[t] |= N_WORKER;
        if (n == "Light" || n == "Heavy" || n == "Ranged") u.flags[t] |= N_COMBAT;
    }
    int maxRange = 0;  // UnitTypeTable.getMaxAttackRange (:341-349)
    for (int t = 0; t < u.ntypes; t++) maxRange = std::max(maxRange, u.range[t]);
    u.maxAttackRadius = 2 * maxRange + 1;
    u.K = 1 + 6 + 4 + 4 + 4 + 4 + u.ntypes + u.maxAttackRadius * u.maxAttackRadius;
    u.mtAttack1 = u.mtAttackFar = u.mtHarvest = u.mtMove = u.mtResource = u.mtStockpile = 0;
    uint64_t prod = 0;
    for (int t = 0; t < u.ntypes; t++) {  // the mask tables (Game::maskTables)
        const uint32_t f = u.flags[t], b = 1u << t;
        if ((f & F_ATTACK) && u.range[t] == 1) u.mtAttack1 |= b;
        if ((f & F_ATTACK) && u.range[t] > 1) u.mtAttackFar |= b;
        if (f & F_HARVEST) u.mtHarvest |= b;
        if (f & F_MOVE) u.mtMove |= b;
        if (f & F_RESOURCE) u.mtResource |= b;
        if (f & F_STOCKPILE) u.mtStockpile |= b;
        for (int i = 0; i < u.nprod[t]; i++) prod |= (uint64_t)1 << (8 * t + u.prod[t][i]);
    }
    u.mtProdLo = (uint32_t)prod;
    u.mtProdHi = (uint32_t)(prod >> 32);
    u.maxSight = 0;
    for (int t = 0; t < u.ntypes; t++) {  // integer floor(sqrt(r^2 - dy^2)): the cells dx^2 + dy^2 <= r^2
        const int r = u.sight[t];
        u.maxSight = std::max(u.maxSight, r);
        u.diskLo[t] = u.diskHi[t] = 0;
        if (r > 15) continue;  // painted with the sqrt form
        for (int dy = 0; dy <= r; dy++) {
            int w = 0;
            while ((w + 1) * (w + 1) + dy * dy <= r * r) w++;
            if (dy < 8) u.diskLo[t] |= (uint32_t)w << (4 * dy);
            else u.diskHi[t] |= (uint32_t)w << (4 * (dy - 8));
        }
    }
}

// new UnitTypeTable(version, crs) — reference src/rts/units/UnitTypeTable.java:104-289
UttInfo makeUtt(int version, int crs) {
    if (version < 1 || version > 3) throw Fail{-EINVAL, "utt_version must be 1, 2 or 3"};
    if (crs < 1 || crs > 3) throw Fail{-EINVAL, "conflict_policy must be 1, 2 or 3"};
    DevUtt u;
    std::memset(&u, 0, sizeof(u));
    u.ntypes = 7;
    for (int t = 0; t < 7; t++) {  // UnitType defaults (rts/units/UnitType.java:33-100)
        u.cost[t] = 1;
        u.hp[t] = 1;
        u.minD[t] = u.maxD[t] = 1;
        u.range[t] = 1;
        u.produceT[t] = u.moveT[t] = u.attackT[t] = u.harvestT[t] = 10;
        u.harvestAmt[t] = 1;
        u.sight[t] = 4;
        u.flags[t] = F_MOVE | F_ATTACK;
    }
    const bool v1 = version == 1, v2 = version == 2, v3 = version == 3;
    // Resource
    u.flags[0] = F_RESOURCE;
    u.sight[0] = 0;
    // Base
    u.cost[1] = 10; u.hp[1] = 10;
    if (v1) u.produceT[1] = 250;
    else if (v2) u.produceT[1] = 200;
    u.flags[1] = F_STOCKPILE;
    u.sight[1] = 5;
    // Barracks
    u.cost[2] = 5; u.hp[2] = 4;
    u.produceT[2] = v1 ? 200 : 100;
    u.flags[2] = 0;
    u.sight[2] = 3;
    // Worker
    u.cost[3] = 1; u.hp[3] = 1;
    if (v3) { u.minD[3] = 0; u.maxD[3] = 2; }
    u.range[3] = 1; u.produceT[3] = 50; u.moveT[3] = 10; u.attackT[3] = 5; u.harvestT[3] = 20;
    u.flags[3] = F_HARVEST | F_MOVE | F_ATTACK;
    u.sight[3] = 3;
    // Light
    u.cost[4] = 2; u.hp[4] = 4;
    if (v3) { u.minD[4] = 1; u.maxD[4] = 3; } else { u.minD[4] = u.maxD[4] = 2; }
    u.produceT[4] = 80; u.moveT[4] = 8; u.attackT[4] = 5;
    u.flags[4] = F_MOVE | F_ATTACK;
    u.sight[4] = 2;
    // Heavy
    if (v3) { u.minD[5] = 0; u.maxD[5] = 6; } else { u.minD[5] = u.maxD[5] = 4; }
    u.produceT[5] = 120;
    if (v1) { u.moveT[5] = 12; u.hp[5] = 4; u.cost[5] = 2; } else { u.moveT[5] = 10; u.hp[5] = 8; u.cost[5] = 3; }
    u.attackT[5] = 5;
    u.flags[5] = F_MOVE | F_ATTACK;
    u.sight[5] = 2;
    // Ranged
    u.cost[6] = 2; u.hp[6] = 1;
    if (v3) { u.minD[6] = 1; u.maxD[6] = 2; }
    u.range[6] = 3; u.produceT[6] = 100; u.moveT[6] = 10; u.attackT[6] = 5;
    u.flags[6] = F_MOVE | F_ATTACK;
    u.sight[6] = 3;
    // produces lists, in declaration order (:283-288)
    u.nprod[1] = 1; u.prod[1][0] = 3;
    u.nprod[2] = 3; u.prod[2][0] = 4; u.prod[2][1] = 5; u.prod[2][2] = 6;
    u.nprod[3] = 2; u.prod[3][0] = 1; u.prod[3][1] = 2;
    u.crs = crs;
    UttInfo I;
    I.dev = u;
    I.names.assign(kTypeNames, kTypeNames + 7);
    I.returnT.assign(7, 10);
    // producedBy in the order of the produces() calls (:283-288): type order here
    I.producedBy.assign(7, {});
    for (int t = 0; t < 7; t++)
        for (int i = 0; i < u.nprod[t]; i++) I.producedBy[(size_t)u.prod[t][i]].push_back(t);
    finishUtt(I);
    return I;
}

// UnitTypeTable.fromJSON (:414-433) + UnitType.createStub / updateFromJSON
// (UnitType.java:156-161, 217-248), including its quirks: harvestTime is read from "produceTime",
// returnTime is not read, and absent members take updateFromJSON's defaults (harvestAmount and sightRadius default to 10,
// canMove / canAttack to false).  Limits of this build: <= 8 types, type IDs equal to their list
// positions, <= 4 produced types, attack range <= 3 (K <= 80 mask slots: an idle unit's mask is
// parked as 80 bits in its free assignment words), hp in int16, positive durations; every produced /
// producedBy name must exist.
UttInfo uttFromJson(const std::string& text) {
    mjson::Value o;
    try {
        o = mjson::parse(text);
    } catch (const std::exception& e) {
        throw Fail{-EINVAL, std::string("utt_json: ") + e.what()};
    }
    try {
        if (o.kind != mjson::Value::OBJ) throw Fail{-EINVAL, "utt_json: not an object"};
        const int crs = o.getInt("moveConflictResolutionStrategy", 1);
        if (crs < 1 || crs > 3) throw Fail{-ENOTSUP, "utt_json: moveConflictResolutionStrategy must be 1, 2 or 3"};
        const mjson::Value& a = o.at("unitTypes");
        if (a.kind != mjson::Value::ARR) throw Fail{-EINVAL, "utt_json: unitTypes is not an array"};
        const int n = (int)a.arr.size();
        if (n < 1 || n > MAX_TYPES) throw Fail{-ENOTSUP, "utt_json: 1..8 unit types supported"};
        UttInfo I;
        DevUtt& u = I.dev;
        std::memset(&u, 0, sizeof(u));
        u.ntypes = n;
        u.crs = crs;
        for (int t = 0; t < n; t++) {  // createStub: ID and name
            const mjson::Value& ut = a.arr[(size_t)t];
            if (ut.getInt("ID", -1) != t) throw Fail{-ENOTSUP, "utt_json: type IDs must equal their list positions"};
            I.names.push_back(ut.getString("name", ""));
        }
        I.returnT.assign((size_t)n, 10);
        I.producedBy.assign((size_t)n, {});
        auto lookup = [&](const mjson::Value& v) {
            if (v.kind != mjson::Value::STR) throw Fail{-EINVAL, "utt_json: type names must be strings"};
            const int k = I.typeOf(v.s);
            if (k < 0) throw Fail{-EINVAL, "utt_json: unknown unit type " + v.s};
            return k;
        };
        for (int t = 0; t < n; t++) {  // updateFromJSON
            const mjson::Value& ut = a.arr[(size_t)t];
            u.cost[t] = ut.getInt("cost", 1);
            u.hp[t] = ut.getInt("hp", 1);
            u.minD[t] = ut.getInt("minDamage", 1);
            u.maxD[t] = ut.getInt("maxDamage", 1);
            u.range[t] = ut.getInt("attackRange", 1);
            u.produceT[t] = ut.getInt("produceTime", 10);
            u.moveT[t] = ut.getInt("moveTime", 10);
            u.attackT[t] = ut.getInt("attackTime", 10);
            u.harvestT[t] = ut.getInt("produceTime", 10);  // sic (UnitType.java:227)
            u.harvestAmt[t] = ut.getInt("harvestAmount", 10);
            u.sight[t] = ut.getInt("sightRadius", 10);
            uint32_t f = 0;
            if (ut.getBool("isResource", false)) f |= F_RESOURCE;
            if (ut.getBool("isStockpile", false)) f |= F_STOCKPILE;
            if (ut.getBool("canHarvest", false)) f |= F_HARVEST;
            if (ut.getBool("canMove", false)) f |= F_MOVE;
            if (ut.getBool("canAttack", false)) f |= F_ATTACK;
            u.flags[t] = f;
            const mjson::Value& pr = ut.at("produces");
            if (pr.kind != mjson::Value::ARR || pr.arr.size() > (size_t)MAX_PRODUCES)
                throw Fail{-ENOTSUP, "utt_json: at most 4 produced types per type"};
            u.nprod[t] = (int)pr.arr.size();
            for (size_t i = 0; i < pr.arr.size(); i++) u.prod[t][i] = lookup(pr.arr[i]);
            const mjson::Value& pb = ut.at("producedBy");
            if (pb.kind != mjson::Value::ARR) throw Fail{-EINVAL, "utt_json: producedBy is not an array"};
            for (auto& v : pb.arr) I.producedBy[(size_t)t].push_back(lookup(v));
            if (u.hp[t] < 1 || u.hp[t] > 32767 || u.cost[t] < 0 || u.cost[t] > 32767 || u.minD[t] < 0 ||
                u.maxD[t] < u.minD[t] || u.maxD[t] > 32767 || u.range[t] < 1 || u.range[t] > 3 ||
                u.produceT[t] < 1 || u.moveT[t] < 1 || u.attackT[t] < 1 || u.harvestT[t] < 1 ||
                u.harvestAmt[t] < 0 || u.harvestAmt[t] > 32767 || u.sight[t] < 0 || u.sight[t] > 64)
                throw Fail{-ENOTSUP, "utt_json: a value of type " + I.names[(size_t)t] + " is outside this build's limits"};
        }
        finishUtt(I);
        return I;
    } catch (const std::runtime_error& e) {
        throw Fail{-EINVAL, std::string("utt_json: ") + e.what()};
    }
}

// UnitTypeTable.toJSON (:372-383) + UnitType.toJSON (UnitType.java:299-343), byte for byte
std::string uttToJson(const UttInfo& I) {
    const DevUtt& u = I.dev;
    auto b = [](bool v) { return v ? "true" : "false"; };
    std::ostringstream w;
    w << "{\"moveConflictResolutionStrategy\":" << u.crs << ",\"unitTypes\":[";
    for (int t = 0; t < u.ntypes; t++) {
        if (t) w << ", ";
        const uint32_t f = u.flags[t];
        w << "{\"ID\":" << t << ", \"name\":\"" << I.names[(size_t)t] << "\", \"cost\":" << u.cost[t] << ", \"hp\":" << u.hp[t]
          << ", \"minDamage\":" << u.minD[t] << ", \"maxDamage\":" << u.maxD[t] << ", \"attackRange\":" << u.range[t]
          << ", \"produceTime\":" << u.produceT[t] << ", \"moveTime\":" << u.moveT[t] << ", \"attackTime\":" << u.attackT[t]
          << ", \"harvestTime\":" << u.harvestT[t] << ", \"returnTime\":" << I.returnT[(size_t)t]
          << ", \"harvestAmount\":" << u.harvestAmt[t] << ", \"sightRadius\":" << u.sight[t]
          << ", \"isResource\":" << b(f & F_RESOURCE) << ", \"isStockpile\":" << b(f & F_STOCKPILE)
          << ", \"canHarvest\":" << b(f & F_HARVEST) << ", \"canMove\":" << b(f & F_MOVE)
          << ", \"canAttack\":" << b(f & F_ATTACK) << ", \"produces\":[";
        for (int i = 0; i < u.nprod[t]; i++) w << (i ? ", " : "") << "\"" << I.names[(size_t)u.prod[t][i]] << "\"";
        w << "], \"producedBy\":[";
        for (size_t i = 0; i < I.producedBy[(size_t)t].size(); i++)
            w << (i ? ", " : "") << "\"" << I.names[(size_t)I.producedBy[(size_t)t][i]] << "\"";
        w << "]}";
    }
    w << "]}";
    return w.str();
}

// ------------------------------------------------------------------ XML map reader
// rts/PhysicalGameState.java:700-726 (fromXML), :765-777 + :577-607 (terrain, raw or A/B RLE),
// rts/units/Unit.java:597-620 (unit attributes).
struct MapDef {
    int W = 0, H = 0;
    std::vector<uint8_t> terrain;
    int res[2] = {0, 0};
    struct U { int type, player, x, y, res, hp; long long id; };
    std::vector<U> units;
};

std::string attrOf(const std::string& tag, const char* name) {
    const std::string key(name);
    size_t p = 0;
    while ((p = tag.find(key, p)) != std::string::npos) {
        const bool start = p == 0 || isspace((unsigned char)tag[p - 1]);
        size_t q = p + key.size();
        while (q < tag.size() && isspace((unsigned char)tag[q])) q++;
        if (start && q < tag.size() && tag[q] == '=') {
            q++;
            while (q < tag.size() && isspace((unsigned char)tag[q])) q++;
            if (q < tag.size() && tag[q] == '"') {
                const size_t e = tag.find('"', q + 1);
                return tag.substr(q + 1, e - q - 1);
            }
        }
        p += key.size();
    }
    throw Fail{-EINVAL, std::string("map: missing attribute ") + name};
}

int toInt(const std::string& s) {
    try {
        return std::stoi(s);
    } catch (...) {
        throw Fail{-EINVAL, "map: bad integer '" + s + "'"};
    }
}

// terrain text, raw digits or the A/B run-length form (PhysicalGameState.java:577-607,765-777)
std::vector<int> decodeTerrain(const std::string& ts, int HW) {
    std::vector<int> terr;
    if (ts.find('A') != std::string::npos || ts.find('B') != std::string::npos) {
        std::string counter;
        for (char ch : ts) {
            if (ch == 'A' || ch == 'B') {
                if (!counter.empty()) {
                    const int n = toInt(counter);
                    if (terr.empty() || n < 1 || n > HW) throw Fail{-EINVAL, "terrain: bad run length"};
                    for (int i = 0; i < n - 1; i++) terr.push_back(terr.back());
                    counter.clear();
                }
                terr.push_back(ch == 'A' ? 0 : 1);
            } else if (!isspace((unsigned char)ch)) {
                counter.push_back(ch);
            }
        }
        if (!counter.empty()) {
            const int n = toInt(counter);
            if (terr.empty() || n < 1 || n > HW) throw Fail{-EINVAL, "terrain: bad run length"};
            for (int i = 0; i < n - 1; i++) terr.push_back(terr.back());
        }
    } else {
        for (char ch : ts)
            if (!isspace((unsigned char)ch)) terr.push_back(ch - '0');
    }
    if ((int)terr.size() < HW) throw Fail{-EINVAL, "terrain too short"};
    return terr;
}

MapDef parseMap(const std::string& path, const UttInfo& utt) {
    std::ifstream f(path);
    if (!f) throw Fail{-ENOENT, "cannot open map " + path};
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string x = ss.str();
    MapDef m;
    size_t p = x.find("<rts.PhysicalGameState");
    if (p == std::string::npos) throw Fail{-EINVAL, "map: no rts.PhysicalGameState in " + path};
    size_t e = x.find('>', p);
    const std::string root = x.substr(p, e - p);
    m.W = toInt(attrOf(root, "width"));
    m.H = toInt(attrOf(root, "height"));
    if (m.W <= 0 || m.H <= 0 || m.W > 250 || m.H > 250) throw Fail{-EINVAL, "map: unsupported size"};
    const size_t t0 = x.find("<terrain>", e), t1 = x.find("</terrain>", t0);
    if (t0 == std::string::npos || t1 == std::string::npos) throw Fail{-EINVAL, "map: no terrain"};
    const std::string ts = x.substr(t0 + 9, t1 - t0 - 9);
    const int HW = m.W * m.H;
    const std::vector<int> terr = decodeTerrain(ts, HW);
    m.terrain.resize((size_t)HW);
    for (int i = 0; i < HW; i++) m.terrain[(size_t)i] = terr[(size_t)i] != 0;
    const size_t end = x.find("</rts.PhysicalGameState>", t1);
    size_t q = t1;
    int np = 0;
    while (true) {
        const size_t a = x.find("<rts.Player", q);
        if (a == std::string::npos || a > end) break;
        const size_t b = x.find('>', a);
        const std::string pt = x.substr(a, b - a);
        const int id = toInt(attrOf(pt, "ID"));
        if (id != np || np >= 2) throw Fail{-EINVAL, "map: players must be 0 and 1 in order"};
        m.res[np++] = toInt(attrOf(pt, "resources"));
        q = b;
    }
    if (np != 2) throw Fail{-EINVAL, "map: need exactly 2 players"};
    q = t1;
    std::vector<long long> ids;
    std::vector<uint8_t> occ((size_t)HW, 0);
    while (true) {
        const size_t a = x.find("<rts.units.Unit ", q);
        if (a == std::string::npos || a > end) break;
        const size_t b = x.find('>', a);
        const std::string ut = x.substr(a, b - a);
        MapDef::U u;
        const std::string tn = attrOf(ut, "type");
        u.type = utt.typeOf(tn);  // utt.getUnitType(name) (Unit.java:610)
        if (u.type < 0) throw Fail{-EINVAL, "map: unknown unit type " + tn};
        u.id = std::stoll(attrOf(ut, "ID"));
        u.player = toInt(attrOf(ut, "player"));
        u.x = toInt(attrOf(ut, "x"));
        u.y = toInt(attrOf(ut, "y"));
        u.res = toInt(attrOf(ut, "resources"));
        u.hp = toInt(attrOf(ut, "hitpoints"));
        if (u.player < -1 || u.player > 1) throw Fail{-EINVAL, "map: unit player out of range"};
        if (u.x < 0 || u.y < 0 || u.x >= m.W || u.y >= m.H) throw Fail{-EINVAL, "map: unit off the map"};
        if (u.res < -32768 || u.res > 32767 || u.hp < -32768 || u.hp > 32767) throw Fail{-EINVAL, "map: value exceeds int16"};
        if (std::find(ids.begin(), ids.end(), u.id) != ids.end()) throw Fail{-EINVAL, "map: repeated unit ID"};
        if (occ[(size_t)(u.y * m.W + u.x)]) throw Fail{-EINVAL, "map: two units in one position"};  // addUnit :192
        occ[(size_t)(u.y * m.W + u.x)] = 1;
        ids.push_back(u.id);
        m.units.push_back(u);
        q = b;
    }
    return m;
}

}  // namespace

struct mrts_env {
    int device = 0;
    hipStream_t stream = nullptr;
    int H = 0, W = 0, HW = 0, CAP = 0, C = 6, K = 79;
    int nSlots = 0, nGames = 0, nSpGames = 0, maxSteps = 0, partialObs = 0;
    int forwardModel = 0;  // games advance through mrts_playout* only (GT_PLAYOUT)
    int maxUnits = 0;      // live-unit bound (H*W unless mrts_config.max_units)
    uint32_t slotIdBase = 0;
    DevUtt utt;
    UttInfo uttInfo;
    std::vector<int> tmplOffHost;
    uint32_t cfgHash = 0;  // game kinds, map templates, max_steps, reward kinds, PO (checkpoint compatibility)
    int32_t* d_state = nullptr;
    int32_t* d_tmpl = nullptr;
    int32_t* d_tmplOff = nullptr;
    int32_t* d_gameKind = nullptr;
    std::vector<int32_t> gameKindHost;
    // library-owned buffers for the host-pointer API
    int32_t* d_actions = nullptr;
    int32_t* d_players = nullptr;
    int32_t* d_obs = nullptr;
    double* d_reward = nullptr;
    uint8_t* d_done = nullptr;
    uint8_t* d_masks = nullptr;
    int32_t* h_obs = nullptr;
    uint8_t* h_masks = nullptr;    // mrts_get_masks_host: pinned, library-owned (Java reuses its mask array)
    int32_t* h_masks32 = nullptr;  // mrts_get_masks_i32_host
    double* h_reward = nullptr;
    uint8_t* h_done = nullptr;
    std::vector<int32_t> h_stateScratch;

    KStatic hstatic;
    KStatic* d_static = nullptr;
    // persistent-buffer observations (mrts_set_obs_delta; partially observable views): the buffer the
    // last launch wrote observations to (null after a launch that changed the state without one, or
    // after an invalidation) and the per-game render records (PO handles on delta-capable maps)
    int obsDelta = 0;
    int16_t* obs16 = nullptr;  // mrts_set_obs16: int16 copy of each observation write (full observability)
    uint8_t* obs8 = nullptr;   // the exchange's uint8 transport (mrts_set_exchange_bytes(env, 1))
    int exBytes = 2;           // bytes per value of the exchanged observation: 2 (int16) or 1 (uint8)
    int multiStep = 1;  // mrts_rollout_fused_dev may run several steps per launch (mrts_set_multi_step)
    const int32_t* lastObsPtr = nullptr;
    int32_t* d_poPrev = nullptr;
    uint32_t* d_prioTab = nullptr;  // multi-step launches: per-SIMD issue-rank table (KDyn.prio_tab)
    int32_t* d_renderErr = nullptr; // the record renders' overflow flag (mrts_render_status)
    int32_t* d_bal = nullptr;       // multi-step launches: balanced game placement (KDyn.bal)
    int obsImg = 0;                 // KDyn.obs_img: every observation value fits a byte
    bool exPending[2] = {false, false};  // exDone[b] was recorded by an earlier (eager) exchange call
    hipStream_t exLastStream = nullptr;  // the stream of the last eager exchange call (already waits for them)
    // native observation exchange (mrts_exchange_init): an RCCL communicator over this handle's ranks,
    // its own communication stream, and per send buffer the step-ready / collective-done events
    ncclComm_t exComm = nullptr;
    int exRanks = 0, exRank = 0;
    bool exLoop = false;  // mrts_exchange_init_loopback: the test transport (no RCCL), see exAllGather
    // compact observation records (mrts_set_records): units per record (0 = off), steps per launch of a
    // records rollout (0 = as many as a launch can run)
    int recUnits = 0, recSteps = 0;
    hipStream_t exStream = nullptr;
    hipEvent_t exReady[2] = {nullptr, nullptr}, exDone[2] = {nullptr, nullptr};
    // mrts_capture_begin / _end / mrts_replay: the calls enqueued in between, as one instantiated graph
    hipGraph_t capGraph = nullptr;
    hipGraphExec_t capExec = nullptr;
    int poWords = 0;
    // delta mask writes: which buffer / player the last mask write went to
    int maskDelta = 0;
    const uint8_t* lastMaskPtr = nullptr;
    int lastMaskPlayer = -1;
    uint32_t* d_source = nullptr;
    // delta policy writes: candidate set of the last source-form policy write, and where it went
    uint32_t* d_polPrev = nullptr;
    // Java row layout (mrts_step_rows*): accepted-pair scratch [n_games][n_rows][2] and host staging
    uint32_t* d_pairs = nullptr;
    int pairsRows = 0;
    int32_t* d_rowsStage = nullptr;
    size_t rowsStageInts = 0;
    int32_t* d_masks32 = nullptr;
    int32_t* d_copyPairs = nullptr;  // mrts_copy_games staging
    int copyPairsCap = 0;
    float* d_eval = nullptr;         // mrts_evaluate staging
    std::vector<int32_t> rewardKinds{RF_WINLOSS};  // a_rfs
    const int32_t* lastPolicyActions = nullptr;
    bool polValid = false;
    const int32_t* fusedActions = nullptr;  // buffer the last fused-policy step wrote (delta base), or null
    // mrts_set_rollout_events: HIP events the next native rollout records around its launches (one shot)
    hipEvent_t evStart = nullptr, evEnd = nullptr;
    mutable uint32_t launchStamp = 0;       // KDyn.fwd_stamp of the last k_env launch (never 0)
    // every step's Responses (mrts_set_step_responses): the ring and its capacity in steps; during a rollout
    // call respK = the call's next step index (each MODE_STEP launch writes its steps there and advances
    // it), -1 outside rollout calls
    double* respRew = nullptr;
    uint8_t* respDone = nullptr;
    int32_t respMax = 0;
    mutable int32_t respK = -1;
    int polParity = 0;
    // the kernels store observations and mask chunks as 16-byte vectors
    static void checkAlign(const KDyn& D) {
        if (((uintptr_t)D.obs & 15) || ((uintptr_t)D.masks & 15)) throw Fail{-EINVAL, "obs / masks buffers must be 16-byte aligned"};
        if (((uintptr_t)D.reward & 7) || ((uintptr_t)D.actions & 3) || ((uintptr_t)D.rows & 3) || ((uintptr_t)D.players & 3))
            throw Fail{-EINVAL, "misaligned buffer"};
    }
    // every launch that changes the state or writes observations; the library-owned buffer of the
    // host-pointer API is always persistent
    void prepObs(KDyn& D) {
        D.obs16 = D.obs ? obs16 : nullptr;
        D.obs8 = D.obs ? obs8 : nullptr;
        D.obs_delta = (D.obs && D.obs == lastObsPtr && (obsDelta || D.obs == d_obs)) ? 1 : 0;
        D.po_prev = D.obs ? d_poPrev : nullptr;
        D.po_words = poWords;
        lastObsPtr = D.obs;
    }
    void prepMasks(KDyn& D) {
        checkAlign(D);
        D.source = D.masks ? d_source : nullptr;
        D.mask_delta = (maskDelta && D.masks && D.masks == lastMaskPtr && D.mask_player == lastMaskPlayer) ? 1 : 0;
        if (D.masks) {
            lastMaskPtr = D.masks;
            lastMaskPlayer = D.mask_player;
        }
    }
    void buildStatic() {
        std::memset(&hstatic, 0, sizeof(hstatic));
        hstatic.utt = utt;
        hstatic.H = H;
        hstatic.W = W;
        hstatic.HW = HW;
        hstatic.CAP = CAP;
        hstatic.n_games = nGames;
        hstatic.n_sp_games = nSpGames;
        hstatic.n_rewards = (int32_t)rewardKinds.size();
        hstatic.reward_need = 0;
        for (size_t j = 0; j < rewardKinds.size(); j++) {
            const int k = rewardKinds[j];
            hstatic.reward_kinds[j] = k;
            if (k >= RF_RESOURCE_GATHER && k <= RF_PRODUCE_COMBAT_UNIT) hstatic.reward_need |= RN_COUNTS;
            if (k == RF_RESOURCE_GATHER) hstatic.reward_need |= RN_RESOURCES;
            if (k == RF_CLOSER_TO_ENEMY_BASE || k == RF_CLOSER_TO_ENEMY_UNIT) hstatic.reward_need |= RN_CLOSER;
        }
        hstatic.max_steps = maxSteps;
        hstatic.C = C;
        hstatic.partial_obs = partialObs;
        hstatic.state = d_state;
        hstatic.tmpl = d_tmpl;
        hstatic.tmpl_off = d_tmplOff;
        hstatic.game_kind = d_gameKind;
    }
    hipError_t launch(int mode, const KDyn& Din, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) const {
        KDyn D = Din;
        D.state = d_state;
        D.state_words = stateWords(CAP, HW);
        D.H = H;
        D.W = W;
        D.HW = HW;
        D.CAP = CAP;
        D.n_sp_games = nSpGames;
        D.n_rewards = hstatic.n_rewards;
        D.max_steps = hstatic.max_steps;
        D.C = hstatic.C;
        D.reward_need = hstatic.reward_need;
        D.reward_kinds4 = 0;
        for (int j = 0; j < hstatic.n_rewards; j++) D.reward_kinds4 |= (uint32_t)hstatic.reward_kinds[j] << (4 * j);
        if (++launchStamp == 0) ++launchStamp;  // H_FWD = 0 means "no forwarded rows"
        D.fwd_stamp = launchStamp;
        D.prio_tab = D.n_iter > 1 ? d_prioTab : nullptr;
        D.bal = D.n_iter > 1 ? d_bal : nullptr;
        D.obs_img = obsImg;
        if (mode == 0 /* MODE_STEP */ && respK >= 0 && respRew) {  // the call's Responses ring (RespScope)
            const size_t stride = (size_t)nSlots * hstatic.n_rewards;
            D.reward = respRew + (size_t)respK * stride;
            D.done = respDone + (size_t)respK * stride;
            D.resp_stride = (int32_t)stride;
            respK += D.n_iter > 1 ? D.n_iter : 1;
        }
        return launchEnv(mode, hstatic, d_static, D, s, e0, e1);
    }
    // a state block about to be injected: if any live unit's hp or resources leaves 0..255, the byte
    // renders (KDyn.obs_img, the uint8 exchange transport) can no longer show it — turn them off for
    // good (300 would have rendered as 44, -5 as 251)
    void noteValues(const int32_t* s) {
        const int nu = s[H_NU];
        const int32_t* A = s + H_WORDS;
        for (int i = 0; i < nu && i < CAP; i++) {
            const int hpv = A[A_HP * CAP + i], rv = A[A_RES * CAP + i];
            if (hpv < 0 || hpv > 255 || rv < 0 || rv > 255) obsImg = 0;
        }
    }
    int gameOfSlot(int slot, int* player) const {
        if (slot < 2 * nSpGames) {
            *player = slot & 1;
            return slot / 2;
        }
        *player = 0;
        return nSpGames + (slot - 2 * nSpGames);
    }
};

namespace {

int fail(const Fail& f) {
    g_err = f.msg;
    return f.code;
}

hipStream_t pickStream(mrts_env*, void* s) { return (hipStream_t)s; }  // NULL = HIP's default stream, like every HIP API

void checkFlagsAfter(mrts_env* env) {  // Java exceptions → error codes
    std::vector<uint32_t> fl((size_t)env->nSlots);
    mrts_error_flags(env, fl.data());
    uint32_t all = 0;
    for (auto f : fl) all |= f;
    if (all & (MRTS_ERR_PRODUCE_TYPE)) throw Fail{-EINVAL, "decoded produce type out of range (Java: IndexOutOfBoundsException)"};
    if (all & (MRTS_ERR_CAPACITY)) throw Fail{-ENOSPC, "unit capacity exhausted"};
    if (all & (MRTS_ERR_ADDUNIT | MRTS_ERR_MOVE_COLLISION)) throw Fail{-EFAULT, "two units in one position (Java: addUnit exception)"};
}

}  // namespace

extern "C" {

const char* mrts_last_error(void) { return g_err.c_str(); }

int mrts_create(const mrts_config* cfg, mrts_env** out) {
    mrts_env* env = nullptr;
    try {
        if (!cfg || !out) throw Fail{-EINVAL, "null argument"};
        if (cfg->n_selfplay_slots < 0 || (cfg->n_selfplay_slots & 1)) throw Fail{-EINVAL, "n_selfplay_slots must be even"};
        if (cfg->n_bot_envs < 0) throw Fail{-EINVAL, "n_bot_envs < 0"};
        const int nSlots = cfg->n_selfplay_slots + cfg->n_bot_envs;
        if (nSlots <= 0) throw Fail{-EINVAL, "no environments"};
        if (!cfg->map_paths) throw Fail{-EINVAL, "map_paths is null"};
        env = new mrts_env();
        env->device = cfg->device;
        env->uttInfo = cfg->utt_json ? uttFromJson(cfg->utt_json) : makeUtt(cfg->utt_version, cfg->conflict_policy);
        env->utt = env->uttInfo.dev;
        env->K = env->utt.K;
        env->C = cfg->partial_obs ? 8 : 6;
        env->partialObs = cfg->partial_obs;
        env->maxSteps = cfg->max_steps;
        env->nSlots = nSlots;
        env->nSpGames = cfg->n_selfplay_slots / 2;
        env->nGames = env->nSpGames + cfg->n_bot_envs;
        env->slotIdBase = (uint32_t)cfg->slot_id_base;
        env->maskDelta = cfg->mask_delta;
        if (cfg->n_rewards < 0 || cfg->n_rewards > MAX_REWARDS) throw Fail{-EINVAL, "n_rewards must be 0..8"};
        if (cfg->n_rewards > 0) {
            if (!cfg->reward_kinds) throw Fail{-EINVAL, "reward_kinds is null"};
            env->rewardKinds.assign(cfg->reward_kinds, cfg->reward_kinds + cfg->n_rewards);
            for (int k : env->rewardKinds)
                if (k < 0 || k >= RF_COUNT) throw Fail{-EINVAL, "unknown reward function"};
        }
        if (cfg->ai1_kinds && cfg->n_selfplay_slots) throw Fail{-EINVAL, "the bot-only client has no self-play slots"};
        env->forwardModel = cfg->forward_model ? 1 : 0;
        if (env->forwardModel && !cfg->ai1_kinds) throw Fail{-EINVAL, "a forward model needs ai1_kinds (player 0's playout policy)"};
        if (env->forwardModel && cfg->partial_obs) throw Fail{-EINVAL, "a forward model plays on the full state (partial_obs must be 0)"};
        env->gameKindHost.assign((size_t)env->nGames, 0);  // self-play = 0
        for (int j = 0; j < cfg->n_bot_envs; j++) {
            const int k2 = cfg->bot_kinds ? cfg->bot_kinds[j] : MRTS_BOT_PASSIVE;
            const int k1 = cfg->ai1_kinds ? cfg->ai1_kinds[j] : MRTS_BOT_PASSIVE;
            if (k1 < 0 || k1 > 1 || k2 < 0 || k2 > 1) throw Fail{-ENOTSUP, "only PassiveAI / RandomBiasedAI are native"};
            const int type = env->forwardModel ? 3 : (cfg->ai1_kinds ? 2 : 1);  // GT_PLAYOUT / BOT_VS_BOT / AGENT_VS_BOT
            env->gameKindHost[(size_t)(env->nSpGames + j)] = type | (k1 << 4) | (k2 << 8);
            // JNIGridnetClient.gameStep runs the opponent on its PartiallyObservableGameState
            // (tests/JNIGridnetClient.java:164-173).  The GPU RandomBiasedAI takes getUnitActions of an
            // owned unit from the full cell map, which equals the view's only when every cell the unit
            // can act on (its 4 neighbours, its attack disk) lies inside its own sight disk.  Every
            // built-in table satisfies that; a custom table that does not is refused, not run with
            // different action lists.
            if (cfg->partial_obs && type == 1 && k2 == MRTS_BOT_RANDOM_BIASED) {
                const DevUtt& u = env->utt;
                for (int t = 0; t < u.ntypes; t++) {
                    const bool acts = (u.flags[t] & (F_MOVE | F_ATTACK | F_HARVEST)) || u.nprod[t] > 0;
                    const int need = std::max(1, (u.flags[t] & F_ATTACK) ? u.range[t] : 1);
                    if (acts && u.sight[t] < need)
                        throw Fail{-ENOTSUP, "partial_obs + RandomBiasedAI: unit type " + env->uttInfo.names[(size_t)t] +
                                                 " has sightRadius < max(1, attackRange); its PO action list would "
                                                 "differ from the full-state one this build computes"};
                }
            }
        }
        // maps: one template per distinct path
        std::map<std::string, int> tmplIndex;
        std::vector<MapDef> maps;
        std::vector<int> gameTmpl((size_t)env->nGames);
        for (int g = 0; g < env->nGames; g++) {
            const int slot = g < env->nSpGames ? 2 * g : 2 * env->nSpGames + (g - env->nSpGames);
            const char* p = cfg->map_paths[slot];
            if (!p) throw Fail{-EINVAL, "null map path"};
            auto it = tmplIndex.find(p);
            if (it == tmplIndex.end()) {
                maps.push_back(parseMap(p, env->uttInfo));
                it = tmplIndex.emplace(p, (int)maps.size() - 1).first;
            }
            gameTmpl[(size_t)g] = it->second;
        }
        env->H = maps[0].H;
        env->W = maps[0].W;
        env->HW = env->H * env->W;
        for (auto& m : maps)
            if (m.H != env->H || m.W != env->W) throw Fail{-EINVAL, "all maps must share env 0's size (JNIGridnetVecClient.java:127-133)"};
        // capacity: one live unit per cell, plus slack for the step's births over its deaths
        // unit slots: at most one live unit per cell, plus slack for the births of a step over its
        // deaths (dead slots are compacted at the end of the step).  max_units lowers the bound on
        // live units (fewer LDS bytes per game -> more games resident per CU); a game that would
        // exceed it sets MRTS_ERR_CAPACITY instead of continuing.
        if (cfg->max_units < 0) throw Fail{-EINVAL, "max_units < 0"};
        const int maxUnits = cfg->max_units ? std::min(cfg->max_units, env->HW) : env->HW;
        env->CAP = maxUnits + std::max(64, maxUnits / 4);
        env->maxUnits = maxUnits;
        if (env->CAP > 0xFFF0) throw Fail{-EINVAL, "map too large"};
        if ((size_t)env->nSlots * env->HW >= (size_t)1 << 31) throw Fail{-EINVAL, "n_slots * H * W must be < 2^31"};
        // everything above is host-only validation (testable without a GPU); device work starts here
        HIPCHK(hipSetDevice(cfg->device));
        HIPCHK(hipStreamCreateWithFlags(&env->stream, hipStreamNonBlocking));
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, cfg->device));
        const size_t lds = ldsBytes(env->HW, env->W, env->CAP, env->partialObs);
        if (lds > 160 * 1024) throw Fail{-EINVAL, "map too large for LDS"};
        if (lds > 64 * 1024) HIPCHK(prepareLds(lds));
        for (auto& m : maps)
            if ((int)m.units.size() > maxUnits) throw Fail{-ENOSPC, "a map holds more units than max_units"};
        {  // the hp / resources range an observation plane can show: the maps' units, the table's types
            // (a unit's hp only falls; its resources fall, or rise by harvestAmount from 0).  A state
            // injected later (mrts_set_state_json, mrts_restore) can hold other values: noteValues.
            int mx = 0, mn = 0;
            for (auto& m : maps)
                for (auto& u : m.units) {
                    mx = std::max(mx, std::max(u.hp, u.res));
                    mn = std::min(mn, std::min(u.hp, u.res));
                }
            for (int t = 0; t < env->utt.ntypes; t++) mx = std::max(mx, std::max(env->utt.hp[t], env->utt.harvestAmt[t]));
            env->obsImg = (mx <= 255 && mn >= 0) ? 1 : 0;
        }
        // templates blob
        std::vector<int32_t> blob;
        std::vector<int> off;
        for (auto& m : maps) {
            off.push_back((int)blob.size());
            const int nu = (int)m.units.size();
            blob.push_back(m.H);
            blob.push_back(m.W);
            blob.push_back(m.res[0]);
            blob.push_back(m.res[1]);
            blob.push_back(nu);
            std::vector<int32_t> terr((size_t)(env->HW + 3) / 4, 0);
            std::memcpy(terr.data(), m.terrain.data(), (size_t)env->HW);
            blob.insert(blob.end(), terr.begin(), terr.end());
            for (auto& u : m.units)
                blob.push_back((int32_t)((uint32_t)u.x | ((uint32_t)u.y << 8) | ((uint32_t)u.type << 16) | ((uint32_t)(u.player + 1) << 20)));
            for (auto& u : m.units) blob.push_back(u.hp);
            for (auto& u : m.units) blob.push_back(u.res);
        }
        env->tmplOffHost.resize((size_t)env->nGames);
        for (int g = 0; g < env->nGames; g++) env->tmplOffHost[(size_t)g] = off[(size_t)gameTmpl[(size_t)g]];
        {  // what a state block does not carry but its meaning depends on: a restore must match it
            uint32_t hv = 2166136261u;
            auto mix = [&hv](const void* p, size_t n) {
                for (size_t i = 0; i < n; i++) hv = (hv ^ ((const uint8_t*)p)[i]) * 16777619u;
            };
            mix(env->gameKindHost.data(), env->gameKindHost.size() * 4);
            mix(blob.data(), blob.size() * 4);
            mix(env->tmplOffHost.data(), env->tmplOffHost.size() * 4);
            mix(&env->maxSteps, 4);
            mix(&env->partialObs, sizeof(env->partialObs));
            const int nrk = (int)env->rewardKinds.size();
            mix(&nrk, 4);
            mix(env->rewardKinds.data(), env->rewardKinds.size() * sizeof(env->rewardKinds[0]));
            env->cfgHash = hv;
        }
        const size_t sw = (size_t)stateWords(env->CAP, env->HW);
        HIPCHK(hipMalloc(&env->d_state, sw * env->nGames * 4));
        if (env->partialObs && poDeltaShape(env->H, env->W)) {  // PO render records (delta observations)
            env->poWords = poPrevWords(env->CAP, env->H, env->HW);
            HIPCHK(hipMalloc(&env->d_poPrev, (size_t)env->poWords * env->nGames * 4));
            HIPCHK(hipMemset(env->d_poPrev, 0, (size_t)env->poWords * env->nGames * 4));
        }
        HIPCHK(hipMalloc(&env->d_tmpl, blob.size() * 4));
        HIPCHK(hipMalloc(&env->d_tmplOff, (size_t)env->nGames * 4));
        HIPCHK(hipMalloc(&env->d_gameKind, (size_t)env->nGames * 4));
        HIPCHK(hipMemcpy(env->d_tmpl, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(env->d_tmplOff, env->tmplOffHost.data(), (size_t)env->nGames * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(env->d_gameKind, env->gameKindHost.data(), (size_t)env->nGames * 4, hipMemcpyHostToDevice));
        // headers: java.util.Random seeds per game (same derivation as the CPU oracle)
        std::vector<int32_t> hdr(sw * env->nGames, 0);
        auto scramble = [](uint64_t s) { return (s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); };
        for (int g = 0; g < env->nGames; g++) {
            const int slot = g < env->nSpGames ? 2 * g : 2 * env->nSpGames + (g - env->nSpGames);
            const uint64_t es = cfg->seed + (uint64_t)(env->slotIdBase + (uint32_t)slot);
            int32_t* h = &hdr[(size_t)g * sw];
            const uint64_t rc = scramble(es ^ 0x9E3779B97F4A7C15ULL), rd = scramble(es ^ 0xC2B2AE3D27D4EB4FULL), rs = scramble(es);
            h[H_RNG_CANCEL] = (int32_t)(uint32_t)rc;
            h[H_RNG_CANCEL + 1] = (int32_t)(uint32_t)(rc >> 32);
            h[H_RNG_DAMAGE] = (int32_t)(uint32_t)rd;
            h[H_RNG_DAMAGE + 1] = (int32_t)(uint32_t)(rd >> 32);
            h[H_RNG_SAMPLER] = (int32_t)(uint32_t)rs;
            h[H_RNG_SAMPLER + 1] = (int32_t)(uint32_t)(rs >> 32);
        }
        HIPCHK(hipMemcpy(env->d_state, hdr.data(), hdr.size() * 4, hipMemcpyHostToDevice));
        // host-API buffers
        const size_t S = (size_t)nSlots;
        HIPCHK(hipMalloc(&env->d_actions, S * env->HW * 7 * 4));
        HIPCHK(hipMalloc(&env->d_players, S * 4));
        HIPCHK(hipMalloc(&env->d_obs, S * env->C * env->HW * 4));
        const size_t R = env->rewardKinds.size();
        HIPCHK(hipMalloc(&env->d_reward, S * R * 8));
        HIPCHK(hipMalloc(&env->d_done, S * R));
        HIPCHK(hipMalloc(&env->d_masks, S * env->HW * env->K));
        HIPCHK(hipHostMalloc(&env->h_obs, S * env->C * env->HW * 4, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&env->h_reward, S * R * 8, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&env->h_done, S * R, hipHostMallocDefault));
        HIPCHK(hipMemset(env->d_players, 0, S * 4));
        // the Java clients' arrays start as zeros (new double[rfs.length], JNIGridnetClientSelfPlay.java:
        // 134-135); a self-play reset leaves slots >= 2 alone, so they must not start as garbage
        HIPCHK(hipMemset(env->d_reward, 0, S * R * 8));
        HIPCHK(hipMemset(env->d_done, 0, S * R));
        // static kernel parameters → device buffer
        env->buildStatic();
        HIPCHK(hipMalloc(&env->d_static, sizeof(KStatic)));
        HIPCHK(hipMemcpy(env->d_static, &env->hstatic, sizeof(KStatic), hipMemcpyHostToDevice));
        if (envIterable(env->hstatic)) {  // entries carry a launch stamp: stale ones are ignored, zero = empty
            HIPCHK(hipMalloc(&env->d_prioTab, (size_t)PRIO_KEYS * 16 * 4));
            HIPCHK(hipMemset(env->d_prioTab, 0, (size_t)PRIO_KEYS * 16 * 4));
            HIPCHK(hipMalloc(&env->d_bal, ((size_t)BAL_COST + 2 * (size_t)env->nGames) * 4));
            // header and costs zero, the permutation the identity: a class slice no launch rewrote stays a
            // permutation of its games (balancePerm writes each XCD class's slice on its own)
            std::vector<int32_t> bal((size_t)BAL_COST + 2 * (size_t)env->nGames, 0);
            for (int g = 0; g < env->nGames; g++) bal[(size_t)BAL_COST + env->nGames + g] = g;
            HIPCHK(hipMemcpy(env->d_bal, bal.data(), bal.size() * 4, hipMemcpyHostToDevice));
        }
        // initial state = reset (the Java constructor loads the maps)
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.players = env->d_players;
        HIPCHK(env->launch(1, D, env->stream));
        HIPCHK(hipStreamSynchronize(env->stream));
        *out = env;
        return 0;
    } catch (const Fail& f) {
        if (env) mrts_destroy(env);
        return fail(f);
    } catch (const std::exception& e) {
        if (env) mrts_destroy(env);
        return fail(Fail{-EINVAL, e.what()});
    }
}

int mrts_dims(const mrts_env* env, int32_t* n_slots, int32_t* H, int32_t* W, int32_t* C, int32_t* K) {
    if (!env) return -EINVAL;
    if (n_slots) *n_slots = env->nSlots;
    if (H) *H = env->H;
    if (W) *W = env->W;
    if (C) *C = env->C;
    if (K) *K = env->K;
    return 0;
}

void* mrts_stream(mrts_env* env) { return env ? (void*)env->stream : nullptr; }

int mrts_reset_dev(mrts_env* env, const int32_t* d_players, int32_t* d_obs, double* d_reward, uint8_t* d_done,
                   uint8_t* d_masks, int32_t mask_player, void* stream) {
    try {
        HIPCHK(hipSetDevice(env->device));
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.players = d_players;
        D.obs = d_obs;
        D.reward = d_reward;
        D.done = d_done;
        D.masks = d_masks;
        D.mask_player = mask_player;
        env->prepMasks(D);
        env->prepObs(D);
        env->fusedActions = nullptr;
        HIPCHK(env->launch(1, D, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_step_dev(mrts_env* env, const int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                  uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, void* stream) {
    try {
        if (env->forwardModel) throw Fail{-EINVAL, "a forward-model handle advances through mrts_playout*"};
        if (!d_actions) throw Fail{-EINVAL, "actions is null"};
        HIPCHK(hipSetDevice(env->device));
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.actions = d_actions;
        D.players = d_players;
        D.obs = d_obs;
        D.reward = d_reward;
        D.done = d_done;
        D.masks = d_masks;
        D.mask_player = mask_player;
        env->prepMasks(D);
        env->prepObs(D);
        if (d_masks || d_actions == env->fusedActions) env->fusedActions = nullptr;
        HIPCHK(env->launch(0, D, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

namespace {
// records rollout (mrts_rollout_*_records_dev): the launch writes its steps' records into `chunk`, the
// part of the receive buffer one all-gather fills, at this rank's place ([rank][steps][games][words]):
// the chunk holds `steps` steps, and this launch's first one is step `first` of them
struct RecPlan {
    uint32_t* chunk;
    int rank;
    int steps, first;
};
void planRecords(const mrts_env* env, KDyn& D, const RecPlan* rec) {
    if (!rec) return;
    D.rec_units = env->recUnits;
    D.rec_out = rec->chunk + ((size_t)rec->rank * rec->steps + rec->first) * env->nGames * recWords(env->recUnits, env->partialObs);
}
// n_iter consecutive fused steps (next_step, next_step + 1, ...) as ONE launch when the handle runs a
// specialised full-observability self-play kernel and is in the steady fused state (the previous
// launch was a fused step on these buffers: delta masks and policy rows, forwarded action words);
// else one step.  Returns the number of steps enqueued.
int stepFused(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward, uint8_t* d_done,
              uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t next_step, int32_t n_iter, void* stream,
              hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr, const RecPlan* rec = nullptr) {
    if (!d_actions || !d_masks) throw Fail{-EINVAL, "actions and masks are required"};
    if (env->forwardModel) throw Fail{-EINVAL, "a forward-model handle advances through mrts_playout*"};
    HIPCHK(hipSetDevice(env->device));
    KDyn D;
    std::memset(&D, 0, sizeof(D));
    D.actions = d_actions;
    D.players = d_players;
    D.obs = d_obs;
    D.reward = d_reward;
    D.done = d_done;
    D.masks = d_masks;
    D.mask_player = mask_player;
    env->prepMasks(D);
    env->prepObs(D);
    D.pol_actions = d_actions;
    D.pol_seed = seed;
    D.pol_step = next_step;
    D.pol_slot_base = env->slotIdBase;
    D.pol_delta = (D.mask_delta && env->fusedActions == d_actions) ? 1 : 0;
    D.fwd_read = env->fusedActions == d_actions ? 1 : 0;  // games check H_FWD == this stamp - 1
    const bool steady = D.pol_delta && D.fwd_read && D.mask_delta && envIterable(env->hstatic);
    D.n_iter = (steady && n_iter > 1) ? n_iter : 1;
    planRecords(env, D, rec);
    HIPCHK(env->launch(0, D, pickStream(env, stream), e0, e1));
    env->fusedActions = d_actions;
    if (env->lastPolicyActions == d_actions) env->polValid = false;  // the standalone policy's delta base is stale
    return D.n_iter;
}
}  // namespace

int mrts_step_fused_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                        uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t next_step,
                        void* stream) {
    try {
        stepFused(env, d_actions, d_players, d_obs, d_reward, d_done, d_masks, mask_player, seed, next_step, 1, stream);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

namespace {
// the one-shot rollout events (mrts_set_rollout_events): recorded on the rollout's stream right
// before its first launch / right after its last, then forgotten
struct RolloutEvents {
    mrts_env* env;
    hipStream_t s;
    hipEvent_t end = nullptr;
    RolloutEvents(mrts_env* e, void* stream) : env(e), s(pickStream(e, stream)) {
        if (env->evStart) HIPCHK(hipEventRecord(env->evStart, s));
        end = env->evEnd;
        env->evStart = env->evEnd = nullptr;
    }
    void done() {
        if (end) HIPCHK(hipEventRecord(end, s));
    }
};
}  // namespace

namespace {
// a rollout call's span of the Responses ring (mrts_set_step_responses): the step launches write step k
// of the call at ring step k instead of d_reward / d_done (launch() points them at the ring; the last
// step's are ring step n_steps - 1 — no copy back, which cost a with_gather window ~5 %)
struct RespScope {
    mrts_env* env;
    RespScope(mrts_env* e, int32_t n_steps) : env(e) {
        if (!env->respRew) return;
        if (n_steps > env->respMax) throw Fail{-EINVAL, "more steps than the Responses ring holds (mrts_set_step_responses)"};
        env->respK = 0;
    }
    ~RespScope() { env->respK = -1; }
};
}  // namespace

int mrts_set_step_responses(mrts_env* env, double* d_rewards, uint8_t* d_dones, int32_t max_steps) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    if (!d_rewards != !d_dones || (d_rewards && max_steps < 1)) return fail(Fail{-EINVAL, "both rings and max_steps >= 1, or both NULL"});
    // the kernel forms a ring step's offset as a 32-bit product (it x n_slots x n_rewards)
    if (d_rewards && (uint64_t)max_steps * (uint64_t)env->nSlots * (uint64_t)env->hstatic.n_rewards >= (1ull << 32))
        return fail(Fail{-EINVAL, "the Responses ring exceeds 2^32 entries"});
    env->respRew = d_rewards;
    env->respDone = d_dones;
    env->respMax = d_rewards ? max_steps : 0;
    return 0;
}

int mrts_set_rollout_events(mrts_env* env, void* start, void* end) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    env->evStart = (hipEvent_t)start;
    env->evEnd = (hipEvent_t)end;
    return 0;
}

int mrts_rollout_fused_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                           uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t first_next_step,
                           int32_t n_steps, void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    try {
        // the timing events ride on the launches: start with the first, end re-recorded by each (the last wins)
        RespScope rs(env, n_steps);
        hipEvent_t e0 = env->evStart, e1 = env->evEnd;
        env->evStart = env->evEnd = nullptr;
        if (n_steps == 0) {
            RolloutEvents ev(env, stream);
            ev.done();
        }
        for (int32_t k = 0; k < n_steps;) {
            const int32_t n = std::min<int32_t>(n_steps - k, env->multiStep ? MRTS_MAX_ITER : 1);
            k += stepFused(env, d_actions, d_players, d_obs, d_reward, d_done, d_masks, mask_player, seed,
                           first_next_step + (uint32_t)k, n, stream, e0, e1);
            e0 = nullptr;
        }
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_set_multi_step(mrts_env* env, int32_t on) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    env->multiStep = on ? 1 : 0;
    return 0;
}

int mrts_multi_step_capable(const mrts_env* env) { return (env && env->multiStep && envIterable(env->hstatic)) ? 1 : 0; }

int mrts_step_rows_dev(mrts_env* env, const int32_t* d_rows, int32_t n_rows, const int32_t* d_players, int32_t* d_obs,
                       double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, void* stream) {
    try {
        if (env->forwardModel) throw Fail{-EINVAL, "a forward-model handle advances through mrts_playout*"};
        if (!d_rows && n_rows > 0) throw Fail{-EINVAL, "rows is null"};
        if (n_rows < 0 || (size_t)n_rows * env->nSlots * 8 >= ((size_t)1 << 31)) throw Fail{-EINVAL, "bad n_rows"};
        HIPCHK(hipSetDevice(env->device));
        if (n_rows > env->pairsRows) {
            hipStream_t s = pickStream(env, stream);
            HIPCHK(hipStreamSynchronize(s));  // the old scratch may still be in use on the stream
            (void)hipFree(env->d_pairs);
            env->d_pairs = nullptr;
            HIPCHK(hipMalloc(&env->d_pairs, (size_t)env->nGames * n_rows * 2 * 4));
            env->pairsRows = n_rows;
        }
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.rows = d_rows;
        D.n_rows = n_rows;
        D.pairs = env->d_pairs;
        D.players = d_players;
        D.obs = d_obs;
        D.reward = d_reward;
        D.done = d_done;
        D.masks = d_masks;
        D.mask_player = mask_player;
        env->prepMasks(D);
        env->prepObs(D);
        if (d_masks) env->fusedActions = nullptr;
        HIPCHK(env->launch(0, D, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_masks_i32_dev(mrts_env* env, int32_t player, int32_t* d_out, void* stream) {
    try {
        if (!d_out) throw Fail{-EINVAL, "out is null"};
        int r = mrts_get_masks_dev(env, player, env->d_masks, stream);
        if (r) return r;
        HIPCHK(launchWiden(env->d_masks, d_out, (size_t)env->nSlots * env->HW * env->K, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_onehot_features(const mrts_env* env) {
    const int base = 5 + 5 + 3 + (env->utt.ntypes + 1) + 6 + 2;
    return base + 2 * (env->C - 6);
}

int mrts_onehot_dev(mrts_env* env, const int32_t* d_obs, uint8_t* d_out, void* stream) {
    try {
        if (!d_obs || !d_out) throw Fail{-EINVAL, "null buffer"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(launchOneHot(d_obs, d_out, env->nSlots, env->HW, env->C, env->utt.ntypes, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_masks_dev(mrts_env* env, int32_t player, uint8_t* d_out, void* stream) {
    try {
        if (!d_out) throw Fail{-EINVAL, "out is null"};
        HIPCHK(hipSetDevice(env->device));
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.masks = d_out;
        D.mask_player = player;
        D.players = env->d_players;
        env->prepMasks(D);
        env->fusedActions = nullptr;
        HIPCHK(env->launch(2, D, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_policy_uniform_dev(mrts_env* env, uint64_t seed, uint32_t step, int32_t* d_actions, void* stream) {
    try {
        if (!env || !d_actions) throw Fail{-EINVAL, "null argument"};
        if ((uintptr_t)d_actions & 3) throw Fail{-EINVAL, "misaligned buffer"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(launchPolicyUniform(d_actions, env->nSlots, env->HW, env->utt.ntypes, env->K - 23 - env->utt.ntypes, seed, step,
                                   (uint32_t)env->slotIdBase, pickStream(env, stream)));
        // the tensor no longer holds what a masked policy or a fused step wrote there
        if (env->fusedActions == d_actions) env->fusedActions = nullptr;
        if (env->lastPolicyActions == d_actions) env->polValid = false;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

namespace {
// n_iter fused uniform steps (step, step + 1, ...) as ONE launch on the multi-step shapes (the rows
// are drawn in the kernel, so no steady state is needed), else one.  Returns the steps enqueued.
int stepUniform(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward, uint8_t* d_done,
                uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t step, int32_t n_iter, void* stream,
                hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr, const RecPlan* rec = nullptr) {
    if (!env || !d_actions) throw Fail{-EINVAL, "null argument"};
    if ((uintptr_t)d_actions & 3) throw Fail{-EINVAL, "misaligned buffer"};
    if (env->forwardModel) throw Fail{-EINVAL, "a forward-model handle advances through mrts_playout*"};
    HIPCHK(hipSetDevice(env->device));
    KDyn D;
    std::memset(&D, 0, sizeof(D));
    D.actions = d_actions;
    D.players = d_players;
    D.obs = d_obs;
    D.reward = d_reward;
    D.done = d_done;
    D.masks = d_masks;
    D.mask_player = mask_player;
    env->prepMasks(D);
    env->prepObs(D);
    D.uni_actions = d_actions;
    D.uni_seed = seed;
    D.uni_step = step;
    D.uni_slot_base = (uint32_t)env->slotIdBase;
    // masks in a loop need the delta row sets of the previous write (kept in LDS between iterations)
    const bool loopable = envIterable(env->hstatic) && (!d_masks || D.mask_delta);
    D.n_iter = (loopable && n_iter > 1) ? n_iter : 1;
    planRecords(env, D, rec);
    if (d_masks || env->fusedActions == d_actions) env->fusedActions = nullptr;
    if (env->lastPolicyActions == d_actions) env->polValid = false;
    HIPCHK(env->launch(0, D, pickStream(env, stream), e0, e1));
    return D.n_iter;
}
}  // namespace

int mrts_step_uniform_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                          uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed, uint32_t step, void* stream) {
    try {
        stepUniform(env, d_actions, d_players, d_obs, d_reward, d_done, d_masks, mask_player, seed, step, 1, stream);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_rollout_uniform_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs, double* d_reward,
                             uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps, int32_t fused,
                             void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    if (fused) {
        try {
            RespScope rs(env, n_steps);
            hipEvent_t e0 = env->evStart, e1 = env->evEnd;  // on the launches (see mrts_rollout_fused_dev)
            env->evStart = env->evEnd = nullptr;
            for (int32_t k = 0; k < n_steps;) {
                const int32_t n = std::min<int32_t>(n_steps - k, env->multiStep ? MRTS_MAX_ITER : 1);
                k += stepUniform(env, d_actions, d_players, d_obs, d_reward, d_done, nullptr, 0, seed, first_step + (uint32_t)k, n,
                                 stream, e0, e1);
                e0 = nullptr;
            }
            return 0;
        } catch (const Fail& f) {
            return fail(f);
        }
    }
    try {
        RespScope rs(env, n_steps);
        for (int32_t k = 0; k < n_steps; k++) {
            int r = mrts_policy_uniform_dev(env, seed, first_step + (uint32_t)k, d_actions, stream);
            if (!r) r = mrts_step_dev(env, d_actions, d_players, d_obs, d_reward, d_done, nullptr, 0, stream);
            if (r) return r;
        }
    } catch (const Fail& f) {
        return fail(f);
    }
    return 0;
}

}  // extern "C" (the exchange loop below is a template)
namespace {
// RCCL entry points, resolved by dlopen / dlsym from the library path the caller names (the one its
// process group already loaded: one RCCL instance per process)
struct Rccl {
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
void loadRccl(const char* path) {
    if (g_rccl.allGather) return;
    void* h = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) throw Fail{-ENOENT, std::string("cannot load RCCL: ") + dlerror()};
    Rccl r;
    r.getUniqueId = (decltype(r.getUniqueId))dlsym(h, "ncclGetUniqueId");
    r.commInitRank = (decltype(r.commInitRank))dlsym(h, "ncclCommInitRank");
    r.allGather = (decltype(r.allGather))dlsym(h, "ncclAllGather");
    r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
    r.errorString = (decltype(r.errorString))dlsym(h, "ncclGetErrorString");
    if (!r.getUniqueId || !r.commInitRank || !r.allGather || !r.commDestroy || !r.errorString)
        throw Fail{-ENOENT, "the RCCL library lacks an entry point"};
    g_rccl = r;
}
void ncclChk(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Fail{-EIO, std::string(what) + ": " + g_rccl.errorString(r)};
}
bool exInited(const mrts_env* env) { return env->exComm != nullptr || env->exLoop; }
// The all-gather of `bytes` per rank from send into recv ([ranks][bytes]) on the exchange stream.  The
// loopback test transport (mrts_exchange_init_loopback) stands in for ranks - 1 peers whose data differ
// from this rank's: the bytes are blocks of `rows` rows of `rowBytes` (a step's games, or
// slots), and peer r's place receives this rank's blocks with the rows rotated by r - rank — peer r's row
// i is this rank's row (i + r - rank) mod rows — while this rank's own place is left as written.  So a
// wrong rank offset, stride or chunk base, or a render that reads another rank's place, shows on one GPU
// as a rotated (wrong) observation, not as a copy of the right one.
void exAllGather(mrts_env* env, const void* send, void* recv, size_t bytes, size_t rowBytes, size_t rows) {
    if (env->exLoop) {
        const size_t blk = rowBytes * rows, nblk = blk ? bytes / blk : 0;
        if (!blk || nblk * blk != bytes) throw Fail{-EINVAL, "loopback exchange: bytes are not whole blocks"};
        for (int r = 0; r < env->exRanks; r++) {
            uint8_t* dst = (uint8_t*)recv + (size_t)r * bytes;
            if (dst == send) continue;
            const size_t d = (size_t)(((r - env->exRank) % (int)rows + (int)rows) % (int)rows);  // rotation in rows
            const uint8_t* src = (const uint8_t*)send;
            // dst rows [0, rows - d) <- src rows [d, rows); dst rows [rows - d, rows) <- src rows [0, d), every block
            if (rows - d)
                HIPCHK(hipMemcpy2DAsync(dst, blk, src + d * rowBytes, blk, (rows - d) * rowBytes, nblk, hipMemcpyDeviceToDevice,
                                        env->exStream));
            if (d)
                HIPCHK(hipMemcpy2DAsync(dst + (rows - d) * rowBytes, blk, src, blk, d * rowBytes, nblk, hipMemcpyDeviceToDevice,
                                        env->exStream));
        }
        return;
    }
    ncclChk(g_rccl.allGather(send, recv, bytes, ncclUint8, env->exComm, env->exStream), "ncclAllGather");
}
// per step: wait until the collective that last read send buffer k % 2 is done, run the step (it
// writes its int16 observation there), then all-gather it into recv on the exchange stream
template <class StepFn>
void exchangeLoop(mrts_env* env, int32_t n_steps, const int32_t* d_obs, int16_t* d_send0, int16_t* d_send1, int16_t* d_recv,
                  void* stream, StepFn step) {
    if (!exInited(env)) throw Fail{-EINVAL, "mrts_exchange_init first"};
    // the step kernel writes the transport as part of its observation write (prepObs)
    if (!d_obs) throw Fail{-EINVAL, "the exchange needs an observation buffer (d_obs)"};
    if (env->exBytes == 1 && !env->obsImg) throw Fail{-ENOTSUP, "uint8 exchange: an observation value no longer fits a byte"};
    if (env->partialObs) throw Fail{-ENOTSUP, "the int16 transport is written for full observability only"};
    if (!d_send0 || !d_send1 || !d_recv || (((uintptr_t)d_send0 | (uintptr_t)d_send1) & 7))
        throw Fail{-EINVAL, "send buffers must be 8-byte aligned, recv non-null"};
    HIPCHK(hipSetDevice(env->device));
    hipStream_t s = pickStream(env, stream);
    int16_t* send[2] = {d_send0, d_send1};
    const bool u8 = env->exBytes == 1;  // the buffers then hold uint8 values (mrts_set_exchange_bytes)
    const size_t bytes = (size_t)env->nSlots * env->C * env->HW * (u8 ? 1 : 2);
    bool pending[2] = {false, false};
    int16_t* const saved = env->obs16;
    // a send buffer an earlier call's collective may still read: that call ended with its own stream
    // waiting for its collectives, so only a call on another stream waits for them here.  Not while
    // capturing: the events were recorded outside the capture, so the graph could not hold
    // that dependency — whoever replays a captured exchange orders it after the eager calls itself.
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(s, &cst));
    const bool capturing = cst != hipStreamCaptureStatusNone;
    for (int b = 0; b < 2; b++)
        if (env->exPending[b] && !capturing && s != env->exLastStream) HIPCHK(hipStreamWaitEvent(s, env->exDone[b], 0));
    try {
        for (int32_t k = 0; k < n_steps; k++) {
            const int b = k & 1;
            if (pending[b]) HIPCHK(hipStreamWaitEvent(s, env->exDone[b], 0));
            if (u8) env->obs8 = (uint8_t*)send[b];
            else env->obs16 = send[b];
            step(k);
            HIPCHK(hipEventRecord(env->exReady[b], s));
            HIPCHK(hipStreamWaitEvent(env->exStream, env->exReady[b], 0));
            exAllGather(env, send[b], d_recv, bytes, bytes / env->nSlots, env->nSlots);  // (loopback: rotate slots)
            HIPCHK(hipEventRecord(env->exDone[b], env->exStream));
            pending[b] = true;
            if (!capturing) env->exPending[b] = true;  // (a captured record is the graph's, not an eager event)
        }
        for (int b = 0; b < 2; b++)  // the caller's stream covers every collective of the call
            if (pending[b]) HIPCHK(hipStreamWaitEvent(s, env->exDone[b], 0));
        if (!capturing && n_steps > 0) env->exLastStream = s;
    } catch (...) {
        env->obs16 = saved;
        env->obs8 = nullptr;
        throw;
    }
    env->obs16 = saved;
    env->obs8 = nullptr;
}
// The compact-record exchange (mrts_rollout_*_records_dev): every step's game records go into the receive
// buffer at this rank's place of its chunk; after each chunk, an in-place all-gather of it on the exchange
// stream (it overlaps the next chunk's launch).  step(k, n, plan) enqueues up to n steps from step k and
// returns how many it enqueued.  The chunk schedule depends on the call's arguments and the handle's
// configuration only — never on whether this handle is in the steady fused state: a chunk
// covers min(steps left, steps per launch) steps on every rank, and a handle that is not steady runs the
// chunk's first step alone and the rest as a second launch into the same chunk, so every rank issues the
// same all-gathers with the same sizes and the same step layout.
template <class StepFn>
void recordsLoop(mrts_env* env, int32_t n_steps, const int32_t* d_obs, uint32_t* d_recv, int64_t* offsets, void* stream,
                 StepFn step) {
    if (!exInited(env)) throw Fail{-EINVAL, "mrts_exchange_init first"};
    if (!env->recUnits) throw Fail{-EINVAL, "mrts_set_records first"};
    // a partially observable record holds the views' snapshot, which the step takes as part of its
    // observation write (an auto-reset's fresh snapshot too): without d_obs it would be empty
    if (env->partialObs && !d_obs) throw Fail{-EINVAL, "partially observable records need an observation buffer (d_obs)"};
    if (!d_recv || ((uintptr_t)d_recv & 15)) throw Fail{-EINVAL, "the receive buffer must be non-null and 16-byte aligned"};
    // (partially observable records carry hp as int8: the kernel flags a value outside the record's range)
    if (!env->obsImg && !env->partialObs) throw Fail{-ENOTSUP, "records: an observation value no longer fits a byte"};
    HIPCHK(hipSetDevice(env->device));
    hipStream_t s = pickStream(env, stream);
    const size_t per = (size_t)env->nGames * recWords(env->recUnits, env->partialObs);  // words per rank and step
    size_t base = 0;                                                   // words of d_recv filled so far
    bool any = false;
    const int32_t cap = env->multiStep ? (env->recSteps > 0 ? env->recSteps : MRTS_MAX_ITER) : 1;
    for (int32_t k = 0; k < n_steps;) {
        const int32_t n = std::min<int32_t>(n_steps - k, cap);  // the chunk's steps, the same on every rank
        for (int32_t j = 0; j < n;) {
            const RecPlan rp{d_recv + base, env->exRank, n, j};
            j += step(k + j, n - j, &rp);
        }
        HIPCHK(hipEventRecord(env->exReady[0], s));
        HIPCHK(hipStreamWaitEvent(env->exStream, env->exReady[0], 0));
        const size_t words = (size_t)n * per;
        exAllGather(env, d_recv + base + (size_t)env->exRank * words, d_recv + base, words * 4,
                    4 * (size_t)recWords(env->recUnits, env->partialObs), (size_t)env->nGames);  // (loopback: rotate games)
        if (offsets)
            for (int32_t j = 0; j < n; j++) {
                offsets[2 * (size_t)(k + j)] = (int64_t)(base + (size_t)j * per);
                offsets[2 * (size_t)(k + j) + 1] = (int64_t)words;
            }
        base += (size_t)env->exRanks * words;
        k += n;
        any = true;
    }
    if (any) {  // the caller's stream covers every collective of the call
        HIPCHK(hipEventRecord(env->exDone[0], env->exStream));
        HIPCHK(hipStreamWaitEvent(s, env->exDone[0], 0));
    }
}
}  // namespace
extern "C" {

int mrts_set_records(mrts_env* env, int32_t units_per_record, int32_t steps_per_launch) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    if (units_per_record == 0) {
        env->recUnits = 0;
        return 0;
    }
    if (units_per_record < 1 || units_per_record > 0xFFFF || steps_per_launch < 0)
        return fail(Fail{-EINVAL, "units per record 1..65535, steps per launch >= 0"});
    if (env->nSpGames != env->nGames || (env->HW & 3))
        return fail(Fail{-ENOTSUP, "records: self-play handles, maps whose cell count is a multiple of 4"});
    if (!env->partialObs && (env->HW > 256 || env->utt.ntypes > 7 || !env->obsImg))
        return fail(Fail{-ENOTSUP, "records (full observability): maps of <= 256 cells, <= 7 unit types, every observation "
                                   "value < 256"});
    if (env->partialObs && (env->HW > 65536 || env->utt.ntypes > 15 || env->hstatic.C != 8 ||
                            4 * (size_t)(2 * env->HW + 4 * env->H * ((env->W + 31) / 32) + recWords(units_per_record, true)) >
                                64 * 1024))
        return fail(Fail{-ENOTSUP, "records (partial observability): <= 15 unit types, the receiver's render state and one "
                                   "record in 64 KB of LDS"});
    try {  // the renders' overflow flag: allocated and zeroed here, never on a render path (a lazy
           // hipMalloc there would break a stream capture, and a null-stream memset is unordered with a
           // non-blocking render stream)
        if (!env->d_renderErr) {
            HIPCHK(hipSetDevice(env->device));
            HIPCHK(hipMalloc(&env->d_renderErr, 4));
            HIPCHK(hipMemset(env->d_renderErr, 0, 4));
            HIPCHK(hipDeviceSynchronize());
        }
    } catch (const Fail& f) {
        return fail(f);
    }
    env->recUnits = units_per_record;
    env->recSteps = steps_per_launch;
    return 0;
}

int mrts_rollout_fused_records_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                   double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed,
                                   uint32_t first_next_step, int32_t n_steps, uint32_t* d_recv, int64_t* step_offsets,
                                   void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    try {
        RespScope rs(env, n_steps);
        RolloutEvents ev(env, stream);
        recordsLoop(env, n_steps, d_obs, d_recv, step_offsets, stream, [&](int32_t k, int32_t n, const RecPlan* rp) {
            return stepFused(env, d_actions, d_players, d_obs, d_reward, d_done, d_masks, mask_player, seed,
                             first_next_step + (uint32_t)k, n, stream, nullptr, nullptr, rp);
        });
        ev.done();
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_rollout_uniform_records_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                     double* d_reward, uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps,
                                     uint32_t* d_recv, int64_t* step_offsets, void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    try {
        RespScope rs(env, n_steps);
        RolloutEvents ev(env, stream);
        recordsLoop(env, n_steps, d_obs, d_recv, step_offsets, stream, [&](int32_t k, int32_t n, const RecPlan* rp) {
            return stepUniform(env, d_actions, d_players, d_obs, d_reward, d_done, nullptr, 0, seed, first_step + (uint32_t)k, n,
                               stream, nullptr, nullptr, rp);
        });
        ev.done();
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_render_records_onehot_dev(mrts_env* env, const uint32_t* d_rec, int64_t rec_words, int32_t n_ranks, int64_t rank_stride,
                                   const int32_t* d_sel, const int64_t* d_step_off, int32_t n_sel, uint8_t* d_out, void* stream) {
    try {
        if (!env || !d_rec || !d_out || (n_sel > 0 && !d_sel) || n_sel < 0 || rank_stride < 0 || rec_words < 0 || n_ranks < 1)
            throw Fail{-EINVAL, "bad argument"};
        if (!env->recUnits || !env->d_renderErr) throw Fail{-EINVAL, "mrts_set_records first"};
        if (env->partialObs) throw Fail{-ENOTSUP, "one-hot from records: full observability only"};
        if (((uintptr_t)d_out & 15) || ((uintptr_t)d_rec & 3)) throw Fail{-EINVAL, "misaligned buffer"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(launchRenderRecordsOneHot(env->hstatic, env->d_static, d_rec, rec_words, n_ranks, env->recUnits, rank_stride, d_sel,
                                         d_step_off, n_sel, d_out, env->d_renderErr, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_render_status(mrts_env* env) {
    try {
        if (!env) throw Fail{-EINVAL, "null handle"};
        if (!env->d_renderErr) return 0;
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(hipDeviceSynchronize());
        int32_t v = 0;
        HIPCHK(hipMemcpy(&v, env->d_renderErr, 4, hipMemcpyDeviceToHost));
        if (v) HIPCHK(hipMemset(env->d_renderErr, 0, 4));
        return v ? 1 : 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int32_t mrts_record_words(const mrts_env* env) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    return env->recUnits ? recWords(env->recUnits, env->partialObs) : 0;
}

int mrts_render_records_dev(mrts_env* env, const uint32_t* d_rec, int64_t rec_words, int32_t n_ranks, int64_t rank_stride,
                            void* d_out, int32_t out_bytes, void* stream) {
    try {
        if (!env || !d_rec || !d_out || n_ranks < 1 || rank_stride < 0 || rec_words < 0) throw Fail{-EINVAL, "bad argument"};
        if (!env->recUnits || !env->d_renderErr) throw Fail{-EINVAL, "mrts_set_records first"};
        if (out_bytes != 1 && out_bytes != 4) throw Fail{-EINVAL, "out_bytes: 1 (uint8) or 4 (int32)"};
        if (((uintptr_t)d_out & (out_bytes == 4 ? 15 : 3)) || ((uintptr_t)d_rec & 3)) throw Fail{-EINVAL, "misaligned buffer"};
        // every rank's records inside the buffer (the kernel reads n_games records per rank)
        const int64_t span = (int64_t)(n_ranks - 1) * rank_stride + (int64_t)env->nGames * recWords(env->recUnits, env->partialObs);
        if (span > rec_words) throw Fail{-EINVAL, "the ranks' records reach past the receive buffer (rec_words)"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(launchRenderRecords(env->hstatic, env->d_static, d_rec, env->recUnits, n_ranks, rank_stride, d_out, out_bytes,
                                   env->d_renderErr, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_capture_begin(mrts_env* env, void* stream) {
    try {
        if (!env || !stream) throw Fail{-EINVAL, "capture needs a handle and a non-default stream"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_capture_end(mrts_env* env, void* stream) {
    try {
        if (!env || !stream) throw Fail{-EINVAL, "capture needs a handle and a non-default stream"};
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamEndCapture((hipStream_t)stream, &g));
        if (env->capExec) (void)hipGraphExecDestroy(env->capExec);
        if (env->capGraph) (void)hipGraphDestroy(env->capGraph);
        env->capExec = nullptr;
        env->capGraph = g;
        HIPCHK(hipGraphInstantiate(&env->capExec, g, nullptr, nullptr, 0));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_replay(mrts_env* env, void* stream) {
    try {
        if (!env || !env->capExec) throw Fail{-EINVAL, "nothing captured"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(hipGraphLaunch(env->capExec, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_rccl_unique_id(const char* rccl_path, void* out) {
    try {
        if (!out) throw Fail{-EINVAL, "null argument"};
        loadRccl(rccl_path);
        ncclUniqueId id;
        ncclChk(g_rccl.getUniqueId(&id), "ncclGetUniqueId");
        std::memcpy(out, &id, sizeof(id));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_exchange_init(mrts_env* env, const char* rccl_path, int32_t nranks, int32_t rank, const void* unique_id) {
    try {
        if (!env || !unique_id || nranks < 1 || rank < 0 || rank >= nranks) throw Fail{-EINVAL, "bad exchange arguments"};
        if (exInited(env)) throw Fail{-EINVAL, "the exchange is already initialised"};
        loadRccl(rccl_path);
        HIPCHK(hipSetDevice(env->device));
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        ncclChk(g_rccl.commInitRank(&env->exComm, nranks, id, rank), "ncclCommInitRank");
        env->exRanks = nranks;
        env->exRank = rank;
        HIPCHK(hipStreamCreateWithFlags(&env->exStream, hipStreamNonBlocking));
        for (int b = 0; b < 2; b++) {
            HIPCHK(hipEventCreateWithFlags(&env->exReady[b], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&env->exDone[b], hipEventDisableTiming));
        }
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_exchange_init_loopback(mrts_env* env, int32_t nranks, int32_t rank) {
    try {
        if (!env || nranks < 1 || rank < 0 || rank >= nranks) throw Fail{-EINVAL, "bad exchange arguments"};
        if (exInited(env)) throw Fail{-EINVAL, "the exchange is already initialised"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(hipStreamCreateWithFlags(&env->exStream, hipStreamNonBlocking));
        for (int b = 0; b < 2; b++) {
            HIPCHK(hipEventCreateWithFlags(&env->exReady[b], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&env->exDone[b], hipEventDisableTiming));
        }
        env->exRanks = nranks;
        env->exRank = rank;
        env->exLoop = true;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_rollout_fused_exchange_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                    double* d_reward, uint8_t* d_done, uint8_t* d_masks, int32_t mask_player, uint64_t seed,
                                    uint32_t first_next_step, int32_t n_steps, int16_t* d_send0, int16_t* d_send1,
                                    int16_t* d_recv, void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    try {
        RespScope rs(env, n_steps);
        RolloutEvents ev(env, stream);
        exchangeLoop(env, n_steps, d_obs, d_send0, d_send1, d_recv, stream, [&](int32_t k) {
            stepFused(env, d_actions, d_players, d_obs, d_reward, d_done, d_masks, mask_player, seed,
                      first_next_step + (uint32_t)k, 1, stream);
        });
        ev.done();
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_rollout_uniform_exchange_dev(mrts_env* env, int32_t* d_actions, const int32_t* d_players, int32_t* d_obs,
                                      double* d_reward, uint8_t* d_done, uint64_t seed, uint32_t first_step, int32_t n_steps,
                                      int16_t* d_send0, int16_t* d_send1, int16_t* d_recv, void* stream) {
    if (!env || n_steps < 0) return fail(Fail{-EINVAL, "bad rollout arguments"});
    try {
        RespScope rs(env, n_steps);
        RolloutEvents ev(env, stream);
        exchangeLoop(env, n_steps, d_obs, d_send0, d_send1, d_recv, stream, [&](int32_t k) {
            stepUniform(env, d_actions, d_players, d_obs, d_reward, d_done, nullptr, 0, seed, first_step + (uint32_t)k, 1,
                        stream);
        });
        ev.done();
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_policy_invalidate(mrts_env* env) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    env->polValid = false;
    env->fusedActions = nullptr;
    return 0;
}

int mrts_set_obs_delta(mrts_env* env, int32_t on) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    env->obsDelta = on ? 1 : 0;
    env->lastObsPtr = nullptr;
    return 0;
}

int mrts_set_exchange_bytes(mrts_env* env, int32_t bytes_per_value) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    if (bytes_per_value == 2) {
        env->exBytes = 2;
        return 0;
    }
    if (bytes_per_value != 1) return fail(Fail{-EINVAL, "bytes per value: 1 or 2"});
    // the uint8 transport is written by the 16x16 byte-image render and the one-cell-per-lane render of
    // maps of <= 64 cells: full observability whose every value fits a byte (checked at create over the
    // maps and the unit-type table)
    if (env->partialObs || !(env->HW == 256 || env->HW <= 64) || !env->obsImg)
        return fail(Fail{-ENOTSUP, "uint8 exchange: full observability on 16x16 or <= 64-cell maps, every value < 256"});
    env->exBytes = 1;
    return 0;
}

int mrts_set_obs16(mrts_env* env, int16_t* d_obs16) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    if (d_obs16 && env->partialObs) return fail(Fail{-EINVAL, "the int16 observation copy is for full observability"});
    if ((uintptr_t)d_obs16 & 7) return fail(Fail{-EINVAL, "misaligned buffer (8 bytes)"});
    env->obs16 = d_obs16;
    return 0;
}

int mrts_obs_invalidate(mrts_env* env) {
    if (!env) return fail(Fail{-EINVAL, "null handle"});
    env->lastObsPtr = nullptr;
    return 0;
}

int mrts_set_source_output(mrts_env* env, uint32_t* d_source) {
    if (!env) return -EINVAL;
    env->d_source = d_source;
    return 0;
}

int mrts_policy_dev(mrts_env* env, const uint8_t* d_masks, const uint32_t* d_source, uint64_t seed, uint32_t step,
                    int32_t* d_actions, void* stream) {
    try {
        HIPCHK(hipSetDevice(env->device));
        PolicyParams Q;
        Q.HW = env->HW;
        Q.K = env->K;
        Q.ntypes = env->utt.ntypes;
        Q.n_slots = env->nSlots;
        Q.slot_id_base = env->slotIdBase;
        Q.step = step;
        Q.seed = seed;
        Q.masks = d_masks;
        Q.source = d_source;
        Q.actions = d_actions;
        Q.prev = nullptr;
        Q.prev_out = nullptr;
        Q.delta = 0;
        const size_t pw = (size_t)env->nSlots * maskWords(env->HW);
        if (d_source && env->maskDelta) {  // double-buffered candidate sets: read one, write the other
            if (!env->d_polPrev) HIPCHK(hipMalloc(&env->d_polPrev, 2 * pw * 4));
            Q.prev = env->d_polPrev + pw * env->polParity;
            Q.prev_out = env->d_polPrev + pw * (1 - env->polParity);
            Q.delta = (env->polValid && d_actions == env->lastPolicyActions) ? 1 : 0;
        }
        bool prevWritten = false;
        if (d_actions == env->fusedActions) env->fusedActions = nullptr;
        HIPCHK(launchPolicy(Q, pickStream(env, stream), &prevWritten));
        env->polValid = prevWritten;
        if (prevWritten) env->polParity ^= 1;
        env->lastPolicyActions = d_actions;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

static void fillResponses(mrts_env* env, mrts_responses* out) {
    const size_t S = (size_t)env->nSlots;
    HIPCHK(hipMemcpyAsync(env->h_obs, env->d_obs, S * env->C * env->HW * 4, hipMemcpyDeviceToHost, env->stream));
    const size_t R = env->rewardKinds.size();
    HIPCHK(hipMemcpyAsync(env->h_reward, env->d_reward, S * R * 8, hipMemcpyDeviceToHost, env->stream));
    HIPCHK(hipMemcpyAsync(env->h_done, env->d_done, S * R, hipMemcpyDeviceToHost, env->stream));
    HIPCHK(hipStreamSynchronize(env->stream));
    if (out) {
        out->obs = env->h_obs;
        out->reward = env->h_reward;
        out->done = env->h_done;
    }
}

int mrts_reset(mrts_env* env, const int32_t* players, mrts_responses* out) {
    try {
        HIPCHK(hipSetDevice(env->device));
        const size_t S = (size_t)env->nSlots;
        if (players) HIPCHK(hipMemcpyAsync(env->d_players, players, S * 4, hipMemcpyHostToDevice, env->stream));
        else HIPCHK(hipMemsetAsync(env->d_players, 0, S * 4, env->stream));
        int r = mrts_reset_dev(env, env->d_players, env->d_obs, env->d_reward, env->d_done, nullptr, 0, env->stream);
        if (r) return r;
        fillResponses(env, out);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_step(mrts_env* env, const int32_t* actions, const int32_t* players, mrts_responses* out) {
    try {
        if (!actions) throw Fail{-EINVAL, "actions is null"};
        HIPCHK(hipSetDevice(env->device));
        const size_t S = (size_t)env->nSlots;
        HIPCHK(hipMemcpyAsync(env->d_actions, actions, S * env->HW * 7 * 4, hipMemcpyHostToDevice, env->stream));
        if (players) HIPCHK(hipMemcpyAsync(env->d_players, players, S * 4, hipMemcpyHostToDevice, env->stream));
        else HIPCHK(hipMemsetAsync(env->d_players, 0, S * 4, env->stream));
        int r = mrts_step_dev(env, env->d_actions, env->d_players, env->d_obs, env->d_reward, env->d_done, nullptr, 0, env->stream);
        if (r) return r;
        fillResponses(env, out);
        checkFlagsAfter(env);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_step_rows(mrts_env* env, const int32_t* rows, int32_t n_rows, const int32_t* players, mrts_responses* out) {
    try {
        if (!rows && n_rows > 0) throw Fail{-EINVAL, "rows is null"};
        if (n_rows < 0) throw Fail{-EINVAL, "bad n_rows"};
        HIPCHK(hipSetDevice(env->device));
        const size_t S = (size_t)env->nSlots, n = S * (size_t)n_rows * 8;
        if (n > env->rowsStageInts) {
            HIPCHK(hipStreamSynchronize(env->stream));
            (void)hipFree(env->d_rowsStage);
            env->d_rowsStage = nullptr;
            HIPCHK(hipMalloc(&env->d_rowsStage, n * 4));
            env->rowsStageInts = n;
        }
        if (n) HIPCHK(hipMemcpyAsync(env->d_rowsStage, rows, n * 4, hipMemcpyHostToDevice, env->stream));
        if (players) HIPCHK(hipMemcpyAsync(env->d_players, players, S * 4, hipMemcpyHostToDevice, env->stream));
        else HIPCHK(hipMemsetAsync(env->d_players, 0, S * 4, env->stream));
        int r = mrts_step_rows_dev(env, env->d_rowsStage, n_rows, env->d_players, env->d_obs, env->d_reward, env->d_done,
                                   nullptr, 0, env->stream);
        if (r) return r;
        fillResponses(env, out);
        checkFlagsAfter(env);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_masks_i32(mrts_env* env, int32_t player, int32_t* out) {
    try {
        if (!out) throw Fail{-EINVAL, "out is null"};
        const size_t n = (size_t)env->nSlots * env->HW * env->K;
        if (!env->d_masks32) HIPCHK(hipMalloc(&env->d_masks32, n * 4));
        int r = mrts_get_masks_i32_dev(env, player, env->d_masks32, env->stream);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(out, env->d_masks32, n * 4, hipMemcpyDeviceToHost, env->stream));
        HIPCHK(hipStreamSynchronize(env->stream));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_masks(mrts_env* env, int32_t player, uint8_t* out) {
    try {
        if (!out) throw Fail{-EINVAL, "out is null"};
        int r = mrts_get_masks_dev(env, player, env->d_masks, env->stream);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(out, env->d_masks, (size_t)env->nSlots * env->HW * env->K, hipMemcpyDeviceToHost, env->stream));
        HIPCHK(hipStreamSynchronize(env->stream));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

// getMasks into a library-owned pinned buffer (valid until the next call on the handle, like the Java
// client's reused mask array, JNIGridnetClient.java:211-215): the D2H copy runs at pinned-memory rate
// instead of staging through a pageable caller buffer
int mrts_get_masks_host(mrts_env* env, int32_t player, const uint8_t** out) {
    try {
        if (!out) throw Fail{-EINVAL, "out is null"};
        const size_t n = (size_t)env->nSlots * env->HW * env->K;
        if (!env->h_masks) HIPCHK(hipHostMalloc(&env->h_masks, n, hipHostMallocDefault));
        int r = mrts_get_masks(env, player, env->h_masks);
        if (r) return r;
        *out = env->h_masks;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_masks_i32_host(mrts_env* env, int32_t player, const int32_t** out) {
    try {
        if (!out) throw Fail{-EINVAL, "out is null"};
        const size_t n = (size_t)env->nSlots * env->HW * env->K;
        if (!env->h_masks32) HIPCHK(hipHostMalloc(&env->h_masks32, n * 4, hipHostMallocDefault));
        int r = mrts_get_masks_i32(env, player, env->h_masks32);
        if (r) return r;
        *out = env->h_masks32;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_get_state(mrts_env* env, int32_t slot, int32_t* buf, int32_t cap) {
    try {
        if (slot < 0 || slot >= env->nSlots) throw Fail{-EINVAL, "slot out of range"};
        int pl;
        const int g = env->gameOfSlot(slot, &pl);
        const size_t sw = (size_t)stateWords(env->CAP, env->HW);
        std::vector<int32_t> s(sw);
        HIPCHK(hipStreamSynchronize(env->stream));
        HIPCHK(hipMemcpy(s.data(), env->d_state + (size_t)g * sw, sw * 4, hipMemcpyDeviceToHost));
        const int CAP = env->CAP;
        const int32_t* A = s.data() + H_WORDS;
        const int nu = s[H_NU];
        std::vector<int32_t> d;
        d.push_back(s[H_TIME]);
        d.push_back(2);
        d.push_back(s[H_RES0]);
        d.push_back(s[H_RES1]);
        d.push_back(nu);
        struct Asg { int seq, unit; };
        std::vector<Asg> asg;
        for (int i = 0; i < nu; i++) {
            const uint32_t c = (uint32_t)A[A_UC * CAP + i];
            d.push_back((int32_t)((c >> 16) & 0xF));
            d.push_back((int32_t)((c >> 20) & 3) - 1);
            d.push_back((int32_t)(c & 0xFF));
            d.push_back((int32_t)((c >> 8) & 0xFF));
            d.push_back(A[A_HP * CAP + i]);
            d.push_back(A[A_RES * CAP + i]);
            if ((uint32_t)A[A_UA * CAP + i] & UA_PRESENT) asg.push_back({A[A_AS * CAP + i], i});
        }
        std::sort(asg.begin(), asg.end(), [](const Asg& a, const Asg& b) { return a.seq < b.seq; });
        d.push_back((int32_t)asg.size());
        for (auto& e : asg) {
            const uint32_t a = (uint32_t)A[A_UA * CAP + e.unit];
            const int t = (int)(a & 0xF);
            d.push_back(e.unit);
            d.push_back(t);
            d.push_back(t == 5 ? -1 : A[A_PAR * CAP + e.unit]);
            d.push_back(t == 5 ? (int32_t)((a >> 8) & 0xFF) : 0);
            d.push_back(t == 5 ? (int32_t)((a >> 16) & 0xFF) : 0);
            d.push_back(t == 4 ? (int32_t)((a >> 4) & 0xF) : -1);
            d.push_back(A[A_AT * CAP + e.unit]);
        }
        if ((int)d.size() > cap) return -(int)d.size();
        std::memcpy(buf, d.data(), d.size() * 4);
        return (int)d.size();
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_utt_json(int32_t utt_version, int32_t conflict_policy, const char* utt_json, char* buf, int32_t cap) {
    try {
        const std::string j = uttToJson(utt_json ? uttFromJson(utt_json) : makeUtt(utt_version, conflict_policy));
        if (!buf || cap < (int32_t)j.size() + 1) return -((int)j.size() + 1);
        std::memcpy(buf, j.c_str(), j.size() + 1);
        return (int)j.size();
    } catch (const Fail& f) {
        return fail(f);
    }
}

static int readHeaderWord(mrts_env* env, int word, int32_t* out_per_slot) {
    const size_t sw = (size_t)stateWords(env->CAP, env->HW);
    HIPCHK(hipStreamSynchronize(env->stream));
    std::vector<int32_t> w((size_t)env->nGames);
    HIPCHK(hipMemcpy2D(w.data(), 4, env->d_state + word, sw * 4, 4, (size_t)env->nGames, hipMemcpyDeviceToHost));
    for (int s = 0; s < env->nSlots; s++) {
        int pl;
        out_per_slot[s] = w[(size_t)env->gameOfSlot(s, &pl)];
    }
    return 0;
}

int mrts_error_flags(mrts_env* env, uint32_t* flags) {
    try {
        return readHeaderWord(env, H_ERR, (int32_t*)flags);
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_env_steps(mrts_env* env, int32_t* out) {
    try {
        return readHeaderWord(env, H_STEPS, out);
    } catch (const Fail& f) {
        return fail(f);
    }
}

void mrts_destroy(mrts_env* env) {
    if (!env) return;
    (void)hipSetDevice(env->device);
    if (env->stream) (void)hipStreamSynchronize(env->stream);
    (void)hipFree(env->d_static);
    (void)hipFree(env->d_poPrev);
    (void)hipFree(env->d_prioTab);
    (void)hipFree(env->d_renderErr);
    (void)hipFree(env->d_bal);
    (void)hipFree(env->d_state);
    (void)hipFree(env->d_polPrev);
    (void)hipFree(env->d_pairs);
    (void)hipFree(env->d_rowsStage);
    (void)hipFree(env->d_masks32);
    (void)hipFree(env->d_copyPairs);
    (void)hipFree(env->d_eval);
    (void)hipFree(env->d_tmpl);
    (void)hipFree(env->d_tmplOff);
    (void)hipFree(env->d_gameKind);
    (void)hipFree(env->d_actions);
    (void)hipFree(env->d_players);
    (void)hipFree(env->d_obs);
    (void)hipFree(env->d_reward);
    (void)hipFree(env->d_done);
    (void)hipFree(env->d_masks);
    (void)hipHostFree(env->h_obs);
    (void)hipHostFree(env->h_masks);
    (void)hipHostFree(env->h_masks32);
    (void)hipHostFree(env->h_reward);
    (void)hipHostFree(env->h_done);
    if (env->stream) (void)hipStreamDestroy(env->stream);
    if (env->exStream) (void)hipStreamSynchronize(env->exStream);
    if (env->exComm) (void)g_rccl.commDestroy(env->exComm);
    if (env->exStream) (void)hipStreamDestroy(env->exStream);
    if (env->capExec) (void)hipGraphExecDestroy(env->capExec);
    if (env->capGraph) (void)hipGraphDestroy(env->capGraph);
    for (int b = 0; b < 2; b++) {
        if (env->exReady[b]) (void)hipEventDestroy(env->exReady[b]);
        if (env->exDone[b]) (void)hipEventDestroy(env->exDone[b]);
    }
    delete env;
}

// ---------------------------------------------------------------- state serialisation (checkpoint / interop)
static void readBlock(mrts_env* env, int g, std::vector<int32_t>& s) {
    const size_t sw = (size_t)stateWords(env->CAP, env->HW);
    s.resize(sw);
    HIPCHK(hipStreamSynchronize(env->stream));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(s.data(), env->d_state + (size_t)g * sw, sw * 4, hipMemcpyDeviceToHost));
}

// GameState.toJSON(w, true, false) (rts/GameState.java:819-837) with PhysicalGameState.toJSON
// (:658-691), Player.toJSON (Player.java:86-88), Unit.toJSON (Unit.java:577-588) and
// UnitAction.toJSON (UnitAction.java:569-582).  Unit IDs are list positions: Java's IDs come from a
// JVM-global counter and are not part of a game's reproducible state.
static std::string gameToJson(const mrts_env* env, const std::vector<int32_t>& s) {
    const int CAP = env->CAP, HW = env->HW;
    const int32_t* A = s.data() + H_WORDS;
    const uint8_t* terr = (const uint8_t*)(s.data() + stateTerrOff(CAP, HW));
    const int nu = s[H_NU];
    std::ostringstream w;
    w << "{\"time\":" << s[H_TIME] << ",\"pgs\":{\"width\":" << env->W << ",\"height\":" << env->H << ",\"terrain\":\"";
    for (int i = 0; i < HW; i++) w << (int)terr[i];
    w << "\",\"players\":[{\"ID\":0, \"resources\":" << s[H_RES0] << "},{\"ID\":1, \"resources\":" << s[H_RES1]
      << "}],\"units\":[";
    struct Asg { int seq, unit; };
    std::vector<Asg> asg;
    for (int i = 0; i < nu; i++) {
        const uint32_t c = (uint32_t)A[A_UC * CAP + i];
        if (i) w << ",";
        w << "{\"type\":\"" << env->uttInfo.names[(c >> 16) & 0xF] << "\", \"ID\":" << i << ", \"player\":"
          << (int)((c >> 20) & 3) - 1 << ", \"x\":" << (c & 0xFF) << ", \"y\":" << ((c >> 8) & 0xFF)
          << ", \"resources\":" << A[A_RES * CAP + i] << ", \"hitpoints\":" << A[A_HP * CAP + i] << "}";
        if ((uint32_t)A[A_UA * CAP + i] & UA_PRESENT) asg.push_back({A[A_AS * CAP + i], i});
    }
    w << "]},\"actions\":[";
    std::sort(asg.begin(), asg.end(), [](const Asg& a, const Asg& b) { return a.seq < b.seq; });
    for (size_t k = 0; k < asg.size(); k++) {
        const int i = asg[k].unit;
        const uint32_t a = (uint32_t)A[A_UA * CAP + i];
        const int t = (int)(a & 0xF), prm = (int16_t)A[A_PAR * CAP + i];
        if (k) w << ",";
        w << "{\"ID\":" << i << ", \"time\":" << A[A_AT * CAP + i] << ", \"action\":{\"type\":" << t;
        if (t == 5) {
            w << ", \"x\":" << ((a >> 8) & 0xFF) << ",\"y\":" << ((a >> 16) & 0xFF);
        } else {
            if (prm != -1) w << ", \"parameter\":" << prm;
            if (t == 4) w << ", \"unitType\":\"" << env->uttInfo.names[(a >> 4) & 0xF] << "\"";
        }
        w << "}}";
    }
    w << "]}";
    return w.str();
}

// GameState.fromJSON (rts/GameState.java:897-915): PhysicalGameState.fromJSON (:735-756, terrain raw
// or A/B), Player.fromJSON, Unit.fromJSON (Unit.java:629-642: hitpoints default 1), the actions by
// unit ID in array order (UnitAction.fromJSON, UnitAction.java:647-658).  A new GameState: time from
// the JSON, unitCancelationCounter 0.  Writes the words of block `s` it describes; everything else
// (random streams, kind, mask row sets) is kept.  Rejects what Java would throw on (unknown type or
// ID, two units in a cell) and what this build cannot hold.
static void jsonToBlock(const mrts_env* env, const std::string& text, std::vector<int32_t>& s) {
    mjson::Value o;
    try {
        o = mjson::parse(text);
    } catch (const std::exception& e) {
        throw Fail{-EINVAL, std::string("state json: ") + e.what()};
    }
    try {
        const int CAP = env->CAP, HW = env->HW, W = env->W, H = env->H;
        const mjson::Value& pg = o.at("pgs");
        if (pg.getInt("width", 8) != W || pg.getInt("height", 8) != H) throw Fail{-EINVAL, "state json: map size differs from the handle's"};
        const std::vector<int> terr = decodeTerrain(pg.getString("terrain", ""), HW);
        const mjson::Value& pl = pg.at("players");
        if (pl.arr.size() != 2 || pl.arr[0].getInt("ID", -1) != 0 || pl.arr[1].getInt("ID", -1) != 1)
            throw Fail{-ENOTSUP, "state json: players must be 0 and 1"};
        const mjson::Value& us = pg.at("units");
        const int nu = (int)us.arr.size();
        if (nu > env->maxUnits) throw Fail{-ENOSPC, "state json: more units than the handle's max_units"};
        int32_t* A = s.data() + H_WORDS;
        std::vector<int64_t> ids((size_t)nu);
        std::vector<char> occ((size_t)HW, 0);
        for (int a = 0; a < N_ARRAYS; a++)
            for (int i = 0; i < CAP; i++) A[a * CAP + i] = 0;
        for (int i = 0; i < nu; i++) {
            const mjson::Value& u = us.arr[(size_t)i];
            const int type = env->uttInfo.typeOf(u.getString("type", ""));
            const int p = u.getInt("player", -1), x = u.getInt("x", 0), y = u.getInt("y", 0);
            const int r = u.getInt("resources", 0), hp = u.getInt("hitpoints", 1);
            ids[(size_t)i] = u.getLong("ID", -1);
            if (type < 0) throw Fail{-EINVAL, "state json: unknown unit type"};
            if (p < -1 || p > 1 || x < 0 || y < 0 || x >= W || y >= H) throw Fail{-EINVAL, "state json: unit out of range"};
            if (r < -32768 || r > 32767 || hp < -32768 || hp > 32767) throw Fail{-EINVAL, "state json: value exceeds int16"};
            if (occ[(size_t)(y * W + x)]) throw Fail{-EINVAL, "state json: two units in one position (addUnit)"};
            for (int j = 0; j < i; j++)
                if (ids[(size_t)j] == ids[(size_t)i]) throw Fail{-EINVAL, "state json: repeated unit ID"};
            occ[(size_t)(y * W + x)] = 1;
            A[A_UC * CAP + i] = (int32_t)((uint32_t)x | ((uint32_t)y << 8) | ((uint32_t)type << 16) | ((uint32_t)(p + 1) << 20));
            A[A_HP * CAP + i] = hp;
            A[A_RES * CAP + i] = r;
            A[A_PAR * CAP + i] = -1;
        }
        const mjson::Value& acts = o.at("actions");
        int seq = 0;
        for (auto& av : acts.arr) {
            const int64_t id = av.getLong("ID", -1);
            int i = 0;
            while (i < nu && ids[(size_t)i] != id) i++;
            if (i == nu) throw Fail{-EINVAL, "state json: action for an unknown unit ID"};
            const uint32_t c = (uint32_t)A[A_UC * CAP + i];
            if ((int)((c >> 20) & 3) - 1 < 0) throw Fail{-EINVAL, "state json: action for a neutral unit"};
            const mjson::Value& ua = av.at("action");
            const int t = ua.getInt("type", 0), prm = ua.getInt("parameter", -1);
            const int tx = ua.getInt("x", -1), ty = ua.getInt("y", -1);
            const std::string utn = ua.getString("unitType", "");
            int ut = 0;
            if (t < 0 || t > 5) throw Fail{-EINVAL, "state json: bad action type"};
            if (t == 5 && (tx < 0 || ty < 0 || tx >= W || ty >= H)) throw Fail{-ENOTSUP, "state json: attack target off the map"};
            if (t >= 1 && t <= 4 && (prm < 0 || prm > 3)) throw Fail{-ENOTSUP, "state json: bad direction"};
            if (t == 0 && (prm < -1 || prm > 32767)) throw Fail{-ENOTSUP, "state json: bad NONE duration"};
            if (t == 4) {
                ut = env->uttInfo.typeOf(utn);
                if (ut < 0) throw Fail{-EINVAL, "state json: unknown produced type"};
            }
            const bool again = (uint32_t)A[A_UA * CAP + i] & UA_PRESENT;  // put() on a present key keeps its place
            A[A_UA * CAP + i] = (int32_t)((uint32_t)t | ((uint32_t)ut << 4) |
                                          (t == 5 ? ((uint32_t)tx << 8) | ((uint32_t)ty << 16) : 0u) | UA_PRESENT);
            A[A_PAR * CAP + i] = t == 5 ? -1 : prm;
            A[A_AT * CAP + i] = av.getInt("time", 0);
            if (!again) A[A_AS * CAP + i] = seq++;
        }
        const mjson::Value& p0 = pl.arr[0];
        const mjson::Value& p1 = pl.arr[1];
        s[H_TIME] = o.getInt("time", 0);
        s[H_NU] = nu;
        s[H_RES0] = p0.getInt("resources", 0);
        s[H_RES1] = p1.getInt("resources", 0);
        s[H_SEQ] = seq;
        s[H_STEPS] = 0;
        s[H_ERR] = 0;
        s[H_CANCEL_CNT] = 0;
        uint8_t* tb = (uint8_t*)(s.data() + stateTerrOff(CAP, HW));
        for (int i = 0; i < HW; i++) tb[i] = terr[(size_t)i] != 0;
        for (int i = HW; i < 4 * ((HW + 3) / 4); i++) tb[i] = 0;
        for (int i = 0; i < nu; i++) {  // units may not stand on walls (the cell map has one owner per cell)
            const uint32_t c = (uint32_t)A[A_UC * CAP + i];
            if (tb[(c & 0xFF) + ((c >> 8) & 0xFF) * W]) throw Fail{-ENOTSUP, "state json: unit on a wall"};
        }
    } catch (const std::runtime_error& e) {
        throw Fail{-EINVAL, std::string("state json: ") + e.what()};
    }
}

int mrts_get_state_json(mrts_env* env, int32_t slot, char* buf, int32_t cap) {
    try {
        if (!env || slot < 0 || slot >= env->nSlots) throw Fail{-EINVAL, "slot out of range"};
        int pl;
        std::vector<int32_t> s;
        readBlock(env, env->gameOfSlot(slot, &pl), s);
        const std::string j = gameToJson(env, s);
        if (!buf || cap < (int32_t)j.size() + 1) return -((int)j.size() + 1);
        std::memcpy(buf, j.c_str(), j.size() + 1);
        return (int)j.size();
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_set_state_json(mrts_env* env, int32_t slot, const char* json) {
    try {
        if (!env || !json || slot < 0 || slot >= env->nSlots) throw Fail{-EINVAL, "bad argument"};
        int pl;
        const int g = env->gameOfSlot(slot, &pl);
        std::vector<int32_t> s;
        readBlock(env, g, s);
        jsonToBlock(env, json, s);
        env->noteValues(s.data());
        const size_t sw = s.size();
        HIPCHK(hipMemcpy(env->d_state + (size_t)g * sw, s.data(), sw * 4, hipMemcpyHostToDevice));
        env->lastMaskPtr = nullptr;  // the next mask and observation writes are full ones
        env->lastObsPtr = nullptr;
        env->polValid = false;
        env->fusedActions = nullptr;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

// whole-handle checkpoint: a header + every game's state block (random streams, envSteps, kind included)
namespace {
struct CkptHeader {
    char magic[8];
    int32_t version, H, W, CAP, nGames, nSpGames, words;
    uint32_t uttHash;
    uint32_t cfgHash;  // mrts_env::cfgHash: game kinds (opponents), map templates, max_steps, reward kinds, PO
    int32_t pad_;
};
uint32_t uttHash(const DevUtt& u) {
    uint32_t h = 2166136261u;
    const uint8_t* p = (const uint8_t*)&u;
    for (size_t i = 0; i < sizeof(DevUtt); i++) h = (h ^ p[i]) * 16777619u;
    return h;
}
}  // namespace

int64_t mrts_checkpoint_size(const mrts_env* env) {
    if (!env) return -EINVAL;
    return (int64_t)sizeof(CkptHeader) + (int64_t)stateWords(env->CAP, env->HW) * env->nGames * 4;
}

int mrts_checkpoint(mrts_env* env, void* buf, int64_t cap) {
    try {
        if (!env || !buf) throw Fail{-EINVAL, "null argument"};
        if (cap < mrts_checkpoint_size(env)) throw Fail{-ENOSPC, "buffer too small"};
        CkptHeader h;
        std::memset(&h, 0, sizeof(h));
        std::memcpy(h.magic, "MRTSCKP1", 8);
        h.version = 3;
        h.H = env->H;
        h.W = env->W;
        h.CAP = env->CAP;
        h.nGames = env->nGames;
        h.nSpGames = env->nSpGames;
        h.words = stateWords(env->CAP, env->HW);
        h.uttHash = uttHash(env->utt);
        h.cfgHash = env->cfgHash;
        std::memcpy(buf, &h, sizeof(h));
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy((char*)buf + sizeof(h), env->d_state, (size_t)h.words * h.nGames * 4, hipMemcpyDeviceToHost));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_restore(mrts_env* env, const void* buf, int64_t size) {
    try {
        if (!env || !buf) throw Fail{-EINVAL, "null argument"};
        CkptHeader h;
        if (size < (int64_t)sizeof(h)) throw Fail{-EINVAL, "checkpoint too short"};
        std::memcpy(&h, buf, sizeof(h));
        if (std::memcmp(h.magic, "MRTSCKP1", 8) != 0 || h.version != 3) throw Fail{-EINVAL, "not a checkpoint"};
        if (h.H != env->H || h.W != env->W || h.CAP != env->CAP || h.nGames != env->nGames || h.nSpGames != env->nSpGames ||
            h.words != stateWords(env->CAP, env->HW) || h.uttHash != uttHash(env->utt))
            throw Fail{-EINVAL, "checkpoint of a different configuration"};
        if (h.cfgHash != env->cfgHash)
            throw Fail{-EINVAL, "checkpoint of a different configuration (opponents, maps, max_steps, reward functions "
                                "or partial observability differ)"};
        if (size != mrts_checkpoint_size(env)) throw Fail{-EINVAL, "checkpoint size mismatch"};
        for (int g = 0; g < h.nGames; g++)
            env->noteValues((const int32_t*)((const char*)buf + sizeof(h)) + (size_t)g * h.words);
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(env->d_state, (const char*)buf + sizeof(h), (size_t)h.words * h.nGames * 4, hipMemcpyHostToDevice));
        env->lastMaskPtr = nullptr;
        env->lastObsPtr = nullptr;
        env->polValid = false;
        env->fusedActions = nullptr;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

// ---------------------------------------------------------------- forward model
static void checkCopy(const mrts_env* dst, const mrts_env* src) {
    if (!dst || !src) throw Fail{-EINVAL, "null handle"};
    if (!dst->forwardModel) throw Fail{-EINVAL, "copy destination must be a forward-model handle"};
    if (src->H != dst->H || src->W != dst->W || src->CAP != dst->CAP) throw Fail{-EINVAL, "handles differ in map size"};
    if (std::memcmp(&src->utt, &dst->utt, sizeof(DevUtt)) != 0) throw Fail{-EINVAL, "handles differ in unit-type table"};
    if (src->device != dst->device) throw Fail{-EINVAL, "handles live on different devices"};
}

int mrts_copy_games_dev(mrts_env* dst, const mrts_env* src, const int32_t* d_pairs, int32_t n, void* stream) {
    try {
        if (!src) src = dst;
        checkCopy(dst, src);
        if (n < 0 || (n > 0 && !d_pairs)) throw Fail{-EINVAL, "bad pairs"};
        HIPCHK(hipSetDevice(dst->device));
        HIPCHK(launchCopyGames(dst->d_state, src->d_state, d_pairs, n, dst->nGames, src->nGames, dst->CAP, dst->HW,
                               pickStream(dst, stream)));
        dst->lastObsPtr = nullptr;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_copy_games(mrts_env* dst, const mrts_env* src, const int32_t* pairs, int32_t n) {
    try {
        if (!src) src = dst;
        checkCopy(dst, src);
        if (n < 0 || (n > 0 && !pairs)) throw Fail{-EINVAL, "bad pairs"};
        std::vector<char> isDst((size_t)dst->nGames, 0), isSrc((size_t)src->nGames, 0);
        for (int i = 0; i < n; i++) {
            const int d = pairs[2 * i], s = pairs[2 * i + 1];
            if (d < 0 || d >= dst->nGames || s < 0 || s >= src->nGames) throw Fail{-EINVAL, "game index out of range"};
            if (isDst[(size_t)d]) throw Fail{-EINVAL, "a destination game appears twice"};
            isDst[(size_t)d] = 1;
            isSrc[(size_t)s] = 1;
        }
        if (src == dst)
            for (int g = 0; g < dst->nGames; g++)
                if (isDst[(size_t)g] && isSrc[(size_t)g]) throw Fail{-EINVAL, "a game is both a source and a destination"};
        if (n == 0) return 0;
        HIPCHK(hipSetDevice(dst->device));
        HIPCHK(hipStreamSynchronize(src->stream));
        if (n > dst->copyPairsCap) {
            HIPCHK(hipStreamSynchronize(dst->stream));
            (void)hipFree(dst->d_copyPairs);
            dst->d_copyPairs = nullptr;
            HIPCHK(hipMalloc(&dst->d_copyPairs, (size_t)n * 2 * 4));
            dst->copyPairsCap = n;
        }
        HIPCHK(hipMemcpyAsync(dst->d_copyPairs, pairs, (size_t)n * 2 * 4, hipMemcpyHostToDevice, dst->stream));
        HIPCHK(launchCopyGames(dst->d_state, src->d_state, dst->d_copyPairs, n, dst->nGames, src->nGames, dst->CAP,
                               dst->HW, dst->stream));
        dst->lastObsPtr = nullptr;
        HIPCHK(hipStreamSynchronize(dst->stream));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_playout_dev(mrts_env* env, int32_t horizon, void* stream) {
    try {
        if (!env || !env->forwardModel) throw Fail{-EINVAL, "not a forward-model handle"};
        if (horizon < -MRTS_MAX_HORIZON || horizon > MRTS_MAX_HORIZON) throw Fail{-EINVAL, "horizon out of range"};
        HIPCHK(hipSetDevice(env->device));
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.horizon = horizon;
        HIPCHK(env->launch(3, D, pickStream(env, stream)));
        env->lastObsPtr = nullptr;
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_playout(mrts_env* env, int32_t horizon) {
    try {
        int r = mrts_playout_dev(env, horizon, env ? env->stream : nullptr);
        if (r) return r;
        HIPCHK(hipStreamSynchronize(env->stream));
        checkFlagsAfter(env);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_trace_step(mrts_env* env, const int32_t* pairs, int32_t n_pairs, const int32_t* until, int32_t* out,
                    int32_t generic) {
    try {
        if (!env || !env->forwardModel) throw Fail{-EINVAL, "not a forward-model handle"};
        if (!until || (n_pairs > 0 && !pairs)) throw Fail{-EINVAL, "null argument"};
        if (n_pairs < 0 || (size_t)n_pairs * env->nGames * 8 >= ((size_t)1 << 31)) throw Fail{-EINVAL, "bad n_pairs"};
        const size_t nr = (size_t)env->nGames * n_pairs;
        for (size_t i = 0; i < nr; i++) {  // what Java could not construct (TraceEntry.fromXML, UnitAction(...))
            const int32_t* r = pairs + 8 * i;
            if (r[0] < -1 || r[0] > 1) throw Fail{-EINVAL, "pair player must be 0, 1 or -1 (padding)"};
            if (r[0] < 0) continue;
            if (r[3] == 4 && (r[7] < 0 || r[7] >= env->utt.ntypes)) throw Fail{-EINVAL, "PRODUCE of an unknown unit type"};
            if (r[4] < -32768 || r[4] > 32767) throw Fail{-EINVAL, "parameter out of the int16 range"};
        }
        for (int g = 0; g < env->nGames; g++)
            if (until[g] < 0 || until[g] > (1 << 30)) throw Fail{-EINVAL, "until out of range"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(hipStreamSynchronize(env->stream));
        const size_t need = nr * 8 + 2 * (size_t)env->nGames;
        if (need > env->rowsStageInts) {
            (void)hipFree(env->d_rowsStage);
            env->d_rowsStage = nullptr;
            HIPCHK(hipMalloc(&env->d_rowsStage, need * 4));
            env->rowsStageInts = need;
        }
        int32_t* d_until = env->d_rowsStage + nr * 8;
        if (nr) HIPCHK(hipMemcpyAsync(env->d_rowsStage, pairs, nr * 8 * 4, hipMemcpyHostToDevice, env->stream));
        HIPCHK(hipMemcpyAsync(d_until, until, (size_t)env->nGames * 4, hipMemcpyHostToDevice, env->stream));
        KDyn D;
        std::memset(&D, 0, sizeof(D));
        D.rows = env->d_rowsStage;
        D.n_rows = n_pairs;
        D.trace_until = d_until;
        D.trace_out = d_until + env->nGames;
        D.trace_generic = generic ? 1 : 0;
        HIPCHK(env->launch(4, D, env->stream));
        env->lastObsPtr = nullptr;
        env->fusedActions = nullptr;
        std::vector<int32_t> o((size_t)env->nGames);
        HIPCHK(hipMemcpyAsync(o.data(), D.trace_out, (size_t)env->nGames * 4, hipMemcpyDeviceToHost, env->stream));
        HIPCHK(hipStreamSynchronize(env->stream));
        if (out) std::memcpy(out, o.data(), o.size() * 4);
        checkFlagsAfter(env);
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_evaluate_dev(mrts_env* env, int32_t maxplayer, float* d_out, void* stream) {
    try {
        if (!env || !d_out) throw Fail{-EINVAL, "null argument"};
        if (maxplayer != 0 && maxplayer != 1) throw Fail{-EINVAL, "maxplayer must be 0 or 1"};
        HIPCHK(hipSetDevice(env->device));
        HIPCHK(launchEvaluate(env->hstatic, env->d_static, maxplayer, d_out, pickStream(env, stream)));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

int mrts_evaluate(mrts_env* env, int32_t maxplayer, float* out) {
    try {
        if (!env || !out) throw Fail{-EINVAL, "null argument"};
        if (!env->d_eval) HIPCHK(hipMalloc(&env->d_eval, (size_t)env->nGames * 4));
        int r = mrts_evaluate_dev(env, maxplayer, env->d_eval, env->stream);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(out, env->d_eval, (size_t)env->nGames * 4, hipMemcpyDeviceToHost, env->stream));
        HIPCHK(hipStreamSynchronize(env->stream));
        return 0;
    } catch (const Fail& f) {
        return fail(f);
    }
}

#ifdef MRTS_LANE_AUDIT
// diagnostic build only: the cross-lane read audit (tests/test_zz_lane_audit.py); synchronises the device
int mrts_lane_audit(int32_t* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -EIO;
    return mrts::laneAudit(out, reset) == hipSuccess ? 0 : -EIO;
}
// the negative control: one launch whose readlane reads an inactive lane (the audit must report it)
int mrts_lane_audit_probe(void) {
    int32_t* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int32_t)) != hipSuccess) return -ENOMEM;
    const hipError_t e = mrts::laneAuditProbe(d);
    const hipError_t s = hipDeviceSynchronize();
    (void)hipFree(d);
    return e == hipSuccess && s == hipSuccess ? 0 : -EIO;
}
#endif
#ifdef MRTS_ABLATE
// diagnostic build only: g_ablate (tools/ablate_price.py)
int mrts_set_ablate(unsigned v) { return mrts::setAblate(v) == hipSuccess ? 0 : -EIO; }
int mrts_get_dbg(unsigned long long* out, int reset) { return mrts::getDbg(out, reset) == hipSuccess ? 0 : -EIO; }
#endif
#ifdef MRTS_PHASE_TIMING
// diagnostic build only: per-phase cycle sums of k_env (tools/phase_timing.py)
int mrts_phase_times(unsigned long long* out, int reset) { return mrts::phaseTimes(out, reset) == hipSuccess ? 0 : -EIO; }
int mrts_phase_spans(unsigned long long* out, int n) { return mrts::phaseSpans(out, n) == hipSuccess ? 0 : -EIO; }
#endif
}  // extern "C"
