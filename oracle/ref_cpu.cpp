// ref_cpu — CPU ORACLE (TEST INFRASTRUCTURE ONLY). See ref_cpu.hpp header.
// Engine restatement: rts/{GameState,PhysicalGameState,UnitAction,ResourceUsage,
// PlayerAction,PartiallyObservableGameState}.java, rts/units/{Unit,UnitTypeTable}.java,
// ai/{PassiveAI,RandomBiasedAI}.java, util/Sampler.java.
#include "ref_cpu.hpp"
#include "../microrts_amd/csrc/mrts_json.hpp"  // a plain JSON reader (minimal-json's role)

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

namespace oref {

static thread_local int64_t g_next_ID = 0;  // rts/units/Unit.java:34 (static next_ID)

// ---------------------------------------------------------------- UnitTypeTable
// rts/units/UnitTypeTable.java:104-289
UnitTypeTable::UnitTypeTable(int ver, int crs) : moveConflictResolutionStrategy(crs), version(ver) {
    auto add = [&](UnitType* ut) {
        ut->ID = (int)unitTypes.size();
        unitTypes.emplace_back(ut);
    };
    auto* resource = new UnitType();
    resource->name = "Resource";
    resource->isResource = true;
    resource->isStockpile = false;
    resource->canHarvest = false;
    resource->canMove = false;
    resource->canAttack = false;
    resource->sightRadius = 0;
    add(resource);

    auto* base = new UnitType();
    base->name = "Base";
    base->cost = 10;
    base->hp = 10;
    if (ver == 1) base->produceTime = 250;
    else if (ver == 2) base->produceTime = 200;  // v3 keeps the UnitType default (10)
    base->isResource = false;
    base->isStockpile = true;
    base->canHarvest = false;
    base->canMove = false;
    base->canAttack = false;
    base->sightRadius = 5;
    add(base);

    auto* barracks = new UnitType();
    barracks->name = "Barracks";
    barracks->cost = 5;
    barracks->hp = 4;
    if (ver == 1) barracks->produceTime = 200;
    else if (ver == 2 || ver == 3) barracks->produceTime = 100;
    barracks->isResource = false;
    barracks->isStockpile = false;
    barracks->canHarvest = false;
    barracks->canMove = false;
    barracks->canAttack = false;
    barracks->sightRadius = 3;
    add(barracks);

    auto* worker = new UnitType();
    worker->name = "Worker";
    worker->cost = 1;
    worker->hp = 1;
    if (ver == 1 || ver == 2) worker->minDamage = worker->maxDamage = 1;
    else if (ver == 3) { worker->minDamage = 0; worker->maxDamage = 2; }
    worker->attackRange = 1;
    worker->produceTime = 50;
    worker->moveTime = 10;
    worker->attackTime = 5;
    worker->harvestTime = 20;
    worker->returnTime = 10;
    worker->isResource = false;
    worker->isStockpile = false;
    worker->canHarvest = true;
    worker->canMove = true;
    worker->canAttack = true;
    worker->sightRadius = 3;
    add(worker);

    auto* light = new UnitType();
    light->name = "Light";
    light->cost = 2;
    light->hp = 4;
    if (ver == 1 || ver == 2) light->minDamage = light->maxDamage = 2;
    else if (ver == 3) { light->minDamage = 1; light->maxDamage = 3; }
    light->attackRange = 1;
    light->produceTime = 80;
    light->moveTime = 8;
    light->attackTime = 5;
    light->isResource = false;
    light->isStockpile = false;
    light->canHarvest = false;
    light->canMove = true;
    light->canAttack = true;
    light->sightRadius = 2;
    add(light);

    auto* heavy = new UnitType();
    heavy->name = "Heavy";
    if (ver == 1 || ver == 2) heavy->minDamage = heavy->maxDamage = 4;
    else if (ver == 3) { heavy->minDamage = 0; heavy->maxDamage = 6; }
    heavy->attackRange = 1;
    heavy->produceTime = 120;
    if (ver == 1) { heavy->moveTime = 12; heavy->hp = 4; heavy->cost = 2; }
    else if (ver == 2 || ver == 3) { heavy->moveTime = 10; heavy->hp = 8; heavy->cost = 3; }
    heavy->attackTime = 5;
    heavy->isResource = false;
    heavy->isStockpile = false;
    heavy->canHarvest = false;
    heavy->canMove = true;
    heavy->canAttack = true;
    heavy->sightRadius = 2;
    add(heavy);

    auto* ranged = new UnitType();
    ranged->name = "Ranged";
    ranged->cost = 2;
    ranged->hp = 1;
    if (ver == 1 || ver == 2) ranged->minDamage = ranged->maxDamage = 1;
    else if (ver == 3) { ranged->minDamage = 1; ranged->maxDamage = 2; }
    ranged->attackRange = 3;
    ranged->produceTime = 100;
    ranged->moveTime = 10;
    ranged->attackTime = 5;
    ranged->isResource = false;
    ranged->isStockpile = false;
    ranged->canHarvest = false;
    ranged->canMove = true;
    ranged->canAttack = true;
    ranged->sightRadius = 3;
    add(ranged);

    base->produces.push_back(worker);
    barracks->produces.push_back(light);
    barracks->produces.push_back(heavy);
    barracks->produces.push_back(ranged);
    worker->produces.push_back(base);
    worker->produces.push_back(barracks);
}

// UnitTypeTable.fromJSON (:414-433): EMPTY table, the policy (default CANCEL_BOTH), then createStub
// for every entry (UnitType.java:156-161) and updateFromJSON by name (UnitType.java:217-248) —
// harvestTime from "produceTime", returnTime untouched, minimal-json defaults for absent members.
UnitTypeTable UnitTypeTable::fromJSON(const std::string& json) {
    const mjson::Value o = mjson::parse(json);
    UnitTypeTable utt(1, 1);
    utt.unitTypes.clear();
    utt.version = 0;  // EMPTY_TYPE_TABLE
    utt.moveConflictResolutionStrategy = o.getInt("moveConflictResolutionStrategy", 1);
    const mjson::Value& a = o.at("unitTypes");
    for (auto& v : a.arr) {
        auto* ut = new UnitType();
        ut->ID = v.getInt("ID", -1);
        ut->name = v.getString("name", "");
        utt.unitTypes.emplace_back(ut);
    }
    for (auto& v : a.arr) {
        UnitType* ut = utt.getUnitType(v.getString("name", ""));
        ut->cost = v.getInt("cost", 1);
        ut->hp = v.getInt("hp", 1);
        ut->minDamage = v.getInt("minDamage", 1);
        ut->maxDamage = v.getInt("maxDamage", 1);
        ut->attackRange = v.getInt("attackRange", 1);
        ut->produceTime = v.getInt("produceTime", 10);
        ut->moveTime = v.getInt("moveTime", 10);
        ut->attackTime = v.getInt("attackTime", 10);
        ut->harvestTime = v.getInt("produceTime", 10);
        ut->produceTime = v.getInt("produceTime", 10);
        ut->harvestAmount = v.getInt("harvestAmount", 10);
        ut->sightRadius = v.getInt("sightRadius", 10);
        ut->isResource = v.getBool("isResource", false);
        ut->isStockpile = v.getBool("isStockpile", false);
        ut->canHarvest = v.getBool("canHarvest", false);
        ut->canMove = v.getBool("canMove", false);
        ut->canAttack = v.getBool("canAttack", false);
        for (auto& p : v.at("produces").arr) ut->produces.push_back(utt.getUnitType(p.s));
    }
    return utt;
}

UnitType* UnitTypeTable::getUnitType(int ID) const {
    if (ID < 0 || ID >= (int)unitTypes.size()) throw std::out_of_range("UnitTypeTable.getUnitType: index out of range");
    return unitTypes[(size_t)ID].get();
}
UnitType* UnitTypeTable::getUnitType(const std::string& name) const {
    for (auto& ut : unitTypes)
        if (ut->name == name) return ut.get();
    return nullptr;
}
int UnitTypeTable::getMaxAttackRange() const {
    int m = 0;
    for (auto& ut : unitTypes)
        if (ut->attackRange > m) m = ut->attackRange;
    return m;
}

// ---------------------------------------------------------------- PhysicalGameState
Unit* PhysicalGameState::getUnitAt(int x, int y) const {  // :263-270
    for (auto& u : units)
        if (u->x == x && u->y == y) return u.get();
    return nullptr;
}
UnitP PhysicalGameState::getUnitAtP(int x, int y) const {
    for (auto& u : units)
        if (u->x == x && u->y == y) return u;
    return nullptr;
}
void PhysicalGameState::addUnit(const UnitP& nu) {  // :189-201
    for (auto& e : units)
        if (nu->x == e->x && nu->y == e->y)
            throw std::invalid_argument("PhysicalGameState.addUnit: added two units in position");
    units.push_back(nu);
}
void PhysicalGameState::removeUnit(const Unit* u) {  // :208-210 (LinkedList.remove by identity)
    for (size_t i = 0; i < units.size(); i++)
        if (units[i].get() == u) {
            units.erase(units.begin() + (long)i);
            return;
        }
}
int PhysicalGameState::winner() const {  // :334-353
    std::vector<int> unitcounts(players.size(), 0);
    for (auto& u : units)
        if (u->player >= 0) unitcounts[(size_t)u->player]++;
    int w = -1;
    for (size_t i = 0; i < unitcounts.size(); i++) {
        if (unitcounts[i] > 0) {
            if (w == -1) w = (int)i;
            else return -1;
        }
    }
    return w;
}
bool PhysicalGameState::gameover() const {  // :361-387
    std::vector<int> unitcounts(players.size(), 0);
    int totalunits = 0;
    for (auto& u : units)
        if (u->player >= 0) {
            unitcounts[(size_t)u->player]++;
            totalunits++;
        }
    if (totalunits == 0) return true;
    int w = -1;
    for (size_t i = 0; i < unitcounts.size(); i++) {
        if (unitcounts[i] > 0) {
            if (w == -1) w = (int)i;
            else return false;
        }
    }
    return w != -1;
}
PGSP PhysicalGameState::clone() const {  // :392-401
    auto p = std::make_shared<PhysicalGameState>();
    p->width = width;
    p->height = height;
    p->terrain = terrain;
    for (auto& pl : players) p->players.push_back(std::make_shared<Player>(*pl));
    for (auto& u : units) p->units.push_back(std::make_shared<Unit>(*u));
    return p;
}
PGSP PhysicalGameState::cloneKeepingUnits() const {  // :409-414
    auto p = std::make_shared<PhysicalGameState>();
    p->width = width;
    p->height = height;
    p->terrain = terrain;
    p->players = players;
    p->units = units;
    return p;
}

// ---------------------------------------------------------------- ResourceUsage
// rts/ResourceUsage.java:31-50
bool ResourceUsage::consistentWith(const ResourceUsage& another, const GameState& gs) const {
    for (int pos : another.positionsUsed)
        if (std::find(positionsUsed.begin(), positionsUsed.end(), pos) != positionsUsed.end()) return false;
    for (int i = 0; i < 2; i++) {
        if (another.resourcesUsed[i] == 0) continue;
        if (resourcesUsed[i] + another.resourcesUsed[i] > 0 &&
            resourcesUsed[i] + another.resourcesUsed[i] > gs.getPlayer(i).resources)
            return false;
    }
    return true;
}
void ResourceUsage::merge(const ResourceUsage& o) {  // :92-97
    positionsUsed.insert(positionsUsed.end(), o.positionsUsed.begin(), o.positionsUsed.end());
    for (int i = 0; i < 2; i++) resourcesUsed[i] += o.resourcesUsed[i];
}

// ---------------------------------------------------------------- UnitAction
bool UnitAction::equals(const UnitAction& a) const {  // rts/UnitAction.java:191-208
    if (a.type != type) return false;
    if (type == TYPE_NONE || type == TYPE_MOVE || type == TYPE_HARVEST || type == TYPE_RETURN)
        return a.parameter == parameter;
    if (type == TYPE_ATTACK_LOCATION) return a.x == x && a.y == y;
    return a.parameter == parameter && a.unitType == unitType;
}

static int adjacentPos(int pos, int parameter, int width) {
    switch (parameter) {
        case UnitAction::DIRECTION_UP: return pos - width;
        case UnitAction::DIRECTION_RIGHT: return pos + 1;
        case UnitAction::DIRECTION_DOWN: return pos + width;
        case UnitAction::DIRECTION_LEFT: return pos - 1;
    }
    return pos;
}

// rts/UnitAction.java:246-296 (memoised in r_cache, :130)
const ResourceUsage& UnitAction::resourceUsage(const Unit& u, const PhysicalGameState& pgs) {
    if (r_cache) return *r_cache;
    r_cache.reset(new ResourceUsage());
    switch (type) {
        case TYPE_MOVE: {
            int pos = u.x + u.y * pgs.width;
            r_cache->positionsUsed.push_back(adjacentPos(pos, parameter, pgs.width));
        } break;
        case TYPE_PRODUCE: {
            r_cache->resourcesUsed[u.player] += unitType->cost;
            int pos = u.x + u.y * pgs.width;
            r_cache->positionsUsed.push_back(adjacentPos(pos, parameter, pgs.width));
        } break;
    }
    return *r_cache;
}

int UnitAction::ETA(const Unit& u) const {  // rts/UnitAction.java:307-329
    switch (type) {
        case TYPE_NONE: return parameter;
        case TYPE_MOVE: return u.type->moveTime;
        case TYPE_ATTACK_LOCATION: return u.type->attackTime;
        case TYPE_HARVEST: return u.type->harvestTime;
        case TYPE_RETURN: return u.type->moveTime;  // returnTime unused (:321-322)
        case TYPE_PRODUCE: return unitType->produceTime;
    }
    return 0;
}

static UnitP getUnitAtInList(const PhysicalGameState& pgs, int x, int y) { return pgs.getUnitAtP(x, y); }

void UnitAction::execute(const UnitP& up, GameState& s) {  // rts/UnitAction.java:338-465
    Unit& u = *up;
    PhysicalGameState& pgs = *s.pgs;
    switch (type) {
        case TYPE_NONE: break;
        case TYPE_MOVE:
            switch (parameter) {
                case DIRECTION_UP: u.y = u.y - 1; break;
                case DIRECTION_RIGHT: u.x = u.x + 1; break;
                case DIRECTION_DOWN: u.y = u.y + 1; break;
                case DIRECTION_LEFT: u.x = u.x - 1; break;
            }
            break;
        case TYPE_ATTACK_LOCATION: {
            UnitP other = getUnitAtInList(pgs, x, y);
            if (other) {
                int damage;
                if (u.type->minDamage == u.type->maxDamage) damage = u.type->minDamage;
                else {
                    if (!s.damageRandom) throw std::runtime_error("non-deterministic UTT needs a damage RNG");
                    damage = u.type->minDamage + s.damageRandom->nextInt(1 + (u.type->maxDamage - u.type->minDamage));
                }
                other->hitpoints = other->hitpoints - damage;
                if (other->hitpoints <= 0) s.removeUnit(other.get());
            }
        } break;
        case TYPE_HARVEST: {
            UnitP r;
            switch (parameter) {
                case DIRECTION_UP: r = getUnitAtInList(pgs, u.x, u.y - 1); break;
                case DIRECTION_RIGHT: r = getUnitAtInList(pgs, u.x + 1, u.y); break;
                case DIRECTION_DOWN: r = getUnitAtInList(pgs, u.x, u.y + 1); break;
                case DIRECTION_LEFT: r = getUnitAtInList(pgs, u.x - 1, u.y); break;
            }
            if (r && r->type->isResource && u.type->canHarvest && u.resources == 0) {
                r->resources = r->resources - u.type->harvestAmount;
                if (r->resources <= 0) s.removeUnit(r.get());
                u.resources = u.type->harvestAmount;
            }
        } break;
        case TYPE_RETURN: {
            UnitP b;
            switch (parameter) {
                case DIRECTION_UP: b = getUnitAtInList(pgs, u.x, u.y - 1); break;
                case DIRECTION_RIGHT: b = getUnitAtInList(pgs, u.x + 1, u.y); break;
                case DIRECTION_DOWN: b = getUnitAtInList(pgs, u.x, u.y + 1); break;
                case DIRECTION_LEFT: b = getUnitAtInList(pgs, u.x - 1, u.y); break;
            }
            if (b && b->type->isStockpile && u.resources > 0) {
                Player& p = pgs.getPlayer(u.player);
                p.resources = p.resources + u.resources;
                u.resources = 0;
            }
        } break;
        case TYPE_PRODUCE: {
            int tx = u.x, ty = u.y;
            switch (parameter) {
                case DIRECTION_UP: ty--; break;
                case DIRECTION_RIGHT: tx++; break;
                case DIRECTION_DOWN: ty++; break;
                case DIRECTION_LEFT: tx--; break;
            }
            auto nu = std::make_shared<Unit>();
            nu->player = u.player;
            nu->type = unitType;
            nu->x = tx;
            nu->y = ty;
            nu->resources = 0;
            nu->hitpoints = unitType->hp;
            nu->ID = g_next_ID++;
            Player& p = pgs.getPlayer(u.player);
            if ((p.resources - unitType->cost) >= 0) {
                pgs.addUnit(nu);  // throws on an occupied cell, like Java
                p.resources = p.resources - unitType->cost;
            } else {
                s.errors++;  // Java prints "Illegal action attempted" (:457-461) and continues
            }
        } break;
    }
}

// ---------------------------------------------------------------- Unit.getUnitActions
// rts/units/Unit.java:382-522
std::vector<UnitActionP> getUnitActions(const Unit& me, const GameState& s, int noneDuration) {
    std::vector<UnitActionP> l;
    const PhysicalGameState& pgs = *s.pgs;
    const Player& p = pgs.getPlayer(me.player < 0 ? 0 : me.player);
    const int x = me.x, y = me.y;
    const UnitType& type = *me.type;
    const Unit *uup = nullptr, *uright = nullptr, *udown = nullptr, *uleft = nullptr;
    for (auto& up : pgs.units) {
        const Unit& u = *up;
        if (u.x == x) {
            if (u.y == y - 1) uup = &u;
            else if (u.y == y + 1) udown = &u;
        } else {
            if (u.y == y) {
                if (u.x == x - 1) uleft = &u;
                else if (u.x == x + 1) uright = &u;
            }
        }
    }
    if (type.canAttack) {
        if (type.attackRange == 1) {
            if (y > 0 && uup && uup->player != me.player && uup->player >= 0) l.push_back(UnitAction::attack(uup->x, uup->y));
            if (x < pgs.width - 1 && uright && uright->player != me.player && uright->player >= 0)
                l.push_back(UnitAction::attack(uright->x, uright->y));
            if (y < pgs.height - 1 && udown && udown->player != me.player && udown->player >= 0)
                l.push_back(UnitAction::attack(udown->x, udown->y));
            if (x > 0 && uleft && uleft->player != me.player && uleft->player >= 0)
                l.push_back(UnitAction::attack(uleft->x, uleft->y));
        } else {
            int sqrange = type.attackRange * type.attackRange;
            for (auto& up : pgs.units) {
                const Unit& u = *up;
                if (u.player < 0 || u.player == me.player) continue;
                int sq_dx = (u.x - x) * (u.x - x);
                int sq_dy = (u.y - y) * (u.y - y);
                if (sq_dx + sq_dy <= sqrange) l.push_back(UnitAction::attack(u.x, u.y));
            }
        }
    }
    if (type.canHarvest) {
        if (me.resources == 0) {
            if (y > 0 && uup && uup->type->isResource) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_HARVEST, UnitAction::DIRECTION_UP));
            if (x < pgs.width - 1 && uright && uright->type->isResource) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_HARVEST, UnitAction::DIRECTION_RIGHT));
            if (y < pgs.height - 1 && udown && udown->type->isResource) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_HARVEST, UnitAction::DIRECTION_DOWN));
            if (x > 0 && uleft && uleft->type->isResource) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_HARVEST, UnitAction::DIRECTION_LEFT));
        }
        if (me.resources > 0) {
            if (y > 0 && uup && uup->type->isStockpile && uup->player == me.player) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_RETURN, UnitAction::DIRECTION_UP));
            if (x < pgs.width - 1 && uright && uright->type->isStockpile && uright->player == me.player) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_RETURN, UnitAction::DIRECTION_RIGHT));
            if (y < pgs.height - 1 && udown && udown->type->isStockpile && udown->player == me.player) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_RETURN, UnitAction::DIRECTION_DOWN));
            if (x > 0 && uleft && uleft->type->isStockpile && uleft->player == me.player) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_RETURN, UnitAction::DIRECTION_LEFT));
        }
    }
    for (UnitType* ut : type.produces) {
        if (p.resources >= ut->cost) {
            int tup = (y > 0 ? pgs.getTerrain(x, y - 1) : 1);
            int tright = (x < pgs.width - 1 ? pgs.getTerrain(x + 1, y) : 1);
            int tdown = (y < pgs.height - 1 ? pgs.getTerrain(x, y + 1) : 1);
            int tleft = (x > 0 ? pgs.getTerrain(x - 1, y) : 1);
            if (tup == 0 && pgs.getUnitAt(x, y - 1) == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_PRODUCE, UnitAction::DIRECTION_UP, ut));
            if (tright == 0 && pgs.getUnitAt(x + 1, y) == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_PRODUCE, UnitAction::DIRECTION_RIGHT, ut));
            if (tdown == 0 && pgs.getUnitAt(x, y + 1) == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_PRODUCE, UnitAction::DIRECTION_DOWN, ut));
            if (tleft == 0 && pgs.getUnitAt(x - 1, y) == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_PRODUCE, UnitAction::DIRECTION_LEFT, ut));
        }
    }
    if (type.canMove) {
        int tup = (y > 0 ? pgs.getTerrain(x, y - 1) : 1);
        int tright = (x < pgs.width - 1 ? pgs.getTerrain(x + 1, y) : 1);
        int tdown = (y < pgs.height - 1 ? pgs.getTerrain(x, y + 1) : 1);
        int tleft = (x > 0 ? pgs.getTerrain(x - 1, y) : 1);
        if (tup == 0 && uup == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_MOVE, UnitAction::DIRECTION_UP));
        if (tright == 0 && uright == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_MOVE, UnitAction::DIRECTION_RIGHT));
        if (tdown == 0 && udown == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_MOVE, UnitAction::DIRECTION_DOWN));
        if (tleft == 0 && uleft == nullptr) l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_MOVE, UnitAction::DIRECTION_LEFT));
    }
    l.push_back(std::make_shared<UnitAction>(UnitAction::TYPE_NONE, noneDuration));
    return l;
}

bool canExecuteAction(const Unit& u, const UnitAction& ua, const GameState& gs) {  // Unit.java:531-534
    auto l = getUnitActions(u, gs, ua.ETA(u));
    for (auto& a : l)
        if (a->equals(ua)) return true;  // List.contains → o.equals(e)
    return false;
}

// rts/UnitAction.java:675-709
UnitActionP actionFromVector(const int* action, const UnitTypeTable& utt, const Unit& u, int maxAttackRange) {
    int actionType = action[1];
    auto ua = std::make_shared<UnitAction>(actionType);
    int center = maxAttackRange / 2;
    switch (actionType) {
        case UnitAction::TYPE_NONE: break;
        case UnitAction::TYPE_MOVE: ua->parameter = action[2]; break;
        case UnitAction::TYPE_HARVEST: ua->parameter = action[3]; break;
        case UnitAction::TYPE_RETURN: ua->parameter = action[4]; break;
        case UnitAction::TYPE_PRODUCE:
            ua->parameter = action[5];
            ua->unitType = utt.getUnitType(action[6]);  // throws like ArrayList.get
            break;
        case UnitAction::TYPE_ATTACK_LOCATION: {
            int rx = (action[7] % maxAttackRange - center);
            int ry = (action[7] / maxAttackRange - center);
            ua->x = u.x + rx;
            ua->y = u.y + ry;
        } break;
    }
    return ua;
}

int maskSlotsPerCell(const UnitTypeTable& utt) {  // tests/JNIGridnetClient.java:138
    int r = utt.getMaxAttackRange() * 2 + 1;
    return 1 + 6 + 4 + 4 + 4 + 4 + (int)utt.unitTypes.size() + r * r;
}

// rts/UnitAction.java:711-751
void getValidActionArray(const Unit& u, const GameState& gs, const UnitTypeTable& utt, uint8_t* mask, int maxAttackRange,
                         int idxOffset) {
    auto uas = getUnitActions(u, gs);
    int center = maxAttackRange / 2;
    int numUnitTypes = (int)utt.unitTypes.size();
    for (auto& ua : uas) {
        mask[idxOffset + ua->type] = 1;
        switch (ua->type) {
            case UnitAction::TYPE_NONE: break;
            case UnitAction::TYPE_MOVE: mask[idxOffset + 6 + ua->parameter] = 1; break;
            case UnitAction::TYPE_HARVEST: mask[idxOffset + 6 + 4 + ua->parameter] = 1; break;
            case UnitAction::TYPE_RETURN: mask[idxOffset + 6 + 8 + ua->parameter] = 1; break;
            case UnitAction::TYPE_PRODUCE:
                mask[idxOffset + 6 + 12 + ua->parameter] = 1;
                mask[idxOffset + 6 + 16 + ua->unitType->ID] = 1;
                break;
            case UnitAction::TYPE_ATTACK_LOCATION: {
                int rx = ua->x - u.x, ry = ua->y - u.y;
                mask[idxOffset + 6 + 16 + numUnitTypes + (center + ry) * maxAttackRange + (center + rx)] = 1;
            } break;
        }
    }
}

// ---------------------------------------------------------------- PlayerAction
void PlayerAction::fillWithNones(const GameState& s, int pID, int duration) {  // PlayerAction.java:217-235
    for (auto& u : s.pgs->units) {
        if (u->player == pID) {
            if (s.unitActions.get(u.get()) == nullptr) {
                bool found = false;
                for (auto& pa : actions)
                    if (pa->m_a.get() == u.get()) {
                        found = true;
                        break;
                    }
                if (!found) actions.push_back(std::make_shared<Pair>(Pair{u, std::make_shared<UnitAction>(UnitAction::TYPE_NONE, duration)}));
            }
        }
    }
}
bool PlayerAction::integrityCheck() const {  // :244-259
    int player = -1;
    for (auto& p : actions) {
        if (player == -1) player = p->m_a->player;
        else if (player != p->m_a->player) return false;
    }
    return true;
}

// PlayerAction.java:384-417 ; rows = nrows × 8 ints (Java layout [pos, a_t, ...])
PlayerAction PlayerAction::fromVectorAction(const std::vector<int>& rows, int nrows, const GameState& gs,
                                            const UnitTypeTable& utt, int currentPlayer, int maxAttackRadius) {
    PlayerAction pa;
    ResourceUsage base_ru;
    for (auto& u : gs.pgs->units) {
        UAAP uaa = gs.unitActions.get(u.get());
        if (uaa) base_ru.merge(uaa->action->resourceUsage(*u, *gs.pgs));
    }
    pa.r = base_ru;
    const int W = gs.pgs->width;
    for (int k = 0; k < nrows; k++) {
        const int* action = &rows[(size_t)k * 8];
        UnitP u = gs.pgs->getUnitAtP(action[0] % W, action[0] / W);
        if (u && u->player == currentPlayer && gs.unitActions.get(u.get()) == nullptr) {
            UnitActionP ua = actionFromVector(action, utt, *u, maxAttackRadius);
            if (ua->resourceUsage(*u, *gs.pgs).consistentWith(pa.r, gs)) {
                pa.r.merge(ua->resourceUsage(*u, *gs.pgs));
                pa.addUnitAction(u, ua);
            }
        }
    }
    return pa;
}

// ---------------------------------------------------------------- GameState
bool GameState::issue(PlayerAction& pa) {  // GameState.java:249-328
    bool returnValue = false;
    for (PairP p : pa.actions) {  // local copy of the reference, like Java's loop variable
        UnitActionP origAction = p->m_b;  // keeps `ru` alive when p.m_b is replaced below
        const ResourceUsage& ru = origAction->resourceUsage(*p->m_a, *pgs);
        for (auto& uaa : unitActions.order) {
            if (!uaa->action->resourceUsage(*uaa->unit, *pgs).consistentWith(ru, *this)) {
                if (uaa->time == time) {
                    bool cancel_old = false, cancel_new = false;
                    switch (utt->moveConflictResolutionStrategy) {
                        default:
                        case 1: cancel_old = cancel_new = true; break;
                        case 2:
                            if (!cancelRandom) throw std::runtime_error("CANCEL_RANDOM needs an RNG");
                            if (cancelRandom->nextInt(2) == 0) cancel_new = true;
                            else cancel_old = true;
                            break;
                        case 3:
                            if ((unitCancelationCounter % 2) == 0) cancel_new = true;
                            else cancel_old = true;
                            unitCancelationCounter++;
                            break;
                    }
                    int duration1 = uaa->action->ETA(*uaa->unit);
                    int duration2 = p->m_b->ETA(*p->m_a);
                    if (cancel_old) uaa->action = std::make_shared<UnitAction>(UnitAction::TYPE_NONE, std::min(duration1, duration2));
                    if (cancel_new)
                        p = std::make_shared<Pair>(Pair{p->m_a, std::make_shared<UnitAction>(UnitAction::TYPE_NONE, std::min(duration1, duration2))});
                } else {
                    errors++;  // "Inconsistent actions were executed!" (:301-313)
                    p->m_b = std::make_shared<UnitAction>(UnitAction::TYPE_NONE);
                }
            }
        }
        auto nu = std::make_shared<UnitActionAssignment>(UnitActionAssignment{p->m_a, p->m_b, time});
        unitActions.put(p->m_a, nu);
        if (p->m_b->type != UnitAction::TYPE_NONE) returnValue = true;
    }
    return returnValue;
}

bool GameState::issueSafe(PlayerAction& pa) {  // GameState.java:338-408
    if (!pa.integrityCheck()) throw std::runtime_error("PlayerAction inconsistent before 'issueSafe'");
    if (!integrityCheck()) throw std::runtime_error("GameState inconsistent before 'issueSafe'");
    for (auto& p : pa.actions) {
        if (!p->m_a) throw std::runtime_error("Issuing an action to a null unit!!!");
        if (!canExecuteAction(*p->m_a, *p->m_b, *this)) {
            int l = p->m_b->ETA(*p->m_a);
            p->m_b = std::make_shared<UnitAction>(UnitAction::TYPE_NONE, l);
        }
        bool foundRealUnit = false;
        UnitP substituteUnit;
        for (auto& u : pgs->units) {
            if (u.get() == p->m_a.get()) {
                foundRealUnit = true;
                break;
            }
            if (!substituteUnit && u->x == p->m_a->x && u->y == p->m_a->y) substituteUnit = u;
        }
        if (!foundRealUnit) {
            if (!substituteUnit) errors++;  // "Inconsistent order" (:374-378)
            else p->m_a = substituteUnit;
        }
        {
            const ResourceUsage& r = p->m_b->resourceUsage(*p->m_a, *pgs);
            std::vector<int> positions = r.positionsUsed;
            for (int position : positions) {
                int y = position / pgs->width;
                int x = position % pgs->width;
                if (pgs->getTerrain(x, y) != 0 || pgs->getUnitAt(x, y) != nullptr) {
                    auto new_ua = std::make_shared<UnitAction>(UnitAction::TYPE_NONE, p->m_b->ETA(*p->m_a));
                    errors++;  // "issued an illegal move action" print (:393-396)
                    p->m_b = new_ua;
                }
            }
        }
    }
    bool returnValue = issue(pa);
    if (!integrityCheck()) throw std::runtime_error("GameState inconsistent after 'issueSafe'");
    return returnValue;
}

bool GameState::canExecuteAnyAction(int pID) const {  // :416-423
    for (auto& u : pgs->units)
        if (u->player == pID && unitActions.get(u.get()) == nullptr) return true;
    return false;
}

bool GameState::isComplete() const {  // :148-157
    for (auto& u : pgs->units) {
        if (u->player != -1) {
            UAAP uaa = unitActions.get(u.get());
            if (!uaa || !uaa->action) return false;
        }
    }
    return true;
}

std::shared_ptr<GameState> GameState::clone() const {  // :591-610
    auto gs = std::make_shared<GameState>(pgs->clone(), utt);
    gs->time = time;
    gs->unitCancelationCounter = unitCancelationCounter;
    for (auto& uaa : unitActions.order) {
        size_t idx = 0;
        while (idx < pgs->units.size() && pgs->units[idx].get() != uaa->unit.get()) idx++;
        if (idx == pgs->units.size()) throw std::runtime_error("Inconsistent game state during cloning...");
        const UnitP& u2 = gs->pgs->units[idx];
        // a new assignment sharing the UnitAction object, as the Java does
        gs->unitActions.put(u2, std::make_shared<UnitActionAssignment>(UnitActionAssignment{u2, uaa->action, uaa->time}));
    }
    return gs;
}

bool GameState::cycle() {  // :553-571
    time++;
    std::vector<UAAP> ready;
    for (auto& uaa : unitActions.order)
        if (uaa->action->ETA(*uaa->unit) + uaa->time <= time) ready.push_back(uaa);
    for (auto& uaa : ready) {
        unitActions.remove(uaa->unit.get());
        UnitActionP act = uaa->action;  // Java evaluates uaa.action at the call
        act->execute(uaa->unit, *this);
    }
    return gameover();
}

bool GameState::integrityCheck() const {  // :703-719
    std::vector<const Unit*> used;
    for (auto& uaa : unitActions.order) {
        const Unit* u = uaa->unit.get();
        bool inList = false;
        for (auto& x : pgs->units)
            if (x.get() == u) { inList = true; break; }
        if (!inList) return false;
        if (std::find(used.begin(), used.end(), u) != used.end()) return false;
        used.push_back(u);
    }
    return true;
}

void GameState::getVectorObservation(int player, int32_t* out) const {  // :922-968
    const int H = pgs->height, W = pgs->width, HW = H * W;
    std::memset(out, 0, sizeof(int32_t) * 6 * (size_t)HW);
    for (auto& up : pgs->units) {
        const Unit& u = *up;
        UAAP uaa = unitActions.get(&u);
        int c = u.y * W + u.x;
        out[0 * HW + c] = u.hitpoints;
        out[1 * HW + c] = u.resources;
        if (u.player >= 0) out[2 * HW + c] = ((u.player + player) % 2) + 1;
        out[3 * HW + c] = u.type->ID + 1;
        if (uaa) out[4 * HW + c] = uaa->action->type;
    }
    for (int i = 0; i < HW; i++) out[5 * HW + i] = (*pgs->terrain)[(size_t)i];
}

// ---------------------------------------------------------------- PartiallyObservableGameState
PartiallyObservableGameState::PartiallyObservableGameState(const GameState& gs, int a_player)  // :35-54
    : GameState(gs.pgs->cloneKeepingUnits(), gs.utt), observer(a_player) {
    unitCancelationCounter = gs.unitCancelationCounter;
    time = gs.time;
    cancelRandom = gs.cancelRandom;
    damageRandom = gs.damageRandom;
    unitActions.order = gs.unitActions.order;  // putAll: same UAA objects, same order
    std::vector<const Unit*> toDelete;
    for (auto& u : pgs->units)
        if (u->player != observer)
            if (!observable(u->x, u->y)) toDelete.push_back(u.get());
    for (const Unit* u : toDelete) removeUnit(u);
}
bool PartiallyObservableGameState::observable(int x, int y) const {  // :61-71
    for (auto& u : pgs->units) {
        if (u->player == observer) {
            int d = (u->x - x) * (u->x - x) + (u->y - y) * (u->y - y);
            if (d <= u->type->sightRadius * u->type->sightRadius) return true;
        }
    }
    return false;
}
static void calculateVisibility(const std::vector<std::array<int, 3>>& us, int W, int H, int32_t* vis) {  // :156-179
    for (auto& un : us) {
        int ux = un[0], uy = un[1], sr = un[2], sr2 = sr * sr;
        for (int dy = -sr; dy <= sr; dy++)
            for (int dx = -sr; dx <= sr; dx++) {
                int x = ux + dx, y = uy + dy;
                if (x >= 0 && x < W && y >= 0 && y < H)
                    if (dx * dx + dy * dy <= sr2) vis[y * W + x] = 1;
            }
    }
}
void PartiallyObservableGameState::getVectorObservation(int player, int32_t* out) const {  // :82-154
    const int H = pgs->height, W = pgs->width, HW = H * W;
    std::memset(out, 0, sizeof(int32_t) * 8 * (size_t)HW);
    std::vector<std::array<int, 3>> friendly, enemy;
    for (auto& up : pgs->units) {
        const Unit& u = *up;
        UAAP uaa = unitActions.get(&u);
        int c = u.y * W + u.x;
        out[0 * HW + c] = u.hitpoints;
        out[1 * HW + c] = u.resources;
        if (u.player >= 0) {
            out[2 * HW + c] = ((u.player + player) % 2) + 1;
            if (u.player == player) friendly.push_back({u.x, u.y, u.type->sightRadius});
            else enemy.push_back({u.x, u.y, u.type->sightRadius});
        }
        out[3 * HW + c] = u.type->ID + 1;
        if (uaa) out[4 * HW + c] = uaa->action->type;
    }
    for (int i = 0; i < HW; i++) out[5 * HW + i] = (*pgs->terrain)[(size_t)i];
    calculateVisibility(friendly, W, H, out + 6 * HW);
    calculateVisibility(enemy, W, H, out + 7 * HW);
}

// ---------------------------------------------------------------- AIs
PlayerAction PassiveAI::getAction(int player, GameState& gs) {  // ai/PassiveAI.java:41-45
    PlayerAction pa;
    pa.fillWithNones(gs, player, 10);
    return pa;
}

// util/Sampler.java:116-135
static int samplerWeighted(JavaRandom& g, const std::vector<double>& distribution) {
    double total = 0, accum = 0, tmp;
    for (double f : distribution) total += f;
    if (total == 0) return g.nextInt((int)distribution.size());
    tmp = g.nextDouble() * total;
    for (size_t i = 0; i < distribution.size(); i++) {
        accum += distribution[i];
        if (accum >= tmp) return (int)i;
    }
    throw std::runtime_error("Input distribution empty in Sampler.weighted!");
}

PlayerAction RandomBiasedAI::getAction(int player, GameState& gs) {  // ai/RandomBiasedAI.java:51-107
    PhysicalGameState& pgs = *gs.pgs;
    PlayerAction pa;
    if (!gs.canExecuteAnyAction(player)) return pa;
    for (auto& u : pgs.units) {
        UAAP uaa = gs.getActionAssignment(u.get());
        if (uaa) pa.r.merge(uaa->action->resourceUsage(*u, pgs));
    }
    for (auto& u : pgs.units) {
        if (u->player == player) {
            if (gs.getActionAssignment(u.get()) == nullptr) {
                auto l = getUnitActions(*u, gs);
                UnitActionP none;
                std::vector<double> distribution(l.size());
                for (size_t i = 0; i < l.size(); i++) {
                    auto& a = l[i];
                    if (a->type == UnitAction::TYPE_NONE) none = a;
                    if (a->type == UnitAction::TYPE_ATTACK_LOCATION || a->type == UnitAction::TYPE_HARVEST ||
                        a->type == UnitAction::TYPE_RETURN)
                        distribution[i] = 5;
                    else
                        distribution[i] = 1;
                }
                UnitActionP ua = l[(size_t)samplerWeighted(*generator, distribution)];
                if (ua->resourceUsage(*u, pgs).consistentWith(pa.r, gs)) {
                    pa.r.merge(ua->resourceUsage(*u, pgs));
                    pa.addUnitAction(u, ua);
                } else {
                    pa.addUnitAction(u, none);
                }
            }
        }
    }
    return pa;
}

// ---------------------------------------------------------------- masks
void computeMasks(const GameState& gs, const UnitTypeTable& utt, int player, uint8_t* out) {  // JNIGridnetClient.java:210-223
    const int K = maskSlotsPerCell(utt);
    const int W = gs.pgs->width, H = gs.pgs->height;
    const int maxAttackRadius = utt.getMaxAttackRange() * 2 + 1;
    std::memset(out, 0, (size_t)H * W * K);
    for (auto& u : gs.pgs->units) {
        if (u->player == player && gs.getActionAssignment(u.get()) == nullptr) {
            uint8_t* m = out + ((size_t)u->y * W + u->x) * K;
            m[0] = 1;
            getValidActionArray(*u, gs, utt, m, maxAttackRadius, 1);
        }
    }
}

// ---------------------------------------------------------------- maps
static std::string attr(const std::string& tag, const std::string& name) {
    size_t p = 0;
    while (true) {
        p = tag.find(name, p);
        if (p == std::string::npos) return "";
        bool startOk = (p == 0) || isspace((unsigned char)tag[p - 1]);
        size_t q = p + name.size();
        while (q < tag.size() && isspace((unsigned char)tag[q])) q++;
        if (startOk && q < tag.size() && tag[q] == '=') {
            q++;
            while (q < tag.size() && isspace((unsigned char)tag[q])) q++;
            if (q < tag.size() && tag[q] == '"') {
                size_t e = tag.find('"', q + 1);
                return tag.substr(q + 1, e - q - 1);
            }
        }
        p = p + name.size();
    }
}

// terrain: PhysicalGameState.java:577-607 (RLE 'A'/'B') and :765-777
static std::vector<int> decodeTerrain(const std::string& t, int size) {
    std::vector<int> terrain;
    if (t.find('A') != std::string::npos || t.find('B') != std::string::npos) {
        std::string counter;
        for (char ch : t) {
            if (ch == 'A' || ch == 'B') {
                if (!counter.empty()) {
                    int n = std::stoi(counter);
                    for (int i = 0; i < n - 1; i++) terrain.push_back(terrain.back());
                    counter.clear();
                }
                terrain.push_back(ch == 'A' ? 0 : 1);
            } else if (!isspace((unsigned char)ch)) {
                counter.push_back(ch);
            }
        }
        if (!counter.empty()) {
            int n = std::stoi(counter);
            for (int i = 0; i < n - 1; i++) terrain.push_back(terrain.back());
        }
    } else {
        std::string digits;
        for (char ch : t)
            if (!isspace((unsigned char)ch)) digits.push_back(ch);
        terrain.resize((size_t)size);
        for (int i = 0; i < size; i++) terrain[(size_t)i] = digits.at((size_t)i) - '0';
    }
    return terrain;
}

MapTemplate parseMapXML(const std::string& xml) {  // PhysicalGameState.java:700-726
    MapTemplate m;
    size_t p = xml.find("<rts.PhysicalGameState");
    if (p == std::string::npos) throw std::runtime_error("no rts.PhysicalGameState element");
    size_t e = xml.find('>', p);
    std::string tag = xml.substr(p, e - p);
    m.width = std::stoi(attr(tag, "width"));
    m.height = std::stoi(attr(tag, "height"));
    size_t t0 = xml.find("<terrain>", e);
    size_t t1 = xml.find("</terrain>", t0);
    m.terrain = decodeTerrain(xml.substr(t0 + 9, t1 - t0 - 9), m.width * m.height);
    size_t q = t1;
    size_t end = xml.find("</rts.PhysicalGameState>", q);
    while (true) {
        size_t a = xml.find("<rts.Player", q);
        if (a == std::string::npos || a > end) break;
        size_t b = xml.find('>', a);
        std::string pt = xml.substr(a, b - a);
        int id = std::stoi(attr(pt, "ID"));
        if (id != (int)m.playerResources.size()) throw std::runtime_error("player added in the wrong order");
        m.playerResources.push_back(std::stoi(attr(pt, "resources")));
        q = b;
    }
    q = t1;
    while (true) {
        size_t a = xml.find("<rts.units.Unit ", q);
        if (a == std::string::npos || a > end) break;
        size_t b = xml.find('>', a);
        std::string ut = xml.substr(a, b - a);
        MapTemplate::U u;
        u.type = attr(ut, "type");
        u.id = std::stoll(attr(ut, "ID"));
        u.player = std::stoi(attr(ut, "player"));
        u.x = std::stoi(attr(ut, "x"));
        u.y = std::stoi(attr(ut, "y"));
        u.resources = std::stoi(attr(ut, "resources"));
        u.hitpoints = std::stoi(attr(ut, "hitpoints"));
        m.units.push_back(u);
        q = b;
    }
    return m;
}

MapTemplate loadMapFile(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open map " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parseMapXML(ss.str());
}

PGSP instantiate(const MapTemplate& t, const UnitTypeTable& utt) {
    auto p = std::make_shared<PhysicalGameState>();
    p->width = t.width;
    p->height = t.height;
    p->terrain = std::make_shared<std::vector<int>>(t.terrain);
    for (size_t i = 0; i < t.playerResources.size(); i++)
        p->players.push_back(std::make_shared<Player>(Player{(int)i, t.playerResources[i]}));
    for (auto& u : t.units) {
        auto nu = std::make_shared<Unit>();
        nu->type = utt.getUnitType(u.type);
        if (!nu->type) throw std::runtime_error("unknown unit type " + u.type);
        nu->ID = u.id;
        if (u.id >= g_next_ID) g_next_ID = u.id + 1;
        nu->player = u.player;
        nu->x = u.x;
        nu->y = u.y;
        nu->resources = u.resources;
        nu->hitpoints = u.hitpoints;
        for (auto& e : p->units)
            if (e->ID == nu->ID) throw std::runtime_error("Repeated unit ID in map!");
        p->addUnit(nu);
    }
    return p;
}

// ---------------------------------------------------------------- state dump
// ai/evaluation/SimpleSqrtEvaluationFunction3.java:31-44.  `score += i * 10f` is a float add; the
// sqrt term is a double (40f * cost is a float, times Math.sqrt of an int quotient) added to the
// float score and rounded back (compound assignment); x86-64 SSE float / double with no FMA contraction
// (the Makefile builds without -mfma) is exactly Java's strictfp arithmetic.
static float baseScoreSqrt3(int player, const GameState& gs) {
    const float RESOURCE = 20, RESOURCE_IN_WORKER = 10, UNIT_BONUS_MULTIPLIER = 40.0f;
    float score = gs.getPlayer(player).resources * RESOURCE;
    bool anyunit = false;
    for (auto& up : gs.pgs->units) {
        const Unit& u = *up;
        if (u.player == player) {
            anyunit = true;
            score += u.resources * RESOURCE_IN_WORKER;
            const float f = UNIT_BONUS_MULTIPLIER * u.type->cost;
            score = (float)((double)score + (double)f * std::sqrt((double)(u.hitpoints / u.type->hp)));
        }
    }
    if (!anyunit) return 0;
    return score;
}
float simpleSqrtEvaluation3(int maxplayer, int minplayer, const GameState& gs) {  // :24-29
    float s1 = baseScoreSqrt3(maxplayer, gs);
    float s2 = baseScoreSqrt3(minplayer, gs);
    if (s1 + s2 == 0) return 0.5f;
    return (2 * s1 / (s1 + s2)) - 1;
}

std::vector<int32_t> dumpState(const GameState& gs) {
    std::vector<int32_t> d;
    const PhysicalGameState& p = *gs.pgs;
    d.push_back(gs.time);
    d.push_back((int32_t)p.players.size());
    for (auto& pl : p.players) d.push_back(pl->resources);
    d.push_back((int32_t)p.units.size());
    for (auto& u : p.units) {
        d.push_back(u->type->ID);
        d.push_back(u->player);
        d.push_back(u->x);
        d.push_back(u->y);
        d.push_back(u->hitpoints);
        d.push_back(u->resources);
    }
    d.push_back((int32_t)gs.unitActions.order.size());
    for (auto& a : gs.unitActions.order) {
        int idx = -1;
        for (size_t i = 0; i < p.units.size(); i++)
            if (p.units[i].get() == a->unit.get()) { idx = (int)i; break; }
        d.push_back(idx);
        d.push_back(a->action->type);
        d.push_back(a->action->parameter);
        d.push_back(a->action->x);
        d.push_back(a->action->y);
        d.push_back(a->action->unitType ? a->action->unitType->ID : -1);
        d.push_back(a->time);
    }
    return d;
}

}  // namespace oref

namespace oref {
// GameState.toJSON (rts/GameState.java:819-837) + PhysicalGameState.toJSON (:658-691) + Player /
// Unit / UnitAction.toJSON (Player.java:86-88, Unit.java:577-588, UnitAction.java:569-582)
std::string gameStateToJSON(const GameState& gs) {
    const PhysicalGameState& p = *gs.pgs;
    std::ostringstream w;
    w << "{\"time\":" << gs.time << ",\"pgs\":";
    w << "{\"width\":" << p.width << ",\"height\":" << p.height << ",\"terrain\":\"";
    for (int i = 0; i < p.height * p.width; i++) w << (*p.terrain)[(size_t)i];
    w << "\",\"players\":[";
    for (size_t i = 0; i < p.players.size(); i++) {
        w << "{\"ID\":" << p.players[i]->ID << ", \"resources\":" << p.players[i]->resources << "}";
        if (i + 1 < p.players.size()) w << ",";
    }
    w << "],\"units\":[";
    for (size_t i = 0; i < p.units.size(); i++) {
        const Unit& u = *p.units[i];
        w << "{\"type\":\"" << u.type->name << "\", \"ID\":" << u.ID << ", \"player\":" << u.player << ", \"x\":" << u.x
          << ", \"y\":" << u.y << ", \"resources\":" << u.resources << ", \"hitpoints\":" << u.hitpoints << "}";
        if (i + 1 < p.units.size()) w << ",";
    }
    w << "]}";
    w << ",\"actions\":[";
    bool first = true;
    for (auto& uaa : gs.unitActions.order) {
        if (!first) w << ",";
        first = false;
        const UnitAction& a = *uaa->action;
        w << "{\"ID\":" << uaa->unit->ID << ", \"time\":" << uaa->time << ", \"action\":";
        w << "{\"type\":" << a.type;
        if (a.type == UnitAction::TYPE_ATTACK_LOCATION) {
            w << ", \"x\":" << a.x << ",\"y\":" << a.y;
        } else {
            if (a.parameter != UnitAction::DIRECTION_NONE) w << ", \"parameter\":" << a.parameter;
            if (a.unitType) w << ", \"unitType\":\"" << a.unitType->name << "\"";
        }
        w << "}}";
    }
    w << "]";
    w << "}";
    return w.str();
}

// GameState.fromJSON (:889-915): PhysicalGameState.fromJSON (:735-756), Player.fromJSON
// (Player.java:106-110), Unit.fromJSON (Unit.java:629-642), UnitAction.fromJSON (UnitAction.java:647-658)
GSP gameStateFromJSON(const std::string& json, const UnitTypeTable& utt) {
    const mjson::Value o = mjson::parse(json);
    const mjson::Value& po = o.at("pgs");
    auto p = std::make_shared<PhysicalGameState>();
    p->width = po.getInt("width", 8);
    p->height = po.getInt("height", 8);
    const std::string ts = po.getString("terrain", "");
    std::vector<int> terr((size_t)(p->width * p->height), 0);
    if (ts.find('A') != std::string::npos || ts.find('B') != std::string::npos) {
        MapTemplate t = parseMapXML("<rts.PhysicalGameState width=\"" + std::to_string(p->width) + "\" height=\"" +
                                    std::to_string(p->height) + "\"><terrain>" + ts +
                                    "</terrain><players></players><units></units></rts.PhysicalGameState>");
        terr = t.terrain;
    } else {
        for (size_t i = 0; i < terr.size(); i++) terr[i] = ts.at(i) - '0';
    }
    p->terrain = std::make_shared<std::vector<int>>(terr);
    for (auto& v : po.at("players").arr) p->players.push_back(std::make_shared<Player>(Player{v.getInt("ID", -1), v.getInt("resources", 0)}));
    for (auto& v : po.at("units").arr) {
        auto u = std::make_shared<Unit>();
        u->ID = v.getLong("ID", -1);
        if (u->ID >= g_next_ID) g_next_ID = u->ID + 1;
        u->player = v.getInt("player", -1);
        u->type = utt.getUnitType(v.getString("type", ""));
        if (!u->type) throw std::runtime_error("unknown unit type");
        u->x = v.getInt("x", 0);
        u->y = v.getInt("y", 0);
        u->resources = v.getInt("resources", 0);
        u->hitpoints = v.getInt("hitpoints", 1);
        p->addUnit(u);
    }
    auto gs = std::make_shared<GameState>(p, &utt);
    gs->time = o.getInt("time", 0);
    for (auto& v : o.at("actions").arr) {
        const int64_t id = v.getLong("ID", -1);
        UnitP u;
        for (auto& x : p->units)
            if (x->ID == id) {
                u = x;
                break;
            }
        if (!u) throw std::runtime_error("action for an unknown unit");
        const mjson::Value& ao = v.at("action");
        auto a = std::make_shared<UnitAction>(ao.getInt("type", UnitAction::TYPE_NONE));
        a->parameter = ao.getInt("parameter", UnitAction::DIRECTION_NONE);
        a->x = ao.getInt("x", UnitAction::DIRECTION_NONE);
        a->y = ao.getInt("y", UnitAction::DIRECTION_NONE);
        const std::string ut = ao.getString("unitType", "");
        if (!ut.empty()) a->unitType = utt.getUnitType(ut);
        gs->unitActions.put(u, std::make_shared<UnitActionAssignment>(UnitActionAssignment{u, a, v.getInt("time", 0)}));
    }
    return gs;
}
}  // namespace oref
