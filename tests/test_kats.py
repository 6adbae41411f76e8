"""Hand-derived known-answer tests for the Java semantics of SURVEY.md Appendix A (and the a12 mask
layout), on 4x4 / 5x5 micro-maps written here.

Every expected value below is worked out from the Java text (the file:line next to each KAT), not
from either implementation.  Each KAT runs on the CPU oracle (unmarked: part of the CPU suite) and on
the HIP path through the C ABI (marked gpu).  Actions are fed as Java rows [pos, type, move dir,
harvest dir, return dir, produce dir, produce type, attack index] through the rows entry points, so a
KAT controls the row order exactly.

Dump layout (mrts_get_state / oracle dumpState): [time, 2, res0, res1, n_units,
(type, player, x, y, hp, resources) * n_units, n_assign, (unit index, action type, parameter, x, y,
unit type or -1, issue time) * n_assign].  Unit type ids (UnitTypeTable.java:104-289): Resource 0,
Base 1, Barracks 2, Worker 3, Light 4, Heavy 5, Ranged 6.  Action types (UnitAction.java:31-60):
NONE 0, MOVE 1, HARVEST 2, RETURN 3, PRODUCE 4, ATTACK 5.  Directions: up 0, right 1, down 2, left 3.
Attack index = (3 + dy) * 7 + (3 + dx) (maxAttackRadius 7, JNIGridnetClient.java:125).
"""

import numpy as np
import pytest

from tests import oracle_py

NONE, MOVE, HARVEST, RETURN, PRODUCE, ATTACK = range(6)
RESOURCE, BASE, BARRACKS, WORKER, LIGHT, HEAVY, RANGED = range(7)
UP, RIGHT, DOWN, LEFT = range(4)
NAMES = {RESOURCE: "Resource", BASE: "Base", BARRACKS: "Barracks", WORKER: "Worker", LIGHT: "Light",
         HEAVY: "Heavy", RANGED: "Ranged"}
HP = {RESOURCE: 1, BASE: 10, BARRACKS: 4, WORKER: 1, LIGHT: 4, HEAVY: 4, RANGED: 1}


def atk(dx, dy):
    return (3 + dy) * 7 + (3 + dx)


def write_map(path, W, H, units, walls=(), res=(5, 5)):
    """units: (type, player, x, y[, resources[, hp]]) in list order."""
    terr = ["0"] * (W * H)
    for x, y in walls:
        terr[y * W + x] = "1"
    lines = [f'<rts.PhysicalGameState width="{W}" height="{H}">', f"  <terrain>{''.join(terr)}</terrain>", "  <players>"]
    for i, r in enumerate(res):
        lines += [f'    <rts.Player ID="{i}" resources="{r}">', "    </rts.Player>"]
    lines += ["  </players>", "  <units>"]
    for i, u in enumerate(units):
        t, p, x, y = u[:4]
        r = u[4] if len(u) > 4 else 0
        hp = u[5] if len(u) > 5 else HP[t]
        lines += [f'    <rts.units.Unit type="{NAMES[t]}" ID="{100 + i}" player="{p}" x="{x}" y="{y}" resources="{r}" '
                  f'hitpoints="{hp}" >', "    </rts.units.Unit>"]
    lines += ["  </units>", "</rts.PhysicalGameState>"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return str(path)


def parse(d):
    d = [int(v) for v in d]
    out = {"time": d[0], "res": (d[2], d[3])}
    n = d[4]
    out["units"] = [tuple(d[5 + 6 * i:11 + 6 * i]) for i in range(n)]
    k = 5 + 6 * n
    out["assign"] = [tuple(d[k + 1 + 7 * i:k + 8 + 7 * i]) for i in range(d[k])]
    return out


def row(pos, t=NONE, move=0, harvest=0, ret=0, pdir=0, ptype=0, attack=0):
    return [pos, t, move, harvest, ret, pdir, ptype, attack]


class Runner:
    """Self-play pair (slots 0 = player 0, 1 = player 1) on the oracle or on the GPU."""

    def __init__(self, backend, map_path, partial_obs=False, max_steps=2000, rfs=None):
        self.backend = backend
        self.po = partial_obs
        if backend == "oracle":
            self.e = oracle_py.OracleVecClient(2, 0, max_steps, [map_path] * 2, partial_obs=partial_obs,
                                               rewards=[oracle_py.REWARD_IDS[r] for r in rfs] if rfs else None)
            self.e.reset()
        else:
            import torch

            assert torch.cuda.is_available(), "GPU KATs need an MI355X"
            from microrts_amd import DeviceVecEnv

            self.torch = torch
            self.e = DeviceVecEnv(2, 0, max_steps, [map_path] * 2, partial_obs=partial_obs, rfs=rfs)
            self.e.reset()

    def step(self, rows0=(), rows1=()):
        n = max(len(rows0), len(rows1), 1)
        r = np.zeros((2, n, 8), np.int32)
        r[:, :, 0] = -1  # padding rows name no unit (ignored, PlayerAction.java:401-407)
        for s, rs in enumerate((rows0, rows1)):
            for i, x in enumerate(rs):
                r[s, i] = x
        if self.backend == "oracle":
            obs, rew, done = self.e.step_rows(r)
            return obs, rew.copy(), done.copy()
        t = self.torch.as_tensor(r, device=self.e.device)
        self.e.step_rows(t)
        self.e.synchronize()
        return self.e.obs.cpu().numpy(), self.e.reward.cpu().numpy().copy(), self.e.done.cpu().numpy().copy()

    def idle(self, k):
        for _ in range(k):
            self.step()

    def state(self):
        return parse(self.e.dump(0) if self.backend == "oracle" else self.e.dump_state(0))

    def masks(self, player=0):
        if self.backend == "oracle":
            return self.e.get_masks(player)
        self.e.synchronize()
        return self.e.masks.cpu().numpy()

    def close(self):
        self.e.close()


# ---------------------------------------------------------------------------------------------- KATs
def kat_illegal_becomes_none_eta(tmp, backend):
    """A.5 — GameState.issueSafe (GameState.java:347-354): an action outside getUnitActions becomes
    NONE(ETA(original)).  Worker move into a wall -> NONE(moveTime 10); Base "move" -> NONE(Base
    moveTime = UnitType default 10, UnitType.java:59-63); produce without resources -> NONE(produceTime
    of the produced type, Worker 50).  ETA: UnitAction.java:307-329."""
    m = write_map(tmp / "k1.xml", 5, 5, [(WORKER, 0, 0, 0), (BASE, 0, 4, 4), (BASE, 1, 4, 0)], walls=[(1, 0)], res=(5, 0))
    r = Runner(backend, m)
    r.step([row(0, MOVE, move=RIGHT), row(24, MOVE, move=UP)], [row(4, PRODUCE, pdir=DOWN, ptype=WORKER)])
    s = r.state()
    assert s["time"] == 1
    # insertion order: player 0's pa in row order, then player 1's (JNIGridnetClientSelfPlay.java:161-169)
    assert s["assign"] == [(0, NONE, 10, 0, 0, -1, 0), (1, NONE, 10, 0, 0, -1, 0), (2, NONE, 50, 0, 0, -1, 0)]
    r.idle(8)
    assert r.state()["time"] == 9 and len(r.state()["assign"]) == 3
    r.idle(1)  # time 10: the two NONE(10) are ready (ETA + issue time <= time, GameState.java:556-559)
    s = r.state()
    assert s["time"] == 10 and s["assign"] == [(2, NONE, 50, 0, 0, -1, 0)]
    r.close()


def kat_resource_quirk_row_order(tmp, backend):
    """A.4 — PlayerAction.fromVectorAction + ResourceUsage.consistentWith (ResourceUsage.java:38-46):
    the resource check is skipped while the running reservation of the player is 0, so the first
    produce row is never resource-checked at decode.  Player 0 has 1 resource.
    Order (Base row, Worker row): Base->Worker (cost 1) accepted unchecked; Worker->Barracks (cost 5)
    then fails 1 + 5 > 1 and the worker gets NONE(1).  The Base's produce is legal; after 50 cycles
    the Worker is appended to the unit list and paid (UnitAction.java:434-463).
    Order (Worker row, Base row): the Barracks row is accepted unchecked, the Base row rejected
    (5 + 1 > 1); issueSafe finds the Barracks produce illegal (resources 1 < 5, Unit.java:475-495)
    -> NONE(Barracks produceTime 200)."""
    units = [(BASE, 0, 1, 1), (WORKER, 0, 3, 3), (BASE, 1, 4, 0)]
    m = write_map(tmp / "k2.xml", 5, 5, units, res=(1, 0))
    base_row = row(6, PRODUCE, pdir=DOWN, ptype=WORKER)
    worker_row = row(18, PRODUCE, pdir=RIGHT, ptype=BARRACKS)
    r = Runner(backend, m)
    r.step([base_row, worker_row])
    s = r.state()
    assert s["assign"] == [(0, PRODUCE, DOWN, 0, 0, WORKER, 0)] and s["res"] == (1, 0)
    r.idle(49)
    s = r.state()
    assert s["time"] == 50 and s["res"] == (0, 0)
    assert s["units"] == [(BASE, 0, 1, 1, 10, 0), (WORKER, 0, 3, 3, 1, 0), (BASE, 1, 4, 0, 10, 0), (WORKER, 0, 1, 2, 1, 0)]
    r.close()

    r = Runner(backend, m)
    r.step([worker_row, base_row])
    s = r.state()
    assert s["assign"] == [(1, NONE, 200, 0, 0, -1, 0)] and s["res"] == (1, 0)
    r.close()


def kat_rows_that_do_not_count(tmp, backend):
    """A.4 — a row counts only if an own unit with no assignment stands at (pos % W, pos / W)
    (PlayerAction.java:401-407): rows naming an enemy, an empty cell, an off-map position or a busy
    unit are ignored."""
    m = write_map(tmp / "k3.xml", 5, 5, [(WORKER, 0, 2, 2), (WORKER, 1, 2, 3), (BASE, 1, 4, 0)])
    r = Runner(backend, m)
    r.step([row(17, MOVE, move=RIGHT), row(0, MOVE, move=RIGHT), row(-5, MOVE), row(25, MOVE), row(12, MOVE, move=UP)])
    assert r.state()["assign"] == [(0, MOVE, UP, 0, 0, -1, 0)]
    r.step([row(12, MOVE, move=DOWN)])  # the worker is busy: ignored, the MOVE up stays
    assert r.state()["assign"] == [(0, MOVE, UP, 0, 0, -1, 0)]
    r.idle(8)
    s = r.state()
    assert s["time"] == 10 and s["units"][0] == (WORKER, 0, 2, 1, 1, 0) and s["assign"] == []
    r.close()


def kat_player1_sees_player0_reservations(tmp, backend):
    """A.3 — self-play decodes player 1 after player 0 is issued (JNIGridnetClientSelfPlay.java:161-169),
    so player 0's MOVE target is in player 1's base reservations (PlayerAction.java:387-394): player 1's
    move into the same cell is rejected and that worker gets NONE(1)."""
    m = write_map(tmp / "k4.xml", 5, 5, [(WORKER, 0, 1, 2), (WORKER, 1, 3, 2)])
    r = Runner(backend, m)
    r.step([row(11, MOVE, move=RIGHT)], [row(13, MOVE, move=LEFT)])
    assert r.state()["assign"] == [(0, MOVE, RIGHT, 0, 0, -1, 0)]
    r.idle(9)
    s = r.state()
    assert s["units"] == [(WORKER, 0, 2, 2, 1, 0), (WORKER, 1, 3, 2, 1, 0)]
    r.close()


def kat_dead_unit_still_executes(tmp, backend):
    """A.7 — GameState.cycle snapshots the ready assignments first and executes each even if its unit
    died earlier in the loop (GameState.java:556-568).  Light L (player 0) and Worker W (player 1)
    attack at time 0 (ETA attackTime 5); L's pair was inserted first, so at time 5 L kills W (hp 1 - 2),
    then W's attack still hits Base B (hp 10 - 1).  W leaves the unit list in place (PhysicalGameState.java:208-210)."""
    units = [(LIGHT, 0, 1, 2), (WORKER, 1, 2, 2), (BASE, 0, 3, 2), (BASE, 1, 4, 4)]
    m = write_map(tmp / "k5.xml", 5, 5, units)
    r = Runner(backend, m)
    r.step([row(11, ATTACK, attack=atk(1, 0))], [row(12, ATTACK, attack=atk(1, 0))])
    s = r.state()
    assert s["assign"][:1] == [(0, ATTACK, -1, 2, 2, -1, 0)] and (1, ATTACK, -1, 3, 2, -1, 0) in s["assign"]
    r.idle(4)
    s = r.state()
    assert s["time"] == 5
    assert s["units"] == [(LIGHT, 0, 1, 2, 4, 0), (BASE, 0, 3, 2, 9, 0), (BASE, 1, 4, 4, 10, 0)]
    r.close()


def kat_simultaneous_kill_is_a_draw(tmp, backend):
    """A.7 + A.8 — both last units kill each other in one cycle (the dead one still attacks); gameover
    with no owned units, winner -1 (PhysicalGameState.java:334-387), WinLoss gives -1 to both players
    (WinLossRewardFunction.java:16-24) and done; the VecClient then resets (JNIGridnetVecClient.java:247-266)."""
    m = write_map(tmp / "k6.xml", 4, 4, [(WORKER, 0, 1, 1), (WORKER, 1, 2, 1), (RESOURCE, -1, 0, 3, 5)])
    r = Runner(backend, m)
    _, rew, done = r.step([row(5, ATTACK, attack=atk(1, 0))], [row(6, ATTACK, attack=atk(-1, 0))])
    assert list(rew) == [0.0, 0.0] and list(done) == [0, 0]
    for _ in range(3):
        _, rew, done = r.step()
        assert list(done) == [0, 0]
    _, rew, done = r.step()  # time 5
    assert list(rew) == [-1.0, -1.0] and list(done) == [1, 1]
    s = r.state()  # auto-reset: the fresh map
    assert s["time"] == 0 and len(s["units"]) == 3 and s["assign"] == []
    r.close()


def kat_harvest_deplete_return(tmp, backend):
    """A.7 — harvest takes harvestAmount 1 and removes the resource at <= 0 in place
    (UnitAction.java:378-404); return credits the player (UnitAction.java:406-432) after moveTime
    (ETA of RETURN = moveTime, UnitAction.java:321-322)."""
    units = [(RESOURCE, -1, 0, 0, 1), (WORKER, 0, 0, 1), (BASE, 0, 1, 1), (RESOURCE, -1, 4, 4, 5), (BASE, 1, 4, 0)]
    m = write_map(tmp / "k7.xml", 5, 5, units, res=(3, 0))
    r = Runner(backend, m)
    r.step([row(5, HARVEST, harvest=UP)])
    r.idle(19)
    s = r.state()
    assert s["time"] == 20
    assert s["units"] == [(WORKER, 0, 0, 1, 1, 1), (BASE, 0, 1, 1, 10, 0), (RESOURCE, -1, 4, 4, 1, 5), (BASE, 1, 4, 0, 10, 0)]
    r.step([row(5, RETURN, ret=RIGHT)])
    assert r.state()["assign"][0] == (0, RETURN, RIGHT, 0, 0, -1, 20)
    r.idle(8)
    assert r.state()["res"] == (3, 0)
    r.idle(1)  # time 30
    s = r.state()
    assert s["time"] == 30 and s["res"] == (4, 0) and s["units"][0] == (WORKER, 0, 0, 1, 1, 0)
    r.close()


def kat_duplicate_row_keeps_map_position(tmp, backend):
    """A.2/A.4 — a unit named by two rows gets two pairs (PlayerAction.java:409-413); issue() puts
    both and LinkedHashMap.put on an existing key replaces the value but keeps the entry's position
    (GameState.java:321-322): rows [X right, Y left, X down] end as [X down, Y left]."""
    m = write_map(tmp / "k8.xml", 5, 5, [(WORKER, 0, 0, 0), (WORKER, 0, 4, 4), (BASE, 1, 4, 0)])
    r = Runner(backend, m)
    r.step([row(0, MOVE, move=RIGHT), row(24, MOVE, move=LEFT), row(0, MOVE, move=DOWN)])
    assert r.state()["assign"] == [(0, MOVE, DOWN, 0, 0, -1, 0), (1, MOVE, LEFT, 0, 0, -1, 0)]
    r.idle(9)
    s = r.state()
    assert s["units"][:2] == [(WORKER, 0, 0, 1, 1, 0), (WORKER, 0, 3, 4, 1, 0)]
    r.close()


def kat_po_killed_unit_in_view(tmp, backend):
    """A.9 — a partially observable view shares Unit objects with the game and is taken at the start
    of gameStep (PartiallyObservableGameState.java:35-54): in the step whose cycle kills a visible
    enemy, that enemy still appears with its post-cycle hp (1 - 2 = -1); a step later it is gone."""
    units = [(LIGHT, 0, 1, 2), (WORKER, 1, 2, 2), (BASE, 0, 0, 0), (BASE, 1, 4, 4)]
    m = write_map(tmp / "k9.xml", 5, 5, units)
    r = Runner(backend, m, partial_obs=True)
    r.step([row(11, ATTACK, attack=atk(1, 0))])
    for _ in range(3):
        r.step()
    obs, _, _ = r.step()  # time 5: the attack kills W in this cycle
    assert obs.shape[1] == 8
    assert obs[0, 0, 2, 2] == -1 and obs[0, 3, 2, 2] == WORKER + 1 and obs[0, 2, 2, 2] == 2
    obs, _, _ = r.step()
    assert obs[0, 0, 2, 2] == 0 and obs[0, 3, 2, 2] == 0
    r.close()


def kat_mask_record(tmp, backend):
    """a12 — getMasks record (JNIGridnetClient.java:210-223, UnitAction.getValidActionArray
    UnitAction.java:711-751 over Unit.getUnitActions Unit.java:382-522).  Worker W at (2,2): resource
    up, own Base right, enemy Worker down, empty left; player 0 has 5 resources (Barracks 5 yes,
    Base 10 no).  Expected W slots: [0] own idle; type bits NONE 1 (getUnitActions always ends with
    NONE), move 2, harvest 3, produce 5, attack 6;
    move left 7+3; harvest up 11+0; produce dir left 19+3; produce type Barracks 23+2; attack (0,+1)
    30+(3+1)*7+3.  Base B at (3,2): produce Worker into up / right / down."""
    units = [(WORKER, 0, 2, 2), (RESOURCE, -1, 2, 1, 10), (BASE, 0, 3, 2), (WORKER, 1, 2, 3), (BASE, 1, 0, 4)]
    m = write_map(tmp / "k10.xml", 5, 5, units, res=(5, 5))
    r = Runner(backend, m)
    k = r.masks(0)[0]  # slot 0 = player 0, [H][W][79]
    assert set(np.flatnonzero(k[2, 2])) == {0, 1, 2, 3, 5, 6, 10, 11, 22, 25, 30 + 4 * 7 + 3}
    assert set(np.flatnonzero(k[2, 3])) == {0, 1, 5, 19 + UP, 19 + RIGHT, 19 + DOWN, 23 + WORKER}
    others = np.ones((5, 5), bool)
    others[2, 2] = others[2, 3] = False
    assert not k[others].any()
    r.close()


def kat_reward_functions(tmp, backend):
    """§8f — src/ai/reward/*.java over the TraceEntry of the step (the pairs issued this step, after
    issueSafe; JNIGridnetClientSelfPlay.java:160-169) and the post-cycle state.  Step 1: player 0
    issues HARVEST (ResourceGather +1), PRODUCE Worker (ProduceWorker +1) and an ATTACK on player 1's
    worker E (Attack +1) — counted when issued, not when executed.  Step 5: the attack executes, E
    dies; player 1 had E at distance sqrt(5) from player 0's Base and now has no mobile unit, so
    CloserToEnemyBase = sqrt(5) - 2000000000 (the initial value of newMinDistance,
    CloserToEnemyBaseRewardFunction.java:52).  Step 6: both minima are 2e9 -> 0."""
    rfs = ["WinLossRewardFunction", "ResourceGatherRewardFunction", "ProduceWorkerRewardFunction", "AttackRewardFunction",
           "CloserToEnemyBaseRewardFunction"]
    units = [(RESOURCE, -1, 0, 0, 5), (WORKER, 0, 0, 1), (BASE, 0, 1, 1), (LIGHT, 0, 2, 2), (WORKER, 1, 3, 2),
             (BASE, 1, 4, 4)]
    m = write_map(tmp / "k11.xml", 5, 5, units)
    r = Runner(backend, m, rfs=rfs)
    _, rew, done = r.step([row(5, HARVEST, harvest=UP), row(6, PRODUCE, pdir=DOWN, ptype=WORKER),
                           row(12, ATTACK, attack=atk(1, 0))])
    assert rew.tolist() == [[0.0, 1.0, 1.0, 1.0, 0.0], [0.0, 0.0, 0.0, 0.0, 0.0]]
    assert done.tolist() == [[0, 0, 0, 0, 0], [0, 0, 0, 0, 0]]
    for _ in range(3):
        _, rew, _ = r.step()
        assert not rew.any()
    _, rew, _ = r.step()  # time 5
    assert rew[0].tolist() == [0.0] * 5
    assert rew[1].tolist() == [0.0, 0.0, 0.0, 0.0, float(np.sqrt(5.0)) - 2000000000.0]
    _, rew, _ = r.step()
    assert not rew.any()
    r.close()


class VecRunner:
    """Two self-play slots + one agent-vs-PassiveAI env through the JNIGridnetVecClient mirror (GPU:
    mrts_reset / mrts_step) or the oracle VecClient; all-zero grid actions (NONE rows)."""

    def __init__(self, backend, map_path, max_steps, rfs=("WinLossRewardFunction",)):
        self.backend = backend
        if backend == "oracle":
            self.e = oracle_py.OracleVecClient(2, 1, max_steps, [map_path] * 3, bot_kinds=[oracle_py.BOT_PASSIVE],
                                               rewards=[oracle_py.REWARD_IDS[r] for r in rfs])
        else:
            from microrts_amd import JNIGridnetVecClient

            self.e = JNIGridnetVecClient(2, 1, max_steps, list(rfs), "", [map_path] * 3, a_ai2s=["PassiveAI"])
        self.S = 3
        self.R = len(rfs)

    def reset(self):
        """-> (reward [S][R], done [S][R]) of the reset Responses."""
        if self.backend == "oracle":
            _, rew, done = self.e.reset([0] * self.S)
        else:
            r = self.e.reset([0] * self.S)
            rew, done = r.reward, r.done
        return (np.asarray(rew, np.float64).reshape(self.S, self.R).copy(),
                np.asarray(done).astype(bool).reshape(self.S, self.R).copy())

    def step_full(self, actions=None):
        """-> (reward [S][R], done [S][R])."""
        a = np.zeros((self.S, 25, 7), np.int32) if actions is None else np.asarray(actions, np.int32)
        if self.backend == "oracle":
            _, rew, done = self.e.step(a, [0] * self.S)
        else:
            r = self.e.gameStep(a, [0] * self.S)
            rew, done = r.reward, r.done
        return (np.asarray(rew, np.float64).reshape(self.S, self.R).copy(),
                np.asarray(done).astype(bool).reshape(self.S, self.R).copy())

    def step(self):
        """-> done[0] per slot (bool[S])."""
        return self.step_full()[1][:, 0]

    def env_steps(self):
        if self.backend == "oracle":
            return [self.e.env_steps(s) for s in range(self.S)]
        return self.e.envSteps.tolist()

    def close(self):
        self.e.close()


def kat_env_steps_survive_reset(tmp, backend):
    """A.10 — JNIGridnetVecClient.reset (JNIGridnetVecClient.java:179-211) reloads every game but never
    touches envSteps[]; only the constructor (:116) and the auto-reset path (:229,264-265,285) zero it.
    So with maxSteps = 10: 4 steps, reset() -> envSteps stays 4 and the next auto-reset comes after 6
    more steps (envSteps 10 >= maxSteps, done[0] forced true), then after every 10 steps.  The map
    keeps both players alive and idle (all rows NONE; the bot is PassiveAI), so gameover never fires."""
    m = write_map(tmp / "k12.xml", 5, 5, [(BASE, 0, 0, 0), (BASE, 1, 4, 4)])
    r = VecRunner(backend, m, 10)
    r.reset()
    assert r.env_steps() == [0, 0, 0]
    for _ in range(4):
        assert not r.step().any()
    assert r.env_steps() == [4, 4, 4]
    r.reset()
    assert r.env_steps() == [4, 4, 4]  # NOT zeroed by reset()
    for k in range(5):
        assert not r.step().any(), f"step {k}"
    assert r.env_steps() == [9, 9, 9]
    assert r.step().all()  # 6th step after reset(): envSteps reaches 10 -> auto-reset
    assert r.env_steps() == [0, 0, 0]
    for k in range(9):
        assert not r.step().any(), f"step {k}"
    assert r.step().all()
    r.close()


def kat_selfplay_reset_keeps_slots_from_two(tmp, backend):
    """A.10 / SURVEY a1 — an explicit reset() of a self-play game zeroes reward/done only for
    j < rewards.length, and rewards = new double[2][] (numPlayers, JNIGridnetClientSelfPlay.java:103-104,
    135-136) so the bound is 2, not rfs.length (:235-238): reward/done slots >= 2 keep the previous
    step's values.  JNIGridnetClient.reset (the agent-vs-bot env) zeroes every slot (:248-251).
    rfs = [WinLoss, Attack, ProduceWorker, ResourceGather] on a map with no Resource units: on step 1
    player 0's Base produces a Worker (PRODUCE right, Worker), so ProduceWorker (slot 2) = 1.0 for
    player 0 (ProduceWorkerRewardFunction.java:20-30: every pair of the TraceEntry), 0.0 for player 1;
    ResourceGather (slot 3) is done = true every step (no Resource left, ResourceGatherRewardFunction.java:
    31-40).  After reset(): self-play slots keep [2] = 1.0 / 0.0 and done[3] = true, slots 0 and 1
    zero; the bot env (slot 2) is all zero."""
    m = write_map(tmp / "k13.xml", 5, 5, [(BASE, 0, 0, 0), (BASE, 1, 4, 4)])
    r = VecRunner(backend, m, 100, rfs=("WinLossRewardFunction", "AttackRewardFunction", "ProduceWorkerRewardFunction",
                                        "ResourceGatherRewardFunction"))
    rew, done = r.reset()
    assert not rew.any() and not done.any()  # new double[rfs.length]: zeros before any step
    a = np.zeros((3, 25, 7), np.int32)
    a[0, 0] = a[2, 0] = [PRODUCE, 0, 0, 0, RIGHT, WORKER, 0]  # player 0's Base at cell 0 (slot 0 and the bot env)
    rew, done = r.step_full(a)
    assert rew.tolist() == [[0, 0, 1, 0], [0, 0, 0, 0], [0, 0, 1, 0]]
    assert done.tolist() == [[False, False, False, True]] * 3
    rew, done = r.reset()
    assert rew.tolist() == [[0, 0, 1, 0], [0, 0, 0, 0], [0, 0, 0, 0]]
    assert done.tolist() == [[False, False, False, True], [False, False, False, True], [False] * 4]
    rew, done = r.step_full()  # every slot recomputed by the step
    assert rew.tolist() == [[0, 0, 0, 0]] * 3
    assert done.tolist() == [[False, False, False, True]] * 3
    r.close()


KATS = [kat_illegal_becomes_none_eta, kat_resource_quirk_row_order, kat_rows_that_do_not_count,
        kat_player1_sees_player0_reservations, kat_dead_unit_still_executes, kat_simultaneous_kill_is_a_draw,
        kat_harvest_deplete_return, kat_duplicate_row_keeps_map_position, kat_po_killed_unit_in_view, kat_mask_record,
        kat_reward_functions, kat_env_steps_survive_reset, kat_selfplay_reset_keeps_slots_from_two]


@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_kat_oracle(kat, tmp_path):
    kat(tmp_path, "oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k.__name__ for k in KATS])
def test_kat_gpu(kat, tmp_path):
    kat(tmp_path, "gpu")


@pytest.mark.gpu
def test_env_steps_survive_reset_bot_only():
    """A.10 for the bot-only constructor (JNIGridnetVecClient.java:157-177): reset (:180-190) leaves
    envSteps[] alone, the bot-only gameStep zeroes it on auto-reset (:217-229)."""
    from microrts_amd import JNIGridnetVecClient

    maps = ["maps/16x16/basesWorkers16x16.xml"] * 2
    cl = JNIGridnetVecClient.bots(10, ["WinLossRewardFunction"], "", maps, ["PassiveAI"] * 2, ["PassiveAI"] * 2)
    cl.reset([0, 0])
    for _ in range(3):
        assert not cl.gameStep(None, [0, 0]).done[:, 0].any()
    assert cl.envSteps.tolist() == [3, 3]
    cl.reset([0, 0])
    assert cl.envSteps.tolist() == [3, 3]
    for _ in range(6):
        assert not cl.gameStep(None, [0, 0]).done[:, 0].any()
    assert cl.gameStep(None, [0, 0]).done[:, 0].all()
    assert cl.envSteps.tolist() == [0, 0]
    cl.close()
