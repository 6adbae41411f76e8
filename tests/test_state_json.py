"""Game-state serialisation (SURVEY.md §4 checkpoint/resume, §8f-4 serialisers): GameState.toJSON /
fromJSON (rts/GameState.java:819-837, 897-915) and whole-handle checkpoints.

CPU: the oracle's writer against the Java text format on a known state (a hand-derived KAT), its
reader round trip.  GPU: the HIP handle's JSON equals the oracle's (unit IDs normalised: the build
writes list positions, Java's IDs come from a JVM-global counter), JSON states injected into both
continue in lockstep, and checkpoint/restore replays bit-identically (random streams included)."""
import json

import numpy as np
import pytest

from tests import oracle_py

M4 = "maps/4x4/base4x4.xml"
M8 = "maps/8x8/basesWorkers8x8.xml"

BASE4X4_JSON = ('{"time":0,"pgs":{"width":4,"height":4,"terrain":"0000000000000000","players":[{"ID":0, "resources":5},'
                '{"ID":1, "resources":5}],"units":[{"type":"Resource", "ID":4, "player":-1, "x":0, "y":0, "resources":10, '
                '"hitpoints":1},{"type":"Base", "ID":5, "player":0, "x":1, "y":1, "resources":0, "hitpoints":10},'
                '{"type":"Base", "ID":6, "player":1, "x":3, "y":3, "resources":0, "hitpoints":10},{"type":"Worker", '
                '"ID":7, "player":0, "x":1, "y":0, "resources":0, "hitpoints":1}]},"actions":[]}')


def normalise(text):
    """IDs -> list positions (units and the actions that name them)."""
    d = json.loads(text)
    pos = {u["ID"]: i for i, u in enumerate(d["pgs"]["units"])}
    for i, u in enumerate(d["pgs"]["units"]):
        u["ID"] = i
    for a in d["actions"]:
        a["ID"] = pos[a["ID"]]
    return d


def dump_xy_free(d):
    """A canonical dump with x/y of non-attack assignments zeroed: UnitAction.fromJSON leaves them at
    DIRECTION_NONE (-1) where a decoded action holds 0; only ATTACK_LOCATION reads them."""
    d = np.array(d)
    nu = int(d[4])
    base = 5 + 6 * nu
    for k in range(int(d[base])):
        r = base + 1 + 7 * k
        if d[r + 1] != 5:
            d[r + 3] = d[r + 4] = 0
    return d


def _masked_step(ref, S, step):
    m = ref.get_masks(0)
    return ref.step(np.stack([oracle_py.policy(m[s], 77, s, step, 0) for s in range(S)]))


def test_oracle_to_json_kat():
    ref = oracle_py.OracleVecClient(2, 0, 2000, [M4] * 2)
    ref.reset()
    assert ref.state_json(0) == BASE4X4_JSON  # Java's separators, map-file IDs, no actions yet
    ref.close()


def test_oracle_json_round_trip_with_assignments():
    ref = oracle_py.OracleVecClient(4, 0, 2000, [M8] * 4, seed=5)
    ref.reset()
    for step in range(40):
        _masked_step(ref, 4, step)
    j = ref.state_json(0)
    d = json.loads(j)
    assert d["actions"], "want in-flight assignments"
    assert any(a["action"]["type"] in (1, 2, 4) and "parameter" in a["action"] for a in d["actions"])
    dump = ref.dump(0)
    ref.set_state_json(2, j)  # game 1 (slots 2, 3) becomes a copy of game 0
    assert ref.state_json(2) == j
    assert np.array_equal(dump_xy_free(ref.dump(2)), dump_xy_free(dump))
    assert ref.env_steps(2) == 0
    ref.close()


# ------------------------------------------------------------------ GPU


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("mp,n_bot", [(M8, 2), ("maps/16x16/basesWorkers16x16.xml", 0)])
def test_gpu_json_matches_oracle_and_injection(mp, n_bot):
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp = 4
    S = n_sp + n_bot
    env = DeviceVecEnv(n_sp, n_bot, 2000, [mp] * S, ai2s=["RandomBiasedAI"] * n_bot, seed=31)
    ref = oracle_py.OracleVecClient(n_sp, n_bot, 2000, [mp] * S, bot_kinds=[1] * n_bot, seed=31)
    env.reset()
    ref.reset()
    for step in range(120):
        if step % 20 == 0:
            for s in range(0, S):
                assert normalise(env.state_json(s)) == normalise(ref.state_json(s)), (step, s)
        if step == 60:
            # inject: game 0 <- the state of game 1 (self-play), bot env <- its own state (IDs renumbered)
            j = ref.state_json(2)
            env.set_state_json(0, j)
            ref.set_state_json(0, j)
            if n_bot:
                jb = env.state_json(S - 1)
                env.set_state_json(S - 1, jb)
                ref.set_state_json(S - 1, jb)
            env.get_masks()
        m = ref.get_masks(0)
        env.synchronize()
        assert np.array_equal(env.masks.cpu().numpy(), m), step
        acts = np.stack([oracle_py.policy(m[s], 77, s, step, 0) for s in range(S)])
        env.actions.copy_(torch.as_tensor(acts))
        env.step()
        ref.step(acts)
        env.synchronize()
        assert np.array_equal(env.obs.cpu().numpy(), ref.obs), step
        assert np.array_equal(env.reward.cpu().numpy(), ref.reward), step
    for s in range(S):
        assert np.array_equal(dump_xy_free(env.dump_state(s)), dump_xy_free(ref.dump(s)))
    env.close()
    ref.close()


@pytest.mark.gpu
def test_gpu_set_state_json_rejects_invalid():
    _torch()
    from microrts_amd import DeviceVecEnv

    env = DeviceVecEnv(2, 0, 2000, [M4] * 2)
    good = json.loads(BASE4X4_JSON)
    bad = []
    b = json.loads(BASE4X4_JSON)
    b["pgs"]["width"] = 5
    bad.append(b)  # size differs
    b = json.loads(BASE4X4_JSON)
    b["pgs"]["units"][1]["x"] = 0
    b["pgs"]["units"][1]["y"] = 0
    bad.append(b)  # two units in a cell
    b = json.loads(BASE4X4_JSON)
    b["actions"] = [{"ID": 99, "time": 0, "action": {"type": 0, "parameter": 10}}]
    bad.append(b)  # unknown ID
    b = json.loads(BASE4X4_JSON)
    b["pgs"]["units"][0]["type"] = "Dragon"
    bad.append(b)
    for x in bad:
        with pytest.raises(RuntimeError):
            env.set_state_json(0, json.dumps(x))
    env.set_state_json(0, json.dumps(good))
    assert json.loads(env.state_json(0))["pgs"]["units"][3]["type"] == "Worker"
    with pytest.raises(RuntimeError):
        env.set_state_json(0, "{broken")
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("crs,bots", [(1, 0), (2, 2)])
def test_gpu_checkpoint_restore_replays_identically(crs, bots):
    """A checkpoint holds the random streams too: CANCEL_RANDOM and RandomBiasedAI opponents replay
    the same after restore."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv, UnitTypeTable

    S = 6 + bots
    env = DeviceVecEnv(6, bots, 2000, [M8] * S, ai2s=["RandomBiasedAI"] * bots, utt=UnitTypeTable(1, crs), seed=4)
    env.reset()
    for step in range(50):
        env.random_policy(9, step)
        env.step()
    ck = env.checkpoint()

    def run():
        out = []
        for step in range(50, 120):
            env.random_policy(9, step)
            env.step()
            env.synchronize()
            out.append((env.obs.cpu().numpy().copy(), env.reward.cpu().numpy().copy(), env.masks.cpu().numpy().copy()))
        return out, [env.dump_state(s) for s in range(S)]

    a, da = run()
    env.restore(ck)
    env.get_masks()
    b, db = run()
    for (o1, r1, m1), (o2, r2, m2) in zip(a, b):
        assert np.array_equal(o1, o2) and np.array_equal(r1, r2) and np.array_equal(m1, m2)
    assert all(np.array_equal(x, y) for x, y in zip(da, db))
    other = DeviceVecEnv(4, 0, 2000, [M8] * 4)
    with pytest.raises(RuntimeError):
        other.restore(ck)  # different configuration
    other.close()
    env.close()
    del torch


@pytest.mark.gpu
def test_gpu_restore_rejects_other_opponents_or_limits():
    """a checkpoint restored into a handle of the same shape but other opponents (PassiveAI
    vs RandomBiasedAI), another max_steps, other reward functions or other maps would silently run
    the checkpoint's game kinds until each game's next auto-reset.  The header carries a hash of
    those, and restore refuses a mismatch; the identical configuration restores."""
    _torch()
    from microrts_amd import DeviceVecEnv

    base = dict(ai2s=["RandomBiasedAI"] * 2, seed=4)
    env = DeviceVecEnv(2, 2, 2000, [M8] * 4, **base)
    env.reset()
    ck = env.checkpoint()
    same = DeviceVecEnv(2, 2, 2000, [M8] * 4, **base)
    same.restore(ck)
    same.close()
    for args, kw in (((2, 2, 2000, [M8] * 4), dict(ai2s=["PassiveAI"] * 2)),
                     ((2, 2, 1000, [M8] * 4), base),
                     ((2, 2, 2000, [M8] * 4), dict(base, rfs=["WinLossRewardFunction", "AttackRewardFunction"])),
                     ((2, 2, 2000, [M8] * 2 + ["maps/8x8/bases8x8.xml"] * 2), base)):
        other = DeviceVecEnv(*args, **kw)
        with pytest.raises(RuntimeError, match="different configuration"):
            other.restore(ck)
        other.close()
    env.close()
