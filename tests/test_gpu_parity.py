"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

Every test feeds the SAME int32 action tensors to libmrts.so and to the oracle and compares,
after every step: observations, rewards, dones, legal-action masks and (periodically) the full
canonical state dump (units in list order + assignments in LinkedHashMap order).
"""
import numpy as np
import pytest

from tests import oracle_py

pytestmark = pytest.mark.gpu

SEED = 0x5EEDC0DE


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _compare_step(env, ref, step, dump_every, tag=""):
    env.synchronize()
    obs, rew, done = ref.obs, ref.reward, ref.done
    g_obs = env.obs.cpu().numpy()
    if not np.array_equal(g_obs, obs):
        bad = np.argwhere(g_obs != obs)[0]
        raise AssertionError(f"{tag} obs mismatch step {step} at {bad}: gpu {g_obs[tuple(bad)]} ref {obs[tuple(bad)]}")
    assert np.array_equal(env.reward.cpu().numpy(), rew), f"{tag} reward mismatch step {step}"
    assert np.array_equal(env.done.cpu().numpy(), done), f"{tag} done mismatch step {step}"
    if dump_every and step % dump_every == 0:
        for s in range(ref.S):
            a, b = env.dump_state(s), ref.dump(s)
            if not np.array_equal(a, b):
                n = min(len(a), len(b))
                i = int(np.argmax(a[:n] != b[:n])) if (a[:n] != b[:n]).any() else n
                raise AssertionError(f"{tag} state mismatch slot {s} step {step} at word {i} (len {len(a)} vs {len(b)}):"
                                     f"\n gpu {a[max(0, i - 14):i + 14]}\n ref {b[max(0, i - 14):i + 14]}\n gpu {a.tolist()}"
                                     f"\n ref {b.tolist()}")


def _rollout(maps, n_sp, n_bot=0, steps=200, max_steps=2000, utt=1, crs=1, policy="masked", dump_every=10, seed=3,
             players=None, partial_obs=False, bots=None, rfs=None, utt_json=None, max_units=0):
    torch = _torch()
    from microrts_amd import DeviceVecEnv, UnitTypeTable

    table = UnitTypeTable.fromJSON(utt_json) if utt_json else UnitTypeTable(utt, crs)
    ntypes = len(table.TYPES)
    env = DeviceVecEnv(n_sp, n_bot, max_steps, maps, utt=table, seed=seed, partial_obs=partial_obs,
                       ai2s=bots, rfs=rfs, max_units=max_units)
    kinds = [1 if b == "RandomBiasedAI" else 0 for b in bots] if bots else None
    ref = oracle_py.OracleVecClient(n_sp, n_bot, max_steps, maps, utt_version=utt, crs=crs, seed=seed,
                                    partial_obs=partial_obs, bot_kinds=kinds,
                                    rewards=[oracle_py.REWARD_IDS[r] for r in rfs] if rfs else None, utt_json=utt_json)
    S = ref.S
    if players is not None:
        env.players.copy_(torch.as_tensor(players, dtype=torch.int32))
    env.reset()
    ref.reset(players)
    _compare_step(env, ref, 0, 1, "reset")
    rng = np.random.default_rng(seed)
    HW = ref.H * ref.W
    for step in range(steps):
        m_ref = ref.get_masks(0)
        env.synchronize()
        g_m = env.masks.cpu().numpy()
        if not np.array_equal(g_m, m_ref):
            bad = np.argwhere(g_m != m_ref)[0]
            raise AssertionError(f"mask mismatch step {step} at {bad}: gpu {g_m[tuple(bad)]} ref {m_ref[tuple(bad)]}")
        if policy == "masked":
            env.random_policy(SEED, step)
            env.synchronize()
            acts = env.actions.cpu().numpy()
            if step < 20 or step % 10 == 0:  # the GPU policy kernel is bit-identical to the oracle's Philox policy
                for s in range(min(S, 8)):
                    assert np.array_equal(acts[s], oracle_py.policy(m_ref[s], SEED, s, step, 0, ntypes))
        else:  # unmasked uniform components (exercises every illegal → NONE path)
            acts = np.stack([rng.integers(0, 6, (S, HW)), rng.integers(0, 4, (S, HW)), rng.integers(0, 4, (S, HW)),
                             rng.integers(0, 4, (S, HW)), rng.integers(0, 4, (S, HW)), rng.integers(0, ntypes, (S, HW)),
                             rng.integers(0, ref.K - 23 - ntypes, (S, HW))], axis=-1).astype(np.int32)
            env.actions.copy_(torch.as_tensor(acts))
        env.step()
        ref.step(acts, players)
        _compare_step(env, ref, step + 1, dump_every)
        if rfs:
            _rollout.nonzero |= (ref.reward != 0).reshape(ref.S, -1).any(axis=0)
    flags = env.error_flags()
    env.close()
    ref.close()
    return flags


@pytest.mark.parametrize("mp", ["maps/4x4/base4x4.xml", "maps/8x8/basesWorkers8x8.xml", "maps/16x16/basesWorkers16x16.xml",
                                "maps/BWDistantResources32x32.xml"])
def test_selfplay_masked_policy(mp):
    _rollout([mp] * 16, 16, steps=300 if "32x32" not in mp else 150)


@pytest.mark.parametrize("mp", ["maps/8x8/basesWorkers8x8.xml", "maps/16x16/basesWorkers16x16.xml"])
def test_selfplay_unmasked_uniform(mp):
    _rollout([mp] * 16, 16, steps=300, policy="uniform")


def test_autoreset_and_short_episodes():
    _rollout(["maps/4x4/base4x4.xml"] * 16, 16, steps=200, max_steps=37)


def test_mixed_maps_same_size():
    maps = ["maps/8x8/basesWorkers8x8.xml", "maps/8x8/basesWorkers8x8.xml", "maps/8x8/bases8x8.xml", "maps/8x8/bases8x8.xml",
            "maps/8x8/TwoBasesWorkers8x8.xml", "maps/8x8/TwoBasesWorkers8x8.xml", "maps/8x8/basesWorkersBarracks8x8.xml",
            "maps/8x8/basesWorkersBarracks8x8.xml"]
    _rollout(maps, 8, steps=250)


@pytest.mark.parametrize("utt,crs", [(2, 1), (3, 1), (1, 2), (1, 3), (3, 2)])
def test_utt_versions_and_conflict_policies(utt, crs):
    _rollout(["maps/8x8/basesWorkers8x8.xml"] * 16, 16, steps=250, utt=utt, crs=crs, policy="uniform")


def test_bot_envs_passive():
    players = [0, 1, 0, 1, 1, 0]
    _rollout(["maps/8x8/basesWorkers8x8.xml"] * 6, 0, n_bot=6, steps=200, players=players, policy="uniform")


def test_selfplay_plus_bots():
    _rollout(["maps/8x8/basesWorkers8x8.xml"] * 6, 4, n_bot=2, steps=200, players=[0, 0, 0, 0, 1, 0])


@pytest.mark.parametrize("mp,policy", [("maps/BWDistantResources32x32.xml", "masked"), ("maps/8x8/basesWorkers8x8.xml", "uniform"),
                                       ("maps/16x16/basesWorkers16x16.xml", "uniform")])
def test_partial_observability(mp, policy):
    """BASELINE config c5 semantics: PartiallyObservableGameState views (8 planes)."""
    _rollout([mp] * 16, 16, steps=200, policy=policy, partial_obs=True)


def test_partial_observability_bots_and_resets():
    _rollout(["maps/8x8/basesWorkers8x8.xml"] * 6, 2, n_bot=4, steps=200, max_steps=45, players=[0, 0, 1, 0, 1, 1],
             partial_obs=True, policy="uniform")


@pytest.mark.parametrize("po", [False, True])
def test_agent_vs_random_biased(po):
    """JNIGridnetClient with a RandomBiasedAI opponent (a2 + a17): java.util.Random sampling on the GPU."""
    players = [0, 1, 0, 1, 0, 1, 1, 0]
    _rollout(["maps/8x8/basesWorkers8x8.xml"] * 8, 0, n_bot=8, steps=300, players=players, partial_obs=po,
             bots=["RandomBiasedAI"] * 8, policy="masked")


@pytest.mark.parametrize("mp", ["maps/4x4/base4x4.xml", "maps/16x16/basesWorkers16x16.xml"])
def test_bot_only_client(mp):
    """Config c1 (JNIBotClient: RandomBiasedAI vs RandomBiasedAI / PassiveAI) on the GPU vs the oracle."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n = 8
    ai1 = ["RandomBiasedAI"] * 6 + ["PassiveAI", "RandomBiasedAI"]
    ai2 = ["RandomBiasedAI"] * 6 + ["RandomBiasedAI", "PassiveAI"]
    players = [0, 1] * 4
    env = DeviceVecEnv(0, n, 300, [mp] * n, ai1s=ai1, ai2s=ai2, seed=9)
    env.players.copy_(torch.as_tensor(players, dtype=torch.int32))
    kind = {"PassiveAI": 0, "RandomBiasedAI": 1}
    refs = [oracle_py.OracleBotClient(mp, kind[a], kind[b], max_steps=300, seed=9 + j) for j, (a, b) in enumerate(zip(ai1, ai2))]
    env.reset()
    for step in range(700):
        env.step()
        env.synchronize()
        rw, dn = env.reward.cpu().numpy(), env.done.cpu().numpy()
        for j, r in enumerate(refs):
            er, ed = r.step(players[j])
            assert rw[j] == er and dn[j] == ed, f"env {j} step {step}"
            if step % 25 == 0:
                assert np.array_equal(env.dump_state(j), r.dump()), f"state env {j} step {step}"
    env.close()


def test_host_api_matches_oracle():
    _torch()
    from microrts_amd import JNIGridnetVecClient

    maps = ["maps/16x16/basesWorkers16x16.xml"] * 8
    cl = JNIGridnetVecClient(8, 0, 2000, ["WinLossRewardFunction"], "", maps, seed=11)
    ref = oracle_py.OracleVecClient(8, 0, 2000, maps, seed=11)
    r = cl.reset([0] * 8)
    o, _, _ = ref.reset()
    assert np.array_equal(r.observation, o)
    for step in range(100):
        m = cl.getMasks(0)
        assert np.array_equal(m, ref.get_masks(0))
        acts = np.stack([oracle_py.policy(m[s], SEED, s, step, 0) for s in range(8)])
        r = cl.gameStep(acts, [0] * 8)
        o, rw, d = ref.step(acts)
        assert np.array_equal(r.observation, o) and np.array_equal(r.reward[:, 0], rw)
        assert np.array_equal(r.done[:, 0], d.astype(bool))
    assert np.array_equal(cl.envSteps, np.array([ref.env_steps(s) for s in range(8)]))
    cl.close()


def test_full_size_properties():
    """BASELINE config c3 size (4096 games, 16x16): size-independent invariants + oracle spot checks."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    E = 4096
    mp = "maps/16x16/basesWorkers16x16.xml"
    env = DeviceVecEnv(2 * E, 0, 2000, [mp] * (2 * E), seed=5)
    env.reset()
    picks = [0, 1, 2 * 1234, 2 * 1234 + 1, 2 * E - 2, 2 * E - 1]
    ref = oracle_py.OracleVecClient(len(picks), 0, 2000, [mp] * len(picks), seed=5)
    ref.reset()
    for step in range(60):
        env.random_policy(SEED, step)
        env.step()
        env.synchronize()
        acts = env.actions.cpu().numpy()
        obs = env.obs.cpu().numpy()
        masks = env.masks.cpu().numpy()
        # invariants: type plane non-zero <=> owner or resource; hp > 0 wherever a unit stands;
        # mask slot 0 set only on own units without an action; player planes are mirror images
        typ, hp, own, act = obs[:, 3], obs[:, 0], obs[:, 2], obs[:, 4]
        assert np.all((typ > 0) == (hp > 0))
        assert np.all(own[0::2] == np.where(own[1::2] == 0, 0, 3 - own[1::2]))
        src = masks[..., 0].reshape(2 * E, -1)
        assert np.all(src <= (own.reshape(2 * E, -1) == 1))
        assert np.all(src[act.reshape(2 * E, -1) != 0] == 0)
        # spot check against the oracle: UTT v1 + CANCEL_BOTH draws no random numbers, so an oracle
        # game fed the same action stream from reset is an exact replica of the picked GPU game
        o, _, _ = ref.step(acts[picks])
        assert np.array_equal(obs[picks], o), f"full-size games diverged at step {step}"
    assert not env.error_flags().any()
    env.close()


def test_full_size_c5_fused():
    """BASELINE config c5 as bench.py runs it (2048 games, 32x32 partially observable, max_units 256,
    the fused random policy with forwarded rows, delta masks, persistent PO views): picked games are
    replayed by the oracle from the actions each launch consumed — observations and masks equal."""
    _torch()
    from microrts_amd import DeviceVecEnv

    E = 2048
    mp = "maps/BWDistantResources32x32.xml"
    env = DeviceVecEnv(2 * E, 0, 2000, [mp] * (2 * E), seed=7, partial_obs=True, max_units=256)
    picks = [0, 1, 2 * 777, 2 * 777 + 1, 2 * E - 2, 2 * E - 1]
    ref = oracle_py.OracleVecClient(len(picks), 0, 2000, [mp] * len(picks), seed=7, partial_obs=True)
    env.reset()
    ref.reset()
    env.random_policy(SEED, 0)
    for step in range(80):
        acts = env.actions.cpu().numpy()[picks]  # what this launch consumes (a read: no invalidation)
        env.step_fused(SEED, step + 1)
        env.synchronize()
        o, _, _ = ref.step(acts)
        assert np.array_equal(env.obs.cpu().numpy()[picks], o), f"c5 observations diverged at step {step}"
        assert np.array_equal(env.masks.cpu().numpy()[picks], ref.get_masks(0)), f"c5 masks diverged at step {step}"
    assert not env.error_flags().any()
    env.close()
    ref.close()


def test_full_size_c2_uniform():
    """BASELINE config c2 as bench.py runs it (1024 games, 8x8, unmasked uniform rows, no masks, the
    native policy + step loop): picked games replayed by the oracle with the oracle's uniform rows."""
    _torch()
    from microrts_amd import DeviceVecEnv

    E = 1024
    mp = "maps/8x8/basesWorkers8x8.xml"
    env = DeviceVecEnv(2 * E, 0, 2000, [mp] * (2 * E), seed=8)
    S, H, W, C, K = env.dims
    picks = [0, 1, 2 * 500, 2 * 500 + 1, 2 * E - 2, 2 * E - 1]
    ref = oracle_py.OracleVecClient(len(picks), 0, 2000, [mp] * len(picks), seed=8)
    env.reset()
    ref.reset()
    for step in range(120):
        env.rollout_uniform(SEED, step, 1)
        env.synchronize()
        acts = np.stack([oracle_py.policy_uniform(H, W, K, SEED, s, step) for s in picks])
        o, _, _ = ref.step(acts)
        assert np.array_equal(env.obs.cpu().numpy()[picks], o), f"c2 observations diverged at step {step}"
    assert not env.error_flags().any()
    env.close()
    ref.close()


@pytest.mark.parametrize("mp,po,n_bot", [("maps/16x16/basesWorkers16x16.xml", False, 0),
                                          ("maps/10x10/basesWorkers10x10.xml", True, 6),
                                          ("maps/4x4/base4x4.xml", False, 4)])
def test_delta_masks_and_source_policy_match_full(mp, po, n_bot):
    """Delta mask and observation writes (only dirty rows / 4-cell chunks rewritten) leave the buffers
    byte-identical to full writes after every step (auto-resets at 150 steps included), and the
    source-bit policy kernel picks exactly the actions of the full-read policy kernel."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp = 16
    maps = [mp] * (n_sp + n_bot)
    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    a = DeviceVecEnv(n_sp, n_bot, 150, maps, seed=11, partial_obs=po, ai2s=bots, mask_delta=True, source_bits=True)
    b = DeviceVecEnv(n_sp, n_bot, 150, maps, seed=11, partial_obs=po, ai2s=bots, mask_delta=False, source_bits=False)
    a.reset()
    b.reset()
    rng = np.random.default_rng(2)
    S, H, W = len(maps), a.dims[1], a.dims[2]
    for step in range(400):
        if step % 37 == 5:  # caller-written actions: the next policy call must rewrite every row
            acts = torch.as_tensor(rng.integers(0, 3, (S, H * W, 7)).astype(np.int32), device=a.actions.device)
            a.actions.copy_(acts)
            b.actions.copy_(acts)
        else:
            a.random_policy(SEED, step)
            b.random_policy(SEED, step)
        a.synchronize()
        b.synchronize()
        assert torch.equal(a.obs, b.obs), f"delta observations differ at step {step}"
        assert torch.equal(a.masks, b.masks), f"delta masks differ at step {step}"
        assert torch.equal(a.actions, b.actions), f"source-bit / delta policy differs at step {step}"
        src = a.source.cpu().numpy().view(np.uint32)
        m0 = b.masks.cpu().numpy()[..., 0].reshape(len(maps), -1)
        bits = (src[:, np.arange(m0.shape[1]) >> 5] >> (np.arange(m0.shape[1]) & 31)) & 1
        assert np.array_equal(bits, m0), f"source bits differ at step {step}"
        a.step()
        b.step()
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.obs, b.obs)
    a.close()
    b.close()


def _java_rows(rng, acts, mode):
    """Java-layout rows [slots][n][8] from grid actions [slots][HW][7]: shuffled order, duplicate rows
    for the same cell (with different actions), out-of-map positions."""
    S, HW, _ = acts.shape
    rows = []
    for s in range(S):
        r = np.concatenate([np.arange(HW, dtype=np.int32)[:, None], acts[s]], axis=1)
        if mode != "ascending":
            dup = r[rng.integers(0, HW, HW // 4)].copy()
            dup[:, 1:] = np.stack([rng.integers(0, 6, len(dup)), rng.integers(0, 4, len(dup)), rng.integers(0, 4, len(dup)),
                                   rng.integers(0, 4, len(dup)), rng.integers(0, 4, len(dup)), rng.integers(0, 7, len(dup)),
                                   rng.integers(0, 49, len(dup))], axis=1)
            junk = np.zeros((4, 8), np.int32)
            junk[:, 0] = [-1, HW, HW + 7, -HW]
            r = np.concatenate([r, dup, junk])
            r = r[rng.permutation(len(r))]
        rows.append(r)
    return np.ascontiguousarray(np.stack(rows), np.int32)


@pytest.mark.parametrize("mp,n_sp,n_bot,po,crs,mode", [
    ("maps/8x8/basesWorkers8x8.xml", 8, 0, False, 1, "ascending"),
    ("maps/8x8/basesWorkers8x8.xml", 8, 0, False, 1, "java"),
    ("maps/16x16/basesWorkers16x16.xml", 4, 4, False, 3, "java"),
    ("maps/10x10/basesWorkers10x10.xml", 4, 3, True, 2, "java"),
    ("maps/4x4/base4x4.xml", 6, 2, False, 1, "java"),
])
def test_java_rows_layout(mp, n_sp, n_bot, po, crs, mode):
    """mrts_step_rows (Java int[][][] rows: any order, duplicate rows, off-map positions) vs the oracle
    running PlayerAction.fromVectorAction over the same row lists; rows in ascending cell order must
    also equal the grid path."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv, JNIGridnetVecClient, UnitTypeTable

    maps = [mp] * (n_sp + n_bot)
    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    kinds = [1] * n_bot if n_bot else None
    env = DeviceVecEnv(n_sp, n_bot, 120, maps, utt=UnitTypeTable(1, crs), seed=4, partial_obs=po, ai2s=bots)
    ref = oracle_py.OracleVecClient(n_sp, n_bot, 120, maps, crs=crs, seed=4, partial_obs=po, bot_kinds=kinds)
    grid = DeviceVecEnv(n_sp, n_bot, 120, maps, utt=UnitTypeTable(1, crs), seed=4, partial_obs=po, ai2s=bots) \
        if mode == "ascending" else None
    env.reset()
    ref.reset()
    if grid is not None:
        grid.reset()
    rng = np.random.default_rng(8)
    S, HW = ref.S, ref.H * ref.W
    for step in range(150):
        m = ref.get_masks(0)
        env.synchronize()
        assert np.array_equal(env.masks.cpu().numpy(), m), f"mask mismatch step {step}"
        acts = np.stack([oracle_py.policy(m[s], SEED, s, step, 0) for s in range(S)])
        if step % 3 == 1:  # unmasked components: illegal actions, conflicts
            acts = np.stack([rng.integers(0, 6, (S, HW)), rng.integers(0, 4, (S, HW)), rng.integers(0, 4, (S, HW)),
                             rng.integers(0, 4, (S, HW)), rng.integers(0, 4, (S, HW)), rng.integers(0, 7, (S, HW)),
                             rng.integers(0, 49, (S, HW))], axis=-1).astype(np.int32)
        rows = _java_rows(rng, acts, mode)
        env.step_rows(torch.as_tensor(rows, device=env.device))
        ref.step_rows(rows)
        _compare_step(env, ref, step + 1, 5, f"rows[{mode}]")
        if grid is not None:
            grid.step(torch.as_tensor(acts, device=grid.device))
            grid.synchronize()
            assert torch.equal(grid.obs, env.obs) and torch.equal(grid.masks, env.masks), f"grid != rows at {step}"
    assert not env.error_flags().any()
    env.close()
    ref.close()
    if grid is not None:
        grid.close()
    # host API: Java rows + int32 masks through the JNIGridnetVecClient mirror
    cl = JNIGridnetVecClient(n_sp, n_bot, 120, ["WinLossRewardFunction"], "", maps, bots, UnitTypeTable(1, crs), po)
    ref = oracle_py.OracleVecClient(n_sp, n_bot, 120, maps, crs=crs, seed=0, partial_obs=po, bot_kinds=kinds)
    cl.reset()
    ref.reset()
    for step in range(20):
        m = ref.get_masks(0)
        m32 = cl.getMasks(0, dtype=np.int32)
        assert m32.dtype == np.int32 and np.array_equal(m32, m.astype(np.int32))
        acts = np.stack([oracle_py.policy(m[s], SEED, s, step, 0) for s in range(S)])
        rows = _java_rows(rng, acts, mode)
        r = cl.gameStep(rows)
        o, rw, d = ref.step_rows(rows)
        assert np.array_equal(r.observation, o) and np.array_equal(r.reward[:, 0], rw)
    cl.close()
    ref.close()


@pytest.mark.parametrize("rows", [False, True])
def test_more_than_64_units(rows):
    """EightBasesWorkers16x16 starts with 64 units and grows past one wave's worth: exercises the
    multi-block (nu > 64) decode / issue / ready-list paths, grid and Java-row layouts."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp = "maps/16x16/EightBasesWorkers16x16.xml"
    n = 4
    env = DeviceVecEnv(n, 0, 2000, [mp] * n, seed=2)
    ref = oracle_py.OracleVecClient(n, 0, 2000, [mp] * n, seed=2)
    env.reset()
    ref.reset()
    rng = np.random.default_rng(1)
    most = 0
    for step in range(160):
        m = ref.get_masks(0)
        env.synchronize()
        assert np.array_equal(env.masks.cpu().numpy(), m), f"mask mismatch step {step}"
        acts = np.stack([oracle_py.policy(m[s], SEED, s, step, 0) for s in range(n)])
        if rows:
            r = _java_rows(rng, acts, "java")
            env.step_rows(torch.as_tensor(r, device=env.device))
            ref.step_rows(r)
        else:
            env.step(torch.as_tensor(acts, device=env.device))
            ref.step(acts)
        _compare_step(env, ref, step + 1, 10, "many-units")
        most = max(most, int(ref.dump(0)[4]))
    assert most > 64, f"test did not reach > 64 units (max {most})"
    assert not env.error_flags().any()
    env.close()
    ref.close()


ALL_RFS = ["WinLossRewardFunction", "ResourceGatherRewardFunction", "ProduceWorkerRewardFunction",
           "ProduceBuildingRewardFunction", "AttackRewardFunction", "ProduceCombatUnitRewardFunction",
           "CloserToEnemyBaseRewardFunction", "CloserToEnemyUnitRewardFunction"]


@pytest.mark.parametrize("mp,n_sp,n_bot,po,policy,crs", [
    ("maps/16x16/basesWorkers16x16.xml", 8, 0, False, "masked", 1),
    ("maps/8x8/basesWorkers8x8.xml", 4, 4, False, "uniform", 1),
    ("maps/10x10/basesWorkers10x10.xml", 4, 4, True, "masked", 1),
    ("maps/8x8/basesWorkers8x8.xml", 4, 4, True, "uniform", 3),
    ("maps/4x4/base4x4.xml", 6, 2, False, "masked", 1),
])
def test_all_reward_functions(mp, n_sp, n_bot, po, policy, crs):
    """The eight reward functions of src/ai/reward in MicroRTS-Py's order: reward [S][8] and done [S][8]
    bit-exact (the Closer* ones are fp64 sqrt differences) after every step, self-play + RandomBiasedAI
    opponents, full and partial observability."""
    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    _rollout.nonzero = np.zeros(len(ALL_RFS), bool)
    assert not _rollout([mp] * (n_sp + n_bot), n_sp, n_bot, steps=400, max_steps=300, crs=crs, policy=policy,
                        partial_obs=po, bots=bots, rfs=ALL_RFS, dump_every=25).any()
    # non-vacuous: under the masked policy the gather / worker / attack / distance functions fire (WinLoss
    # and the building / combat-unit ones can stay 0 in 400 random steps); unmasked actions are mostly
    # illegal, so only the distance functions are certain to
    must = [1, 2, 4, 6, 7] if policy == "masked" else [6, 7]
    assert _rollout.nonzero[must].all(), _rollout.nonzero


def test_first_reward_function_drives_reset():
    """done[0] of the FIRST reward function triggers the auto-reset (JNIGridnetVecClient.java:247):
    with ResourceGather first, a game resets only when its resources are gone, not at gameover."""
    rfs = ["ResourceGatherRewardFunction", "WinLossRewardFunction", "AttackRewardFunction"]
    _rollout.nonzero = np.zeros(len(rfs), bool)
    assert not _rollout(["maps/4x4/base4x4.xml"] * 8, 8, 0, steps=600, max_steps=5000, rfs=rfs, dump_every=50).any()


def test_bot_only_reward_functions():
    """Config c1 clients with all eight reward functions (JNIBotClient.java:108-135)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n, mp = 4, "maps/8x8/basesWorkers8x8.xml"
    env = DeviceVecEnv(0, n, 300, [mp] * n, ai1s=["RandomBiasedAI"] * n, ai2s=["RandomBiasedAI"] * n, seed=5, rfs=ALL_RFS)
    refs = [oracle_py.OracleBotClient(mp, 1, 1, max_steps=300, seed=5 + j,
                                      rewards=[oracle_py.REWARD_IDS[r] for r in ALL_RFS]) for j in range(n)]
    env.reset()
    for step in range(500):
        env.step()
        env.synchronize()
        rw, dn = env.reward.cpu().numpy(), env.done.cpu().numpy()
        for j, r in enumerate(refs):
            er, ed = r.step(0)
            assert np.array_equal(rw[j], er) and np.array_equal(dn[j], ed), f"env {j} step {step}: {rw[j]} {er}"
    env.close()


def _encode_obs_np(obs, ntypes=7):
    """numpy restatement of MicroRTS-Py's GridnetVecEnv `_encode_obs` (gym_microrts, external to the
    reference — parity unpinned): per env, planes clipped to [0, n-1] and one-hot encoded, channels
    last, plane sizes [5, 5, 3, ntypes + 1, 6, 2] (+ [2] per extra partial-observability plane)."""
    S, C, H, W = obs.shape
    sizes = [5, 5, 3, ntypes + 1, 6, 2] + [2] * (C - 6)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    out = np.zeros((S, H * W, sum(sizes)), np.uint8)
    flat = obs.reshape(S, C, H * W)
    for p in range(C):
        v = np.clip(flat[:, p], 0, sizes[p] - 1)
        np.put_along_axis(out, (v + offs[p])[..., None], 1, axis=2)
    return out.reshape(S, H, W, -1)


@pytest.mark.parametrize("mp,po", [("maps/16x16/basesWorkers16x16.xml", False), ("maps/10x10/basesWorkers10x10.xml", True),
                                   ("maps/4x4/base4x4.xml", False)])
def test_onehot_encoder(mp, po):
    """mrts_onehot_dev = MicroRTS-Py's observation encoding of the step's int32 observation."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    env = DeviceVecEnv(6, 0, 2000, [mp] * 6, seed=3, partial_obs=po)
    env.reset()
    for step in range(60):
        env.random_policy(SEED, step)
        env.step()
        if step % 10 == 9:
            got = env.onehot_obs()
            env.synchronize()
            ref = _encode_obs_np(env.obs.cpu().numpy())
            assert got.shape == ref.shape and got.shape[-1] == (33 if po else 29)
            assert np.array_equal(got.cpu().numpy(), ref), f"step {step}"
    env.close()


# ------------------------------------------------------------------ JSON unit-type tables
def _fixture_utt():
    import os

    return open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "utts", "TestUnitTypeTable.json")).read()


@pytest.mark.parametrize("mp,n_sp,n_bot,po,policy", [
    ("maps/8x8/basesWorkers8x8.xml", 8, 4, False, "masked"),
    ("maps/16x16/basesWorkers16x16.xml", 4, 2, True, "uniform"),
])
def test_utt_from_json_fixture(mp, n_sp, n_bot, po, policy):
    """The reference's utts/TestUnitTypeTable.json (Base hp 50, Barracks hp 25, harvestTime taken
    from produceTime by UnitType.updateFromJSON) with every reward function."""
    S = n_sp + n_bot
    _rollout.nonzero = np.zeros(len(ALL_RFS), bool)
    assert not _rollout([mp] * S, n_sp, n_bot, steps=300, policy=policy, partial_obs=po, bots=["RandomBiasedAI"] * n_bot,
                        rfs=ALL_RFS, utt_json=_fixture_utt(), dump_every=25).any()
    assert _rollout.nonzero[[6, 7]].all()


def test_utt_from_json_eight_types():
    """A table unlike any built-in one: an 8th type (produced by Workers, defaults for absent
    members, attack range 2) -> K = 1+6+16+8+49 = 80 mask slots, this build's maximum."""
    from microrts_amd.vec_client import UnitTypeTable
    import json

    t = json.loads(UnitTypeTable(2, 3).toJSON())
    t["unitTypes"][3]["produces"].append("Tower")
    t["unitTypes"].append({"ID": 7, "name": "Tower", "cost": 3, "hp": 6, "attackRange": 2, "minDamage": 1,
                           "maxDamage": 3, "canAttack": True, "sightRadius": 4, "produces": [],
                           "producedBy": ["Worker"]})
    js = json.dumps(t)
    mp = "maps/8x8/basesWorkers8x8.xml"
    _rollout.nonzero = np.zeros(len(ALL_RFS), bool)
    assert not _rollout([mp] * 8, 6, 2, steps=300, policy="masked", bots=["RandomBiasedAI"] * 2, rfs=ALL_RFS,
                        utt_json=js, dump_every=25, seed=12).any()
    assert _rollout.nonzero[[1, 2, 4, 6, 7]].all()


@pytest.mark.parametrize("mp,po,mu", [("maps/BWDistantResources32x32.xml", True, 96), ("maps/16x16/basesWorkers16x16.xml", False, 40)])
def test_max_units_bound(mp, po, mu):
    """mrts_config.max_units: a smaller unit-slot capacity plays identically (generic kernel: bot envs)."""
    assert not _rollout([mp] * 8, 6, 2, steps=200, partial_obs=po, bots=["RandomBiasedAI"] * 2, max_units=mu,
                        dump_every=20).any()


@pytest.mark.parametrize("mp,po,mu,policy", [("maps/BWDistantResources32x32.xml", True, 256, "masked"),
                                             ("maps/BWDistantResources32x32.xml", True, 256, "uniform"),
                                             ("maps/8x8/basesWorkers8x8.xml", False, 0, "uniform")])
def test_specialised_shapes(mp, po, mu, policy):
    """The compile-time specialisations of the step kernel: c5 (32x32 PO, 320 slots) and c2 (8x8)."""
    assert not _rollout([mp] * 16, 16, steps=250, partial_obs=po, max_units=mu, policy=policy, dump_every=25).any()


def test_max_units_below_map_units_rejected():
    _torch()
    from microrts_amd import DeviceVecEnv

    with pytest.raises(RuntimeError):
        DeviceVecEnv(2, 0, 100, ["maps/16x16/basesWorkers16x16.xml"] * 2, max_units=3)


@pytest.mark.parametrize("mp,n_sp,n_bot,po,delta", [
    ("maps/16x16/basesWorkers16x16.xml", 8, 0, False, True),
    ("maps/8x8/basesWorkers8x8.xml", 8, 0, False, False),
    ("maps/10x10/basesWorkers10x10.xml", 4, 2, True, True),     # H*W*K % 16 != 0: full mask path
    ("maps/BWDistantResources32x32.xml", 4, 0, True, True),
])
def test_fused_policy_matches_separate_kernels(mp, n_sp, n_bot, po, delta):
    """mrts_step_fused_dev = mrts_step_dev followed by mrts_policy_dev(next step), bit for bit, including
    after a reset and a standalone mask write in between."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    S = n_sp + n_bot
    bots = ["RandomBiasedAI"] * n_bot
    mk = lambda: DeviceVecEnv(n_sp, n_bot, 400, [mp] * S, ai2s=bots, partial_obs=po, seed=6, mask_delta=delta)  # noqa: E731
    A, B = mk(), mk()
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    for k in range(250):
        A.step()
        A.random_policy(SEED, k + 1)
        B.step_fused(SEED, k + 1)
        A.synchronize()
        B.synchronize()
        for name in ("obs", "reward", "done", "masks", "actions"):
            a, b = getattr(A, name).cpu().numpy(), getattr(B, name).cpu().numpy()
            assert np.array_equal(a, b), f"{name} differs after step {k}"
        if k == 90:
            for e in (A, B):
                e.reset()
                e.random_policy(SEED, k + 1)
        if k == 170:
            B.get_masks()
    A.close()
    B.close()
    del torch


@pytest.mark.parametrize("mp", ["maps/16x16/basesWorkers16x16.xml", "maps/8x8/basesWorkers8x8.xml"])
def test_fused_forwarding_respects_action_writes(mp):
    """A fused step forwards its sampled rows to the next launch in the state block (KDyn.fwd_read):
    when the caller overwrites the action tensor in between (uniform random rows, every 7th step), or
    runs a plain step or a mask write on the handle, the next fused step must read the tensor.  Twin A
    always reads the tensor (step + standalone policy kernel)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp = 16
    mk = lambda: DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=5)  # noqa: E731
    A, B = mk(), mk()
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    g = torch.Generator(device="cpu").manual_seed(11)
    hi = torch.tensor([6, 4, 4, 4, 4, 7, 49], dtype=torch.int32)
    for k in range(200):
        if k % 7 == 3:
            alt = (torch.rand(tuple(A.actions.shape), generator=g) * hi).to(torch.int32)
            for e in (A, B):
                e.actions.copy_(alt.to(e.actions.device))
        if k % 29 == 11:  # a plain step on the fused handle, then a fresh policy write
            B.step()
            A.step()
            for e in (A, B):
                e.random_policy(SEED, 1000 + k)
        if k % 31 == 17:
            B.get_masks()
        A.step()
        A.random_policy(SEED, k + 1)
        B.step_fused(SEED, k + 1)
        for name in ("obs", "reward", "done", "masks", "actions"):
            assert np.array_equal(getattr(A, name).cpu().numpy(), getattr(B, name).cpu().numpy()), f"{name} after {k}"
    for s in range(0, n_sp, 2):
        assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s}"
    A.close()
    B.close()


@pytest.mark.parametrize("mp,n_sp", [("maps/16x16/basesWorkers16x16.xml", 64), ("maps/8x8/basesWorkers8x8.xml", 16)])
def test_native_rollout_matches_fused_steps(mp, n_sp):
    """mrts_rollout_fused_dev(n) = n mrts_step_fused_dev calls (the bench's timed launch form), bit for
    bit: observations, rewards, dones, masks, next actions and every game's state."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mk = lambda: DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=3)  # noqa: E731
    A, B = mk(), mk()
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    k = 0
    for n in (1, 7, 0, 40, 180):  # crosses max_steps 300: auto-resets inside a rollout
        for i in range(n):
            A.step_fused(SEED, k + i + 1)
        B.rollout_fused(SEED, k + 1, n)
        k += n
        A.synchronize()
        B.synchronize()
        for name in ("obs", "reward", "done", "masks", "actions"):
            assert np.array_equal(getattr(A, name).cpu().numpy(), getattr(B, name).cpu().numpy()), f"{name} after {k}"
        for s in range(0, n_sp, 2):
            assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s} after {k}"
    assert np.array_equal(A._h.env_steps(), B._h.env_steps())
    A.close()
    B.close()
    del torch


@pytest.mark.parametrize("mp,n_sp,max_steps,po", [("maps/16x16/basesWorkers16x16.xml", 48, 300, False),
                                                   # 1024 games: balanced placement on (balancePerm: n % 512 == 0)
                                                   ("maps/16x16/basesWorkers16x16.xml", 2048, 300, False),
                                                   ("maps/8x8/basesWorkers8x8.xml", 64, 150, False),
                                                   ("maps/16x16/EightBasesWorkers16x16.xml", 8, 2000, False),
                                                   ("maps/BWDistantResources32x32.xml", 32, 200, True)])
def test_multi_step_rollout_matches_single_launches(mp, n_sp, max_steps, po):
    """Multi-step launches (mrts_rollout_fused_dev running up to MRTS_MAX_ITER steps per game in one
    launch, state kept in LDS between steps) = one launch per step (mrts_set_multi_step(0)), bit for
    bit: observations, rewards, dones, masks, source bits, next actions, env steps and every game's
    state — rollouts of 1 .. 250 steps across auto-resets, games above 64 units (EightBasesWorkers:
    the multi-block decode, mask and non-forwarded row paths inside the loop), then single fused
    steps, a plain step and a mask write after the multi-step launches (handle bookkeeping); the 32x32
    partially observable views (persistent-buffer delta renders whose record is re-read per step)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mk = lambda: DeviceVecEnv(n_sp, 0, max_steps, [mp] * n_sp, seed=5, partial_obs=po,  # noqa: E731
                              max_units=256 if po else 0)
    A, B = mk(), mk()
    A.set_multi_step(False)
    assert B.multi_step_capable
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    names = ("obs", "reward", "done", "masks", "actions", "source")

    def same(tag):
        A.synchronize()
        B.synchronize()
        for name in names:
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{name} {tag}"
        for s in range(0, n_sp, 2 if n_sp <= 64 else 14):
            assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s} {tag}"
        assert np.array_equal(A._h.env_steps(), B._h.env_steps()), f"env steps {tag}"

    k = 0
    for n in (1, 2, 5, 64, 250):
        A.rollout_fused(SEED, k + 1, n)
        B.rollout_fused(SEED, k + 1, n)
        k += n
        same(f"after rollout to {k}")
    for e in (A, B):
        e.step_fused(SEED, k + 1)
        e.step_fused(SEED, k + 2)
    same("after single fused steps")
    for e in (A, B):
        e.rollout_fused(SEED, k + 3, 30)
        e.step()
        e.rollout_fused(SEED, k + 40, 20)  # not in the steady state: first step alone, then a loop
    same("after a plain step between rollouts")
    assert not A.error_flags().any() and not B.error_flags().any()
    A.close()
    B.close()


def test_multi_step_uniform_po_matches_single_launches():
    """The c5 helper-wave instance under the uniform rollout (mrts_rollout_uniform_dev: no masks, so
    the game wave hands the helper no mask records): multi-step launches = one launch per step, bit for
    bit — observations, rewards, dones, the drawn rows and every game's state."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp, n_sp = "maps/BWDistantResources32x32.xml", 32
    mk = lambda: DeviceVecEnv(n_sp, 0, 200, [mp] * n_sp, seed=7, partial_obs=True, max_units=256)  # noqa: E731
    A, B = mk(), mk()
    A.set_multi_step(False)
    assert B.multi_step_capable
    for e in (A, B):
        e.reset()
    k = 0
    for n in (1, 3, 64, 180):
        A.rollout_uniform(SEED, k, n)
        B.rollout_uniform(SEED, k, n)
        k += n
        A.synchronize()
        B.synchronize()
        for name in ("obs", "reward", "done", "actions"):
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{name} after {k}"
        for s in range(0, n_sp, 2):
            assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s} after {k}"
    assert not A.error_flags().any() and not B.error_flags().any()
    A.close()
    B.close()


def _crowded_32x32(tmp_path, per_player):
    """BWDistantResources32x32 plus `per_player` extra Workers per player:
    the map file is written by the test (the reference's XML layout, PhysicalGameState.java:700-726)."""
    import re

    src = open("maps/BWDistantResources32x32.xml").read()
    terrain = re.search(r"<terrain>([01]+)</terrain>", src).group(1)
    taken = {(int(x), int(y)) for x, y in re.findall(r'x="(\d+)" y="(\d+)"', src)}
    free = [(x, y) for y in range(32) for x in range(32) if terrain[y * 32 + x] == "0" and (x, y) not in taken]
    left = [c for c in free if c[0] < 12 and 8 <= c[1] < 24]
    right = [c for c in free if c[0] >= 20 and 8 <= c[1] < 24]
    extra, uid = [], 1000
    for p, cells in ((0, left), (1, right)):
        for x, y in cells[:per_player]:
            extra.append(f'    <rts.units.Unit type="Worker" ID="{uid}" player="{p}" x="{x}" y="{y}" resources="0" '
                         f'hitpoints="1" >\n    </rts.units.Unit>\n')
            uid += 1
    path = tmp_path / "crowded32x32.xml"
    path.write_text(src.replace("  </units>", "".join(extra) + "  </units>"))
    return str(path)


def test_po_helper_wave_over_64_units(tmp_path):
    """The partially observable multi-step launch (c5's shape) renders through a helper wave (helperLoopPO):
    from the game's packed step (renderPOPacked) while the game's units fit one wave; a step with more than
    64 units is rendered by the helper from the game's live state (the general writeObsPO) while the game
    waits at a second barrier, and the packed form takes over again after the auto-reset.  The crowded map
    starts at 60 units and the games produce past 64 (oracle: steps ~249-298 of 300): multi-step = one
    launch per step, bit for bit, across both transitions."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp = _crowded_32x32(tmp_path, 22)
    n_sp = 16
    mk = lambda: DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=9, partial_obs=True, max_units=256)  # noqa: E731
    A, B = mk(), mk()
    A.set_multi_step(False)
    assert B.multi_step_capable
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    assert int(B.dump_state(0)[4]) <= 64
    names = ("obs", "reward", "done", "masks", "actions", "source")
    k, high = 0, 0
    for n in (1, 3, 40, 60, 60, 60, 60, 80, 60):
        A.rollout_fused(SEED, k + 1, n)
        B.rollout_fused(SEED, k + 1, n)
        k += n
        A.synchronize()
        B.synchronize()
        for name in names:
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{name} after {k}"
        for s in range(0, n_sp, 2):
            d = B.dump_state(s)
            high = max(high, int(d[4]))
            assert np.array_equal(A.dump_state(s), d), f"state slot {s} after {k}"
    assert high > 64, f"no game grew past 64 units (most {high})"
    assert not A.error_flags().any() and not B.error_flags().any()
    A.close()
    B.close()


@pytest.mark.parametrize("mp,n_sp,n_bot,rows,max_units", [
    ("maps/BWDistantResources32x32.xml", 8, 4, False, 256),
    ("maps/16x16/basesWorkers16x16.xml", 16, 4, False, 0),
    ("maps/8x8/basesWorkers8x8.xml", 8, 4, True, 0),          # Java rows (shuffled, duplicates)
    ("maps/24x24/basesWorkers24x24.xml", 8, 2, False, 0),
    ("maps/10x10/basesWorkers10x10.xml", 8, 2, False, 0),     # W % 4 != 0: always full renders
])
def test_po_obs_delta_matches_full(mp, n_sp, n_bot, rows, max_units):
    """Persistent-buffer partially observable observations (only the 4-cell chunks whose cells can have
    changed are re-rendered: units whose view membership or rendered fields changed, units that died
    in the last render, the XOR of old and new sight rows) stay byte-identical to full renders after
    every step: self-play and agent-vs-RandomBiasedAI games (the agent's side flips every 7 steps),
    auto-resets (max_steps 120), a caller's in-place edit of env.obs, a checkpoint restore and a
    GameState.fromJSON injection."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    S = n_sp + n_bot
    maps = [mp] * S
    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    mk = lambda d: DeviceVecEnv(n_sp, n_bot, 120, maps, seed=8, ai2s=bots, partial_obs=True, obs_delta=d,  # noqa: E731
                                max_units=max_units)
    a, b = mk(True), mk(False)
    a.reset()
    b.reset()
    rng = np.random.default_rng(6)
    ck = None
    for step in range(320):
        if n_bot and step % 7 == 3:
            side = torch.tensor([(step // 7) % 2] * S, dtype=torch.int32, device=a.device)
            a.players.copy_(side)
            b.players.copy_(side)
        a.random_policy(SEED, step)
        b.random_policy(SEED, step)
        if rows:
            r = torch.as_tensor(_java_rows(rng, a.actions.cpu().numpy(), "shuffled_dups"), device=a.device)
            a.step_rows(r)
            b.step_rows(r)
        else:
            a.step()
            b.step()
        if step == 60:
            a.obs[1, 6, 0, 0] += 3  # caller writes the buffer: the next write must be a full one
        if step == 80:
            ck = (a.checkpoint(), b.checkpoint())
        if step == 150:
            a.restore(ck[0])
            b.restore(ck[1])
            a.get_masks()
            b.get_masks()
        if step == 200:
            j = b.state_json(2)
            a.set_state_json(2, j)
            b.set_state_json(2, j)
            a.get_masks()
            b.get_masks()
        if step in (60, 150, 200):
            continue  # the buffers differ / are stale until the next step
        a.synchronize()
        b.synchronize()
        assert torch.equal(a.obs, b.obs), f"delta PO observations differ after step {step}"
    assert not a.error_flags().any()
    a.close()
    b.close()


def test_uniform_policy_matches_oracle():
    """mrts_policy_uniform_dev (BASELINE config c2's unmasked uniform rows) = the oracle's restatement,
    for every slot, several steps, with a non-zero slot_id_base."""
    _torch()
    from microrts_amd import DeviceVecEnv

    env = DeviceVecEnv(12, 0, 300, ["maps/8x8/basesWorkers8x8.xml"] * 12, seed=2, slot_id_base=40)
    S, H, W, C, K = env.dims
    for step in (0, 1, 7, 123456):
        env.uniform_policy(SEED, step)
        acts = env.actions.cpu().numpy().reshape(S, H * W, 7)
        for s in range(S):
            assert np.array_equal(acts[s], oracle_py.policy_uniform(H, W, K, SEED, 40 + s, step)), f"slot {s} step {step}"
    env.close()


@pytest.mark.parametrize("mp", ["maps/8x8/basesWorkers8x8.xml", "maps/16x16/basesWorkers16x16.xml"])
def test_uniform_rollout_matches_oracle(mp):
    """The c2 workload: rollout_uniform (uniform rows + a step without masks, native loop) against the
    oracle VecClient stepped with the oracle's uniform rows — observations, rewards and dones every
    step, the canonical state every 20 steps, and across auto-resets (max_steps 150)."""
    _torch()
    from microrts_amd import DeviceVecEnv

    n = 16
    env = DeviceVecEnv(n, 0, 150, [mp] * n, seed=4, with_masks=False)
    ref = oracle_py.OracleVecClient(n, 0, 150, [mp] * n, seed=4)
    S, H, W, C, K = env.dims
    env.reset()
    ref.reset(None)
    _compare_step(env, ref, 0, 1, "reset")
    for step in range(260):
        env.rollout_uniform(SEED, step, 1)
        acts = np.stack([oracle_py.policy_uniform(H, W, K, SEED, s, step) for s in range(S)])
        ref.step(acts, None)
        _compare_step(env, ref, step + 1, 20, "uniform")
    assert not env.error_flags().any()
    env.close()
    ref.close()


@pytest.mark.parametrize("mp,n_sp,n_bot,po,masks", [("maps/16x16/basesWorkers16x16.xml", 24, 0, False, False),
                                                     ("maps/8x8/basesWorkers8x8.xml", 32, 0, False, False),
                                                     ("maps/8x8/basesWorkers8x8.xml", 16, 6, False, True),
                                                     ("maps/10x10/basesWorkers10x10.xml", 12, 6, True, False)])
def test_uniform_fused_matches_split(mp, n_sp, n_bot, po, masks):
    """mrts_step_uniform_dev (the step kernel writes the uniform rows and draws its idle units' rows
    itself, one launch) = mrts_policy_uniform_dev + mrts_step_dev (two launches): the action tensor,
    observations, rewards, dones (and masks) after every step, every slot's canonical state every 25
    steps — specialised 16x16 / 8x8 kernels, the generic kernel with agent-vs-RandomBiasedAI games and
    partially observable views, across auto-resets (max_steps 120)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    maps = [mp] * (n_sp + n_bot)
    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    mk = lambda: DeviceVecEnv(n_sp, n_bot, 120, maps, seed=9, partial_obs=po, ai2s=bots, with_masks=masks,
                              slot_id_base=7)
    a, b = mk(), mk()
    a.reset()
    b.reset()
    for step in range(300):
        a.uniform_policy(SEED, step)
        a.step(masks=masks)
        b.step_uniform(SEED, step, masks=masks)
        a.synchronize()
        b.synchronize()
        assert torch.equal(a.actions, b.actions), f"actions differ at step {step}"
        assert torch.equal(a.obs, b.obs), f"observations differ at step {step}"
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), f"rewards / dones differ at step {step}"
        if masks:
            assert torch.equal(a.masks, b.masks), f"masks differ at step {step}"
        if step % 25 == 0:
            for s in range(a.dims[0]):
                assert np.array_equal(a.dump_state(s), b.dump_state(s)), f"state of slot {s} differs at step {step}"
    assert not a.error_flags().any() and not b.error_flags().any()
    # the native rollout's fused and split forms agree too (fused: multi-step launches on the
    # self-play-only 16x16 / 8x8 handles), across an auto-reset
    assert b.multi_step_capable == (n_bot == 0)
    a.rollout_uniform(SEED, 300, 100, fused=False)
    b.rollout_uniform(SEED, 300, 100, fused=True)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.actions, b.actions)
    assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done)
    for s in range(a.dims[0]):
        assert np.array_equal(a.dump_state(s), b.dump_state(s)), f"state of slot {s} differs after the rollout"
    assert np.array_equal(a._h.env_steps(), b._h.env_steps())
    a.close()
    b.close()


@pytest.mark.parametrize("mp,n_sp,n_bot", [("maps/16x16/basesWorkers16x16.xml", 24, 0),
                                          ("maps/8x8/basesWorkers8x8.xml", 16, 6),
                                          ("maps/NoWhereToRun9x8.xml", 8, 2)])
def test_obs16_copy_matches_obs(mp, n_sp, n_bot):
    """mrts_set_obs16: every observation write also leaves the planes as int16 in the given buffer —
    after reset, plain steps, fused steps and multi-step rollouts (auto-resets included), on the
    specialised and generic kernels; switching the buffer and turning it off work too."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    bots = ["RandomBiasedAI"] * n_bot if n_bot else None
    env = DeviceVecEnv(n_sp, n_bot, 120, [mp] * (n_sp + n_bot), seed=12, ai2s=bots)
    bufs = [torch.full(tuple(env.obs.shape), -7, dtype=torch.int16, device=env.device) for _ in range(2)]
    env.set_obs16(bufs[0])
    env.reset()
    env.synchronize()
    assert torch.equal(bufs[0], env.obs.to(torch.int16)), "after reset"
    env.random_policy(SEED, 0)
    for k in range(200):
        b = bufs[k & 1]
        env.set_obs16(b)
        if k % 3 == 0:
            env.step()
            env.random_policy(SEED, k + 1)
        else:
            env.step_fused(SEED, k + 1)
        env.synchronize()
        assert torch.equal(b, env.obs.to(torch.int16)), f"step {k}"
    env.set_obs16(bufs[0])
    env.rollout_fused(SEED, 300, 50)  # multi-step launches on the self-play-only 16x16 handle
    env.synchronize()
    assert torch.equal(bufs[0], env.obs.to(torch.int16)), "after a rollout"
    env.set_obs16(None)
    before = bufs[0].clone()
    env.step_fused(SEED, 400)
    env.synchronize()
    assert torch.equal(bufs[0], before), "written after set_obs16(None)"
    assert not env.error_flags().any()
    env.close()


def test_host_mask_views_match_copies():
    """getMasks(copy=False): views of the library-owned pinned arrays (mrts_get_masks_host /
    mrts_get_masks_i32_host) hold the same masks as the copying form, and the next call refills them."""
    _torch()
    from microrts_amd import JNIGridnetVecClient, UnitTypeTable

    mp = "maps/8x8/basesWorkers8x8.xml"
    vc = JNIGridnetVecClient(8, 0, 100, ["WinLossRewardFunction"], ".", [mp] * 8, [], UnitTypeTable(), False)
    vc.reset([0] * 8)
    rng = np.random.default_rng(1)
    for step in range(30):
        a = np.stack([rng.integers(0, 6, (8, 64)), rng.integers(0, 4, (8, 64)), rng.integers(0, 4, (8, 64)),
                      rng.integers(0, 4, (8, 64)), rng.integers(0, 4, (8, 64)), rng.integers(0, 7, (8, 64)),
                      rng.integers(0, 49, (8, 64))], axis=-1).astype(np.int32)
        vc.gameStep(a)
        for dt in (np.uint8, np.int32):
            v = vc.getMasks(0, dtype=dt, copy=False)
            c = vc.getMasks(0, dtype=dt)
            assert v.dtype == dt and v.shape == c.shape and np.array_equal(v, c), f"step {step} {dt}"
    vc.close()


def test_full_obs_without_byte_image(tmp_path):
    """16x16 full observability renders through the LDS byte image only when every plane value fits a
    byte (KDyn.obs_img); a resource pile of 300 sends the same maps through the cell-map gather — both
    against the oracle, every step (observations, rewards, dones, masks, states every 10 steps)."""
    src = open("maps/16x16/basesWorkers16x16.xml").read()
    assert 'resources="25"' in src
    big = tmp_path / "bigpile16x16.xml"
    big.write_text(src.replace('resources="25"', 'resources="300"', 1))
    _rollout([str(big)] * 8, 8, steps=120)
