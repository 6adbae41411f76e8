"""Batched forward model for search AIs: GameState.clone()
(rts/GameState.java:591-610), NaiveMCTS.simulate (ai/mcts/naivemcts/NaiveMCTS.java:297-308) and
SimpleSqrtEvaluationFunction3 (ai/evaluation/SimpleSqrtEvaluationFunction3.java:24-44).

CPU tests pin the oracle's new pieces: the clone reproduces the source exactly (dump + continuation),
the playout loop follows the do-while (first-iteration and gameover exits), and the evaluation's Java
float arithmetic matches an independent numpy float32/float64 restatement.  The reference holds no
fixtures for search AIs, so the playout loop and the evaluation are "parity unpinned" beyond the engine
semantics the trace fixtures and KATs already pin.  GPU tests compare the HIP forward model with the
oracle bit for bit (state dumps, float32 evaluations) through the C ABI."""
import numpy as np
import pytest

from tests import oracle_py

RB, PASSIVE = oracle_py.BOT_RANDOM_BIASED, oracle_py.BOT_PASSIVE
M8 = "maps/8x8/basesWorkers8x8.xml"
M16 = "maps/16x16/basesWorkers16x16.xml"
M4 = "maps/4x4/base4x4.xml"
# UnitTypeTable VERSION_ORIGINAL (rts/units/UnitTypeTable.java:111-259): type id -> (cost, hp)
UTT1 = {0: (1, 1), 1: (10, 10), 2: (5, 4), 3: (1, 1), 4: (2, 4), 5: (2, 4), 6: (2, 1)}


def eval_from_dump(d, maxplayer):
    """numpy restatement of SimpleSqrtEvaluationFunction3 over a canonical state dump."""
    f32, f64 = np.float32, np.float64
    res = [int(d[2]), int(d[3])]
    nu = int(d[4])
    units = np.asarray(d[5:5 + 6 * nu]).reshape(nu, 6)

    def base(p):
        score = f32(res[p]) * f32(20)
        any_unit = False
        for t, pl, _x, _y, hp, r in units:
            if pl != p:
                continue
            any_unit = True
            score = f32(score + f32(r) * f32(10))
            cost, mhp = UTT1[int(t)]
            bonus = f64(f32(40.0) * f32(cost)) * np.sqrt(f64(int(hp) // mhp))
            score = f32(f64(score) + bonus)
        return score if any_unit else f32(0)

    s1, s2 = base(maxplayer), base(1 - maxplayer)
    if f32(s1 + s2) == 0:
        return f32(0.5)
    return f32(f32(f32(2) * s1) / f32(s1 + s2)) - f32(1)


# ------------------------------------------------------------------ CPU: the oracle's new pieces


def test_initial_evaluation_kat():
    fm = oracle_py.OracleForwardModel(1, M8, RB, RB, seed=3)
    # per player: 5 resources * 20 + Base 40*10*sqrt(1) + Worker 40*1*sqrt(1) = 540 -> 2*540/1080 - 1
    assert fm.evaluate(0, 0) == np.float32(0.0) and fm.evaluate(0, 1) == np.float32(0.0)


def test_clone_reproduces_source():
    fm = oracle_py.OracleForwardModel(4, M8, RB, RB, seed=11)
    fm.playout(0, 37)  # mid-game, with in-flight assignments
    d0 = fm.dump(0)
    assert d0[5 + 6 * d0[4]] > 0, "want assignments in the cloned state"
    fm.copy(1, 0)
    assert np.array_equal(fm.dump(1), d0)
    # same state + same seeds -> same continuation; the clone is independent of its source
    fm.copy(2, 0)
    fm2 = oracle_py.OracleForwardModel(4, M8, RB, RB, seed=11)
    fm2.playout(0, 37)
    fm2.playout(0, 50)
    fm.playout(0, 50)
    assert np.array_equal(fm.dump(0), fm2.dump(0))
    assert np.array_equal(fm.dump(1), d0) and np.array_equal(fm.dump(2), d0)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_evaluation_matches_numpy_restatement(seed):
    fm = oracle_py.OracleForwardModel(6, M8, [RB, RB, PASSIVE, RB, RB, RB], [RB, PASSIVE, RB, RB, RB, RB], seed=seed)
    seen = set()
    for chunk in range(12):
        for g in range(6):
            fm.playout(g, 40 + 7 * g)
            d = fm.dump(g)
            for mp in (0, 1):
                v = fm.evaluate(g, mp)
                assert v == eval_from_dump(d, mp), (chunk, g, mp)
                seen.add(float(v))
    assert len(seen) > 5  # not vacuous: many distinct scores


def test_playout_loop_exits():
    fm = oracle_py.OracleForwardModel(3, M4, RB, RB, seed=5)
    # horizon 0 on an incomplete state: the do-while issues once and stops before the cycle
    fm.playout(0, 0)
    d = fm.dump(0)
    assert d[0] == 0 and d[5 + 6 * d[4]] > 0
    # then the next call cycles first (the state is complete)
    fm.playout(0, 1)
    assert fm.dump(0)[0] == 1
    # a long horizon ends at gameover (base4x4 RandomBiased games finish)
    fm.playout(1, 20000)
    d = fm.dump(1)
    owners = set(int(p) for p in np.asarray(d[5:5 + 6 * d[4]]).reshape(-1, 6)[:, 1]) - {-1}
    assert len(owners) <= 1 and d[0] < 20000


# ------------------------------------------------------------------ GPU: HIP forward model vs oracle


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def _mixed(n):
    ai1 = [RB, RB, PASSIVE, RB] * (n // 4)
    ai2 = [RB, PASSIVE, RB, RB] * (n // 4)
    name = {RB: "RandomBiasedAI", PASSIVE: "PassiveAI"}
    return ai1, ai2, [name[k] for k in ai1], [name[k] for k in ai2]


def _compare(gpu, ref, n, tag, evals=True):
    for g in range(n):
        assert np.array_equal(gpu.dump_state(g), ref.dump(g)), f"{tag}: state of game {g}"
    if evals:
        for mp in (0, 1):
            v = gpu.evaluate(mp).cpu().numpy()
            for g in range(n):
                assert v[g] == ref.evaluate(g, mp), f"{tag}: evaluation of game {g} for player {mp}"
    assert not gpu.error_flags().any()


@pytest.mark.gpu
@pytest.mark.parametrize("mp", [M8, M16])
def test_gpu_playouts_match_oracle(mp):
    _torch()
    from microrts_amd import ForwardModel

    n = 16
    ai1, ai2, n1, n2 = _mixed(n)
    gpu = ForwardModel(n, mp, policies=(n1, n2), seed=21)
    ref = oracle_py.OracleForwardModel(n, mp, ai1, ai2, seed=21)
    _compare(gpu, ref, n, "initial")
    for chunk, horizon in enumerate([0, 1, 13, 50, 100, 0, 200, 300]):
        gpu.playout(horizon)
        for g in range(n):
            ref.playout(g, horizon)
        _compare(gpu, ref, n, f"chunk {chunk} (horizon {horizon})")
    gpu.close()


@pytest.mark.gpu
def test_gpu_clone_within_forward_model():
    torch = _torch()
    from microrts_amd import ForwardModel

    n = 16
    gpu = ForwardModel(n, M8, seed=4)
    ref = oracle_py.OracleForwardModel(n, M8, RB, RB, seed=4)
    rng = np.random.default_rng(0)
    for rnd in range(6):
        gpu.playout(23 + rnd)
        for g in range(n):
            ref.playout(g, 23 + rnd)
        # a tree-search expansion: half the games become clones of the other half
        src = rng.choice(n, n // 2, replace=False)
        dst = np.setdiff1d(np.arange(n), src)
        rng.shuffle(dst)
        pairs = np.stack([dst, src], 1).astype(np.int32)
        if rnd % 2:
            gpu.copy_from(torch.as_tensor(pairs, device="cuda"))
        else:
            gpu.copy_from(pairs)
        for d, s in pairs:
            ref.copy(int(d), int(s))
        _compare(gpu, ref, n, f"round {rnd} after clone")
    gpu.close()


@pytest.mark.gpu
def test_gpu_clone_from_vec_env_then_playout():
    """MCTS use: clone the live self-play games of a DeviceVecEnv (stepped with the Philox policy in
    lockstep with the oracle VecClient), then run playouts from those roots."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv, ForwardModel

    S = 8
    env = DeviceVecEnv(S, 0, 2000, [M8] * S, seed=17)
    vref = oracle_py.OracleVecClient(S, 0, 2000, [M8] * S, seed=17)
    env.reset()
    vref.reset()
    seed = 0x5EEDC0DE
    for step in range(60):
        m = vref.get_masks(0)
        acts = np.stack([oracle_py.policy(m[s], seed, s, step, 0) for s in range(S)])
        env.actions.copy_(torch.as_tensor(acts))
        env.step()
        vref.step(acts)
    n = 8
    gpu = ForwardModel(n, M8, seed=99)
    ref = oracle_py.OracleForwardModel(n, M8, RB, RB, seed=99)
    pairs = np.array([[j, j % (S // 2)] for j in range(n)], np.int32)  # two clones of each game
    gpu.copy_from(pairs, src=env)
    for d, g in pairs:
        ref.copy_from_vec(int(d), vref, int(2 * g))
    _compare(gpu, ref, n, "cloned roots")
    gpu.playout(100)
    for g in range(n):
        ref.playout(g, 100)
    _compare(gpu, ref, n, "after playout")
    env.close()
    gpu.close()


@pytest.mark.gpu
def test_gpu_playout_to_gameover_and_argument_checks():
    _torch()
    from microrts_amd import DeviceVecEnv, ForwardModel

    n = 8
    gpu = ForwardModel(n, M4, seed=8)
    ref = oracle_py.OracleForwardModel(n, M4, RB, RB, seed=8)
    gpu.playout(20000)
    for g in range(n):
        ref.playout(g, 20000)
    _compare(gpu, ref, n, "gameover")
    gpu.playout(5)  # a finished game still runs the do-while's first pass, as the Java does
    for g in range(n):
        ref.playout(g, 5)
    _compare(gpu, ref, n, "after gameover")
    with pytest.raises(RuntimeError):
        gpu.copy_from([[0, 1], [0, 2]])  # a destination twice
    with pytest.raises(RuntimeError):
        gpu.copy_from([[0, 1], [1, 2]])  # game 1 both source and destination
    with pytest.raises(ValueError):
        gpu.playout(1 << 20)
    other = DeviceVecEnv(2, 0, 100, [M8] * 2)
    with pytest.raises(RuntimeError):
        gpu.copy_from([[0, 0]], src=other)  # different map size
    from microrts_amd import _lib

    with pytest.raises(RuntimeError):  # a forward model is not stepped
        _lib.check(gpu._h.L.mrts_step_dev(gpu._h.h, None, None, None, None, None, None, 0, None))
    other.close()
    gpu.close()


@pytest.mark.gpu
def test_gpu_full_size_playouts_deterministic():
    """4096 games of 16x16 with NaiveMCTS's default lookahead (MAXSIMULATIONTIME = 1024): clones of
    one root replay identically when their streams are identical, a sample matches the oracle."""
    torch = _torch()
    from microrts_amd import ForwardModel

    n = 4096
    gpu = ForwardModel(n, M16, seed=1000)
    gpu.playout(1024)
    torch.cuda.synchronize()
    sample = [0, 1, 777, 2048, 4095]
    ref = oracle_py.OracleForwardModel(n, M16, RB, RB, seed=1000)
    for g in sample:
        ref.playout(g, 1024)
        assert np.array_equal(gpu.dump_state(g), ref.dump(g)), g
    v = gpu.evaluate(0).cpu().numpy()
    for g in sample:
        assert v[g] == ref.evaluate(g, 0)
    assert np.all((v >= -1) & (v <= 1))
    assert not gpu.error_flags().any()
    gpu.close()
