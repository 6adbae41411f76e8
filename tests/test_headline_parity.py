"""The shipped benchmark forms against the CPU oracle, at the BASELINE configs' full sizes.

bench.py times each config as ONE native rollout call that runs K steps per `k_env` launch
(multi-step launches).  Here the same calls run at the bench's sizes (c3: 4096
self-play games on 16x16; c2: 1024 games on 8x8; c5: 2048 partially observable games on 32x32 with
max_units 256) after a 1000-step burn-in, followed by K = 20 and K = 200 step launches.  65-66
picked games (two for each of the 8 XCD classes in each of the 4 SIMD slots of the launch's
placement, plus the first and the last game; _pick_games) are replayed by the oracle with its OWN policy stream: the oracle computes its masks
(JNIGridnetVecClient.getMasks, :307-316) and samples the same Philox masked-uniform (or unmasked
uniform) rows from them, so no GPU-produced action ever enters the oracle.  UTT v1 + CANCEL_BOTH
draws no Java random numbers, so such an oracle game is an exact replica of the picked GPU game.  At
each launch end: observations, rewards, dones, masks, the next action rows and the canonical state
dumps (units in list order, assignments in LinkedHashMap order) must be bit-identical.

Also here: TestLoadingMaps (test/microrts/TestLoadingMaps.java:24-51) on the product path — all 140
maps through the host parser + on-device reset, against the oracle's parser — and the C-ABI
contract that a write to d_actions between fused calls needs mrts_policy_invalidate().
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from tests import oracle_py

pytestmark = pytest.mark.gpu

SEED = 0x5EEDC0DE
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BURNIN = 1000


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _pick_games(n_games, per=2):
    """64 games spread over the launch's placement classes: the dispatcher puts blocks
    b, b + n/4, b + 2n/4, b + 3n/4 on one SIMD and block b on XCD b % 8, and balanced placement
    (mrts_kernels.hip balancePerm) permutes games within their XCD class — so `per` games for each of
    the 8 XCD classes in each of the 4 SIMD-slot quarters, at scattered offsets; plus the first and
    the last game."""
    q = n_games // 4
    g = {k * q + 8 * ((37 * k + 101 * j + 11 * c + 3) % (q // 8)) + c for k in range(4) for c in range(8) for j in range(per)}
    g |= {0, n_games - 1}
    return sorted(g)


def _picks(n_games):
    """The slots (both players) of _pick_games."""
    return [s for k in _pick_games(n_games) for s in (2 * k, 2 * k + 1)]


class _MaskedReplica:
    """Oracle self-play games replaying picked GPU slots under the masked-uniform policy: the
    actions of step t are oracle_py.policy(the oracle's own masks, SEED, global slot id, t)."""

    def __init__(self, mp, picks, seed, partial_obs=False):
        self.picks = picks
        self.ref = oracle_py.OracleVecClient(len(picks), 0, 2000, [mp] * len(picks), seed=seed, partial_obs=partial_obs)
        self.ref.reset()
        self.t = 0

    def actions(self, step):
        m = self.ref.get_masks(0)
        return m, np.stack([oracle_py.policy(m[i], SEED, s, step, 0) for i, s in enumerate(self.picks)])

    def run(self, n):
        for _ in range(n):
            _, a = self.actions(self.t)
            self.ref.step(a)
            self.t += 1


def _compare_launch_end(env, rep, tag):
    env.synchronize()
    ref, picks = rep.ref, rep.picks
    assert np.array_equal(env.obs.cpu().numpy()[picks], ref.obs), f"{tag}: observations"
    assert np.array_equal(env.reward.cpu().numpy()[picks], ref.reward), f"{tag}: rewards"
    assert np.array_equal(env.done.cpu().numpy()[picks], ref.done), f"{tag}: dones"
    m, nxt = rep.actions(rep.t)  # the rows the launch sampled for the next step
    assert np.array_equal(env.masks.cpu().numpy()[picks], m), f"{tag}: masks"
    assert np.array_equal(env.actions.cpu().numpy()[picks], nxt), f"{tag}: next action rows"
    for i, s in enumerate(picks):
        assert np.array_equal(env.dump_state(s), ref.dump(i)), f"{tag}: state of slot {s}"


def _masked_multi_step(mp, n_games, seed, partial_obs=False, max_units=0):
    _torch()
    from microrts_amd import DeviceVecEnv

    S = 2 * n_games
    env = DeviceVecEnv(S, 0, 2000, [mp] * S, seed=seed, partial_obs=partial_obs, max_units=max_units)
    assert env.fused_multi_step, "the bench's shape must run multi-step launches"
    rep = _MaskedReplica(mp, _picks(n_games), seed, partial_obs)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, BURNIN)  # the first launch is a single step, then multi-step launches
    rep.run(BURNIN)
    _compare_launch_end(env, rep, f"after the {BURNIN}-step burn-in")
    k = BURNIN
    for K in (20, 200):  # the driver's K and the bench default
        env.rollout_fused(SEED, k + 1, K)
        rep.run(K)
        k += K
        _compare_launch_end(env, rep, f"after a {K}-step launch (step {k})")
    assert not env.error_flags().any()
    env.close()
    rep.ref.close()


def test_full_size_c3_multi_step():
    """BASELINE configs[2] (c3) as bench.py times it: 4096 self-play games on basesWorkers16x16, the
    fused masked policy, delta masks, K steps per k_env launch."""
    _masked_multi_step("maps/16x16/basesWorkers16x16.xml", 4096, seed=5)


def test_full_size_c5_multi_step():
    """BASELINE configs[4] (c5) per GPU: 2048 partially observable self-play games on
    BWDistantResources32x32, max_units 256, multi-step launches with incremental PO views."""
    _masked_multi_step("maps/BWDistantResources32x32.xml", 2048, seed=7, partial_obs=True, max_units=256)


def test_full_size_c2_multi_step():
    """BASELINE configs[1] (c2) as bench.py times it: 1024 games on basesWorkers8x8, unmasked uniform
    rows drawn by the step kernel, K steps per launch.  The oracle draws the same rows itself
    (oracle_py.policy_uniform = mrts_policy_uniform_dev's Philox stream)."""
    _torch()
    from microrts_amd import DeviceVecEnv

    E = 1024
    mp = "maps/8x8/basesWorkers8x8.xml"
    env = DeviceVecEnv(2 * E, 0, 2000, [mp] * (2 * E), seed=8)
    assert env.multi_step_capable
    S, H, W, C, K = env.dims
    picks = _picks(E)
    ref = oracle_py.OracleVecClient(len(picks), 0, 2000, [mp] * len(picks), seed=8)
    env.reset()
    ref.reset()
    t = 0

    def ref_run(n):
        nonlocal t
        for _ in range(n):
            ref.step(np.stack([oracle_py.policy_uniform(H, W, K, SEED, s, t) for s in picks]))
            t += 1

    for n in (BURNIN, 20, 200):
        env.rollout_uniform(SEED, t, n, fused=True)
        ref_run(n)
        env.synchronize()
        tag = f"c2 after a {n}-step rollout (step {t})"
        assert np.array_equal(env.obs.cpu().numpy()[picks], ref.obs), f"{tag}: observations"
        assert np.array_equal(env.reward.cpu().numpy()[picks], ref.reward), f"{tag}: rewards"
        assert np.array_equal(env.done.cpu().numpy()[picks], ref.done), f"{tag}: dones"
        last = np.stack([oracle_py.policy_uniform(H, W, K, SEED, s, t - 1) for s in picks])
        assert np.array_equal(env.actions.cpu().numpy()[picks], last), f"{tag}: the last step's rows"
        for i, s in enumerate(picks):
            assert np.array_equal(env.dump_state(s), ref.dump(i)), f"{tag}: state of slot {s}"
    assert not env.error_flags().any()
    env.close()
    ref.close()


MAPS = sorted(glob.glob(os.path.join(ROOT, "maps", "**", "*.xml"), recursive=True))


def test_all_maps_load_product_path():
    """TestLoadingMaps (test/microrts/TestLoadingMaps.java:24-51) on the product path: every one of
    the 140 maps goes through libmrts's host XML parser (terrain RLE, PhysicalGameState.java:577-607,
    765-777; units in file order, Unit.java:597-620) into a device template and an on-device reset.
    The reset observation and the canonical state dump equal the oracle's parse.  Maps above 64x64
    cells run with max_units 1024 (their full unit capacity does not fit one CU's LDS; the largest
    map holds 64 units)."""
    _torch()
    from microrts_amd import DeviceVecEnv

    assert len(MAPS) == 140
    for m in MAPS:
        rel = os.path.relpath(m, ROOT)
        ref = oracle_py.OracleVecClient(2, 0, 100, [rel, rel])
        obs, _, _ = ref.reset()
        mu = 1024 if ref.H * ref.W > 64 * 64 else 0
        env = DeviceVecEnv(2, 0, 100, [rel, rel], max_units=mu)
        env.reset()
        env.synchronize()
        assert env.dims[1:3] == (ref.H, ref.W), rel
        assert np.array_equal(env.obs.cpu().numpy(), obs), f"{rel}: reset observation"
        assert np.array_equal(env.masks.cpu().numpy(), ref.get_masks(0)), f"{rel}: reset masks"
        for s in (0, 1):
            assert np.array_equal(env.dump_state(s), ref.dump(s)), f"{rel}: state"
        env.close()
        ref.close()


def test_c_abi_fused_write_needs_invalidate():
    """include/mrts.h: a fused call keeps the rows it sampled and the next fused call on
    the same d_actions decodes from that copy.  Through the raw C entry points (no Python version
    counter involved): rows written into d_actions between fused calls are used iff
    mrts_policy_invalidate() is called — then the step equals a plain mrts_step_dev of those rows on
    a twin handle; without it they are ignored (the documented contract, shown here to hold)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n = 16
    mp = "maps/16x16/basesWorkers16x16.xml"
    A, B, C = (DeviceVecEnv(n, 0, 300, [mp] * n, seed=5) for _ in range(3))
    L = B._h.L
    p = DeviceVecEnv._p

    def raw_fused(e, k):
        s = ctypes.c_void_p(torch.cuda.current_stream(e.device).cuda_stream)
        r = L.mrts_step_fused_dev(e._h.h, p(e.actions), p(e.players), p(e.obs), p(e.reward), p(e.done), p(e.masks), 0,
                                  SEED, k, s)
        assert r == 0

    for e in (A, B, C):
        e.reset()
        e.random_policy(SEED, 0)
    for k in range(12):
        A.step()
        A.random_policy(SEED, k + 1)
        raw_fused(B, k + 1)
        raw_fused(C, k + 1)
    torch.cuda.synchronize()
    for name in ("obs", "masks", "actions"):
        assert torch.equal(getattr(A, name), getattr(B, name)) and torch.equal(getattr(A, name), getattr(C, name))
    g = torch.Generator(device="cpu").manual_seed(3)
    hi = torch.tensor([6, 4, 4, 4, 4, 7, 49], dtype=torch.int32)
    alt = (torch.rand(tuple(A.actions.shape), generator=g) * hi).to(torch.int32).to(A.device)
    for e in (A, B, C):
        e.actions.copy_(alt)
    assert L.mrts_policy_invalidate(B._h.h) == 0
    A.step()  # the plain step decodes every row of d_actions
    raw_fused(B, 100)
    raw_fused(C, 100)  # no invalidate: decodes the kept copy of the previous sample
    torch.cuda.synchronize()
    for s in range(0, n, 2):
        assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"invalidated fused step, slot {s}"
    assert any(not np.array_equal(A.dump_state(s), C.dump_state(s)) for s in range(0, n, 2)), \
        "without invalidate the written rows should have been ignored"
    for e in (A, B, C):
        e.close()


def _exchange_env(env, world=1, rank=0):
    import ctypes

    from microrts_amd import _lib
    from microrts_amd.dist import rccl_library_path

    L, h = env._h.L, env._h.h
    path = rccl_library_path().encode()
    uid = (ctypes.c_char * 128)()
    _lib.check(L.mrts_rccl_unique_id(path, uid))
    _lib.check(L.mrts_exchange_init(h, path, world, rank, uid))
    return path, uid


@pytest.mark.parametrize("mp,uniform,u8", [("maps/16x16/basesWorkers16x16.xml", False, False),
                                           ("maps/16x16/basesWorkers16x16.xml", False, True),
                                           ("maps/8x8/basesWorkers8x8.xml", True, False),
                                           ("maps/8x8/basesWorkers8x8.xml", True, True)])
def test_native_exchange_one_rank(mp, uniform, u8):
    """mrts_rollout_{fused,uniform}_exchange_dev on a one-rank RCCL communicator: every output equals the
    same rollout with one launch per step and no exchange (observations, rewards, dones, masks, next
    actions, states), the last step's int16 observation arrived in recv[0], and the send buffers alternate
    (the last step's in send[(n - 1) % 2]); with mrts_set_exchange_bytes(1) the same as uint8 (refused
    on a shape no uint8 render writes); a second mrts_exchange_init and a partially observable
    handle are refused."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp = 64
    A = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=21, with_masks=not uniform)
    B = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=21, with_masks=not uniform)
    A.set_multi_step(False)
    for e in (A, B):
        e.reset()
        if not uniform:
            e.random_policy(SEED, 0)
    path, uid = _exchange_env(B)
    dt = torch.uint8 if u8 else torch.int16
    if u8:
        assert B._h.L.mrts_set_exchange_bytes(B._h.h, 1) == 0
    else:
        assert B._h.L.mrts_set_exchange_bytes(B._h.h, 3) != 0  # 1 or 2 bytes only
    send = [torch.zeros(tuple(B.obs.shape), dtype=dt, device=B.device) for _ in range(2)]
    recv = torch.zeros((1,) + tuple(B.obs.shape), dtype=dt, device=B.device)
    k = 0
    for n in (1, 2, 7, 120):
        if uniform:
            A.rollout_uniform(SEED, k, n)
            B.rollout_uniform_exchange(SEED, k, n, send, recv)
        else:
            A.rollout_fused(SEED, k + 1, n)
            B.rollout_fused_exchange(SEED, k + 1, n, send, recv)
        k += n
        A.synchronize()
        B.synchronize()
        for name in ("obs", "reward", "done", "actions") + (() if uniform else ("masks",)):
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{name} after {k}"
        for s in range(0, n_sp, 2):
            assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s} after {k}"
        assert int(B.obs.max()) < 256 and int(B.obs.min()) >= 0
        ox = B.obs.to(dt)
        assert torch.equal(recv[0], ox), f"recv after {k}"
        assert torch.equal(send[(n - 1) % 2], ox), f"send buffer after {k}"
    assert B._h.L.mrts_exchange_init(B._h.h, path, 1, 0, uid) != 0  # already initialised
    P = DeviceVecEnv(8, 0, 300, ["maps/BWDistantResources32x32.xml"] * 8, seed=1, partial_obs=True, max_units=256)
    assert P._h.L.mrts_set_exchange_bytes(P._h.h, 1) != 0
    P.reset()
    P.random_policy(SEED, 0)
    _exchange_env(P)
    with pytest.raises(Exception):
        P.rollout_fused_exchange(SEED, 1, 2, [torch.zeros(tuple(P.obs.shape), dtype=torch.int16, device=P.device)] * 2,
                                 torch.zeros((1,) + tuple(P.obs.shape), dtype=torch.int16, device=P.device))
    for e in (A, B, P):
        assert not e.error_flags().any()
        e.close()


def test_native_exchange_graph_replay():
    """mrts_capture_begin / _end / mrts_replay around an exchange rollout: the replay reruns the
    captured steps verbatim — from the same start state it produces the same buffers as the eager call
    (observations, masks, next actions, states, and the all-gathered int16 observation)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp, n_sp = "maps/16x16/basesWorkers16x16.xml", 32
    A = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=4)
    B = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=4)
    bufs = []
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
        e.rollout_fused(SEED, 1, 30)
        _exchange_env(e)
        bufs.append(([torch.zeros(tuple(e.obs.shape), dtype=torch.int16, device=e.device) for _ in range(2)],
                     torch.zeros((1,) + tuple(e.obs.shape), dtype=torch.int16, device=e.device)))
    A.rollout_fused_exchange(SEED, 31, 12, *bufs[0])
    ck = B.checkpoint()
    cap = torch.cuda.Stream(B.device)
    cap.wait_stream(torch.cuda.current_stream(B.device))
    B.capture(lambda: B.rollout_fused_exchange(SEED, 31, 12, *bufs[1]), cap)
    torch.cuda.current_stream(B.device).wait_stream(cap)
    torch.cuda.synchronize()
    B.restore(ck)  # capture ran nothing: the replay starts from the same state
    B.replay()
    A.synchronize()
    B.synchronize()
    for name in ("obs", "reward", "done", "masks", "actions"):
        assert torch.equal(getattr(A, name), getattr(B, name)), name
    for s in range(0, n_sp, 2):
        assert np.array_equal(A.dump_state(s), B.dump_state(s)), f"state slot {s}"
    assert torch.equal(bufs[0][1], bufs[1][1])
    for e in (A, B):
        assert not e.error_flags().any()
        e.close()


def test_values_beyond_a_byte_after_injection():
    """the 16x16 byte-image render and the uint8 exchange transport hold values 0..255
    only.  A state injected by GameState.fromJSON (rts/GameState.java:897-915) may carry more: a Resource
    with 300 resources and a Base with 1000 must still show exactly in the int32 observation — in single
    steps and in multi-step launches — and the uint8 transport must then be refused."""
    import json

    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp, n_sp = "maps/16x16/basesWorkers16x16.xml", 8
    env = DeviceVecEnv(n_sp, 0, 2000, [mp] * n_sp, seed=9)
    assert env.fused_multi_step
    rep = _MaskedReplica(mp, list(range(n_sp)), 9)
    assert env._h.L.mrts_set_exchange_bytes(env._h.h, 1) == 0  # every map value fits a byte
    env.reset()
    d = json.loads(rep.ref.state_json(0))
    res = [u for u in d["pgs"]["units"] if u["type"] == "Resource"]
    base = [u for u in d["pgs"]["units"] if u["type"] == "Base"]
    res[0]["resources"] = 300
    base[0]["hitpoints"] = 1000
    j = json.dumps(d)
    for s in (0, 4):
        env.set_state_json(s, j)
        rep.ref.set_state_json(s, j)
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, 1)  # a single step, then multi-step launches
    rep.run(1)
    _compare_launch_end(env, rep, "after one step")
    ob = env.obs.cpu().numpy()
    assert ob[0, 1].max() == 300 and ob[0, 0].max() == 1000, "the injected values must show unclipped"
    env.rollout_fused(SEED, 2, 40)
    rep.run(40)
    _compare_launch_end(env, rep, "after a 40-step launch")
    assert env._h.L.mrts_set_exchange_bytes(env._h.h, 1) != 0, "uint8 transport after values > 255"
    env.close()
    rep.ref.close()


def test_exchange_needs_an_observation_buffer():
    """the exchange's send buffers are written by the step's observation write, so an
    exchange rollout without d_obs would all-gather stale data — it is refused (-EINVAL)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    mp, n_sp = "maps/16x16/basesWorkers16x16.xml", 4
    B = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=3)
    B.reset()
    B.random_policy(SEED, 0)
    _exchange_env(B)
    send = [torch.zeros(tuple(B.obs.shape), dtype=torch.int16, device=B.device) for _ in range(2)]
    recv = torch.zeros((1,) + tuple(B.obs.shape), dtype=torch.int16, device=B.device)
    p = DeviceVecEnv._p
    st = ctypes.c_void_p(torch.cuda.current_stream(B.device).cuda_stream)
    r = B._h.L.mrts_rollout_fused_exchange_dev(B._h.h, p(B.actions), p(B.players), None, p(B.reward), p(B.done), p(B.masks), 0,
                                               SEED, 1, 2, p(send[0]), p(send[1]), p(recv), st)
    assert r == -22
    B.close()


@pytest.mark.parametrize("mp,uniform,spl,max_steps,po", [("maps/16x16/basesWorkers16x16.xml", False, 0, 300, False),
                                                         ("maps/16x16/basesWorkers16x16.xml", False, 7, 300, False),
                                                         ("maps/16x16/basesWorkers16x16.xml", False, 0, 13, False),
                                                         ("maps/8x8/basesWorkers8x8.xml", True, 0, 300, False),
                                                         ("maps/8x8/basesWorkers8x8.xml", True, 0, 11, False),
                                                         ("maps/BWDistantResources32x32.xml", False, 0, 300, True),
                                                         ("maps/BWDistantResources32x32.xml", False, 9, 17, True),
                                                         ("maps/16x16/basesWorkers16x16.xml", False, 0, 300, True),
                                                         ("maps/8x8/basesWorkers8x8.xml", True, 0, 300, True),
                                                         ("maps/8x8/basesWorkers8x8.xml", False, 0, 400, "dead"),
                                                         ("maps/16x16/EightBasesWorkers16x16.xml", False, 0, 300, "many")])
def test_record_exchange_one_rank(mp, uniform, spl, max_steps, po):
    """the compact observation exchange (mrts_rollout_*_records_dev) on a one-rank
    RCCL communicator.  Every step's records, all-gathered and rendered back on the receiving side
    (mrts_render_records_dev, int32 and uint8 / int8), equal the sender's own int32 observation of that
    step — taken from a twin handle stepped one launch per step — while the records rollout runs its steps
    as multi-step launches (spl = steps per launch, 0 = one launch); every other output equals the twin's.
    A small max_steps puts auto-resets inside the launches (the record then holds the reset state).
    po: partially observable handles (two record words per unit of either view; the receiver paints the
    sight disks) — the 32x32 map runs c5's helper-wave kernel in the records rollout; po = "dead": 266
    masked random steps on 8x8, long enough that a view shows units that died in the step (their hp <= 0,
    kept by the view's snapshot until the compaction), and the test checks that one did.  po = "many"
    (the 64-unit record): full observability on a map that starts with 64 units, records
    sized to the map's cell count (one unit per cell at most, so no game can overflow them) — the games pass
    64 live units (the general paths beyond one wave) and every step still renders exactly."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    many = po == "many"
    po = False if many else po
    n_sp = 64
    kw = dict(partial_obs=True, max_units=256) if po else dict(max_units=256) if many else {}
    A = DeviceVecEnv(n_sp, 0, max_steps, [mp] * n_sp, seed=23, with_masks=not uniform, **kw)
    B = DeviceVecEnv(n_sp, 0, max_steps, [mp] * n_sp, seed=23, with_masks=not uniform, **kw)
    A.set_multi_step(False)
    for e in (A, B):
        e.reset()
        if not uniform:
            e.random_policy(SEED, 0)
    _exchange_env(B)
    units = 256 if many else 64
    words = B.set_records(units, spl)
    assert words == units + 1 or po
    B.set_step_responses(100)  # every step's reward / done
    S = n_sp
    k = 0
    dead_seen = False
    most = 0
    for n in (1, 40, 25) + ((100, 100) if po == "dead" else ()):
        want, wantR, wantD = [], [], []
        for j in range(n):
            if uniform:
                A.rollout_uniform(SEED, k + j, 1)
            else:
                A.rollout_fused(SEED, k + j + 1, 1)
            A.synchronize()
            want.append(A.obs.clone())
            wantR.append(A.reward.clone())
            wantD.append(A.done.clone())
            if po:
                dead_seen |= bool(((want[-1][:, 0] <= 0) & (want[-1][:, 3] > 0)).any())
        recv = B.records_buffer(n)
        off = B.rollout_uniform_records(SEED, k, n, recv) if uniform else B.rollout_fused_records(SEED, k + 1, n, recv)
        k += n
        B.synchronize()
        assert off.shape == (n, 2) and (off[:, 1] % ((S // 2) * words) == 0).all()
        for j in range(n):
            got = torch.zeros_like(B.obs)
            B.render_records(recv, off[j, 0], off[j, 1], 1, got)
            g8 = torch.zeros(tuple(B.obs.shape), dtype=torch.int8 if po else torch.uint8, device=B.device)
            B.render_records(recv, off[j, 0], off[j, 1], 1, g8)
            B.synchronize()
            assert torch.equal(got, want[j]), f"step {k - n + j}: rendered int32 observation"
            assert torch.equal(g8.to(torch.int32), want[j]), f"step {k - n + j}: rendered byte observation"
            assert torch.equal(B.step_rewards[j], wantR[j]), f"step {k - n + j}: the Responses ring's reward"
            assert torch.equal(B.step_dones[j], wantD[j]), f"step {k - n + j}: the Responses ring's done"
        for name in ("obs", "actions") + (() if uniform else ("masks",)):  # (reward / done: the ring's, above)
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{name} after {k}"
        for s in range(0, n_sp, 2):
            d = A.dump_state(s)
            assert np.array_equal(d, B.dump_state(s)), f"state slot {s} after {k}"
            most = max(most, int(d[4]))
    for e in (A, B):
        assert not e.error_flags().any()
    if po == "dead":
        assert dead_seen, "no view showed a unit that died in its step"
    if many:
        assert most > 64, f"the games never passed 64 units (most {most})"
    # a record too small for the games' unit lists is an error, not a silent truncation
    assert B.set_records(2, 0) == (5 if po else 3)
    recv = B.records_buffer(2)
    if uniform:
        B.rollout_uniform_records(SEED, k, 2, recv)
    else:
        B.rollout_fused_records(SEED, k + 1, 2, recv)
    B.synchronize()
    assert (B.error_flags() & (1 << 6)).any(), "MRTS_ERR_RECORD"
    for e in (A, B):
        e.close()


def test_step_responses_every_reward_function():
    """mrts_set_step_responses with all 8 reward functions (reward / done [slots][8]) and
    both rollout forms the benchmark shapes run as multi-step launches (c3's masked fused rollout, c2's
    uniform one): every step's ring entry equals the reward / done a twin returns from one launch per step,
    across auto-resets (max_steps 60 and gameovers); d_reward / d_done are left alone while the ring is on;
    a call longer than the ring is refused; NULL turns it off (then the plain buffers again)."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv
    from microrts_amd._lib import REWARD_FUNCTIONS

    rfs = list(REWARD_FUNCTIONS)
    for mp, uniform in (("maps/16x16/basesWorkers16x16.xml", False), ("maps/8x8/basesWorkers8x8.xml", True)):
        n_sp = 32
        A = DeviceVecEnv(n_sp, 0, 60, [mp] * n_sp, seed=31, rfs=rfs, with_masks=not uniform)
        B = DeviceVecEnv(n_sp, 0, 60, [mp] * n_sp, seed=31, rfs=rfs, with_masks=not uniform)
        A.set_multi_step(False)
        for e in (A, B):
            e.reset()
            if not uniform:
                e.random_policy(SEED, 0)
        B.set_step_responses(150)
        k = 0
        saw_done = False
        for n in (1, 150, 37):
            wantR, wantD = [], []
            for j in range(n):
                if uniform:
                    A.rollout_uniform(SEED, k + j, 1)
                else:
                    A.rollout_fused(SEED, k + j + 1, 1)
                A.synchronize()
                wantR.append(A.reward.clone())
                wantD.append(A.done.clone())
            if uniform:
                B.rollout_uniform(SEED, k, n)
            else:
                B.rollout_fused(SEED, k + 1, n)
            k += n
            B.synchronize()
            for j in range(n):
                assert torch.equal(B.step_rewards[j], wantR[j]), f"{mp}: step {k - n + j} reward"
                assert torch.equal(B.step_dones[j], wantD[j]), f"{mp}: step {k - n + j} done"
                saw_done |= bool(wantD[j][:, 0].any())
            for name in ("obs", "actions"):
                assert torch.equal(getattr(A, name), getattr(B, name)), f"{mp}: {name} after {k}"
            assert not bool(B._reward.any()) and not bool(B._done.any()), "the plain buffers are left alone"
            #  env.reward / env.done read the call's last ring step, not the stale plain buffers
            assert torch.equal(B.reward, wantR[-1]) and torch.equal(B.done, wantD[-1])
        assert saw_done, "no auto-reset inside the checked steps"
        with pytest.raises(RuntimeError):
            B.rollout_uniform(SEED, k, 151) if uniform else B.rollout_fused(SEED, k + 1, 151)
        B.set_step_responses(0)
        for e in (A, B):  # off again: the plain buffers receive the step
            if uniform:
                e.rollout_uniform(SEED, k, 3)
            else:
                e.rollout_fused(SEED, k + 1, 3)
        for name in ("obs", "reward", "done", "actions"):
            assert torch.equal(getattr(A, name), getattr(B, name)), f"{mp}: {name} with the ring off"
        for e in (A, B):
            assert not e.error_flags().any()
            e.close()


@pytest.mark.parametrize("mp,spl", [("maps/16x16/basesWorkers16x16.xml", 0), ("maps/8x8/basesWorkers8x8.xml", 7)])
def test_records_onehot_batch(mp, spl):
    """mrts_render_records_onehot_dev: a learner's batch — random slots of every rank of an
    8-rank loopback exchange — rendered from the records straight into MicroRTS-Py's one-hot layout equals
    the twin's int32 observation of the same slot (rank r's slot s = the twin's slot s + 2 (r - rank), the
    loopback's rotation) through mrts_onehot_dev, every step of 1 + 30 + 12 records steps."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp, world, rank = 64, 8, 3
    A = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=37)
    B = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=37)
    A.set_multi_step(False)
    for e in (A, B):
        e.reset()
        e.random_policy(SEED, 0)
    assert B._h.L.mrts_exchange_init_loopback(B._h.h, world, rank) == 0
    B.set_records(64, spl)
    g = torch.Generator(device="cpu").manual_seed(5)
    S, k = n_sp, 0
    for n in (1, 30, 12):
        want = []
        for j in range(n):
            A.rollout_fused(SEED, k + j + 1, 1)
            A.synchronize()
            want.append(A.onehot_obs().clone())
        recv = B.records_buffer(n, world)
        off = B.rollout_fused_records(SEED, k + 1, n, recv)
        k += n
        for j in range(n):
            sel = torch.randperm(world * S, generator=g)[:100].to(torch.int32)
            got = B.render_records_onehot(recv, off[j, 0], off[j, 1], sel.to(B.device))
            B.synchronize()
            r, s = sel // S, sel % S
            twin = (s + 2 * (r - rank)) % S
            assert torch.equal(got.cpu(), want[j].cpu()[twin.long()]), f"step {k - n + j}: one-hot batch"
        # one launch for a minibatch of random (step, slot) pairs over the whole call (per-sample step offsets)
        js = torch.randint(0, n, (300,), generator=g)
        sel = torch.randint(0, world * S, (300,), generator=g).to(torch.int32)
        so = torch.from_numpy(off[js.numpy()]).contiguous()  # each sample's step's (offset, rank stride)
        got = B.render_records_onehot(recv, 0, 0, sel.to(B.device), step_off=so.to(B.device)).cpu()
        B.synchronize()
        r, s = sel // S, sel % S
        twin = ((s + 2 * (r - rank)) % S).long()
        for i in range(300):
            assert torch.equal(got[i], want[int(js[i])][int(twin[i])].cpu()), f"minibatch sample {i}"
    assert not B.render_overflow()
    # a sample outside the buffer — an index outside [0, ranks x slots), a step_off row past the
    # receive buffer — renders as zeros and raises the render flag instead of reading past the buffer
    o, st = int(off[-1, 0]), int(off[-1, 1])
    bad = torch.tensor([-1, world * S, 5], dtype=torch.int32, device=B.device)
    got = B.render_records_onehot(recv, o, st, bad, n_ranks=world).cpu()
    assert not got[0].any() and not got[1].any() and got[2].any() and B.render_overflow()
    so = torch.tensor([[o, st], [recv.numel(), st], [o, 10 * recv.numel()]], dtype=torch.int64, device=B.device)
    bad = torch.tensor([5, 5, S + 5], dtype=torch.int32, device=B.device)  # (rank 1: its stride is out of range)
    got = B.render_records_onehot(recv, 0, 0, bad, step_off=so).cpu()
    assert got[0].any() and not got[1].any() and not got[2].any() and B.render_overflow()
    assert not B.render_overflow(), "the flag resets when read"
    with pytest.raises(RuntimeError):  # a rank stride reaching past the receive buffer
        B.render_records(recv, o, recv.numel(), 2, torch.zeros((2 * S,) + tuple(B.obs.shape[1:]), dtype=torch.int32,
                                                                device=B.device))
    for e in (A, B):
        assert not e.error_flags().any()
        e.close()


@pytest.mark.parametrize("mp,po,spl,world,rank", [("maps/16x16/basesWorkers16x16.xml", False, 0, 8, 3),
                                                  ("maps/16x16/basesWorkers16x16.xml", False, 7, 8, 7),
                                                  ("maps/BWDistantResources32x32.xml", True, 9, 4, 1)])
def test_record_exchange_loopback_ranks(mp, po, spl, world, rank):
    """The records exchange's multi-rank layout on one GPU (mrts_exchange_init_loopback: rank `rank` of
    `world`; peer r's place receives this rank's records with the games rotated by r - rank, so every
    rank's data differ — VERDICT r4 #4).  Every step's chunk: this rank's records sit unrotated at
    offset + rank x stride (the in-place all-gather's send = recv + rank x bytes) and peer r's place holds
    them rotated by r - rank games; rendering all `world` ranks gives, for rank r, the twin's int32
    observation with its slots rotated by 2 (r - rank) — a wrong rank offset, stride or chunk base, or a
    render that reads another rank's place, fails here (shown below by rendering a neighbour's place as
    this rank's), where RCCL cannot put two ranks on one device.  The tensor exchange's [ranks][...]
    receive buffer too (rotated by slots).  And the chunk schedule does not depend on whether a handle is
    in the steady fused state: a twin made unsteady by a get_masks call reports the same
    per-step offsets."""
    torch = _torch()
    from microrts_amd import DeviceVecEnv

    n_sp = 64
    kw = dict(partial_obs=True, max_units=256) if po else {}
    A = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=29, **kw)
    B = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=29, **kw)
    C = DeviceVecEnv(n_sp, 0, 300, [mp] * n_sp, seed=29, **kw)  # B's twin, never in the steady state at a call
    A.set_multi_step(False)
    for e in (A, B, C):
        e.reset()
        e.random_policy(SEED, 0)
    L, h = B._h.L, B._h.h
    assert L.mrts_exchange_init_loopback(h, world, world) != 0  # rank out of range
    assert L.mrts_exchange_init_loopback(h, world, rank) == 0
    assert L.mrts_exchange_init_loopback(h, world, rank) != 0  # already initialised
    assert L.mrts_exchange_init_loopback(C._h.h, world, rank) == 0
    words = B.set_records(64, spl)
    assert C.set_records(64, spl) == words
    distinct = 0  # steps whose games differed, so that a wrong rank place would have shown
    G = n_sp // 2
    k = 0
    for n in (1, 40, 25):
        want = []
        for j in range(n):
            A.rollout_fused(SEED, k + j + 1, 1)
            A.synchronize()
            want.append(A.obs.clone())
        recv = B.records_buffer(n, world)
        recv.fill_(-7)  # every record header the exchange owes must be written (unit words past n are don't-care)
        off = B.rollout_fused_records(SEED, k + 1, n, recv)
        C.get_masks()  # C leaves the steady fused state: its first launch of the call runs one step alone
        recvC = C.records_buffer(n, world)
        recvC.fill_(-7)  # (as recv: unit words past a record's n stay as they were)
        offC = C.rollout_fused_records(SEED, k + 1, n, recvC)
        assert np.array_equal(off, offC), "the chunk schedule must not depend on the steady state"
        k += n
        B.synchronize()
        C.synchronize()
        assert torch.equal(recv, recvC)
        for j in range(n):
            o, stride = int(off[j, 0]), int(off[j, 1])
            assert stride >= G * words and (o + (world - 1) * stride + G * words) <= recv.numel()
            mine = recv[o + rank * stride:o + rank * stride + G * words]
            assert not bool((mine.view(G, words)[:, 0] == -7).any()), f"step {k - n + j}: a record header never written"
            for r in range(world):  # peer r: this rank's game (g + r - rank) mod G at its game g
                peer = recv[o + r * stride:o + r * stride + G * words].view(G, words)
                assert torch.equal(peer, torch.roll(mine.view(G, words), -(r - rank), 0)), f"step {k - n + j}: rank {r}"
            out = torch.zeros((world * 2 * G,) + tuple(B.obs.shape[1:]), dtype=torch.int32, device=B.device)
            B.render_records(recv, o, stride, world, out)
            B.synchronize()
            for r in range(world):
                assert torch.equal(out[r * 2 * G:(r + 1) * 2 * G], torch.roll(want[j], -2 * (r - rank), 0)), \
                    f"step {k - n + j}: rendered rank {r}"
            # the check can fail: once the games differ, the neighbour's place rendered as this rank's is not
            # this rank's observation (right after a reset every game may still look the same)
            if not torch.equal(torch.roll(want[j], -2, 0), want[j]):
                nb = (rank + 1) % world
                wrong = torch.zeros_like(B.obs)
                B.render_records(recv, o + nb * stride, stride, 1, wrong)
                B.synchronize()
                assert not torch.equal(wrong, want[j]), f"step {k - n + j}: a neighbour's place renders like this rank's"
                distinct += 1
        assert torch.equal(A.obs, B.obs) and torch.equal(A.masks, B.masks)
    if not po:  # the per-step tensor exchange: [ranks][slots][C][H][W]
        send = [torch.zeros(tuple(B.obs.shape), dtype=torch.int16, device=B.device) for _ in range(2)]
        tr = torch.full((world,) + tuple(B.obs.shape), -7, dtype=torch.int16, device=B.device)
        A.rollout_fused(SEED, k + 1, 3)
        B.rollout_fused_exchange(SEED, k + 1, 3, send, tr)
        A.synchronize()
        B.synchronize()
        for r in range(world):  # peer r: this rank's slot (i + r - rank) mod slots at its slot i
            assert torch.equal(tr[r], torch.roll(A.obs.to(torch.int16), -(r - rank), 0)), f"tensor exchange rank {r}"
    assert distinct > 10, "the games never differed: the rank checks could not fail"
    for e in (A, B, C):
        assert not e.error_flags().any()
        e.close()
