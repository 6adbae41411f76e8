"""The multi-GPU configurations' observation exchange at full size, on one GPU (VERDICT r5 "next" #1).

BASELINE configs[3] (c4: basesWorkers16x16, 4096 self-play games per GPU x 8 GPUs, observation all-gather) and
configs[4] (c5: BWDistantResources32x32, 2048 partially observable games per GPU x 8) exchange every step's
compact game records (mrts_rollout_fused_records_dev).  RCCL cannot put two ranks on one device,
so the 8-rank layout runs through mrts_exchange_init_loopback: this handle is rank 3 of 8 and peer r's place of
every all-gather receives this rank's records with the games rotated by r - 3, so every rank's data differ
and a wrong rank offset, stride, chunk base or render shows as a wrong observation.

Each test runs the shipped form at the full per-GPU size — fused masked policy, delta masks, multi-step
launches — for a 1000-step burn-in, then three records calls: K = 20 (the driver's window), K = 200 (the bench
default) and K = 1040, whose receive buffer (8 ranks x 1040 steps x every game's record, > 2^31 words) puts the
second chunk's offsets past 2^31 words, so every offset / stride / base on the path must be 64-bit.  At every
step of every call the Responses ring (reward / done, mrts_set_step_responses) is compared; at the checked steps
all 8 ranks' observations are rendered from the records, each rank's render must be this rank's rotated by
2 (r - 3) slots (checked on the GPU) and this rank's must equal the oracle's observation (so rank r's equals the
oracle replica of the rotated games); for c4 a one-hot minibatch of random (step, slot) pairs over all 8 ranks
and the whole call (mrts_render_records_onehot_dev) must equal MicroRTS-Py's encoding (numpy restatement) of the
oracle replica's observation of the rotated slot.  After each call: every slot's observation, mask buffer,
action rows and canonical state dump.  What the exchange must deliver per rank is every step's Responses:
/root/reference/src/tests/JNIGridnetVecClient.java:213-297, src/ai/jni/Responses.java:12-30.

Oracle side: as tests/test_full_size_every_game.py — one OracleVecClient per shard of games on 16 threads,
stepping in native code with the same Philox rows (oref_rollout_policy), here one step at a time so that every
step's responses can be compared.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from tests import oracle_py
from tests.test_full_size_every_game import _threads
from tests.test_gpu_parity import _encode_obs_np

pytestmark = pytest.mark.gpu

SEED = 0x5EEDC0DE
WORLD, RANK = 8, 3
BURN = 1000
CALLS = (20, 200, 1040)
# config: map, games per GPU, partially observable, max_units, seed, record units
SHAPES = {"c4": ("maps/16x16/basesWorkers16x16.xml", 4096, False, 0, 11, 64),
          "c5x8": ("maps/BWDistantResources32x32.xml", 2048, True, 256, 13, 64)}
N_ONEHOT = 768  # samples per call (c4)


def _checked_steps(n):
    """The steps of an n-step call whose rendered observations are compared (every step's ring is)."""
    if n <= 20:
        return list(range(n))
    if n <= 200:
        return sorted(set(range(0, n, 25)) | {n - 1})
    return [0, 511, 1023, 1024, n - 1]  # the last step of chunk 0 and the first of chunk 1 (offset > 2^31 words)


def _gpu_run(cfg):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from microrts_amd import DeviceVecEnv

    mp, G, po, mu, seed, units = SHAPES[cfg]
    S = 2 * G
    env = DeviceVecEnv(S, 0, 2000, [mp] * S, seed=seed, partial_obs=po, max_units=mu)
    assert env.fused_multi_step, "the bench's shape must run multi-step launches"
    L, h = env._h.L, env._h.h
    assert L.mrts_exchange_init_loopback(h, WORLD, RANK) == 0
    words = env.set_records(units, 0)
    env.reset()
    env.random_policy(SEED, 0)
    env.rollout_fused(SEED, 1, BURN)
    t = BURN
    env.set_step_responses(max(CALLS))
    gen = torch.Generator(device="cpu").manual_seed(17)
    points = []
    for n in CALLS:
        recv = env.records_buffer(n, WORLD)
        off = env.rollout_fused_records(SEED, t + 1, n, recv)
        env.synchronize()
        # the per-step (offset, rank stride) table: 64-bit, chunked as the host plans it (MRTS_MAX_ITER steps
        # per chunk), every rank's place inside the buffer
        per = G * words
        assert off.dtype == np.int64 and off.shape == (n, 2)
        base = 0
        for c0 in range(0, n, 1024):
            m = min(1024, n - c0)
            for j in range(c0, c0 + m):
                assert off[j, 1] == m * per and off[j, 0] == base + (j - c0) * per, f"{cfg}: offsets of step {j}"
            base += WORLD * m * per
        assert base == recv.numel() and int(off[-1, 0]) + (WORLD - 1) * int(off[-1, 1]) + per <= recv.numel()
        if n > 1024:
            assert recv.numel() > 2 ** 31 and off[1024, 0] >= 2 ** 31, "the long call must pass 2^31 words"
        pt = {"t0": t, "n": n,
              "ring_r": env.step_rewards[:n].cpu().numpy().copy(), "ring_d": env.step_dones[:n].cpu().numpy().copy(),
              "obs": {}}
        out = torch.zeros((WORLD * S,) + tuple(env.obs.shape[1:]), dtype=torch.int32, device=env.device)
        for j in _checked_steps(n):
            env.render_records(recv, int(off[j, 0]), int(off[j, 1]), WORLD, out)
            env.synchronize()
            own = out[RANK * S:(RANK + 1) * S]
            for r in range(WORLD):  # rank r's place: this rank's games rotated by r - RANK
                assert torch.equal(out[r * S:(r + 1) * S], torch.roll(own, -2 * (r - RANK), 0)), \
                    f"{cfg}: step {t + j}: rendered rank {r}"
            # the rank checks can fail: neighbouring ranks' observations differ (the games diverged in the burn-in)
            assert not torch.equal(torch.roll(own, -2, 0), own), f"{cfg}: step {t + j}: every rank looks the same"
            assert int(own.min()) >= -32768 and int(own.max()) < 32768
            pt["obs"][j] = own.to(torch.int16).cpu().numpy()
        del out
        if not po:  # a learner's minibatch over every rank and the whole call, in one launch
            js = torch.randint(0, n, (N_ONEHOT,), generator=gen)
            sel = torch.randint(0, WORLD * S, (N_ONEHOT,), generator=gen).to(torch.int32)
            so = torch.from_numpy(off[js.numpy()]).contiguous()
            got = env.render_records_onehot(recv, 0, 0, sel.to(env.device), step_off=so.to(env.device)).cpu().numpy()
            r_, s_ = sel.numpy() // S, sel.numpy() % S
            twin = (s_ + 2 * (r_ - RANK)) % S
            pt["onehot"] = (js.numpy(), twin, got)
        assert not env.render_overflow(), f"{cfg}: a record overflowed"
        del recv
        t += n
        pt["end"] = {"obs": env.obs.cpu().numpy(), "masks": env.masks.cpu().numpy(), "actions": env.actions.cpu().numpy(),
                     "state": [env._h.dump(s) for s in range(S)]}
        points.append(pt)
    assert not env.error_flags().any()
    env.close()
    return points


def _shard(cfg, g0, g1, points):
    """Oracle replicas of games [g0, g1), one step at a time -> ({what: mismatching slots}, examples, samples)."""
    mp, G, po, mu, seed, units = SHAPES[cfg]
    sl = slice(2 * g0, 2 * g1)
    slots = np.arange(2 * g0, 2 * g1)
    ns = len(slots)
    ref = oracle_py.OracleVecClient(ns, 0, 2000, [mp] * ns, seed=seed, partial_obs=po)
    ref.reset()
    bad, ex, nsamp = {}, [], 0

    def chk(what, got, want, t):
        ok = (np.asarray(got).reshape(ns, -1) == np.asarray(want).reshape(ns, -1)).all(axis=1)
        if not ok.all():
            bad[f"{what}"] = bad.get(what, 0) + int((~ok).sum())
            ex.append((t, what, [int(s) for s in slots[~ok][:4]]))

    ref.rollout_policy(BURN, SEED, 2 * g0, 0)
    t = BURN
    for pt in points:
        assert pt["t0"] == t
        oh = pt.get("onehot")
        for j in range(pt["n"]):
            ref.rollout_policy(1, SEED, 2 * g0, t)
            t += 1
            chk("ring reward", pt["ring_r"][j][sl], ref.reward, t)
            chk("ring done", pt["ring_d"][j][sl], ref.done, t)
            if j in pt["obs"]:
                chk("rendered obs", pt["obs"][j][sl], ref.obs, t)
            if oh is not None:
                js, twin, got = oh
                mine = np.nonzero((js == j) & (twin >= 2 * g0) & (twin < 2 * g1))[0]
                if len(mine):
                    want = _encode_obs_np(ref.obs[twin[mine] - 2 * g0])
                    for i, w in zip(mine, want):
                        if not np.array_equal(got[i], w):
                            bad["one-hot sample"] = bad.get("one-hot sample", 0) + 1
                            ex.append((t, "one-hot sample", [int(twin[i])]))
                    nsamp += len(mine)
        e = pt["end"]
        chk("obs", e["obs"][sl], ref.obs, t)
        m = ref.get_masks(0)
        chk("masks", e["masks"][sl], m, t)
        chk("actions", e["actions"][sl], np.stack([oracle_py.policy(m[i], SEED, int(s), t, 0) for i, s in enumerate(slots)]), t)
        nst = [int(s) for i, s in enumerate(slots) if not np.array_equal(e["state"][s], ref.dump(i))]
        if nst:
            bad["state"] = bad.get("state", 0) + len(nst)
            ex.append((t, "state", nst[:4]))
    ref.close()
    return bad, ex, nsamp


def _loopback_full_size(cfg):
    import time

    t0 = time.time()
    points = _gpu_run(cfg)
    print(f"{cfg}: GPU rollout + renders {time.time() - t0:.1f} s; oracle replicas next", flush=True)
    G = SHAPES[cfg][1]
    nt = _threads()
    step = (G + nt - 1) // nt
    bad, ex, nsamp = {}, [], 0
    with cf.ThreadPoolExecutor(nt) as pool:  # the oracle steps in native code with the GIL released
        for b, e, k in pool.map(lambda g0: _shard(cfg, g0, min(g0 + step, G), points), range(0, G, step)):
            for key, v in b.items():
                bad[key] = bad.get(key, 0) + v
            ex += e
            nsamp += k
    print(f"{cfg}: oracle done at {time.time() - t0:.1f} s", flush=True)
    assert not bad, f"{cfg}: mismatches {bad}; first cases (step, field, slots) {ex[:8]}"
    if not SHAPES[cfg][2]:
        assert nsamp == N_ONEHOT * len(CALLS), "every one-hot sample must have been checked"


def test_loopback_full_size_c4():
    """BASELINE configs[3]: 4096 games on this rank of 8, the records exchange at K = 20 / 200 / 1040."""
    _loopback_full_size("c4")


def test_loopback_full_size_c5x8():
    """BASELINE configs[4]: 2048 partially observable games on this rank of 8 (the render helper wave), the
    records exchange at K = 20 / 200 / 1040."""
    _loopback_full_size("c5x8")
