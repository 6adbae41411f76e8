"""ctypes binding of the CPU oracle (oracle/build/liboref.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboref.so")
_lib = None

BOT_PASSIVE, BOT_RANDOM_BIASED = 0, 1


def build():
    srcs = [os.path.join(ROOT, "oracle", f) for f in ("ref_cpu.cpp", "ref_cpu.hpp", "oracle_capi.cpp", "Makefile")]
    srcs.append(os.path.join(ROOT, "microrts_amd", "csrc", "mrts_json.hpp"))
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in srcs):
        return LIB
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return LIB


def load():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P, I, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.oref_create.restype = P
        L.oref_create.argtypes = [I, I, P, I, I, I, I, P, U64, ctypes.c_char_p]
        L.oref_destroy.argtypes = [P]
        L.oref_dims.argtypes = [P, P, P, P, P, P]
        L.oref_reset.argtypes = [P, P, P, P, P]
        L.oref_step.argtypes = [P, P, P, P, P, P]
        L.oref_step_rows.argtypes = [P, P, I, P, P, P, P]
        L.oref_set_rewards.argtypes = [P, P, I]
        L.oref_botclient_set_rewards.argtypes = [P, P, I]
        L.oref_get_masks.argtypes = [P, I, P]
        L.oref_dump_state.argtypes = [P, I, P, I]
        L.oref_env_steps.argtypes = [P, I]
        L.oref_errors.argtypes = [P, I]
        L.oref_last_error.restype = ctypes.c_char_p
        L.oref_trace_replay.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, I]
        L.oref_trace_dumps.argtypes = [ctypes.c_char_p, ctypes.c_char_p, P, ctypes.c_int64, P, P, I, ctypes.c_char_p, I]
        L.oref_policy.argtypes = [P, I, I, I, U64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, P]
        L.oref_botclient_create.restype = P
        L.oref_botclient_create.argtypes = [ctypes.c_char_p, I, I, I, I, I, ctypes.c_int64, ctypes.c_char_p]
        L.oref_botclient_destroy.argtypes = [P]
        L.oref_botclient_step.argtypes = [P, I, P, P]
        L.oref_botclient_dump.argtypes = [P, P, I]
        L.oref_state_json.argtypes = [P, I, ctypes.c_char_p, I]
        L.oref_set_state_json.argtypes = [P, I, ctypes.c_char_p]
        L.oref_fm_create.restype = P
        L.oref_fm_create.argtypes = [ctypes.c_char_p, I, P, P, I, I, ctypes.c_int64, ctypes.c_char_p]
        L.oref_fm_destroy.argtypes = [P]
        L.oref_fm_copy.argtypes = [P, I, I]
        L.oref_fm_copy_from_vec.argtypes = [P, I, P, I]
        L.oref_fm_playout.argtypes = [P, I, I]
        L.oref_fm_evaluate.restype = ctypes.c_float
        L.oref_fm_evaluate.argtypes = [P, I, I]
        L.oref_fm_dump.argtypes = [P, I, P, I]
        L.oref_fm_errors.argtypes = [P, I]
        L.oref_bench.restype = ctypes.c_double
        L.oref_bench.argtypes = [ctypes.c_char_p, I, I, I, U64, I]
        L.oref_bench2.restype = ctypes.c_double
        L.oref_bench2.argtypes = [ctypes.c_char_p, I, I, I, U64, I, I]
        L.oref_bench3.restype = ctypes.c_double
        L.oref_bench3.argtypes = [ctypes.c_char_p, I, I, I, U64, I, I]
        L.oref_bench_bots.restype = ctypes.c_double
        L.oref_bench_bots.argtypes = [ctypes.c_char_p, I, ctypes.c_int64, I]
        L.oref_policy_uniform.argtypes = [I, I, I, U64, ctypes.c_uint32, ctypes.c_uint32, P]
        L.oref_rollout_policy.argtypes = [P, I, I, I, U64, ctypes.c_uint32, ctypes.c_uint32, P, P, P]
        _lib = L
    return _lib


def trace_dumps(map_path, fixture_text):
    """Replay one converted reference trace (tests/golden/make_trace_fixtures.py) on the oracle with the
    rule of TestTracesIntegrity.java:72-127: the canonical state dump at every entry (after catching up
    with its time, before its actions) and issueSafe's combined return value per entry."""
    L = load()
    n = int(fixture_text.split(None, 2)[1])
    cap = 1 << 22
    buf = np.zeros(cap, dtype=np.int32)
    off = np.zeros(n + 1, dtype=np.int32)
    iss = np.zeros(max(n, 1), dtype=np.int32)
    msg = ctypes.create_string_buffer(1024)
    r = L.oref_trace_dumps(map_path.encode(), fixture_text.encode(), _ptr(buf), cap, _ptr(off), _ptr(iss), n, msg, 1024)
    if r != n:
        raise RuntimeError(f"oracle trace replay: {r}: {msg.value.decode()}")
    return [buf[off[e]:off[e + 1]].copy() for e in range(n)], iss[:n].copy()


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleVecClient:
    """Mirror of tests.JNIGridnetVecClient (src/tests/JNIGridnetVecClient.java) on the CPU oracle."""

    def __init__(self, n_selfplay_slots, n_bot_envs, max_steps, map_paths, partial_obs=False, utt_version=1, crs=1,
                 bot_kinds=None, seed=0, slot_id_base=0, rewards=None, utt_json=None):
        """rewards: reward function ids (REWARD_IDS); None = [WinLoss].  reward / done are [S] for one
        reward function, [S][R] otherwise."""
        L = load()
        self.L = L
        paths = (ctypes.c_char_p * len(map_paths))(*[os.path.join(ROOT, p).encode() for p in map_paths])
        bk = np.asarray(bot_kinds if bot_kinds is not None else [0] * n_bot_envs, dtype=np.int32)
        self.h = L.oref_create(n_selfplay_slots, n_bot_envs, _ptr(bk) if n_bot_envs else None, max_steps, int(partial_obs),
                               utt_version, crs, ctypes.cast(paths, ctypes.c_void_p), seed + slot_id_base,
                               utt_json.encode() if utt_json else None)
        if not self.h:
            raise RuntimeError(L.oref_last_error().decode())
        d = [ctypes.c_int32() for _ in range(5)]
        L.oref_dims(self.h, *[ctypes.byref(x) for x in d])
        self.S, self.H, self.W, self.C, self.K = [x.value for x in d]
        self.obs = np.zeros((self.S, self.C, self.H, self.W), np.int32)
        R = 1
        if rewards is not None:
            k = np.asarray(rewards, np.int32)
            self._chk(L.oref_set_rewards(self.h, _ptr(k), len(k)))
            R = len(k)
        shape = (self.S,) if R == 1 else (self.S, R)
        self.reward = np.zeros(shape, np.float64)
        self.done = np.zeros(shape, np.uint8)

    def _chk(self, r):
        if r != 0:
            raise RuntimeError(self.L.oref_last_error().decode())

    def reset(self, players=None):
        p = np.asarray(players, np.int32) if players is not None else None
        self._chk(self.L.oref_reset(self.h, _ptr(p), _ptr(self.obs), _ptr(self.reward), _ptr(self.done)))
        return self.obs.copy(), self.reward.copy(), self.done.copy()

    def step(self, actions, players=None):
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.S, self.H * self.W, 7)
        p = np.asarray(players, np.int32) if players is not None else None
        self._chk(self.L.oref_step(self.h, _ptr(a), _ptr(p), _ptr(self.obs), _ptr(self.reward), _ptr(self.done)))
        return self.obs.copy(), self.reward.copy(), self.done.copy()

    def step_rows(self, rows, players=None):
        """gameStep with Java rows [slots][n_rows][8] (PlayerAction.fromVectorAction list semantics)."""
        r = np.ascontiguousarray(rows, dtype=np.int32)
        assert r.ndim == 3 and r.shape[0] == self.S and r.shape[2] == 8
        p = np.asarray(players, np.int32) if players is not None else None
        self._chk(self.L.oref_step_rows(self.h, _ptr(r), r.shape[1], _ptr(p), _ptr(self.obs), _ptr(self.reward),
                                        _ptr(self.done)))
        return self.obs.copy(), self.reward.copy(), self.done.copy()

    def rollout_policy(self, n_steps, seed, slot_base, step0, uniform=False, n_types=7):
        """n_steps gameSteps in native code with the GPU benchmark's own policy streams: the masked-uniform
        rows of each slot from its own masks (slot id slot_base + s, player 0), or the unmasked uniform
        rows; obs / reward / done then hold the last step's responses.  Releases the GIL while it runs."""
        self._chk(self.L.oref_rollout_policy(self.h, n_steps, int(uniform), n_types, seed, slot_base, step0, _ptr(self.obs),
                                             _ptr(self.reward), _ptr(self.done)))

    def get_masks(self, player=0):
        m = np.zeros((self.S, self.H, self.W, self.K), np.uint8)
        self._chk(self.L.oref_get_masks(self.h, player, _ptr(m)))
        return m

    def dump(self, slot):
        buf = np.zeros(1 << 16, np.int32)
        n = self.L.oref_dump_state(self.h, slot, _ptr(buf), buf.size)
        assert n >= 0
        return buf[:n].copy()

    def env_steps(self, slot):
        return self.L.oref_env_steps(self.h, slot)

    def state_json(self, slot):
        """GameState.toJSON of the game behind `slot` (Java's unit IDs)."""
        n = self.L.oref_state_json(self.h, slot, None, 0)
        buf = ctypes.create_string_buffer(-n)
        self.L.oref_state_json(self.h, slot, buf, -n)
        return buf.value.decode()

    def set_state_json(self, slot, text):
        self._chk(self.L.oref_set_state_json(self.h, slot, text.encode()))

    def close(self):
        if self.h:
            self.L.oref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


# reward function ids (oracle_capi.cpp RewardKind = include/mrts.h MRTS_RF_*)
REWARD_IDS = {"WinLossRewardFunction": 0, "ResourceGatherRewardFunction": 1, "ProduceWorkerRewardFunction": 2,
              "ProduceBuildingRewardFunction": 3, "AttackRewardFunction": 4, "ProduceCombatUnitRewardFunction": 5,
              "CloserToEnemyBaseRewardFunction": 6, "CloserToEnemyUnitRewardFunction": 7}


def policy(mask, seed, env_id, step, player, n_types=7):
    """Philox masked-uniform policy (bit-identical to the GPU policy kernel). mask: u8[H,W,K]."""
    L = load()
    H, W, K = mask.shape
    m = np.ascontiguousarray(mask, np.uint8)
    out = np.zeros((H * W, 7), np.int32)
    L.oref_policy(_ptr(m), H * W, K, n_types, seed, env_id, step, player, _ptr(out))
    return out


def policy_uniform(H, W, K, seed, slot_id, step, n_types=7):
    """Unmasked uniform random rows of one slot (bit-identical to mrts_policy_uniform_dev)."""
    L = load()
    out = np.zeros((H * W, 7), np.int32)
    L.oref_policy_uniform(H * W, K, n_types, seed, slot_id, step, _ptr(out))
    return out


class OracleBotClient:
    """tests.JNIBotClient (src/tests/JNIBotClient.java) + the bot-only VecClient auto-reset, one game."""

    def __init__(self, map_path, ai1, ai2, max_steps=2000, utt_version=1, crs=1, seed=0, rewards=None, utt_json=None):
        L = load()
        self.L = L
        self.h = L.oref_botclient_create(os.path.join(ROOT, map_path).encode(), ai1, ai2, max_steps, utt_version, crs, seed,
                                         utt_json.encode() if utt_json else None)
        if not self.h:
            raise RuntimeError(L.oref_last_error().decode())
        self.R = 1
        if rewards is not None:
            k = np.asarray(rewards, np.int32)
            if L.oref_botclient_set_rewards(self.h, _ptr(k), len(k)) != 0:
                raise RuntimeError("bad reward functions")
            self.R = len(k)

    def step(self, player=0):
        """-> (reward, done): scalars for one reward function, arrays [R] otherwise."""
        r = np.zeros(self.R, np.float64)
        d = np.zeros(self.R, np.uint8)
        if self.L.oref_botclient_step(self.h, player, _ptr(r), _ptr(d)) != 0:
            raise RuntimeError(self.L.oref_last_error().decode())
        if self.R == 1:
            return float(r[0]), int(d[0])
        return r, d

    def dump(self):
        buf = np.zeros(1 << 16, np.int32)
        n = self.L.oref_botclient_dump(self.h, _ptr(buf), buf.size)
        return buf[:n].copy()

    def close(self):
        if self.h:
            self.L.oref_botclient_destroy(self.h)
            self.h = None


class OracleForwardModel:
    """Batched forward model (GameState.clone + NaiveMCTS.simulate + SimpleSqrtEvaluationFunction3)
    on the CPU oracle; game j's random streams are seeded from seed + j like the GPU ForwardModel."""

    def __init__(self, n, map_path, ai1, ai2, utt_version=1, crs=1, seed=0, utt_json=None):
        L = load()
        self.L = L
        a1 = np.asarray(ai1 if isinstance(ai1, (list, tuple, np.ndarray)) else [ai1] * n, np.int32)
        a2 = np.asarray(ai2 if isinstance(ai2, (list, tuple, np.ndarray)) else [ai2] * n, np.int32)
        self.h = L.oref_fm_create(os.path.join(ROOT, map_path).encode(), n, _ptr(a1), _ptr(a2), utt_version, crs, seed,
                                  utt_json.encode() if utt_json else None)
        if not self.h:
            raise RuntimeError(L.oref_last_error().decode())
        self.n = n

    def copy(self, dst, src):
        self.L.oref_fm_copy(self.h, dst, src)

    def copy_from_vec(self, dst, vec, slot):
        self.L.oref_fm_copy_from_vec(self.h, dst, vec.h, slot)

    def playout(self, game, horizon):
        if self.L.oref_fm_playout(self.h, game, horizon) != 0:
            raise RuntimeError(self.L.oref_last_error().decode())

    def evaluate(self, game, maxplayer=0):
        return np.float32(self.L.oref_fm_evaluate(self.h, game, maxplayer))

    def dump(self, game):
        buf = np.zeros(1 << 16, np.int32)
        n = self.L.oref_fm_dump(self.h, game, _ptr(buf), buf.size)
        assert n >= 0
        return buf[:n].copy()

    def errors(self, game):
        return self.L.oref_fm_errors(self.h, game)

    def close(self):
        if self.h:
            self.L.oref_fm_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()
