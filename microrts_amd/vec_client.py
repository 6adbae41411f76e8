"""Host-side mirror of the reference's env-client interface over the libmrts C ABI.

* ``JNIGridnetVecClient`` mirrors ``tests.JNIGridnetVecClient`` (reference
  src/tests/JNIGridnetVecClient.java:17-335): same constructor arguments, ``reset`` / ``gameStep``
  / ``getMasks`` / ``close``, host numpy arrays that are library-owned views reused by the next
  call (like the Java ``Response`` buffers, GameState.java:923-925).
* ``DeviceVecEnv`` is the zero-copy rollout form: every buffer is a torch tensor in HBM and all
  calls are ordered on torch's current HIP stream (no host sync).

There is no CPU fallback: constructing either class without a GPU or without libmrts.so raises.
"""
import ctypes
import os

import numpy as np

from . import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class UnitTypeTable:
    """rts.units.UnitTypeTable(version, crs) (src/rts/units/UnitTypeTable.java:22-349)."""

    EMPTY_TYPE_TABLE = -1
    VERSION_ORIGINAL = 1
    VERSION_ORIGINAL_FINETUNED = 2
    VERSION_NON_DETERMINISTIC = 3
    MOVE_CONFLICT_RESOLUTION_CANCEL_BOTH = 1
    MOVE_CONFLICT_RESOLUTION_CANCEL_RANDOM = 2
    MOVE_CONFLICT_RESOLUTION_CANCEL_ALTERNATING = 3

    def __init__(self, version=VERSION_ORIGINAL, crs=MOVE_CONFLICT_RESOLUTION_CANCEL_BOTH):
        if version not in (1, 2, 3) or crs not in (1, 2, 3):
            raise ValueError("unsupported UnitTypeTable version / conflict policy")
        self.version, self.crs = version, crs
        self.json = None  # set by fromJSON: the table is then the JSON's (version / crs unused)
        self._desc = None

    @classmethod
    def fromJSON(cls, text):
        """UnitTypeTable.fromJSON (UnitTypeTable.java:414-433), validated by the native parser (its
        quirks included: harvestTime is read from "produceTime", returnTime is not read)."""
        utt = cls()
        utt.json = text if isinstance(text, str) else text.decode()
        utt.toJSON()  # raises on a table this build cannot run
        return utt

    def toJSON(self):
        """UnitTypeTable.toJSON (UnitTypeTable.java:372-383), byte for byte."""
        L = _lib.load()
        j = self.json.encode() if self.json else None
        n = L.mrts_utt_json(self.version, self.crs, j, None, 0)
        if n >= 0 or n == -22 or n == -95:
            raise ValueError(L.mrts_last_error().decode() or "invalid unit-type table")
        buf = ctypes.create_string_buffer(-n)
        _lib.check(0 if L.mrts_utt_json(self.version, self.crs, j, buf, -n) >= 0 else -1)
        return buf.value.decode()

    def _table(self):
        if self._desc is None:
            import json

            self._desc = json.loads(self.toJSON())
        return self._desc

    @property
    def TYPES(self):
        return [t["name"] for t in self._table()["unitTypes"]]

    def getUnitTypes(self):
        return self._table()["unitTypes"]

    def getMoveConflictResolutionStrategy(self):
        return self._table()["moveConflictResolutionStrategy"]

    def getMaxAttackRange(self):
        """UnitTypeTable.getMaxAttackRange (:341-349)."""
        return max(t["attackRange"] for t in self._table()["unitTypes"])


class _ClientView:
    """The per-env client objects the Java VecClient exposes (clients / selfPlayClients); only
    sendUTT() (JNIGridnetClient.java:225-233) is meaningful on this build."""

    def __init__(self, utt):
        self._utt = utt

    def sendUTT(self):
        return self._utt.toJSON()


class Responses:
    """ai.jni.Responses (src/ai/jni/Responses.java:12-30)."""

    def __init__(self, observation, reward, done):
        self.observation, self.reward, self.done = observation, reward, done


def _bot_kind(ai):
    name = ai if isinstance(ai, str) else type(ai).__name__
    if name in ("PassiveAI", "passive"):
        return _lib.MRTS_BOT_PASSIVE
    if name in ("RandomBiasedAI", "random_biased"):
        return _lib.MRTS_BOT_RANDOM_BIASED
    raise NotImplementedError(f"opponent AI {name!r} has no native implementation (only PassiveAI / RandomBiasedAI)")


def _check_rfs(rfs):
    """a_rfs (RewardFunctionInterface[], :106) -> MRTS_RF_* ids: class names or instances/classes with
    those names (src/ai/reward/*.java); None = [WinLossRewardFunction]."""
    out = []
    for r in (rfs or ["WinLossRewardFunction"]):
        name = r if isinstance(r, str) else (r.__name__ if isinstance(r, type) else type(r).__name__)
        name = name.rsplit(".", 1)[-1]
        if name not in _lib.REWARD_FUNCTIONS:
            raise NotImplementedError(f"reward function {name!r} is not implemented on the GPU path "
                                      f"(available: {sorted(_lib.REWARD_FUNCTIONS)})")
        out.append(_lib.REWARD_FUNCTIONS[name])
    if len(out) > 8:
        raise ValueError("at most 8 reward functions")
    return out


def _kinds(ais, n):
    kinds = [_bot_kind(a) for a in (ais or [])][:n]
    kinds += [_lib.MRTS_BOT_PASSIVE] * (n - len(kinds))
    return (ctypes.c_int32 * max(1, n))(*(kinds or [0]))


def _last_map_index(n_selfplay, n_bot):
    """The largest a_mapPaths index Java reads: mapPaths[i*2] per self-play client
    (JNIGridnetVecClient.java:119), mapPaths[a_num_selfplayenvs + i] per bot env (:123), and
    mapPaths[0] for the storage sizing (:127)."""
    return max([0] + ([2 * (n_selfplay // 2 - 1)] if n_selfplay >= 2 else []) +
               ([n_selfplay + n_bot - 1] if n_bot > 0 else []))


class _Handle:
    def __init__(self, n_selfplay, n_bot, max_steps, map_paths, ai2s, utt, partial_obs, device, seed, slot_id_base,
                 ai1s=None, mask_delta=False, rewards=None, forward_model=False, max_units=0):
        need = _last_map_index(n_selfplay, n_bot)
        if len(map_paths) <= need:
            raise ValueError(f"{len(map_paths)} map paths; Java reads mapPaths[{need}]")
        L = _lib.load()
        self.L = L
        self._paths = (ctypes.c_char_p * len(map_paths))(*[p.encode() for p in map_paths])
        self._kinds = _kinds(ai2s, n_bot)
        self._ai1 = _kinds(ai1s, n_bot) if ai1s is not None else None
        P32 = ctypes.POINTER(ctypes.c_int32)
        self.rewards = list(rewards) if rewards else [0]
        self._rk = (ctypes.c_int32 * len(self.rewards))(*self.rewards)
        self.R = len(self.rewards)
        cfg = _lib.MrtsConfig(n_selfplay, n_bot, max_steps, int(bool(partial_obs)), utt.version, utt.crs,
                              ctypes.cast(self._kinds, P32),
                              ctypes.cast(self._ai1, P32) if self._ai1 is not None else None,
                              ctypes.cast(self._paths, ctypes.POINTER(ctypes.c_char_p)), device, seed, slot_id_base,
                              int(bool(mask_delta)), ctypes.cast(self._rk, P32), self.R, int(bool(forward_model)),
                              utt.json.encode() if utt.json else None, int(max_units))
        h = ctypes.c_void_p()
        _lib.check(L.mrts_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        d = [ctypes.c_int32() for _ in range(5)]
        L.mrts_dims(self.h, *[ctypes.byref(x) for x in d])
        self.S, self.H, self.W, self.C, self.K = [x.value for x in d]

    def close(self):
        if getattr(self, "h", None):
            self.L.mrts_destroy(self.h)
            self.h = None

    def dump(self, slot):
        buf = np.zeros(1 << 16, np.int32)
        n = self.L.mrts_get_state(self.h, slot, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
        if n < 0:
            raise RuntimeError(self.L.mrts_last_error().decode())
        return buf[:n].copy()

    def error_flags(self):
        f = np.zeros(self.S, np.uint32)
        _lib.check(self.L.mrts_error_flags(self.h, f.ctypes.data_as(ctypes.c_void_p)))
        return f

    def state_json(self, slot):
        n = self.L.mrts_get_state_json(self.h, slot, None, 0)  # -(length + 1), or an errno
        if n > -64:
            _lib.check(n if n < 0 else -22)
        buf = ctypes.create_string_buffer(-n)
        n = self.L.mrts_get_state_json(self.h, slot, buf, -n)
        _lib.check(0 if n >= 0 else n)
        return buf.value.decode()

    def set_state_json(self, slot, text):
        _lib.check(self.L.mrts_set_state_json(self.h, slot, text.encode() if isinstance(text, str) else text))

    def checkpoint(self):
        n = self.L.mrts_checkpoint_size(self.h)
        buf = ctypes.create_string_buffer(n)
        _lib.check(self.L.mrts_checkpoint(self.h, buf, n))
        return buf.raw

    def restore(self, data):
        _lib.check(self.L.mrts_restore(self.h, ctypes.c_char_p(bytes(data)), len(data)))

    def env_steps(self):
        f = np.zeros(self.S, np.int32)
        _lib.check(self.L.mrts_env_steps(self.h, f.ctypes.data_as(ctypes.c_void_p)))
        return f


def _resolve(micrortsPath, p):
    if micrortsPath:
        return os.path.join(micrortsPath, p)
    return p if os.path.isabs(p) or os.path.exists(p) else os.path.join(ROOT, p)


class JNIGridnetVecClient:
    """tests.JNIGridnetVecClient (src/tests/JNIGridnetVecClient.java:106-142) on MI355X."""

    def __init__(self, a_num_selfplayenvs, a_num_envs, a_max_steps, a_rfs, a_micrortsPath, a_mapPaths, a_ai2s=None,
                 a_utt=None, partial_obs=False, device=0, seed=0, slot_id_base=0, _ai1s=None):
        rewards = _check_rfs(a_rfs)
        # Java indexes a_ai2s[i] (and a_ai1s[i] in the bot-only constructor) for every bot env
        # (JNIGridnetVecClient.java:121-123,163-165) and throws on a null or short array; no silent
        # PassiveAI default here (DeviceVecEnv keeps one, documented there)
        for name, ais in (("a_ai2s", a_ai2s), ("a_ai1s", _ai1s)):
            if (name == "a_ai2s" or _ai1s is not None) and a_num_envs > 0 and (ais is None or len(ais) < a_num_envs):
                raise ValueError(f"{name} names {0 if ais is None else len(ais)} bots for {a_num_envs} bot environments")
        utt = a_utt or UnitTypeTable()
        paths = [_resolve(a_micrortsPath, p) for p in a_mapPaths]
        self._h = _Handle(a_num_selfplayenvs, a_num_envs, a_max_steps, paths, a_ai2s, utt, partial_obs, device, seed,
                          slot_id_base, ai1s=_ai1s, rewards=rewards)
        self.botOnly = _ai1s is not None
        self.maxSteps = a_max_steps
        self.utt = utt
        self.partialObs = partial_obs
        self.mapPaths = list(a_mapPaths)
        h = self._h
        self.num_slots, self.height, self.width, self.num_planes, self.mask_slots = h.S, h.H, h.W, h.C, h.K
        self._resp = _lib.MrtsResponses()
        # the Java fields of per-env clients (:22-26); each offers sendUTT()
        self.selfPlayClients = [_ClientView(utt)] * (a_num_selfplayenvs // 2)
        self.clients = [_ClientView(utt)] * a_num_envs

    def sendUTT(self):
        """The unit-type table as JSON (JNIGridnetClient.sendUTT, :225-233)."""
        return self.utt.toJSON()

    def getGameStateJSON(self, slot):
        """GameState.toJSON of the game behind `slot` (unit IDs = list positions)."""
        return self._h.state_json(slot)

    def setGameStateJSON(self, slot, text):
        """GameState.fromJSON into the game behind `slot` (envSteps restarts at 0)."""
        self._h.set_state_json(slot, text)

    def checkpoint(self):
        """bytes holding every game's state (random streams and envSteps included)."""
        return self._h.checkpoint()

    def restore(self, data):
        self._h.restore(data)

    @classmethod
    def bots(cls, a_max_steps, a_rfs, a_micrortsPath, a_mapPaths, a_ai1s, a_ai2s, a_utt=None, partial_obs=False, device=0,
             seed=0, slot_id_base=0):
        """The bot-only constructor JNIGridnetVecClient(maxSteps, rfs, path, mapPaths, ai1s, ai2s, utt, po)
        (src/tests/JNIGridnetVecClient.java:157-177): JNIBotClients, reward/done only."""
        return cls(0, len(a_ai2s), a_max_steps, a_rfs, a_micrortsPath, a_mapPaths, a_ai2s, a_utt, partial_obs, device, seed,
                   slot_id_base, _ai1s=list(a_ai1s))

    def _responses(self):
        h, r = self._h, self._resp
        obs = None if getattr(self, "botOnly", False) else np.ctypeslib.as_array(r.obs, shape=(h.S, h.C, h.H, h.W))
        rew = np.ctypeslib.as_array(r.reward, shape=(h.S, h.R))
        done = np.ctypeslib.as_array(r.done, shape=(h.S, h.R)).view(np.bool_)
        return Responses(obs, rew, done)

    def reset(self, players=None):
        """reset(int[] players) (:179-211)."""
        p = None if players is None else np.ascontiguousarray(players, np.int32)
        _lib.check(self._h.L.mrts_reset(self._h.h, None if p is None else p.ctypes.data_as(ctypes.c_void_p),
                                        ctypes.byref(self._resp)))
        return self._responses()

    def gameStep(self, action, players=None):
        """gameStep(int[][][] action, int[] players) (:213-297).

        action is either the Java layout [slots][n_rows][8] (rows [pos, 7 components], any order,
        duplicates allowed: PlayerAction.fromVectorAction list semantics) or the grid layout
        [slots][H*W][7] (row r = cell r, ascending — what MicroRTS-Py sends)."""
        h = self._h
        if action is None:  # bot-only clients take no actions (JNIGridnetVecClient.java:214-216)
            action = np.zeros((h.S, h.H * h.W, 7), np.int32)
        a = np.ascontiguousarray(action, np.int32)
        p = None if players is None else np.ascontiguousarray(players, np.int32)
        pp = None if p is None else p.ctypes.data_as(ctypes.c_void_p)
        if a.ndim == 3 and a.shape[0] == h.S and a.shape[2] == 8:
            _lib.check(h.L.mrts_step_rows(h.h, a.ctypes.data_as(ctypes.c_void_p), a.shape[1], pp, ctypes.byref(self._resp)))
        else:
            a = a.reshape(h.S, h.H * h.W, 7)
            _lib.check(h.L.mrts_step(h.h, a.ctypes.data_as(ctypes.c_void_p), pp, ctypes.byref(self._resp)))
        return self._responses()

    def getMasks(self, player=0, dtype=np.uint8, copy=True):
        """getMasks(int player) (:307-316) → [slots][H][W][79]; dtype np.int32 gives the Java int[][][][]
        element type.  copy=False returns a view of a library-owned pinned array that the next call
        refills (the Java client reuses its mask array the same way, JNIGridnetClient.java:211-215) —
        the fast form: the device-to-host copy runs at pinned-memory rate."""
        h = self._h
        if not copy:
            i32 = np.dtype(dtype) == np.int32
            ptr = ctypes.c_void_p()
            fn = h.L.mrts_get_masks_i32_host if i32 else h.L.mrts_get_masks_host
            _lib.check(fn(h.h, player, ctypes.byref(ptr)))
            ct = ctypes.c_int32 if i32 else ctypes.c_uint8
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(h.S, h.H, h.W, h.K))
        if np.dtype(dtype) == np.int32:
            m = np.empty((h.S, h.H, h.W, h.K), np.int32)
            _lib.check(h.L.mrts_get_masks_i32(h.h, player, m.ctypes.data_as(ctypes.c_void_p)))
            return m
        m = np.empty((h.S, h.H, h.W, h.K), np.uint8)
        _lib.check(h.L.mrts_get_masks(h.h, player, m.ctypes.data_as(ctypes.c_void_p)))
        return m

    @property
    def envSteps(self):
        return self._h.env_steps()

    def dump_state(self, slot):
        return self._h.dump(slot)

    def error_flags(self):
        return self._h.error_flags()

    def close(self):
        """close() (:318-334)."""
        self._h.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceVecEnv:
    """Zero-copy rollout backend: torch HBM tensors; every call is ordered on torch's CURRENT HIP
    stream of the env's device (or an explicit `stream=`), so ordinary torch ops on the tensors need
    no extra synchronisation."""

    def __init__(self, num_selfplay_slots, num_bot_envs, max_steps, map_paths, ai2s=None, utt=None, partial_obs=False,
                 device=0, seed=0, slot_id_base=0, with_masks=True, ai1s=None, mask_delta=True, source_bits=True,
                 rfs=None, max_units=0, obs_delta=True):
        """ai2s / ai1s: the bot of each bot env (names or objects named like the Java classes); a missing
        or short list is padded with PassiveAI (the JNIGridnetVecClient mirror raises instead, like
        Java).  mask_delta: `masks` is owned by this object and reused every call, so only changed rows are
        rewritten (the tensor must not be written by the caller).  source_bits: also keep mask slot 0
        as bits in `source` ([slots][ceil(H*W/32)] int32), which random_policy uses.  rfs: reward
        function names (a_rfs); reward / done are [S] for one function, [S][R] otherwise.  obs_delta:
        `obs` is persistent too (mrts_set_obs_delta: partially observable views re-render only the chunks
        that can have changed); an in-place torch write to `obs` (its version counter moves) makes the
        next write a full one."""
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("DeviceVecEnv needs an MI355X (torch.cuda is unavailable); there is no CPU fallback")
        self.torch = torch
        utt = utt or UnitTypeTable()
        paths = [_resolve("", p) for p in map_paths]
        self._h = _Handle(num_selfplay_slots, num_bot_envs, max_steps, paths, ai2s, utt, partial_obs, device, seed,
                          slot_id_base, ai1s=ai1s, mask_delta=mask_delta and with_masks, rewards=_check_rfs(rfs),
                          max_units=max_units)
        h = self._h
        self.mask_delta = bool(mask_delta and with_masks)
        dev = torch.device("cuda", device)
        self.device = dev
        S, H, W, C, K = h.S, h.H, h.W, h.C, h.K
        self.obs = torch.zeros((S, C, H, W), dtype=torch.int32, device=dev)
        rshape = (S,) if h.R == 1 else (S, h.R)
        self._reward = torch.zeros(rshape, dtype=torch.float64, device=dev)
        self._done = torch.zeros(rshape, dtype=torch.uint8, device=dev)
        self._ring_last = None  # ring step holding the last rollout call's responses (set_step_responses)
        self.masks = torch.zeros((S, H, W, K), dtype=torch.uint8, device=dev) if with_masks else None
        self.actions = torch.zeros((S, H * W, 7), dtype=torch.int32, device=dev)
        self.players = torch.zeros((S,), dtype=torch.int32, device=dev)
        self.source = torch.zeros((S, (H * W + 31) // 32), dtype=torch.int32, device=dev) if (with_masks and source_bits) else None
        if self.source is not None:
            _lib.check(h.L.mrts_set_source_output(h.h, self._p(self.source)))
        self.mask_player = 0
        self.partial_obs = bool(partial_obs)
        self.step_rewards = self.step_dones = None
        self._policy_out, self._policy_version = None, -1
        _lib.check(h.L.mrts_set_obs_delta(h.h, int(bool(obs_delta))))
        self._obs_version = -1
        self._ptr_cache = None
        torch.cuda.synchronize(dev)

    @property
    def reward(self):
        """The last step's reward ([slots] or [slots][R], float64).  After a rollout call that wrote the Responses
        ring (set_step_responses), this is the ring's last step of that call (a view: no copy), else
        the plain buffer the step calls write."""
        return self._reward if self._ring_last is None else self.step_rewards[self._ring_last]

    @property
    def done(self):
        """The last step's done flags (uint8, as reward; the ring's last step after a ring-writing rollout)."""
        return self._done if self._ring_last is None else self.step_dones[self._ring_last]

    def _ring_written(self, n_steps):
        """After a rollout call: with the ring on, its responses are in ring steps 0 .. n_steps - 1."""
        if self.step_rewards is not None and n_steps > 0:
            self._ring_last = n_steps - 1

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def _s(self, stream):
        if stream is None:  # torch's current stream, without building a Stream object per call
            return ctypes.c_void_p(self.torch._C._cuda_getCurrentRawStream(self.device.index))
        return ctypes.c_void_p(stream.cuda_stream)

    def _bufs(self):
        """actions, players, obs, reward, done, masks as ctypes pointers, cached while the same tensor
        objects stay attached (the rollout calls' per-call host cost)."""
        key = (self.actions, self.players, self.obs, self._reward, self._done, self.masks)
        c = self._ptr_cache
        if c is None or any(a is not b for a, b in zip(c[0], key)):
            c = self._ptr_cache = (key, tuple(self._p(t) for t in key))
        return c[1]

    def set_rollout_events(self, start, end):
        """The next rollout_fused / rollout_uniform call records these hipEvent_t handles (ints or
        ctypes pointers, None = skip) right before its first and after its last kernel launch
        (mrts_set_rollout_events): a benchmark's events bracket exactly the rollout's kernels."""
        _lib.check(self._h.L.mrts_set_rollout_events(self._h.h, start, end))

    def _obs_guard(self):
        """Before a call that writes `obs`: a torch in-place write since our last one voids the delta base."""
        if self.obs._version != self._obs_version:
            _lib.check(self._h.L.mrts_obs_invalidate(self._h.h))

    def _obs_written(self):
        self._obs_version = self.obs._version

    def reset(self, stream=None):
        h = self._h
        self._obs_guard()
        _lib.check(h.L.mrts_reset_dev(h.h, self._p(self.players), self._p(self.obs), self._p(self._reward),
                                      self._p(self._done), self._p(self.masks), self.mask_player, self._s(stream)))
        self._ring_last = None
        self._obs_written()

    def step(self, actions=None, stream=None, masks=True):
        """masks=False: this step writes no masks (the masks tensor keeps its previous contents)."""
        h = self._h
        a = self.actions if actions is None else actions
        self._obs_guard()
        _lib.check(h.L.mrts_step_dev(h.h, self._p(a), self._p(self.players), self._p(self.obs), self._p(self._reward),
                                     self._p(self._done), self._p(self.masks) if masks else None, self.mask_player,
                                     self._s(stream)))
        self._ring_last = None
        self._obs_written()

    def uniform_policy(self, seed, step, out=None, stream=None):
        """Unmasked uniform random rows for every cell (BASELINE config c2; mrts_policy_uniform_dev):
        type in [0,6), directions in [0,4), produce type in [0,ntypes), attack index in [0,K-23-ntypes)."""
        h = self._h
        out = self.actions if out is None else out
        _lib.check(h.L.mrts_policy_uniform_dev(h.h, seed, step, self._p(out), self._s(stream)))
        return out

    def step_uniform(self, seed, step, masks=False, stream=None):
        """uniform_policy(seed, step) into env.actions, then step() on it — in one launch
        (mrts_step_uniform_dev: the step kernel writes the rows and draws its idle units' rows itself)."""
        h = self._h
        self._obs_guard()
        _lib.check(h.L.mrts_step_uniform_dev(h.h, self._p(self.actions), self._p(self.players), self._p(self.obs),
                                             self._p(self._reward), self._p(self._done),
                                             self._p(self.masks) if masks else None, self.mask_player, seed, step,
                                             self._s(stream)))
        self._ring_last = None
        self._obs_written()

    def rollout_uniform(self, seed, first_step, n_steps, fused=True, stream=None):
        """n_steps x (uniform_policy(seed, first_step + k), then a step without masks), enqueued by
        native code (mrts_rollout_uniform_dev): the c2 random-policy rollout.  fused: one
        step_uniform launch per step (same results) instead of a policy launch + a step launch."""
        h = self._h
        self._obs_guard()
        a, pl, o, r, d, _ = self._bufs()
        _lib.check(h.L.mrts_rollout_uniform_dev(h.h, a, pl, o, r, d, seed, first_step, n_steps, 1 if fused else 0,
                                                self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()

    def step_fused(self, seed, next_step, stream=None):
        """step() on env.actions, then env.actions := random_policy(seed, next_step) from the masks this
        step wrote (mrts_step_fused_dev: one launch, identical result)."""
        h = self._h
        assert self.masks is not None, "the fused policy samples from the masks"
        if self._policy_out is not None and self._policy_out is self.actions and self.actions._version != self._policy_version:
            _lib.check(h.L.mrts_policy_invalidate(h.h))  # written by someone else since
        self._obs_guard()
        a, pl, o, r, d, m = self._bufs()
        _lib.check(h.L.mrts_step_fused_dev(h.h, a, pl, o, r, d, m, self.mask_player, seed, next_step, self._s(stream)))
        self._ring_last = None
        self._obs_written()
        self._policy_out, self._policy_version = self.actions, self.actions._version

    def set_obs16(self, out):
        """Every later observation write also fills `out` (int16 [n_slots][C][H][W], or None = off) —
        the observation exchange's compact transport, written by the step kernel
        (mrts_set_obs16; full observability)."""
        import torch
        if out is not None:
            assert out.dtype == torch.int16 and tuple(out.shape) == tuple(self.obs.shape) and out.is_contiguous()
        _lib.check(self._h.L.mrts_set_obs16(self._h.h, self._p(out) if out is not None else None))
        self._obs16 = out  # keep it alive while the handle writes into it

    def set_multi_step(self, on):
        """rollout_fused may run several steps per launch (default; mrts_set_multi_step)."""
        _lib.check(self._h.L.mrts_set_multi_step(self._h.h, 1 if on else 0))

    @property
    def multi_step_capable(self):
        """The handle's shape and switch allow multi-step launches (mrts_multi_step_capable):
        rollout_uniform uses them; rollout_fused only with mask_delta (see fused_multi_step)."""
        return bool(self._h.L.mrts_multi_step_capable(self._h.h))

    @property
    def fused_multi_step(self):
        """rollout_fused runs several steps per launch on this handle: the shape allows it and the
        handle keeps delta masks (the steady fused state needs them)."""
        return self.multi_step_capable and bool(self.mask_delta)

    def rollout_fused(self, seed, first_next_step, n_steps, stream=None):
        """n_steps step_fused calls (next_step = first_next_step, first_next_step + 1, ...) enqueued by
        native code (mrts_rollout_fused_dev): no Python between them; on the specialised
        full-observability self-play shapes, in the steady fused state, up to MRTS_MAX_ITER steps per
        launch (each game's state kept in LDS between its steps) — bit-identical results."""
        h = self._h
        assert self.masks is not None, "the fused policy samples from the masks"
        if self._policy_out is not None and self._policy_out is self.actions and self.actions._version != self._policy_version:
            _lib.check(h.L.mrts_policy_invalidate(h.h))
        self._obs_guard()
        a, pl, o, r, d, m = self._bufs()
        _lib.check(h.L.mrts_rollout_fused_dev(h.h, a, pl, o, r, d, m, self.mask_player, seed, first_next_step, n_steps,
                                              self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()
        self._policy_out, self._policy_version = self.actions, self.actions._version

    def rollout_fused_exchange(self, seed, first_next_step, n_steps, send, recv, stream=None):
        """rollout_fused with one launch per step and the all-gather of every step's int16 observation
        into recv (mrts_rollout_fused_exchange_dev; microrts_amd.dist.NativeExchange sets it up)."""
        h = self._h
        if self._policy_out is not None and self._policy_out is self.actions and self.actions._version != self._policy_version:
            _lib.check(h.L.mrts_policy_invalidate(h.h))
        self._obs_guard()
        a, pl, o, r, d, m = self._bufs()
        _lib.check(h.L.mrts_rollout_fused_exchange_dev(h.h, a, pl, o, r, d, m, self.mask_player, seed, first_next_step,
                                                       n_steps, self._p(send[0]), self._p(send[1]), self._p(recv),
                                                       self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()
        self._policy_out, self._policy_version = self.actions, self.actions._version

    def capture(self, fn, stream):
        """Capture the calls fn() makes on this handle on `stream` (a non-default torch stream, made
        current during fn) as one graph (mrts_capture_begin / _end); replay() launches it."""
        h = self._h
        s = ctypes.c_void_p(stream.cuda_stream)
        with self.torch.cuda.stream(stream):
            _lib.check(h.L.mrts_capture_begin(h.h, s))
            try:
                fn()
            finally:
                _lib.check(h.L.mrts_capture_end(h.h, s))

    def replay(self, stream=None):
        """Launch the graph capture() built (the same calls, verbatim) on `stream` (default: current)."""
        _lib.check(self._h.L.mrts_replay(self._h.h, self._s(stream)))

    def rollout_uniform_exchange(self, seed, first_step, n_steps, send, recv, stream=None):
        """rollout_uniform (fused form) with the all-gather of every step's int16 observation
        (mrts_rollout_uniform_exchange_dev)."""
        h = self._h
        self._obs_guard()
        a, pl, o, r, d, _ = self._bufs()
        _lib.check(h.L.mrts_rollout_uniform_exchange_dev(h.h, a, pl, o, r, d, seed, first_step, n_steps, self._p(send[0]),
                                                         self._p(send[1]), self._p(recv), self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()

    def set_records(self, units_per_record=64, steps_per_launch=0):
        """Enable the compact observation records (mrts_set_records): units per game record (0 = off) and
        steps per launch of a records rollout (0 = as many as a launch runs).  Returns words per record."""
        _lib.check(self._h.L.mrts_set_records(self._h.h, int(units_per_record), int(steps_per_launch)))
        self.record_units = int(units_per_record)
        self.record_words = int(self._h.L.mrts_record_words(self._h.h))
        return self.record_words

    def records_buffer(self, n_steps, world=1):
        """A receive buffer for n_steps of a records rollout over `world` ranks (uint32 words)."""
        return self.torch.zeros(n_steps * world * (self._h.S // 2) * self.record_words, dtype=self.torch.int32,
                                device=self.device)

    def rollout_fused_records(self, seed, first_next_step, n_steps, recv, stream=None):
        """rollout_fused whose every step's game records are all-gathered into recv
        (mrts_rollout_fused_records_dev; microrts_amd.dist.RecordExchange sets it up).  Returns the
        per-step (word offset of rank 0's records, rank stride) as int64 [n_steps, 2]."""
        h = self._h
        if self._policy_out is not None and self._policy_out is self.actions and self.actions._version != self._policy_version:
            _lib.check(h.L.mrts_policy_invalidate(h.h))
        self._obs_guard()
        a, pl, o, r, d, m = self._bufs()
        off = np.zeros((max(n_steps, 1), 2), dtype=np.int64)
        _lib.check(h.L.mrts_rollout_fused_records_dev(h.h, a, pl, o, r, d, m, self.mask_player, seed, first_next_step, n_steps,
                                                      self._p(recv), off.ctypes.data_as(ctypes.c_void_p), self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()
        self._policy_out, self._policy_version = self.actions, self.actions._version
        return off[:n_steps]

    def rollout_uniform_records(self, seed, first_step, n_steps, recv, stream=None):
        """rollout_uniform (fused form) whose every step's game records are all-gathered into recv
        (mrts_rollout_uniform_records_dev).  Returns the per-step offsets as rollout_fused_records."""
        h = self._h
        self._obs_guard()
        a, pl, o, r, d, _ = self._bufs()
        off = np.zeros((max(n_steps, 1), 2), dtype=np.int64)
        _lib.check(h.L.mrts_rollout_uniform_records_dev(h.h, a, pl, o, r, d, seed, first_step, n_steps, self._p(recv),
                                                        off.ctypes.data_as(ctypes.c_void_p), self._s(stream)))
        self._ring_written(n_steps)
        self._obs_written()
        return off[:n_steps]

    def render_records(self, recv, offset, rank_stride, n_ranks, out, stream=None):
        """The observations of n_ranks x games records (rank r's at recv[offset + r * rank_stride:]) into
        out [n_ranks * slots, C, H, W] (uint8 or int32; int8 or int32 for a partially observable handle) —
        mrts_render_records_dev."""
        h = self._h
        ob = out.element_size()
        T = self.torch
        # a partially observable view shows a dead unit's hp (<= 0): int8, never uint8
        ok = (T.int8, T.int32) if self.partial_obs else (T.uint8, T.int32)
        assert out.dtype in ok, f"render_records: out must be one of {ok}, not {out.dtype}"
        assert out.is_contiguous() and out.numel() == n_ranks * self.obs.numel()
        assert recv.dtype == T.int32 and recv.is_contiguous() and 0 <= int(offset) <= recv.numel()
        ptr = ctypes.c_void_p(recv.data_ptr() + 4 * int(offset))
        _lib.check(h.L.mrts_render_records_dev(h.h, ptr, recv.numel() - int(offset), int(n_ranks), int(rank_stride), self._p(out),
                                               ob, self._s(stream)))
        return out

    def render_records_onehot(self, recv, offset, rank_stride, sel, out=None, step_off=None, stream=None, n_ranks=None):
        """A learner minibatch from records in one launch: the MicroRTS-Py one-hot observations (onehot_obs'
        layout, uint8 [n][H][W][F]) of the slots sel (int32 tensor of global indices r * slots + slot over the
        ranks in recv) of the step whose records start at recv[offset] with rank_stride — or, with step_off
        (int64 tensor [n, 2]: each sample's step's row of the rollout's offsets table), each sample's own
        step — mrts_render_records_onehot_dev.  n_ranks (default: as many as recv holds) bounds sel; a sample
        outside recv or n_ranks renders as zeros and raises render_overflow()."""
        h, T = self._h, self.torch
        F = h.L.mrts_onehot_features(h.h)
        assert sel.dtype == T.int32 and sel.is_contiguous() and sel.device == self.device
        if step_off is not None:
            assert step_off.dtype == T.int64 and step_off.is_contiguous() and step_off.numel() == 2 * sel.numel()
        if out is None:
            out = T.empty((sel.numel(), h.H, h.W, F), dtype=T.uint8, device=self.device)
        assert out.dtype == T.uint8 and out.is_contiguous() and out.numel() == sel.numel() * h.H * h.W * F
        assert recv.dtype == T.int32 and recv.is_contiguous() and 0 <= int(offset) <= recv.numel()
        if n_ranks is None:  # every rank place a records buffer of this handle's games can hold
            n_ranks = max(1, recv.numel() // max(1, (h.S // 2) * self.record_words))
        ptr = ctypes.c_void_p(recv.data_ptr() + 4 * int(offset))
        _lib.check(h.L.mrts_render_records_onehot_dev(h.h, ptr, recv.numel() - int(offset), int(n_ranks), int(rank_stride),
                                                      self._p(sel), self._p(step_off), int(sel.numel()), self._p(out),
                                                      self._s(stream)))
        return out

    def render_overflow(self):
        """True if a record rendered since the last call had its overflow bit set (units missing from the
        rendered observation; the sender flagged MRTS_ERR_RECORD) — mrts_render_status, synchronises."""
        r = self._h.L.mrts_render_status(self._h.h)
        if r < 0:
            _lib.check(r)
        return bool(r)

    def set_step_responses(self, max_steps):
        """Every step's reward / done from each rollout call of at most max_steps steps
        (mrts_set_step_responses; Java's gameStep returns them on every call): step k of the next call
        lands in self.step_rewards[k] / self.step_dones[k] ([slots] or [slots][R], as reward / done) INSTEAD
        of the plain reward / done buffers, which rollout calls then leave untouched; after such a call
        self.reward / self.done are views of its last ring step (step_rewards[n_steps - 1]), so they never
        read stale.  0 turns it off."""
        h, T = self._h, self.torch
        if not max_steps:
            _lib.check(h.L.mrts_set_step_responses(h.h, None, None, 0))
            self.step_rewards = self.step_dones = None
            self._ring_last = None
            return
        self._ring_last = None
        self.step_rewards = T.zeros((max_steps,) + tuple(self._reward.shape), dtype=T.float64, device=self.device)
        self.step_dones = T.zeros((max_steps,) + tuple(self._done.shape), dtype=T.uint8, device=self.device)
        _lib.check(h.L.mrts_set_step_responses(h.h, self._p(self.step_rewards), self._p(self.step_dones), int(max_steps)))

    def step_rows(self, rows, stream=None):
        """gameStep with Java rows: int32 [slots][n_rows][8] on this device (any order, duplicates ok)."""
        h = self._h
        assert rows.dtype == self.torch.int32 and rows.is_contiguous() and rows.dim() == 3 and rows.shape[2] == 8
        assert rows.shape[0] == h.S and rows.device == self.device
        self._obs_guard()
        _lib.check(h.L.mrts_step_rows_dev(h.h, self._p(rows), rows.shape[1], self._p(self.players), self._p(self.obs),
                                          self._p(self._reward), self._p(self._done),
                                          self._p(self.masks) if self.masks is not None else None, self.mask_player,
                                          self._s(stream)))
        self._ring_last = None
        self._obs_written()

    def onehot_obs(self, obs=None, out=None, stream=None):
        """MicroRTS-Py's encoding of the observation (gym_microrts `_encode_obs`: clip + one-hot,
        channels last): uint8 [slots][H][W][F], F = 29 (33 with partial observability)."""
        h = self._h
        F = h.L.mrts_onehot_features(h.h)
        src = self.obs if obs is None else obs
        if out is None:
            out = self.torch.empty((h.S, h.H, h.W, F), dtype=self.torch.uint8, device=self.device)
        _lib.check(h.L.mrts_onehot_dev(h.h, self._p(src), self._p(out), self._s(stream)))
        return out

    def get_masks(self, out=None, stream=None):
        h = self._h
        out = self.masks if out is None else out
        _lib.check(h.L.mrts_get_masks_dev(h.h, self.mask_player, self._p(out), self._s(stream)))
        return out

    def random_policy(self, seed, step, masks=None, out=None, stream=None):
        h = self._h
        m = self.masks if masks is None else masks
        out = self.actions if out is None else out
        src = self.source if masks is None else None
        # the library rewrites only changed rows when `out` still holds its previous output; an
        # in-place write by anyone else bumps the tensor's version counter -> full rewrite
        if self._policy_out is not out or out._version != self._policy_version:
            _lib.check(h.L.mrts_policy_invalidate(h.h))
        _lib.check(h.L.mrts_policy_dev(h.h, self._p(m), self._p(src), seed, step, self._p(out), self._s(stream)))
        self._policy_out, self._policy_version = out, out._version
        return out

    def synchronize(self):
        self.torch.cuda.current_stream(self.device).synchronize()

    def dump_state(self, slot):
        self.synchronize()
        return self._h.dump(slot)

    def error_flags(self):
        self.synchronize()
        return self._h.error_flags()

    def state_json(self, slot):
        """GameState.toJSON of the game behind `slot` (unit IDs = list positions)."""
        self.synchronize()
        return self._h.state_json(slot)

    def set_state_json(self, slot, text):
        """GameState.fromJSON into the game behind `slot`; call get_masks() before a policy reads masks."""
        self.synchronize()
        self._h.set_state_json(slot, text)
        self._policy_out = None

    def checkpoint(self):
        self.synchronize()
        return self._h.checkpoint()

    def restore(self, data):
        """Every game's state from checkpoint(); call get_masks() before a policy reads masks."""
        self.synchronize()
        self._h.restore(data)
        self._policy_out = None

    @property
    def dims(self):
        h = self._h
        return h.S, h.H, h.W, h.C, h.K

    def close(self):
        self.synchronize()
        self._h.close()


class ForwardModel:
    """Batched forward model for search AIs: n games kept in HBM, each advanced by
    NaiveMCTS.simulate (ai/mcts/naivemcts/NaiveMCTS.java:297-308) with its own playout policies
    (RandomBiasedAI / PassiveAI for players 0 and 1), cloned from any handle's games with
    GameState.clone() semantics (rts/GameState.java:591-610), and scored with
    SimpleSqrtEvaluationFunction3.  Game j's java.util.Random streams are seeded from seed + j (see
    DESIGN.md).  Device calls are ordered on torch's current stream of the device."""

    def __init__(self, n_games, map_path, policies=("RandomBiasedAI", "RandomBiasedAI"), utt=None, device=0, seed=0,
                 max_units=0):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("ForwardModel needs an MI355X (torch.cuda is unavailable); there is no CPU fallback")
        self.torch = torch
        utt = utt or UnitTypeTable()
        p0, p1 = policies
        p0 = p0 if isinstance(p0, (list, tuple)) else [p0] * n_games
        p1 = p1 if isinstance(p1, (list, tuple)) else [p1] * n_games
        maps = list(map_path) if isinstance(map_path, (list, tuple)) else [map_path] * n_games  # one per game, same size
        self._h = _Handle(0, n_games, 1 << 30, [_resolve("", m) for m in maps], p1, utt, False, device, seed, 0,
                          ai1s=p0, forward_model=True, max_units=max_units)
        self.n = n_games
        self.device = torch.device("cuda", device)
        self.value = torch.zeros(n_games, dtype=torch.float32, device=self.device)
        torch.cuda.synchronize(self.device)

    def _s(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self):
        """Every game back to its map's initial state (random streams continue)."""
        h = self._h
        _lib.check(h.L.mrts_reset_dev(h.h, None, None, None, None, None, 0, self._s()))

    def copy_from(self, pairs, src=None):
        """gs[dst] = src_games[src_game].clone() for (dst, src_game) rows of `pairs` (int32 [n, 2]: a
        torch tensor on this device, or anything numpy accepts).  src: a DeviceVecEnv,
        JNIGridnetVecClient or ForwardModel with the same map size (None = self)."""
        h = self._h
        sh = h.h if src is None else src._h.h
        if isinstance(pairs, self.torch.Tensor) and pairs.is_cuda:
            assert pairs.dtype == self.torch.int32 and pairs.is_contiguous() and pairs.dim() == 2 and pairs.shape[1] == 2
            if src is not None and hasattr(src, "synchronize"):
                src.synchronize()
            _lib.check(h.L.mrts_copy_games_dev(h.h, sh, ctypes.c_void_p(pairs.data_ptr()), pairs.shape[0], self._s()))
        else:
            pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
            self.synchronize()
            _lib.check(h.L.mrts_copy_games(h.h, sh, pr.ctypes.data_as(ctypes.c_void_p), pr.shape[0]))

    def playout(self, horizon):
        """NaiveMCTS.simulate(gs, gs.getTime() + horizon) on every game (one launch)."""
        if not -_lib.MRTS_MAX_HORIZON <= horizon <= _lib.MRTS_MAX_HORIZON:
            raise ValueError("horizon out of range")
        h = self._h
        _lib.check(h.L.mrts_playout_dev(h.h, int(horizon), self._s()))

    def trace_step(self, pairs, until, generic=False):
        """One entry of TestTracesIntegrity.testTrace (test/microrts/TestTracesIntegrity.java:72-127) on
        every game: issueSafe(player 0's rows), issueSafe(player 1's rows), then cycle() until time ==
        until[g].  pairs: int32 [n_games, n_pairs, 8] rows [player (-1 = padding), x, y, type, parameter,
        target x, target y, unit type].  Returns the MRTS_TRACE_* bits per game (int32 [n_games])."""
        h = self._h
        pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32))
        assert pr.ndim == 3 and pr.shape[0] == self.n and pr.shape[2] == 8
        un = np.ascontiguousarray(np.asarray(until, dtype=np.int32).reshape(self.n))
        out = np.zeros(self.n, dtype=np.int32)
        self.synchronize()
        _lib.check(h.L.mrts_trace_step(h.h, pr.ctypes.data_as(ctypes.c_void_p), pr.shape[1], un.ctypes.data_as(ctypes.c_void_p),
                                       out.ctypes.data_as(ctypes.c_void_p), int(bool(generic))))
        return out

    def evaluate(self, maxplayer=0, out=None):
        """SimpleSqrtEvaluationFunction3.evaluate(maxplayer, 1 - maxplayer, gs): float32 [n] on device."""
        h = self._h
        out = self.value if out is None else out
        _lib.check(h.L.mrts_evaluate_dev(h.h, int(maxplayer), ctypes.c_void_p(out.data_ptr()), self._s()))
        return out

    def synchronize(self):
        self.torch.cuda.current_stream(self.device).synchronize()

    def dump_state(self, game):
        self.synchronize()
        return self._h.dump(game)

    def error_flags(self):
        self.synchronize()
        return self._h.error_flags()

    def state_json(self, game):
        self.synchronize()
        return self._h.state_json(game)

    def set_state_json(self, game, text):
        self.synchronize()
        self._h.set_state_json(game, text)

    def close(self):
        self.synchronize()
        self._h.close()
