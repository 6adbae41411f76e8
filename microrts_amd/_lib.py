"""ctypes binding of libmrts.so (include/mrts.h).  The product path is GPU-only: if the HIP
library is missing this module raises — there is no CPU fallback."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRTS_LIB_PATH") or os.path.join(HERE, "libmrts.so")  # override: diagnostics builds only

MRTS_BOT_PASSIVE, MRTS_BOT_RANDOM_BIASED = 0, 1
MRTS_MAX_HORIZON = 65536
# a_rfs names (src/ai/reward/*.java) -> MRTS_RF_* ids
REWARD_FUNCTIONS = {"WinLossRewardFunction": 0, "ResourceGatherRewardFunction": 1, "ProduceWorkerRewardFunction": 2,
                    "ProduceBuildingRewardFunction": 3, "AttackRewardFunction": 4, "ProduceCombatUnitRewardFunction": 5,
                    "CloserToEnemyBaseRewardFunction": 6, "CloserToEnemyUnitRewardFunction": 7}
ERR_BITS = {
    1 << 0: "CAPACITY", 1 << 1: "ADDUNIT", 1 << 2: "PRODUCE_TYPE", 1 << 3: "OLDER_CONFLICT",
    1 << 4: "NEG_RESOURCES", 1 << 5: "MOVE_COLLISION", 1 << 6: "RECORD",
}

def _code_sections(obj):
    """The .text and .rodata sections (the kernels' machine code and kernel descriptors) of an amdgcn code
    object, concatenated: what the kernels run, without the symbol tables (hipcc's per-compile __hip_cuid_*
    symbol differs between builds of the same source under different -D flags)."""
    import struct

    shoff = struct.unpack_from("<Q", obj, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", obj, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", obj, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    out = b""
    for want in (b".text", b".rodata"):
        for name, _, _, _, off, size in secs:
            if obj[stroff + name:obj.index(b"\0", stroff + name)] == want:
                out += obj[off:off + size]
    if not out:
        raise RuntimeError("amdgcn code object without .text")
    return out


def device_code_sha256(path=None):
    """SHA-256 of the gfx950 code inside libmrts.so (the .hip_fatbin offload bundle's amdgcn entry): its
    .text and .rodata, the kernels' machine code and descriptors.  Counter files (profiles/pmc_*.json) name
    the code they describe with it, so a host-only change to the library keeps them valid and any kernel
    change voids them."""
    import hashlib
    import struct

    data = open(path or LIB_PATH, "rb").read()
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _, _, _, off, size in secs:
        if data[stroff + name:data.index(b"\0", stroff + name)] != b".hip_fatbin":
            continue
        b = data[off:off + size]
        if not b.startswith(b"__CLANG_OFFLOAD_BUNDLE__"):
            break
        n, p = struct.unpack_from("<Q", b, 24)[0], 32
        for _ in range(n):
            eoff, esize, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if "amdgcn" in triple:
                return hashlib.sha256(_code_sections(b[eoff:eoff + esize])).hexdigest()
    raise RuntimeError(f"{path or LIB_PATH}: no amdgcn code object in .hip_fatbin")


# every symbol include/mrts.h declares
EXPORTS = [
    "mrts_create", "mrts_dims", "mrts_reset", "mrts_step", "mrts_get_masks", "mrts_step_rows", "mrts_get_masks_i32",
    "mrts_get_masks_host", "mrts_get_masks_i32_host",
    "mrts_reset_dev", "mrts_step_dev", "mrts_get_masks_dev", "mrts_step_rows_dev", "mrts_get_masks_i32_dev", "mrts_onehot_features", "mrts_onehot_dev", "mrts_policy_dev", "mrts_step_fused_dev", "mrts_rollout_fused_dev", "mrts_set_rollout_events", "mrts_rccl_unique_id", "mrts_exchange_init", "mrts_exchange_init_loopback", "mrts_rollout_fused_exchange_dev", "mrts_rollout_uniform_exchange_dev", "mrts_set_exchange_bytes", "mrts_set_records", "mrts_record_words", "mrts_rollout_fused_records_dev", "mrts_rollout_uniform_records_dev", "mrts_render_records_dev", "mrts_render_status", "mrts_render_records_onehot_dev", "mrts_set_step_responses", "mrts_capture_begin", "mrts_capture_end", "mrts_replay", "mrts_set_multi_step", "mrts_multi_step_capable", "mrts_set_obs16", "mrts_policy_uniform_dev", "mrts_step_uniform_dev", "mrts_rollout_uniform_dev", "mrts_policy_invalidate", "mrts_set_obs_delta", "mrts_obs_invalidate", "mrts_set_source_output", "mrts_copy_games", "mrts_copy_games_dev", "mrts_playout", "mrts_playout_dev", "mrts_trace_step",
    "mrts_evaluate", "mrts_evaluate_dev", "mrts_utt_json", "mrts_get_state_json",
    "mrts_set_state_json", "mrts_checkpoint_size", "mrts_checkpoint", "mrts_restore", "mrts_get_state", "mrts_error_flags", "mrts_env_steps", "mrts_stream",
    "mrts_destroy", "mrts_last_error",
]


class MrtsConfig(ctypes.Structure):
    _fields_ = [
        ("n_selfplay_slots", ctypes.c_int32),
        ("n_bot_envs", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("partial_obs", ctypes.c_int32),
        ("utt_version", ctypes.c_int32),
        ("conflict_policy", ctypes.c_int32),
        ("bot_kinds", ctypes.POINTER(ctypes.c_int32)),
        ("ai1_kinds", ctypes.POINTER(ctypes.c_int32)),
        ("map_paths", ctypes.POINTER(ctypes.c_char_p)),
        ("device", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("slot_id_base", ctypes.c_int32),
        ("mask_delta", ctypes.c_int32),
        ("reward_kinds", ctypes.POINTER(ctypes.c_int32)),
        ("n_rewards", ctypes.c_int32),
        ("forward_model", ctypes.c_int32),
        ("utt_json", ctypes.c_char_p),
        ("max_units", ctypes.c_int32),
    ]


class MrtsResponses(ctypes.Structure):
    _fields_ = [
        ("obs", ctypes.POINTER(ctypes.c_int32)),
        ("reward", ctypes.POINTER(ctypes.c_double)),
        ("done", ctypes.POINTER(ctypes.c_uint8)),
    ]


_lib = None


def load(path=LIB_PATH):
    """Load libmrts.so; raises ImportError (loudly) when the HIP extension has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libmrts.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (no CPU fallback exists)")
    # A process may hold only ONE HIP/HSA runtime.  PyTorch-ROCm bundles its own libamdhip64.so;
    # importing torch first makes libmrts.so bind to that same runtime (its DT_NEEDED soname is
    # already satisfied), which is also what lets torch tensors be passed as device pointers.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    P, I32, U32, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
    L.mrts_create.argtypes = [ctypes.POINTER(MrtsConfig), ctypes.POINTER(P)]
    L.mrts_create.restype = ctypes.c_int
    L.mrts_dims.argtypes = [P, P, P, P, P, P]
    L.mrts_reset.argtypes = [P, P, ctypes.POINTER(MrtsResponses)]
    L.mrts_step.argtypes = [P, P, P, ctypes.POINTER(MrtsResponses)]
    L.mrts_get_masks.argtypes = [P, I32, P]
    L.mrts_step_rows.argtypes = [P, P, I32, P, ctypes.POINTER(MrtsResponses)]
    L.mrts_get_masks_i32.argtypes = [P, I32, P]
    L.mrts_get_masks_host.argtypes = [P, I32, ctypes.POINTER(ctypes.c_void_p)]
    L.mrts_get_masks_i32_host.argtypes = [P, I32, ctypes.POINTER(ctypes.c_void_p)]
    L.mrts_step_rows_dev.argtypes = [P, P, I32, P, P, P, P, P, I32, P]
    L.mrts_get_masks_i32_dev.argtypes = [P, I32, P, P]
    L.mrts_onehot_features.argtypes = [P]
    L.mrts_onehot_dev.argtypes = [P, P, P, P]
    L.mrts_reset_dev.argtypes = [P, P, P, P, P, P, I32, P]
    L.mrts_step_dev.argtypes = [P, P, P, P, P, P, P, I32, P]
    L.mrts_get_masks_dev.argtypes = [P, I32, P, P]
    L.mrts_policy_dev.argtypes = [P, P, P, U64, U32, P, P]
    L.mrts_policy_invalidate.argtypes = [P]
    L.mrts_step_fused_dev.argtypes = [P, P, P, P, P, P, P, I32, U64, U32, P]
    L.mrts_rollout_fused_dev.argtypes = [P, P, P, P, P, P, P, I32, U64, U32, I32, P]
    L.mrts_policy_uniform_dev.argtypes = [P, U64, U32, P, P]
    L.mrts_step_uniform_dev.argtypes = [P, P, P, P, P, P, P, I32, U64, U32, P]
    L.mrts_rollout_uniform_dev.argtypes = [P, P, P, P, P, P, U64, U32, I32, I32, P]
    L.mrts_set_obs_delta.argtypes = [P, I32]
    L.mrts_set_multi_step.argtypes = [P, I32]
    L.mrts_set_rollout_events.argtypes = [P, P, P]
    C = ctypes.c_char_p
    L.mrts_rccl_unique_id.argtypes = [C, P]
    L.mrts_exchange_init.argtypes = [P, C, I32, I32, P]
    L.mrts_exchange_init_loopback.argtypes = [P, I32, I32]
    L.mrts_rollout_fused_exchange_dev.argtypes = [P, P, P, P, P, P, P, I32, U64, U32, I32, P, P, P, P]
    L.mrts_rollout_uniform_exchange_dev.argtypes = [P, P, P, P, P, P, U64, U32, I32, P, P, P, P]
    L.mrts_set_exchange_bytes.argtypes = [P, I32]
    I64 = ctypes.c_int64
    L.mrts_set_records.argtypes = [P, I32, I32]
    L.mrts_record_words.argtypes = [P]
    L.mrts_rollout_fused_records_dev.argtypes = [P, P, P, P, P, P, P, I32, U64, U32, I32, P, P, P]
    L.mrts_rollout_uniform_records_dev.argtypes = [P, P, P, P, P, P, U64, U32, I32, P, P, P]
    L.mrts_render_records_dev.argtypes = [P, P, I64, I32, I64, P, I32, P]
    L.mrts_render_status.argtypes = [P]
    L.mrts_render_records_onehot_dev.argtypes = [P, P, I64, I32, I64, P, P, I32, P, P]
    L.mrts_set_step_responses.argtypes = [P, P, P, I32]
    L.mrts_capture_begin.argtypes = [P, P]
    L.mrts_capture_end.argtypes = [P, P]
    L.mrts_replay.argtypes = [P, P]
    L.mrts_multi_step_capable.argtypes = [P]
    L.mrts_set_obs16.argtypes = [P, P]
    L.mrts_obs_invalidate.argtypes = [P]
    L.mrts_set_source_output.argtypes = [P, P]
    L.mrts_copy_games.argtypes = [P, P, P, I32]
    L.mrts_copy_games_dev.argtypes = [P, P, P, I32, P]
    L.mrts_playout.argtypes = [P, I32]
    L.mrts_playout_dev.argtypes = [P, I32, P]
    L.mrts_trace_step.argtypes = [P, P, I32, P, P, I32]
    L.mrts_evaluate.argtypes = [P, I32, P]
    L.mrts_evaluate_dev.argtypes = [P, I32, P, P]
    L.mrts_utt_json.argtypes = [I32, I32, ctypes.c_char_p, ctypes.c_char_p, I32]
    L.mrts_get_state.argtypes = [P, I32, P, I32]
    L.mrts_get_state_json.argtypes = [P, I32, ctypes.c_char_p, I32]
    L.mrts_set_state_json.argtypes = [P, I32, ctypes.c_char_p]
    L.mrts_checkpoint_size.argtypes = [P]
    L.mrts_checkpoint_size.restype = ctypes.c_int64
    L.mrts_checkpoint.argtypes = [P, P, ctypes.c_int64]
    L.mrts_restore.argtypes = [P, P, ctypes.c_int64]
    L.mrts_error_flags.argtypes = [P, P]
    L.mrts_env_steps.argtypes = [P, P]
    L.mrts_stream.argtypes = [P]
    L.mrts_stream.restype = P
    L.mrts_destroy.argtypes = [P]
    L.mrts_destroy.restype = None
    L.mrts_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise RuntimeError(f"mrts error {rc}: {load().mrts_last_error().decode()}")
