"""ctypes binding of libhockey_hip.so (include/hockey.h).

The library is built in-tree (hockey-env_amd/csrc/Makefile -> hockey_amd/_lib/libhockey_hip.so) and is
the ONLY compute path: there is no CPU fallback.  Loading fails loudly when the library is missing, and
context creation fails loudly when no gfx950 device is visible.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HK_LIB") or os.path.join(_HERE, "_lib", "libhockey_hip.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

OBS_DIM, ACT_DIM, INFO_DIM, STATE_DIM, AUX_DIM, PARAM_DIM, DEBUG_DIM, NUM_COUNTERS = 18, 8, 4, 18, 5, 6, 13, 16
RECORD_DIM = 16
HOST_RECORD_BYTES = 280  # hk_step_host output: obs f32[18], obs2 f32[18], done u8 (+7), record f64[16]

POLICY_EXTERNAL, POLICY_RANDOM, POLICY_BASIC_WEAK, POLICY_BASIC_STRONG = 0, 1, 2, 3
STEP_SKIP_PHYSICS = 1
DIAG_LARGE_ISLANDS = 1
CNT_STEPS, CNT_EPISODES, CNT_GOALS_P1, CNT_GOALS_P2, CNT_TOI, CNT_OVERFLOW, CNT_LARGE_ISLANDS, CNT_BAD_POLICY = range(8)


class HockeyNativeError(RuntimeError):
    pass


class Config(ctypes.Structure):
    _fields_ = [("keep_mode", ctypes.c_int32), ("mode", ctypes.c_int32), ("auto_reset", ctypes.c_int32),
                ("vel_ref_semantics", ctypes.c_int32), ("policy", ctypes.c_int32 * 2), ("seed", ctypes.c_uint64),
                ("arena_offset", ctypes.c_int64), ("diag_flags", ctypes.c_int32)]


class StepIO(ctypes.Structure):
    _fields_ = [("actions", ctypes.c_void_p), ("opp_inc", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("obs2", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("reward2", ctypes.c_void_p),
                ("done", ctypes.c_void_p), ("info", ctypes.c_void_p), ("info2", ctypes.c_void_p),
                ("actions_out", ctypes.c_void_p), ("debug", ctypes.c_void_p), ("final_obs", ctypes.c_void_p),
                ("flags", ctypes.c_int32), ("policy2", ctypes.c_void_p), ("record", ctypes.c_void_p)]


EXPORTS = ["hk_last_error", "hk_version", "hk_create", "hk_destroy", "hk_num_arenas", "hk_set_policy", "hk_reset",
           "hk_step", "hk_step_host", "hk_rollout", "hk_get_state", "hk_set_state", "hk_opponent_phase", "hk_opponent_phase3",
           "hk_observe", "hk_counters",
           "hk_reset_counters",
           "hk_bytes_per_step", "hk_info"]

_lib = None

# the files csrc/Makefile hashes into <lib>.srchash (HASHSRC = $(SRC) $(HDR) Makefile), in its order
HASH_SOURCES = ["hk_kernels.hip", "hk_capi.cpp", "hk_core.h", "hk_geom.h", "hk_arena.h", "hk_solver.h", "hk_step.h",
                "hk_kernels.h", "hk_scene_data.inc", "../../include/hockey.h", "Makefile"]


def source_hash():
    """12-hex sha256 of the library's sources as they are in this tree (== the Makefile's .srchash)."""
    import hashlib

    h = hashlib.sha256()
    for name in HASH_SOURCES:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:12]


def built_hash():
    """Source hash the in-tree libhockey_hip.so was built from (its .srchash sidecar), or None."""
    try:
        with open(LIB_PATH + ".srchash") as f:
            return f.read().strip() or None
    except OSError:
        return None


def build(force=False, arch="gfx950"):
    """Compile the HIP library in-tree (hipcc cross-compiles gfx950 without a GPU)."""
    cmd = ["make", "-s", "-C", CSRC, f"ARCH={arch}"]
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(cmd)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HockeyNativeError(
            f"native library {LIB_PATH} is missing: run `make -C {CSRC}` (or __graft_entry__.build()); "
            "there is no CPU fallback for the hot path")
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    L.hk_last_error.restype = ctypes.c_char_p
    L.hk_version.restype = ctypes.c_char_p
    L.hk_create.argtypes = [i32, i64, ctypes.POINTER(Config), ctypes.POINTER(vp)]
    L.hk_destroy.argtypes = [vp]
    L.hk_num_arenas.argtypes = [vp]
    L.hk_num_arenas.restype = i64
    L.hk_set_policy.argtypes = [vp, i32, i32]
    L.hk_reset.argtypes = [vp, vp, vp, vp, vp, vp]
    L.hk_step.argtypes = [vp, ctypes.POINTER(StepIO), vp]
    L.hk_rollout.argtypes = [vp, i32, ctypes.POINTER(StepIO), vp]
    L.hk_step_host.argtypes = [vp, vp, vp, i32, vp, vp]
    L.hk_get_state.argtypes = [vp, vp, vp, vp]
    L.hk_set_state.argtypes = [vp, vp, vp, vp, vp]
    L.hk_observe.argtypes = [vp, vp, vp, vp]
    L.hk_info.argtypes = [vp, vp, vp, vp, vp, vp]
    L.hk_opponent_phase.argtypes = [vp, vp, vp, vp]
    L.hk_opponent_phase3.argtypes = [vp, vp, vp, vp]
    L.hk_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), vp]
    L.hk_reset_counters.argtypes = [vp, vp]
    L.hk_bytes_per_step.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    for name in ["hk_create", "hk_destroy", "hk_set_policy", "hk_reset", "hk_step", "hk_step_host", "hk_rollout", "hk_get_state",
                 "hk_set_state",
                 "hk_observe", "hk_info", "hk_opponent_phase", "hk_opponent_phase3", "hk_counters", "hk_reset_counters", "hk_bytes_per_step"]:
        getattr(L, name).restype = i32
    _lib = L
    return L


def check(status, what):
    if status != 0:
        msg = lib().hk_last_error().decode(errors="replace")
        raise HockeyNativeError(f"{what} failed ({status}): {msg}")


def ptr(t):
    """Raw device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
