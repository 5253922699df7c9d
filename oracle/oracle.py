"""ctypes binding of the C oracle (oracle/hk_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; it is the
checker, never the product.  See hk_oracle.h for what it restates (reference file:line citations).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libhk_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "hk_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.hko_create.restype = ctypes.c_void_p
        L.hko_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.hko_destroy.argtypes = [ctypes.c_void_p]
        L.hko_geometry.restype = ctypes.c_int
        L.hko_geometry.argtypes = [_f32p, ctypes.c_int]
        L.hko_reset.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int]
        L.hko_set_raw.argtypes = [ctypes.c_void_p, _f32p, _i32p]
        L.hko_get_raw.argtypes = [ctypes.c_void_p, _f32p, _i32p]
        L.hko_step.restype = ctypes.c_int
        L.hko_step.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int, _f32p, ctypes.POINTER(ctypes.c_double),
                               _f64p, _f32p]
        L.hko_obs.argtypes = [ctypes.c_void_p, _f32p]
        L.hko_obs_two.argtypes = [ctypes.c_void_p, _f32p]
        L.hko_info_two.argtypes = [ctypes.c_void_p, _f64p, ctypes.POINTER(ctypes.c_double)]
        L.hko_basic_opponent.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                         ctypes.c_double, _f64p, _f64p]
        L.hko_stats.argtypes = [ctypes.c_void_p, _i32p]
        L.hko_bench_random.restype = ctypes.c_int64
        L.hko_bench_random.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


class OracleWorld:
    """One arena of the CPU restatement (HockeyEnv + Box2D-2.3 step)."""

    def __init__(self, keep_mode=True, mode=0):
        self._L = lib()
        self.keep_mode = bool(keep_mode)
        self.mode = int(mode)
        self._w = self._L.hko_create(int(keep_mode), int(mode))

    def __del__(self):
        try:
            if self._w:
                self._L.hko_destroy(self._w)
                self._w = None
        except Exception:  # noqa: BLE001
            pass

    def reset(self, params6, max_t):
        self._L.hko_reset(self._w, np.ascontiguousarray(params6, np.float32), int(max_t))

    def set_raw(self, st18, aux5):
        self._L.hko_set_raw(self._w, np.ascontiguousarray(st18, np.float32), np.ascontiguousarray(aux5, np.int32))

    def get_raw(self):
        st = np.zeros(18, np.float32)
        aux = np.zeros(5, np.int32)
        self._L.hko_get_raw(self._w, st, aux)
        return st, aux

    def step(self, action8, skip_physics=False):
        obs = np.zeros(18, np.float32)
        info = np.zeros(4, np.float64)
        dbg = np.zeros(13, np.float32)
        r = ctypes.c_double()
        d = self._L.hko_step(self._w, np.ascontiguousarray(action8, np.float32), int(skip_physics), obs,
                             ctypes.byref(r), info, dbg)
        return obs, r.value, bool(d), info, dbg

    def obs(self):
        o = np.zeros(18, np.float32)
        self._L.hko_obs(self._w, o)
        return o

    def obs_two(self):
        o = np.zeros(18, np.float32)
        self._L.hko_obs_two(self._w, o)
        return o

    def info_two(self):
        info = np.zeros(4, np.float64)
        r = ctypes.c_double()
        self._L.hko_info_two(self._w, info, ctypes.byref(r))
        return info, r.value

    def stats(self):
        o = np.zeros(4, np.int32)
        self._L.hko_stats(self._w, o)
        return o


def basic_opponent(weak, keep_mode, phase, inc, obs18):
    ph = ctypes.c_double(phase)
    act = np.zeros(4, np.float64)
    lib().hko_basic_opponent(int(weak), int(keep_mode), ctypes.byref(ph), float(inc),
                             np.ascontiguousarray(obs18, np.float64), act)
    return act, ph.value


def geometry():
    out = np.zeros(256, np.float32)
    n = lib().hko_geometry(out, 256)
    return out[:n]


def bench_random(n_arenas, steps, threads=0, seed=0, policy="random"):
    sec = ctypes.c_double()
    pol = {"random": 0, "basic": 1}[policy]
    total = lib().hko_bench_random(int(n_arenas), int(steps), int(threads), int(seed), pol, ctypes.byref(sec))
    return int(total), sec.value
