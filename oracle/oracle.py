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
        L.hko_set_vel_ref.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.hko_begin_contact.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        L.hko_philox.argtypes = [ctypes.c_uint64, u32p, u32p]
        vp = ctypes.c_void_p
        L.hkov_create.restype = vp
        L.hkov_create.argtypes = [ctypes.c_int64, _i32p, ctypes.c_uint64, ctypes.c_int64]
        L.hkov_destroy.argtypes = [vp]
        L.hkov_reset.argtypes = [vp, vp, vp, vp, vp]
        L.hkov_set_policy.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.hkov_step.argtypes = [vp] * 13
        L.hkov_get_state.argtypes = [vp, vp, vp]
        L.hkov_set_state.argtypes = [vp, vp, vp, vp]
        L.hkov_observe.argtypes = [vp, vp, vp]
        L.hkov_phase.argtypes = [vp, vp, vp]
        L.hkov_counters.argtypes = [vp, vp]
        L.hkov_time_steps.restype = ctypes.c_double
        L.hkov_time_steps.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.hko_set_variant.argtypes = [ctypes.c_int]
        L.hko_run_c1.restype = ctypes.c_int
        L.hko_run_c1.argtypes = [ctypes.c_int, _f32p, _f64p, ctypes.c_double, _f32p, ctypes.c_int, vp, vp,
                                 ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


class OracleWorld:
    """One arena of the CPU restatement (HockeyEnv + Box2D-2.3 step)."""

    def __init__(self, keep_mode=True, mode=0, vel_ref=False):
        self._L = lib()
        self.keep_mode = bool(keep_mode)
        self.mode = int(mode)
        self._w = self._L.hko_create(int(keep_mode), int(mode))
        if vel_ref:
            self._L.hko_set_vel_ref(self._w, 1)

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

    def begin_contact(self, body_a, body_b):
        self._L.hko_begin_contact(self._w, int(body_a), int(body_b))

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


VAR_REVERSE, VAR_NO_BLOCK, VAR_NO_SLEEP, VAR_ITERS_8_3 = 1, 2, 4, 8
# deliberately wrong physics: negative controls of the behavioural pins (scripts/pin_power_study.py)
VAR_REST_THRESH0, VAR_ARITH_FRIC, VAR_NO_TOI, VAR_REST_MIN = 16, 32, 64, 128
# goal-path variants (hk_oracle.c HKO_VAR_SENSOR_* / HKO_VAR_KEEP_COM)
VAR_SENSOR_SKIN_PLUS, VAR_SENSOR_SKIN_MINUS, VAR_SENSOR_SWEPT, VAR_KEEP_COM = 256, 512, 1024, 2048
VAR_SENSOR_CORE = 4096


def set_variant(flags):
    """Process-wide sensitivity-study variant of the Box2D restatement (hk_oracle.c hko_set_variant); 0 restores
    the restatement the kernel is pinned to."""
    lib().hko_set_variant(int(flags))


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


def philox(key, ctr):
    """Philox4x32-10 block: key (uint64), counter (4 x uint32) -> 4 x uint32."""
    out = np.zeros(4, np.uint32)
    lib().hko_philox(int(key), np.ascontiguousarray(ctr, np.uint32), out)
    return out


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


POLICY = {"external": 0, "random": 1, "weak": 2, "strong": 3}


class OracleVec:
    """N arenas of the CPU restatement behind the hk_create / hk_reset / hk_step contract (include/hockey.h):
    fused policies, Philox randomness keyed by global arena id, auto-reset.  numpy in / out, [N, k] arrays."""

    def __init__(self, n, keep_mode=True, mode=0, auto_reset=False, vel_ref=False, policies=("external", "external"),
                 seed=0, arena_offset=0):
        self._L = lib()
        self.n = int(n)
        cfg = np.array([int(keep_mode), int(mode), int(auto_reset), int(vel_ref), POLICY[policies[0]],
                        POLICY[policies[1]]], np.int32)
        self._v = self._L.hkov_create(self.n, cfg, int(seed) & ((1 << 64) - 1), int(arena_offset))

    def close(self):
        if getattr(self, "_v", None):
            self._L.hkov_destroy(self._v)
            self._v = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reset(self, mask=None, params=None, max_t=None, one_starts=None):
        c = np.ascontiguousarray
        m = None if mask is None else c(mask, np.uint8)
        p = None if params is None else c(params, np.float32)
        t = None if max_t is None else c(max_t, np.int32)
        o = None if one_starts is None else c(one_starts, np.uint8)
        self._L.hkov_reset(self._v, _p(m), _p(p), _p(t), _p(o))

    def set_policy(self, player, policy):
        self._L.hkov_set_policy(self._v, int(player), POLICY[policy] if isinstance(policy, str) else int(policy))

    def step(self, actions=None, opp_inc=None, with_agent_two=False, final_obs=False, policy2=None):
        n = self.n
        p2 = None if policy2 is None else np.ascontiguousarray(policy2, np.uint8).reshape(n)
        a = None if actions is None else np.ascontiguousarray(actions, np.float32).reshape(n, 8)
        inc = None if opp_inc is None else np.ascontiguousarray(opp_inc, np.float64).reshape(n, 2)
        out = {"obs": np.zeros((n, 18), np.float32), "reward": np.zeros(n, np.float32),
               "done": np.zeros(n, np.uint8), "info": np.zeros((n, 4), np.float32),
               "actions": np.zeros((n, 8), np.float32)}
        if with_agent_two:
            out.update(obs2=np.zeros((n, 18), np.float32), reward2=np.zeros(n, np.float32),
                       info2=np.zeros((n, 4), np.float32))
        if final_obs:
            out["final_obs"] = np.zeros((n, 18), np.float32)
        g = out.get
        self._L.hkov_step(self._v, _p(a), _p(inc), _p(g("obs")), _p(g("obs2")), _p(g("reward")), _p(g("reward2")),
                          _p(g("done")), _p(g("info")), _p(g("info2")), _p(g("actions")), _p(g("final_obs")),
                          _p(p2))
        return out

    def get_state(self):
        st = np.zeros((self.n, 18), np.float32)
        aux = np.zeros((self.n, 5), np.int32)
        self._L.hkov_get_state(self._v, _p(st), _p(aux))
        return st, aux

    def set_state(self, state=None, aux=None, mask=None):
        c = np.ascontiguousarray
        st = None if state is None else c(state, np.float32)
        ax = None if aux is None else c(aux, np.int32)
        m = None if mask is None else c(mask, np.uint8)
        self._L.hkov_set_state(self._v, _p(m), _p(st), _p(ax))

    def observe(self):
        o, o2 = np.zeros((self.n, 18), np.float32), np.zeros((self.n, 18), np.float32)
        self._L.hkov_observe(self._v, _p(o), _p(o2))
        return o, o2

    def phase(self, new=None):
        out = np.zeros((self.n, 2), np.float64)
        ph = None if new is None else np.ascontiguousarray(new, np.float64)
        self._L.hkov_phase(self._v, _p(out), _p(ph))
        return out

    def counters(self):
        out = np.zeros(16, np.int64)
        self._L.hkov_counters(self._v, _p(out))
        return out

    def time_steps(self, steps, threads=0):
        """Wall seconds of `steps` batched steps on `threads` OpenMP threads (the CPU baseline)."""
        return self._L.hkov_time_steps(self._v, int(steps), int(threads))


def run_c1(p2_actions, p1_inc, p1_phase0, params, record=True):
    """BASELINE C1 on one arena, one thread: weak BasicOpponent (player 1) vs the given player-2 actions,
    reset on done from ``params`` ([E, 6], one row per reset(seed=episode)).  Returns (obs, done, episodes,
    seconds)."""
    p2 = np.ascontiguousarray(p2_actions, np.float32)
    steps = p2.shape[0]
    inc = np.ascontiguousarray(p1_inc, np.float64)
    prm = np.ascontiguousarray(params, np.float32)
    obs = np.zeros((steps, 18), np.float32) if record else None
    done = np.zeros(steps, np.uint8) if record else None
    sec = ctypes.c_double()
    ep = lib().hko_run_c1(steps, p2, inc, float(p1_phase0), prm, prm.shape[0], _p(obs), _p(done), ctypes.byref(sec))
    return obs, done, ep, sec.value
