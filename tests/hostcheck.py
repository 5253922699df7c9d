"""ctypes wrapper of libhockey_hostcheck.so: the kernel's per-arena source (hk_step.h and below) compiled
for the host CPU.  TEST / DEBUG HARNESS ONLY -- the product package never loads it.

It runs the exact device code paths (register arena, contact solver, TOI) lane by lane on the CPU, so the
CPU suite can hold the kernel logic to the oracle bit for bit without a GPU, and gdb can step through it.
"""
import ctypes
import os
import subprocess
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hockey-env_amd", "csrc")
LIB = os.environ.get("HKH_LIB") or os.path.join(ROOT, "hockey-env_amd", "hockey_amd", "_lib", "libhockey_hostcheck.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", CSRC, "hostcheck"])


def lib():
    global _lib
    if _lib is None:
        if not os.environ.get("HKH_LIB"):
            build()
        L = ctypes.CDLL(LIB)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.hkh_create.restype = vp
        L.hkh_create.argtypes = [i64, vp, ctypes.c_uint64, i64]
        for name, n in (("hkh_destroy", 1), ("hkh_reset", 5), ("hkh_step", 2), ("hkh_get_state", 3),
                        ("hkh_set_state", 4), ("hkh_observe", 3), ("hkh_counters", 2)):
            getattr(L, name).restype = None
            getattr(L, name).argtypes = [vp] * n
        L.hkh_diag.restype = None
        L.hkh_diag.argtypes = [vp]
        _lib = L
    return _lib


def velocity_diag():
    """Velocity-loop coverage counters of the host build since the last call (and clears them): [0] islands
    retired while another island of the lane kept iterating, [1] live contacts swapped into slots 0/1, [2] S3 lanes
    entering the three-contact shape family, [3] S2 two-contact shape chunks (hk_solver.h)."""
    out = np.zeros(4, np.uint64)
    lib().hkh_diag(out.ctypes.data)
    return out


def _p(a):
    return None if a is None else a.ctypes.data


class StepIO(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("actions", "opp_inc", "obs", "obs2", "reward", "reward2", "done",
                                               "info", "info2", "actions_out", "debug", "final_obs")] + [
                    ("flags", ctypes.c_int32), ("policy2", ctypes.c_void_p), ("record", ctypes.c_void_p)]


POLICY = {"external": 0, "random": 1, "weak": 2, "strong": 3}


class HostVec:
    """Same call shapes as hockey_amd.vec_env.VecHockeyEnv for the calls the parity tests make (numpy)."""

    def __init__(self, n, keep_mode=True, mode=0, auto_reset=False, vel_ref=False,
                 policies=("external", "external"), seed=0, arena_offset=0, diag_flags=0):
        self.n = n
        cfg = np.array([int(keep_mode), int(mode), int(auto_reset), int(vel_ref), POLICY[policies[0]],
                        POLICY[policies[1]], int(diag_flags)], np.int32)
        self._cfg = cfg
        self.L = lib()
        self.h = self.L.hkh_create(n, cfg.ctypes.data, seed, arena_offset)
        self.L.hkh_reset(self.h, None, None, None, None)  # hk_create's device-placement reset

    def close(self):
        if self.h:
            self.L.hkh_destroy(self.h)
            self.h = None

    __del__ = close

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.L.hkh_reset(self.h, _p(m), None, None, None)

    def reset_params(self, params, mask=None, max_t=None):
        p = np.ascontiguousarray(params, np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        mt = None if max_t is None else np.ascontiguousarray(max_t, np.int32)
        self.L.hkh_reset(self.h, _p(m), _p(p), _p(mt), None)

    def step(self, actions=None, with_agent_two=False, opp_inc=None, debug=False, skip_physics=False,
             record_actions=False, final_obs=False, policy2=None, record=False):
        n = self.n
        out = SimpleNamespace(obs=np.zeros((n, 18), np.float32), reward=np.zeros(n, np.float32),
                              done=np.zeros(n, np.uint8), info=np.zeros((n, 4), np.float32))
        io = StepIO()
        a = None if actions is None else np.ascontiguousarray(actions, np.float32)
        inc = None if opp_inc is None else np.ascontiguousarray(opp_inc, np.float64)
        io.actions, io.opp_inc = _p(a), _p(inc)
        io.obs, io.reward, io.done, io.info = _p(out.obs), _p(out.reward), _p(out.done), _p(out.info)
        if with_agent_two:
            out.obs2, out.reward2 = np.zeros((n, 18), np.float32), np.zeros(n, np.float32)
            out.info2 = np.zeros((n, 4), np.float32)
            io.obs2, io.reward2, io.info2 = _p(out.obs2), _p(out.reward2), _p(out.info2)
        if debug:
            out.debug = np.zeros((n, int(debug) if not isinstance(debug, bool) else 13), np.float32)
            io.debug = _p(out.debug)
        if record_actions:
            out.actions = np.zeros((n, 8), np.float32)
            io.actions_out = _p(out.actions)
        if final_obs:
            out.final_obs = np.zeros((n, 18), np.float32)
            io.final_obs = _p(out.final_obs)
        if record:
            out.record = np.zeros((n, 16), np.float64)
            io.record = _p(out.record)
        io.flags = 1 if skip_physics else 0
        p2 = None if policy2 is None else np.ascontiguousarray(policy2, np.uint8)
        io.policy2 = _p(p2)
        self.L.hkh_step(self.h, ctypes.byref(io))
        return out

    def get_state(self):
        st = np.zeros((self.n, 18), np.float32)
        aux = np.zeros((self.n, 5), np.int32)
        self.L.hkh_get_state(self.h, _p(st), _p(aux))
        return st, aux

    def set_state(self, state, aux=None, mask=None):
        st = None if state is None else np.ascontiguousarray(state, np.float32)
        ax = None if aux is None else np.ascontiguousarray(aux, np.int32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.L.hkh_set_state(self.h, _p(m), _p(st), _p(ax))

    def counters(self):
        c = np.zeros(16, np.uint64)
        self.L.hkh_counters(self.h, _p(c))
        return c


def _observe(self):
    o, o2 = np.zeros((self.n, 18), np.float32), np.zeros((self.n, 18), np.float32)
    self.L.hkh_observe(self.h, _p(o), _p(o2))
    return o, o2


HostVec.observe = _observe


class HostTorchEnv:
    """VecHockeyEnv-shaped torch (CPU) view of HostVec, so hockey_amd.td3.train can run its collection loop on
    the kernel source's host build in the CPU suite.  Every step records the actions the kernel applied."""

    def __init__(self, n, **kw):
        import torch

        self.torch = torch
        self.n = n
        self.h = HostVec(n, **kw)

    def reset(self):
        self.h.reset()
        return self.observe()

    def reset_params(self, params, mask=None, max_t=None):
        self.h.reset_params(np.asarray(params, np.float32), mask, max_t)

    def observe(self):
        o, o2 = self.h.observe()
        return self.torch.from_numpy(o), self.torch.from_numpy(o2)

    def step(self, actions=None, with_agent_two=False, policy2=None, **kw):
        t = self.torch
        a = None if actions is None else np.ascontiguousarray(t.as_tensor(actions).cpu().numpy(), np.float32)
        p2 = None if policy2 is None else np.ascontiguousarray(t.as_tensor(policy2).cpu().numpy(), np.uint8)
        r = self.h.step(a, with_agent_two=with_agent_two, policy2=p2, record_actions=True)
        conv = {k: t.from_numpy(v) for k, v in vars(r).items()}
        return SimpleNamespace(**conv)

    def close(self):
        self.h.close()
