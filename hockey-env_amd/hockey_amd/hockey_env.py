"""Drop-in single-environment facades over the batched GPU simulator.

Same names, constructor arguments, return types and quirks as ``hockey/hockey_env.py``:
``HockeyEnv`` (:83-779), ``HockeyEnv_BasicOpponent`` (:875-886), ``BasicOpponent`` (:781-833), ``Mode``
(:78-81) and the ``Hockey-v0`` / ``Hockey-One-v0`` registrations (:889-903).  Each facade owns a
one-arena :class:`~hockey_amd.vec_env.VecHockeyEnv`; the step itself always runs on the MI355X.

Every value a facade returns is the kernel's: obs / obs_agent_two from hk_step / hk_observe, and info,
info_agent_two, both rewards and the has_puck / time / done / winner fields in float64 from the step kernel's
record (hk_step_io.record; hk_info after a reset or set_state), exactly as the reference computes them.  A
step is ONE call into the library (hk_step_host): the action and the opponent's phase increment go in through
pinned staging, the step kernel runs, and the packed result (obs, obs2, done, the float64 record) comes back
before the call returns.  The fused
``HockeyEnv_BasicOpponent`` opponent draws its phase from the global ``np.random`` exactly like the
reference's ``BasicOpponent`` (:785, :796), so seeded reference scripts reproduce.  ``render`` is out of scope.
"""
import ctypes
import struct
import warnings

import numpy as np

from . import _native as N
from .constants import CENTER_X, CENTER_Y, FPS, MAX_ANGLE, SCALE, Mode, parse_mode
from .placement import np_random, placement
from .spaces import Box, Discrete

__all__ = ["HockeyEnv", "HockeyEnv_BasicOpponent", "BasicOpponent", "PolicyOpponent", "Mode", "register_envs",
           "make"]

# packed per-env output record (one device buffer, one D2H copy): byte offsets.  _F64 holds hk_step_io.record
# (f64[16]: info, info2, reward, reward2, has1, has2, time, done, winner); hk_info writes its first 10 words
# after a reset / set_state, and _AUXI the int32 aux of hk_get_state then
_OBS, _OBS2, _DONE, _F64, _AUXI, _REC = 0, 72, 144, 152, 280, 304
_INFO, _INFO2, _REW, _REW2 = _F64, _F64 + 32, _F64 + 64, _F64 + 72


def set_state_raw(state, keep_mode=True):
    """HockeyEnv.set_state (hockey_env.py:594-608) as a raw hk_set_state row: body origins / angles /
    velocities in float32 as the pybox2d setters store them, NaN where set_state calls no setter (the puck's
    angle and angular velocity); plus has_puck (int counters) or None when keep_mode is off."""
    state = np.asarray(state, np.float64)
    raw = np.full(18, np.nan, np.float32)
    for b, o in ((0, 0), (1, 6)):
        raw[6 * b + 0:6 * b + 2] = (state[[o, o + 1]] + [CENTER_X, CENTER_Y]).astype(np.float32)
        raw[6 * b + 2:6 * b + 6] = state[o + 2:o + 6].astype(np.float32)
    raw[12:14] = (state[[12, 13]] + [CENTER_X, CENTER_Y]).astype(np.float32)
    raw[15:17] = state[14:16].astype(np.float32)
    has = (int(state[16]), int(state[17])) if keep_mode else None
    return raw, has


class _Snap:
    """The current state's values as the kernel returned them: obs (float64), obs2 (float32, widened when read),
    f (float64 info[0:4], info2[4:8], reward[8], reward2[9]; after a step also has1, has2, time, done, winner in
    [10:15]) and aux (int32 has1, has2, time, done, winner; decoded from f when first read after a step)."""
    __slots__ = ("obs", "obs2_f32", "f", "_aux")

    def __init__(self, obs, obs2_f32, f, aux=None):
        self.obs, self.obs2_f32, self.f, self._aux = obs, obs2_f32, f, aux

    @property
    def aux(self):
        if self._aux is None:
            self._aux = self.f[10:15].astype(np.int32)
        return self._aux


_PACK_ACT = struct.Struct("<8f").pack_into  # the 8 staged actions (float32, as astype rounds)
_PACK_INC = struct.Struct("<d").pack_into


def _stage_actions(buf, action):
    """buf[0:8] (float32) = float32(np.clip(np.asarray(action, np.float64)[0:4], -1, 1)) followed by four zeros
    (hockey_env.py:659, 875-886), packed in one call without numpy temporaries for the common inputs (a float
    ndarray or a list of floats).  min(max(x, -1), 1) with x first returns x for NaN and keeps -0.0, as np.clip
    does; the float32 pack rounds to nearest like astype."""
    if isinstance(action, np.ndarray) and action.dtype.kind == "f" and action.ndim == 1 and action.shape[0] >= 4:
        v = action[0:4].tolist()
    elif isinstance(action, (list, tuple)) and len(action) >= 4 and all(type(x) is float for x in action[0:4]):
        v = action
    else:
        v = np.clip(np.asarray(action, np.float64)[0:4], -1, 1).tolist()
    _PACK_ACT(buf, 0, min(max(v[0], -1.0), 1.0), min(max(v[1], -1.0), 1.0), min(max(v[2], -1.0), 1.0),
              min(max(v[3], -1.0), 1.0), 0.0, 0.0, 0.0, 0.0)


class HockeyEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": FPS}
    continuous = False

    def __init__(self, keep_mode: bool = True, mode=Mode.NORMAL, verbose: bool = False, device=None,
                 _policies=("external", "external")):
        import torch

        from .vec_env import VecHockeyEnv

        self.mode = mode
        self.keep_mode = keep_mode
        self.verbose = verbose
        self.seed()
        self._vec = VecHockeyEnv(1, keep_mode=keep_mode, mode=self._mode, device=device, policies=_policies)
        # reset / set_state refresh: a device record and its pinned host twin (one transfer)
        self._rec = torch.zeros(_REC, dtype=torch.uint8, device=self._vec.device)
        self._rec_h = torch.zeros(_REC, dtype=torch.uint8, pin_memory=True)
        base = self._rec.data_ptr()
        # hk_step_host: host-side in / out buffers of one step (include/hockey.h HK_HOST_RECORD_BYTES)
        self._act_np = np.zeros(N.ACT_DIM, np.float32)
        self._inc_np = np.zeros(2, np.float64)
        self._out_np = np.zeros(N.HOST_RECORD_BYTES, np.uint8)
        self._out_obs = np.frombuffer(self._out_np, np.float32, 18, _OBS)  # views into the step's out buffer
        self._out_obs2 = np.frombuffer(self._out_np, np.float32, 18, _OBS2)
        self._out_f = np.frombuffer(self._out_np, np.float64, 16, _F64)
        self._step_flags = 0  # HK_STEP_* (the golden harness sets HK_STEP_SKIP_PHYSICS)
        self._host_ptrs = (self._act_np.ctypes.data_as(ctypes.c_void_p), self._inc_np.ctypes.data_as(ctypes.c_void_p),
                           self._out_np.ctypes.data_as(ctypes.c_void_p))
        # the step's fixed call argument; the context, flags and torch's current stream are read per call, so a
        # step is ordered on the same stream as the reset / set_state / observe calls around it
        self._step_fn = self._vec.L.hk_step_host
        self._ptr = {k: ctypes.c_void_p(base + off) for k, off in
                     (("obs", _OBS), ("obs2", _OBS2), ("info", _INFO), ("info2", _INFO2), ("reward", _REW),
                      ("reward2", _REW2), ("aux", _AUXI))}
        self._snap = None
        self.observation_space = Box(-np.inf, np.inf, shape=(18,), dtype=np.float32)
        self.num_actions = 3 if not self.keep_mode else 4
        self.action_space = Box(-1, +1, (self.num_actions * 2,), dtype=np.float32)
        self.discrete_action_space = Discrete(7)  # sic (hockey_env.py:151): 8 actions are defined
        self.timeStep = 1.0 / FPS
        self.one_starts = True
        self.max_timesteps = None  # see reset
        self.closest_to_goal_dist = 1000
        self.reset(self.one_starts)

    # --------------------------------------------------------------- mode (hockey_env.py:754-779)
    @property
    def mode(self):
        return self._mode

    @mode.setter
    def mode(self, value):
        self._mode = parse_mode(value)

    def seed(self, seed=None):
        self.np_random, seed = np_random(seed)
        self._seed = seed
        return [seed]

    # --------------------------------------------------------------- device record
    def _refresh(self):
        """The obs, info / rewards and aux of the current state after a reset / set_state: computed on the device
        and copied to the host in one transfer (after a step, hk_step_host returned them; see _launch_step)."""
        L, ctx, st = self._vec.L, self._vec._ctx, self._vec._stream()
        p = self._ptr
        N.check(L.hk_observe(ctx, p["obs"], p["obs2"], st), "hk_observe")
        N.check(L.hk_info(ctx, p["info"], p["info2"], p["reward"], p["reward2"], st), "hk_info")
        N.check(L.hk_get_state(ctx, None, p["aux"], st), "hk_get_state")
        import torch

        self._rec_h.copy_(self._rec, non_blocking=True)
        torch.cuda.current_stream(self._vec.device).synchronize()
        b = self._rec_h.numpy()
        self._snap = _Snap(np.frombuffer(b, np.float32, 18, _OBS).astype(np.float64),
                           np.frombuffer(b, np.float32, 18, _OBS2).copy(),
                           np.frombuffer(b, np.float64, 10, _F64).copy(), np.frombuffer(b, np.int32, 5, _AUXI).copy())
        return self._snap

    # --------------------------------------------------------------- reset / step
    def reset(self, one_starting=None, mode=None, seed=None, options=None):
        self.seed(seed)
        if mode is not None:
            # the reference evaluates hasattr(Mode, self.mode) with an Enum, which raises
            hasattr(Mode, self._mode)
        if self._mode == Mode.NORMAL:
            self.max_timesteps = 250
            self.one_starts = bool(one_starting) if one_starting is not None else (not self.one_starts)
        else:
            self.max_timesteps = 80
        self.closest_to_goal_dist = 1000
        params, max_t = placement(self._mode, self.one_starts, self.np_random)
        self._vec.one_starts[:] = self.one_starts
        # max_t travels explicitly: the kernel's info / time limit follow the mode of THIS reset even after
        # the mode setter changed it (hockey_env.py:357-365)
        self._vec.reset_params(params[None, :], max_t=[max_t])
        s = self._refresh()
        return self._obs_out(s.obs), self._get_info()

    def _launch_step(self, a8, opp_inc=None):
        """a8: the 8 actions, or None when the caller wrote them into _act_np; opp_inc: the two phase increments,
        True when the caller wrote them into _inc_np, or None (the kernel draws its own)."""
        if a8 is not None:
            self._act_np[:] = a8
        act_p, inc_p, out_p = self._host_ptrs
        if opp_inc is None:
            inc_p = None
        elif opp_inc is not True:
            self._inc_np[:] = opp_inc
        rc = self._step_fn(self._vec._ctx, act_p, inc_p, self._step_flags, out_p, self._vec._stream())
        if rc:
            N.check(rc, "hk_step_host")
        # the snapshot: obs2 / f stay views of the step's out buffer, which only
        # the next step rewrites
        o = self._out_obs.astype(np.float64)
        self._snap = _Snap(o, self._out_obs2, self._out_f)
        f = self._out_f.tolist()  # Python floats of the record (one conversion instead of one per field)
        # a fresh float64 array either way: the snapshot keeps o, so an in-place change of the returned obs
        # must not reach _get_obs() (the reference returns an independent array)
        obs = o.copy() if self.keep_mode else o[:16].copy()
        return obs, f[8], bool(f[13]), False, {"winner": int(f[0]), "reward_closeness_to_puck": f[1],
                                               "reward_touch_puck": f[2], "reward_puck_direction": f[3]}

    def step(self, action):
        a = np.clip(np.asarray(action, np.float64), -1, +1).astype(np.float32)  # hockey_env.py:659
        if not self.keep_mode:
            a = np.concatenate([a[0:3], [0.0], a[3:6], [0.0]]).astype(np.float32)
        return self._launch_step(a)

    # --------------------------------------------------------------- observations / info
    def _obs_out(self, o):
        return o.copy() if self.keep_mode else o[:16].copy()

    def _get_obs(self):
        return self._obs_out(self._snap.obs)

    def obs_agent_two(self):
        return self._obs_out(self._snap.obs2_f32.astype(np.float64))

    @staticmethod
    def _info_dict(v):
        return {"winner": int(v[0]), "reward_closeness_to_puck": float(v[1]), "reward_touch_puck": float(v[2]),
                "reward_puck_direction": float(v[3])}

    def _get_info(self):
        return self._info_dict(self._snap.f[0:4])

    def get_info_agent_two(self):
        return self._info_dict(self._snap.f[4:8])

    def _compute_reward(self):
        """hockey_env.py:518-527 from the kernel's done / winner."""
        aux = self._snap.aux
        if not aux[3]:
            return 0.0
        return 10.0 if aux[4] == 1 else (-10.0 if aux[4] != 0 else 0.0)

    def get_reward(self, info):
        return float(self._compute_reward() + info["reward_closeness_to_puck"])

    def get_reward_agent_two(self, info_two):
        return float(-self._compute_reward() + info_two["reward_closeness_to_puck"])

    # --------------------------------------------------------------- state access (hockey_env.py:594-608)
    def set_state(self, state):
        """pybox2d setters in the reference's order; the puck's angle and angular velocity are not assigned
        (NaN = setter not called, include/hockey.h hk_set_state).  has_puck is stored as an int counter."""
        raw, has = set_state_raw(state, self.keep_mode)
        aux = self._snap.aux.copy()
        if has is not None:
            aux[0], aux[1] = has
        self._vec.set_state(raw[None, :], aux[None, :])
        self._refresh()

    @property
    def time(self):
        return int(self._snap.aux[2])

    @property
    def done(self):
        return bool(self._snap.aux[3])

    @property
    def winner(self):
        return int(self._snap.aux[4])

    @property
    def player1_has_puck(self):
        return int(self._snap.aux[0])

    @property
    def player2_has_puck(self):
        return int(self._snap.aux[1])

    def discrete_to_continous_action(self, discrete_action):
        """hockey_env.py:637-656"""
        action_cont = [(discrete_action == 1) * -1.0 + (discrete_action == 2) * 1.0,
                       (discrete_action == 3) * -1.0 + (discrete_action == 4) * 1.0,
                       (discrete_action == 5) * -1.0 + (discrete_action == 6) * 1.0]
        if self.keep_mode:
            action_cont.append((discrete_action == 7) * 1.0)
        return action_cont

    def render(self, mode="human"):  # pragma: no cover - UI is out of scope
        warnings.warn("hockey_amd: render() is not part of the accelerated hot path; nothing is drawn")
        return None

    def close(self):
        self._vec.close()

    @property
    def unwrapped(self):
        return self


class BasicOpponent:
    """Scripted PD opponent (hockey_env.py:781-833) for single observations on the host.

    Batched arenas evaluate the same controller inside the step kernel (policy 'weak'/'strong')."""

    def __init__(self, weak=True, keep_mode=True):
        self.weak = weak
        self.keep_mode = keep_mode
        self.phase = np.random.uniform(0, np.pi)

    def act(self, obs, verbose=False):
        alpha = obs[2]
        p1 = np.asarray([obs[0], obs[1], alpha])
        v1 = np.asarray(obs[3:6])
        puck = np.asarray(obs[12:14])
        puckv = np.asarray(obs[14:16])
        target_pos = p1[0:2]
        self.phase += np.random.uniform(0, 0.2)
        time_to_break = 0.1
        kp = 0.5 if self.weak else 10
        kd = 0.5
        if puckv[0] < 30.0 / SCALE:
            dist = np.sqrt(np.sum((p1[0:2] - puck) ** 2))
            if p1[0] < puck[0] and abs(p1[1] - puck[1]) < 30.0 / SCALE:
                target_pos = [puck[0] + 0.2, puck[1] + puckv[1] * dist * 0.1]
            else:
                target_pos = [-210 / SCALE, puck[1]]
        else:
            target_pos = [-210 / SCALE, 0]
        target_angle = MAX_ANGLE * np.sin(self.phase)
        shoot = 0.0
        if self.keep_mode and obs[16] > 0 and obs[16] < 7:
            shoot = 1.0
        target = np.asarray([target_pos[0], target_pos[1], target_angle])
        error = target - p1
        need_break = abs((error / (v1 + 0.01))) < [time_to_break, time_to_break, time_to_break * 10]
        action = np.clip(error * [kp, kp / 5, kp / 2] - v1 * need_break * [kd, kd, kd], -1, 1)
        if self.keep_mode:
            return np.hstack([action, [shoot]])
        return action


class HockeyEnv_BasicOpponent(HockeyEnv):
    """Hockey-One-v0 (hockey_env.py:875-886): the opponent runs fused inside the GPU step kernel on the
    kernel's own obs_agent_two, with the phase stream of the reference's BasicOpponent: U(0, pi) from the
    global ``np.random`` at construction (:785) and U(0, 0.2) per act (:796), fed as ``opp_inc``."""

    def __init__(self, mode=Mode.NORMAL, weak_opponent=False, device=None):
        super().__init__(mode=mode, keep_mode=True, device=device,
                         _policies=("external", "weak" if weak_opponent else "strong"))
        self.opponent = BasicOpponent(weak=weak_opponent)  # draws the phase from np.random, as the reference
        self.weak_opponent = weak_opponent
        self.action_space = Box(-1, +1, (4,), dtype=np.float32)
        self._vec.opponent_phase(np.array([[0.0, self.opponent.phase]]))

    def step(self, action):
        # the draw opponent.act(obs_agent_two()) makes (hockey_env.py:796): RandomState.uniform(0, 0.2) is
        # 0.0 + (0.2 - 0.0) * random_sample(), the same double as 0.2 * random() from the same global stream
        inc = 0.2 * np.random.random()
        self.opponent.phase += inc  # host mirror of the kernel's phase
        _stage_actions(self._act_np, action)
        _PACK_INC(self._inc_np, 8, inc)
        return self._launch_step(None, opp_inc=True)


class PolicyOpponent:
    """hockey_env.py:908-922: a torch policy as an opponent, ``act(obs) -> np.ndarray`` (4,)."""

    def __init__(self, policy, device=None):
        self.policy = policy
        self.device = device

    def act(self, obs):
        import torch

        with torch.no_grad():
            x = torch.tensor(obs, dtype=torch.float32, device=self.device).unsqueeze(0)
            return self.policy(x).squeeze(0).cpu().numpy()


_REGISTRY = {
    "Hockey-v0": (HockeyEnv, {"mode": 0}),
    "Hockey-One-v0": (HockeyEnv_BasicOpponent, {"mode": 0, "weak_opponent": False}),
}


def make(env_id, **kwargs):
    """gym.make replacement when gymnasium is absent."""
    cls, kw = _REGISTRY[env_id]
    kw = dict(kw)
    kw.update(kwargs)
    return cls(**kw)


def register_envs():
    """Register Hockey-v0 / Hockey-One-v0 with gymnasium when it is importable (hockey_env.py:889-903)."""
    try:
        from gymnasium.envs.registration import register
    except Exception:  # noqa: BLE001
        return False
    for env_id, (cls, kw) in _REGISTRY.items():
        try:
            register(id=env_id, entry_point=f"hockey_amd.hockey_env:{cls.__name__}", kwargs=kw)
        except Exception as e:  # noqa: BLE001
            print(e)
    return True


register_envs()
