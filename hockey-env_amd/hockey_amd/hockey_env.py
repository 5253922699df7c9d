"""Drop-in single-environment facades over the batched GPU simulator.

Same names, constructor arguments, return types and quirks as ``hockey/hockey_env.py``:
``HockeyEnv`` (:83-779), ``HockeyEnv_BasicOpponent`` (:875-886), ``BasicOpponent`` (:781-833), ``Mode``
(:78-81) and the ``Hockey-v0`` / ``Hockey-One-v0`` registrations (:889-903).  Each facade owns a
one-arena :class:`~hockey_amd.vec_env.VecHockeyEnv`; the step itself always runs on the MI355X.

Documented differences: rewards/info are float32-rounded (the kernel computes them in
double and emits float32); ``HockeyEnv_BasicOpponent`` evaluates the opponent inside the step kernel
with a per-arena Philox phase stream instead of the global ``np.random``; ``render`` is out of scope.
"""
import warnings

import numpy as np

from .constants import (CENTER_X, CENTER_Y, FPS, MAX_ANGLE, MAX_TIME_KEEP_PUCK, SCALE, Mode, parse_mode)
from .placement import np_random, placement
from .spaces import Box, Discrete

__all__ = ["HockeyEnv", "HockeyEnv_BasicOpponent", "BasicOpponent", "Mode", "register_envs", "make"]


class HockeyEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "render_fps": FPS}
    continuous = False

    def __init__(self, keep_mode: bool = True, mode=Mode.NORMAL, verbose: bool = False, device=None,
                 _policies=("external", "external")):
        from .vec_env import VecHockeyEnv

        self.mode = mode
        self.keep_mode = keep_mode
        self.verbose = verbose
        self.seed()
        self._vec = VecHockeyEnv(1, keep_mode=keep_mode, mode=self._mode, device=device, policies=_policies)
        self.observation_space = Box(-np.inf, np.inf, shape=(18,), dtype=np.float32)
        self.num_actions = 3 if not self.keep_mode else 4
        self.action_space = Box(-1, +1, (self.num_actions * 2,), dtype=np.float32)
        self.discrete_action_space = Discrete(7)  # sic (hockey_env.py:151): 8 actions are defined
        self.timeStep = 1.0 / FPS
        self.one_starts = True
        self.max_timesteps = 250 if self._mode == Mode.NORMAL else 80
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
        self._vec.reset_params(params[None, :])
        obs, _ = self._vec.observe()
        return self._obs_np(obs[0]), self._get_info()

    def step(self, action):
        a = np.clip(np.asarray(action), -1, +1).astype(np.float32)
        if not self.keep_mode:
            a = np.concatenate([a[0:3], [0.0], a[3:6], [0.0]]).astype(np.float32)
        res = self._vec.step(a[None, :])
        obs = self._obs_np(res.obs[0])
        r = float(res.reward[0].item())
        d = bool(res.done[0].item())
        info = self._info_dict(res.info[0].cpu().numpy())
        return obs, r, d, False, info

    # --------------------------------------------------------------- observations / info
    def _obs_np(self, t):
        o = t.cpu().numpy().astype(np.float64)
        return o if self.keep_mode else o[:16]

    def _get_obs(self):
        return self._obs_np(self._vec.observe()[0][0])

    def obs_agent_two(self):
        return self._obs_np(self._vec.observe()[1][0])

    @staticmethod
    def _info_dict(v):
        return {"winner": int(v[0]), "reward_closeness_to_puck": float(v[1]), "reward_touch_puck": float(v[2]),
                "reward_puck_direction": float(v[3])}

    def _state(self):
        st, aux = self._vec.get_state()
        return st[0].cpu().numpy(), aux[0].cpu().numpy()

    def _info_for(self, two):
        st, aux = self._state()
        me = st[6:8] if two else st[0:2]
        puck, pv = st[12:14], st[15:17]
        T = self.max_timesteps
        close = 0.0
        cond = (puck[0] > CENTER_X and pv[0] >= 0) if two else (puck[0] < CENTER_X and pv[0] <= 0)
        if cond:
            d = np.asarray(np.float32(me - puck), np.float64)
            close += float(np.sqrt(np.sum(d ** 2))) * (-30. / (250. / SCALE * T / 2))
        touch = 1. if aux[1 if two else 0] == MAX_TIME_KEEP_PUCK else 0.
        f = (-1. if two else 1.) / (T * 25)
        winner = int(aux[4])
        return {"winner": -winner if two else winner, "reward_closeness_to_puck": float(close),
                "reward_touch_puck": float(touch), "reward_puck_direction": float(pv[0]) * f}

    def _get_info(self):
        return self._info_for(False)

    def get_info_agent_two(self):
        return self._info_for(True)

    def _compute_reward(self):
        _, aux = self._state()
        r = 0
        if aux[3]:
            if aux[4] == 1:
                r += 10
            elif aux[4] != 0:
                r -= 10
        return float(r)

    def get_reward(self, info):
        return float(self._compute_reward() + info["reward_closeness_to_puck"])

    def get_reward_agent_two(self, info_two):
        return float(-self._compute_reward() + info_two["reward_closeness_to_puck"])

    # --------------------------------------------------------------- state access (hockey_env.py:594-608)
    def set_state(self, state):
        state = np.asarray(state, np.float64)
        st, aux = self._state()
        raw = st.copy()
        for b, o in ((0, 0), (1, 6)):
            raw[6 * b + 0] = np.float32(state[o + 0] + CENTER_X)
            raw[6 * b + 1] = np.float32(state[o + 1] + CENTER_Y)
            raw[6 * b + 2:6 * b + 6] = np.float32(state[o + 2:o + 6])
        raw[12] = np.float32(state[12] + CENTER_X)
        raw[13] = np.float32(state[13] + CENTER_Y)
        raw[15] = np.float32(state[14])
        raw[16] = np.float32(state[15])
        if self.keep_mode:
            aux[0], aux[1] = int(state[16]), int(state[17])
        self._vec.set_state(raw[None, :], aux[None, :])

    @property
    def time(self):
        return int(self._state()[1][2])

    @property
    def done(self):
        return bool(self._state()[1][3])

    @property
    def winner(self):
        return int(self._state()[1][4])

    @property
    def player1_has_puck(self):
        return int(self._state()[1][0])

    @property
    def player2_has_puck(self):
        return int(self._state()[1][1])

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
    """Hockey-One-v0 (hockey_env.py:875-886): the opponent runs fused inside the GPU step kernel."""

    def __init__(self, mode=Mode.NORMAL, weak_opponent=False, device=None):
        super().__init__(mode=mode, keep_mode=True, device=device,
                         _policies=("external", "weak" if weak_opponent else "strong"))
        self.weak_opponent = weak_opponent
        self.action_space = Box(-1, +1, (4,), dtype=np.float32)

    def step(self, action):
        a = np.zeros(8, np.float32)
        a[0:4] = np.clip(np.asarray(action, np.float64)[0:4], -1, 1).astype(np.float32)
        res = self._vec.step(a[None, :])
        return (self._obs_np(res.obs[0]), float(res.reward[0].item()), bool(res.done[0].item()), False,
                self._info_dict(res.info[0].cpu().numpy()))


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
