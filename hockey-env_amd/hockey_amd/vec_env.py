"""VecHockeyEnv: N independent arenas resident in HBM, stepped by the gfx950 kernel.

This is the batched form of ``HockeyEnv`` (hockey/hockey_env.py:83-779): every call maps one-to-one
onto the reference's per-env call, vectorised over a leading arena axis and kept on the device:

  ========================================  ================================================
  reference (one env, numpy, host)          VecHockeyEnv (N arenas, torch tensors on cuda)
  ========================================  ================================================
  reset(seed=s)            :345              reset(seeds=[...]) / reset() (device placement)
  step(a[8]) -> obs,r,d,_,info :658          step(actions[N,8]) -> obs[N,18], r[N], d[N], info
  obs_agent_two()          :500              obs_agent_two()  (or step(..., with_agent_two=True))
  get_info_agent_two()/get_reward_agent_two  returned by step(..., with_agent_two=True)
  set_state(s[18])         :594              set_state(state[N,18] raw, aux[N,5])
  BasicOpponent.act        :787              policy=('external'|'random'|'weak'|'strong') per player
  ========================================  ================================================

Torch is plumbing only (device memory + the current HIP stream); the compute is libhockey_hip.so.
"""
import ctypes

import numpy as np
import torch

from . import _native as N

from .constants import Mode, parse_mode
from .placement import np_random, placement

# torch's private accessor for the current raw stream (no Stream object per call); the public form is the fallback,
# and tests/test_gpu_facade.py holds the two equal inside and outside a torch.cuda.stream context
_getraw = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(index):
    """torch's current stream on device ``index`` as an integer hipStream_t."""
    if _getraw is not None:
        return _getraw(index)
    return torch.cuda.current_stream(index).cuda_stream


_POLICIES = {"external": N.POLICY_EXTERNAL, "random": N.POLICY_RANDOM, "weak": N.POLICY_BASIC_WEAK,
             "strong": N.POLICY_BASIC_STRONG}


def _policy_id(p):
    if isinstance(p, int):
        return p
    return _POLICIES[p]


class StepResult:
    __slots__ = ("obs", "reward", "done", "info", "obs2", "reward2", "info2", "actions", "final_obs", "record")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw.get(k))


class VecHockeyEnv:
    """Batched hockey arenas on one MI355X (one context per device and stream)."""

    def __init__(self, n_arenas, keep_mode=True, mode=Mode.NORMAL, device=None, policies=("external", "external"),
                 auto_reset=False, seed=0, vel_ref_semantics=False, arena_offset=0, diag_flags=0):
        if not torch.cuda.is_available():
            raise N.HockeyNativeError("VecHockeyEnv needs a ROCm GPU (gfx950); the hot path has no CPU fallback")
        self.L = N.lib()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.n = int(n_arenas)
        self.keep_mode = bool(keep_mode)
        self.mode = parse_mode(mode)
        self.auto_reset = bool(auto_reset)
        cfg = N.Config()
        cfg.keep_mode = int(self.keep_mode)
        cfg.mode = self.mode.value
        cfg.auto_reset = int(self.auto_reset)
        cfg.vel_ref_semantics = int(bool(vel_ref_semantics))
        cfg.policy[0] = _policy_id(policies[0])
        cfg.policy[1] = _policy_id(policies[1])
        cfg.seed = int(seed) & ((1 << 64) - 1)
        cfg.arena_offset = int(arena_offset)
        cfg.diag_flags = int(diag_flags)
        self.arena_offset = int(arena_offset)
        self.policies = [cfg.policy[0], cfg.policy[1]]
        ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            N.check(self.L.hk_create(self.device.index, self.n, ctypes.byref(cfg), ctypes.byref(ctx)), "hk_create")
        self._ctx = ctx
        self.one_starts = np.ones(self.n, bool)  # HockeyEnv.__init__ resets with one_starting=True
        self._alloc()

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        d, n = self.device, self.n
        self.obs_buf = torch.zeros((n, N.OBS_DIM), dtype=torch.float32, device=d)
        self.obs2_buf = torch.zeros((n, N.OBS_DIM), dtype=torch.float32, device=d)
        self.reward_buf = torch.zeros((n,), dtype=torch.float32, device=d)
        self.reward2_buf = torch.zeros((n,), dtype=torch.float32, device=d)
        self.done_buf = torch.zeros((n,), dtype=torch.uint8, device=d)
        self.info_buf = torch.zeros((n, N.INFO_DIM), dtype=torch.float32, device=d)
        self.info2_buf = torch.zeros((n, N.INFO_DIM), dtype=torch.float32, device=d)
        self.actions_buf = torch.zeros((n, N.ACT_DIM), dtype=torch.float32, device=d)
        self.final_obs_buf = torch.zeros((n, N.OBS_DIM), dtype=torch.float32, device=d)
        self.record_buf = torch.zeros((n, N.RECORD_DIM), dtype=torch.float64, device=d)

    def _stream(self):
        # torch's current stream on this device as a raw hipStream_t: the C accessor, without building a
        # torch.cuda.Stream object (the single-env facade reads it on every step)
        return ctypes.c_void_p(_raw_stream(self._dev_index))

    def close(self):
        if getattr(self, "_ctx", None):
            self.L.hk_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def set_policy(self, player, policy):
        pid = _policy_id(policy)
        N.check(self.L.hk_set_policy(self._ctx, int(player), pid), "hk_set_policy")
        self.policies[player] = pid

    # ------------------------------------------------------------------ reset
    def reset(self, seeds=None, mask=None, one_starting=None):
        """HockeyEnv.reset for the selected arenas.

        seeds: None -> device Philox placement; int / sequence -> the reference's PCG64 draws per arena
        (bit-identical placement to ``HockeyEnv.reset(seed=s)``).  one_starting: None toggles like the
        reference (NORMAL mode), a bool / bool array forces the puck side.
        Returns (obs[N,18], info[N,4]) tensors (agent-1 frame) for all arenas.
        """
        n = self.n
        sel = np.ones(n, bool) if mask is None else np.asarray(mask.cpu() if torch.is_tensor(mask) else mask, bool)
        if self.mode == Mode.NORMAL:
            if one_starting is None:
                self.one_starts = np.where(sel, ~self.one_starts, self.one_starts)
            else:
                self.one_starts = np.where(sel, np.broadcast_to(np.asarray(one_starting, bool), (n,)), self.one_starts)
        one_t = torch.as_tensor(self.one_starts.astype(np.uint8), device=self.device)
        mask_t = None if mask is None else torch.as_tensor(sel.astype(np.uint8), device=self.device)
        params_t = None
        if seeds is not None:
            seeds = np.broadcast_to(np.asarray(seeds, dtype=object), (n,))
            params = np.zeros((n, N.PARAM_DIM), np.float32)
            for i in np.nonzero(sel)[0]:
                rng, _ = np_random(None if seeds[i] is None else int(seeds[i]))
                params[i], _ = placement(self.mode, bool(self.one_starts[i]), rng)
            params_t = torch.as_tensor(params, device=self.device)
        N.check(self.L.hk_reset(self._ctx, N.ptr(mask_t), N.ptr(params_t), None, N.ptr(one_t), self._stream()),
                "hk_reset")
        return self.observe()

    def reset_params(self, params, mask=None, max_t=None):
        """Reset from explicit placement vectors [N,6] (float32 on device)."""
        mask_t = None if mask is None else torch.as_tensor(mask, dtype=torch.uint8, device=self.device)
        mt = None if max_t is None else torch.as_tensor(max_t, dtype=torch.int32, device=self.device)
        params = torch.as_tensor(params, dtype=torch.float32, device=self.device).contiguous()
        N.check(self.L.hk_reset(self._ctx, N.ptr(mask_t), N.ptr(params), N.ptr(mt), None, self._stream()), "hk_reset")

    # ------------------------------------------------------------------ step
    def step(self, actions=None, with_agent_two=False, opp_inc=None, debug=None, skip_physics=False,
             record_actions=False, final_obs=False, policy2=None, record=False):
        """HockeyEnv.step for every arena.  actions: [N,8] float (clipped in-kernel), may be None when no
        player is external.  Returns a StepResult of device tensors (views of persistent buffers).

        With auto_reset, an arena that is done after this step is reset at its end: done / reward / info are
        the terminal step's, obs / obs2 the new episode's first state, and ``final_obs`` (when requested) the
        terminal observation (== obs for arenas that did not reset).

        policy2 ([N] uint8 / policy ids, optional): player 2's policy of each arena for this step, overriding
        the context's (rl/training/opponent_manager.py draws the opponent per step); 'external' arenas read
        actions[:, 4:8].

        record: also return the [N,16] float64 step record (include/hockey.h hk_step_io.record: info, info2,
        reward, reward2 in float64 and has_puck1/2, time, done, winner after the step)."""
        a = None
        if actions is not None:
            a = torch.as_tensor(actions, dtype=torch.float32, device=self.device)
            if a.shape != (self.n, N.ACT_DIM):
                raise ValueError(f"actions must have shape ({self.n}, {N.ACT_DIM}), got {tuple(a.shape)}")
            a = a.contiguous()
        inc = None
        if opp_inc is not None:
            inc = torch.as_tensor(opp_inc, dtype=torch.float64, device=self.device).contiguous()
        io = N.StepIO()
        io.actions = None if a is None else a.data_ptr()
        io.opp_inc = None if inc is None else inc.data_ptr()
        io.obs = self.obs_buf.data_ptr()
        io.reward = self.reward_buf.data_ptr()
        io.done = self.done_buf.data_ptr()
        io.info = self.info_buf.data_ptr()
        if with_agent_two:
            io.obs2 = self.obs2_buf.data_ptr()
            io.reward2 = self.reward2_buf.data_ptr()
            io.info2 = self.info2_buf.data_ptr()
        if record_actions:
            io.actions_out = self.actions_buf.data_ptr()
        if debug is not None:
            io.debug = debug.data_ptr()
        if final_obs:
            io.final_obs = self.final_obs_buf.data_ptr()
        if record:
            io.record = self.record_buf.data_ptr()
        io.flags = N.STEP_SKIP_PHYSICS if skip_physics else 0
        p2 = None
        if policy2 is not None:
            p2 = torch.as_tensor(policy2, dtype=torch.uint8, device=self.device).contiguous()
            if p2.shape != (self.n,):
                raise ValueError(f"policy2 must have shape ({self.n},), got {tuple(p2.shape)}")
            io.policy2 = p2.data_ptr()
        N.check(self.L.hk_step(self._ctx, ctypes.byref(io), self._stream()), "hk_step")
        return StepResult(obs=self.obs_buf, reward=self.reward_buf, done=self.done_buf, info=self.info_buf,
                          obs2=self.obs2_buf if with_agent_two else None,
                          reward2=self.reward2_buf if with_agent_two else None,
                          info2=self.info2_buf if with_agent_two else None,
                          actions=self.actions_buf if record_actions else None,
                          final_obs=self.final_obs_buf if final_obs else None,
                          record=self.record_buf if record else None)

    def step_raw(self, io):
        """Launch one step with a prepared StepIO (no Python-side allocation; for benchmarks)."""
        N.check(self.L.hk_step(self._ctx, ctypes.byref(io), self._stream()), "hk_step")

    def rollout(self, n_steps, actions=None, with_agent_two=False, record_actions=False, final_obs=False):
        """``n_steps`` consecutive steps in one launch (hk_rollout).  Returns a StepResult whose tensors carry a
        leading [n_steps] dimension.  ``actions`` ([n_steps, N, 8]) is needed only for external players."""
        k, n = int(n_steps), self.n
        d = self.device
        a = None
        if actions is not None:
            a = torch.as_tensor(actions, dtype=torch.float32, device=d)
            if a.shape != (k, n, N.ACT_DIM):
                raise ValueError(f"actions must have shape ({k}, {n}, {N.ACT_DIM}), got {tuple(a.shape)}")
            a = a.contiguous()
        obs = torch.empty((k, n, N.OBS_DIM), dtype=torch.float32, device=d)
        rew = torch.empty((k, n), dtype=torch.float32, device=d)
        done = torch.empty((k, n), dtype=torch.uint8, device=d)
        info = torch.empty((k, n, N.INFO_DIM), dtype=torch.float32, device=d)
        io = N.StepIO()
        io.actions = None if a is None else a.data_ptr()
        io.obs, io.reward, io.done, io.info = obs.data_ptr(), rew.data_ptr(), done.data_ptr(), info.data_ptr()
        obs2 = rew2 = info2 = acts = None
        if with_agent_two:
            obs2 = torch.empty_like(obs)
            rew2 = torch.empty_like(rew)
            info2 = torch.empty_like(info)
            io.obs2, io.reward2, io.info2 = obs2.data_ptr(), rew2.data_ptr(), info2.data_ptr()
        if record_actions:
            acts = torch.empty((k, n, N.ACT_DIM), dtype=torch.float32, device=d)
            io.actions_out = acts.data_ptr()
        fobs = None
        if final_obs:
            fobs = torch.empty_like(obs)
            io.final_obs = fobs.data_ptr()
        N.check(self.L.hk_rollout(self._ctx, k, ctypes.byref(io), self._stream()), "hk_rollout")
        return StepResult(obs=obs, reward=rew, done=done, info=info, obs2=obs2, reward2=rew2, info2=info2,
                          actions=acts, final_obs=fobs)

    def rollout_raw(self, n_steps, io):
        """hk_rollout with a prepared StepIO whose arrays have a leading [n_steps] dimension."""
        N.check(self.L.hk_rollout(self._ctx, int(n_steps), ctypes.byref(io), self._stream()), "hk_rollout")

    # ------------------------------------------------------------------ state / obs
    def observe(self):
        N.check(self.L.hk_observe(self._ctx, N.ptr(self.obs_buf), N.ptr(self.obs2_buf), self._stream()), "hk_observe")
        return self.obs_buf, self.obs2_buf

    def info(self):
        """(info[N,4], info2[N,4], reward[N], reward2[N]) float64 of the current state (hk_info): _get_info,
        get_info_agent_two and the matching get_reward / get_reward_agent_two of hockey_env.py:518-591."""
        d, n = self.device, self.n
        i1 = torch.empty((n, N.INFO_DIM), dtype=torch.float64, device=d)
        i2 = torch.empty((n, N.INFO_DIM), dtype=torch.float64, device=d)
        r1 = torch.empty((n,), dtype=torch.float64, device=d)
        r2 = torch.empty((n,), dtype=torch.float64, device=d)
        N.check(self.L.hk_info(self._ctx, N.ptr(i1), N.ptr(i2), N.ptr(r1), N.ptr(r2), self._stream()), "hk_info")
        return i1, i2, r1, r2

    def obs_agent_two(self):
        return self.observe()[1]

    def get_state(self):
        st = torch.zeros((self.n, N.STATE_DIM), dtype=torch.float32, device=self.device)
        aux = torch.zeros((self.n, N.AUX_DIM), dtype=torch.int32, device=self.device)
        N.check(self.L.hk_get_state(self._ctx, N.ptr(st), N.ptr(aux), self._stream()), "hk_get_state")
        return st, aux

    def set_state(self, state=None, aux=None, mask=None):
        st = None if state is None else torch.as_tensor(state, dtype=torch.float32, device=self.device).contiguous()
        ax = None if aux is None else torch.as_tensor(aux, dtype=torch.int32, device=self.device).contiguous()
        mk = None if mask is None else torch.as_tensor(mask, dtype=torch.uint8, device=self.device).contiguous()
        N.check(self.L.hk_set_state(self._ctx, N.ptr(mk), N.ptr(st), N.ptr(ax), self._stream()), "hk_set_state")

    def opponent_phase(self, new_phase=None, rows=2):
        """Return the BasicOpponent phases [N,rows] (float64, device); optionally overwrite them.  rows=2:
        player 1 / player 2 (hk_opponent_phase); rows=3 adds player 2's weak bot under a policy2 override
        (hk_opponent_phase3, include/hockey.h states which step walks which row)."""
        if rows not in (2, 3):
            raise ValueError("rows must be 2 or 3")
        out = torch.zeros((self.n, rows), dtype=torch.float64, device=self.device)
        ph = None if new_phase is None else torch.as_tensor(new_phase, dtype=torch.float64,
                                                            device=self.device).contiguous()
        if ph is not None and ph.shape != (self.n, rows):
            raise ValueError(f"new_phase must have shape ({self.n}, {rows})")
        fn = self.L.hk_opponent_phase if rows == 2 else self.L.hk_opponent_phase3
        N.check(fn(self._ctx, N.ptr(out), N.ptr(ph), self._stream()), "hk_opponent_phase")
        return out

    def counters(self):
        out = (ctypes.c_int64 * N.NUM_COUNTERS)()
        N.check(self.L.hk_counters(self._ctx, out, self._stream()), "hk_counters")
        return np.array(out[:], np.int64)

    def reset_counters(self):
        N.check(self.L.hk_reset_counters(self._ctx, self._stream()), "hk_reset_counters")

    def bytes_per_step(self):
        a, b = ctypes.c_int64(), ctypes.c_int64()
        N.check(self.L.hk_bytes_per_step(self._ctx, ctypes.byref(a), ctypes.byref(b)), "hk_bytes_per_step")
        return a.value, b.value
