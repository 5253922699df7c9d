"""GPU-resident TD3 over batched arenas (BASELINE config C5).

Mirrors the reference's learner, acting and collection semantics on device tensors end to end:

* config: ``TD3Config`` carries the fields of rl/td3/config.py with the reference's defaults;
  ``TD3Config.from_json`` reads a run's ``config.json`` (e.g. pretrained/stage_1/config/config.json);
* networks: rl/td3/networks.py -- actor 18-256-256-4 (tanh, tanh); twin Q critics 22-256-256-1 (tanh
  hidden, identity out) fed with the action unscaled to [-1, 1]; state-dict names match the reference's
  td3_*.pt checkpoints, so ``TD3.checkpoint()`` and ``evaluate.load_actor`` interoperate with them;
* update: rl/td3/learner.py:55-218 -- target policy smoothing N(0, 0.2) clipped to +-0.3, clipped double Q,
  weighted smooth-L1 critic loss (rl/utils/torch_utils.py:12-24; importance weights under prioritized
  replay), delayed actor update every ``policy_update_freq`` critic updates with -Q1 as the actor loss, Polyak
  averaging rho = 1 - tau; Adam(lr, eps 1e-6, weight decay wd) for both (rl/td3/agent.py:174-182);
* replay: rl/replay/uniform_buffer.py (``ReplayRing``) and rl/replay/prioritized_buffer.py:6-69
  (``PrioritizedRing``), both device-resident;
* acting: rl/td3/agent.py:198-264 -- uniform random actions while the agent's step count is below
  ``start_steps``, then actor + exploration noise of the configured kind (``hockey_amd.noise``: Gaussian, OU,
  pink, uniform; rl/common/noise.py) scaled by the annealed / constant noise scale, clamped to [-1, 1];
* collection: rl/training/train.py:135-207 -- an episode is ``max_steps`` environment steps WITHOUT
  breaking on done (the env's done is sticky, so post-goal steps repeat the terminal reward), every
  transition is stored with ``done``, and learner updates follow at the reference's replay ratio.

Learner updates are launch-bound at the reference's batch of 256 (a few dozen small kernels each), so a pair
of updates (critic-only, then critic + delayed actor + Polyak) is captured once as a HIP graph and replayed
(``Learner``); the first pairs run eagerly on a side stream to initialise the optimiser state, as graph
capture requires.  Results are the same updates, just launched as one graph.

Batched differences (by design): N episodes run side by side (one arena each) and enter one device ring; the
updates of those N episodes run after the round (the reference runs ``train_iters`` after each episode), at
the reference's replay ratio (samples drawn per stored transition, ``train_iters * batch_size / max_steps``
= 16.4 for the reference) -- so a larger batch means proportionally fewer updates; see
``hockey_amd.opponents`` for the opponent draws.
"""
import json
import math
from dataclasses import dataclass, fields

import torch

from .constants import Mode
from .evaluate import Actor, reset_params
from .noise import make_noise


class _QNet(torch.nn.Module):
    """ActorNetwork shape with identity output (the reference builds its critics from ActorNetwork)."""

    def __init__(self, n_in, h=256):
        super().__init__()
        self.fc1 = torch.nn.Linear(n_in, h)
        self.fc2 = torch.nn.Linear(h, h)
        self.fc3 = torch.nn.Linear(h, 1)

    def forward(self, x):
        x = torch.tanh(self.fc1(x))
        x = torch.tanh(self.fc2(x))
        return self.fc3(x).squeeze(-1)


class TwinQ(torch.nn.Module):
    """rl/td3/networks.py TwinQNetwork; parameter / buffer names match the reference checkpoints."""

    def __init__(self, n_obs=18, n_act=4, h=256):
        super().__init__()
        self.register_buffer("action_low", -torch.ones(n_act))
        self.register_buffer("action_high", torch.ones(n_act))
        self.register_buffer("action_range", self.action_high - self.action_low)
        self.q1 = _QNet(n_obs + n_act, h)
        self.q2 = _QNet(n_obs + n_act, h)

    def _input(self, state, action):
        action = ((action - self.action_low) / self.action_range) * 2 - 1.0  # TwinQNetwork._unscale_action
        return torch.cat([state, action], dim=-1)

    def forward(self, state, action):
        x = self._input(state, action)
        return self.q1(x), self.q2(x)

    def q1_only(self, state, action):
        """The first head alone: the actor update uses only q1 (learner.py update_actor), the same values as
        forward()[0] without the second head's forward."""
        return self.q1(self._input(state, action))


def smooth_l1(x, y, weights=None):
    """rl/utils/torch_utils.py weighted_smooth_l1_loss (unit weights when ``weights`` is None)."""
    diff = x - y
    if weights is None:
        return torch.where(diff.abs() < 1, 0.5 * diff ** 2, diff.abs() - 0.5).mean()
    return torch.where(diff.abs() < 1, 0.5 * weights * diff ** 2, (diff.abs() - 0.5) * weights).mean()


@dataclass
class TD3Config:  # rl/td3/config.py (same fields and defaults)
    max_steps: int = 500
    train_iters: int = 32
    eval_interval: int = 200
    eval_episodes: int = 100
    gamma: float = 0.99
    tau_actor: float = 0.005
    tau_critic: float = 0.005
    policy_update_freq: int = 2
    lr_q: float = 4e-4
    lr_pol: float = 4e-4
    wd_q: float = 0.0
    wd_pol: float = 0.0
    prioritized_replay: bool = False
    beta: float = 0.15
    buffer_size: int = 300_000
    batch_size: int = 256
    start_steps: int = 2000
    action_noise_scale: float = 0.2
    target_action_noise_scale: float = 0.2
    target_action_noise_clip: float = 0.3
    noise_mode: str = "gaussian"
    use_noise_annealing: bool = True
    noise_anneal_mode: str = "linear"
    noise_min_scale: float = 0.07
    early_stopping: bool = False
    early_patience: int = 15
    early_min_delta: float = 0.01
    use_self_play: bool = True
    self_play_interval: int = 250
    self_play_pool_size: int = 12
    curriculum_name: str = "ablation"

    @classmethod
    def from_json(cls, path, **overrides):
        """A run's saved config.json (rl/experiment/tracking.py writes it); unknown keys are ignored."""
        with open(path) as f:
            d = json.load(f)
        names = {f.name for f in fields(cls)}
        kw = {k: v for k, v in d.items() if k in names}
        kw.update(overrides)
        return cls(**kw)

    @property
    def replay_ratio(self):
        """Samples the learner draws per stored transition: train_iters updates of batch_size per max_steps
        transitions (rl/training/train.py:145-207) -- 16.4 for the reference's 32 x 256 / 500."""
        return self.train_iters * self.batch_size / self.max_steps


class ReplayRing:
    """Device-resident FIFO replay buffer with uniform sampling (rl/replay/uniform_buffer.py: indices
    ``(rand(batch) * size).astype(int)``).  The fill level lives on the device too, so sampling can sit inside
    a captured HIP graph while the ring fills."""

    prioritized = False

    def __init__(self, capacity, n_obs=18, n_act=4, device="cuda:0"):
        self.cap, self.size, self.pos = int(capacity), 0, 0
        d = self.device = torch.device(device)
        self.s = torch.zeros((self.cap, n_obs), device=d)
        self.a = torch.zeros((self.cap, n_act), device=d)
        self.r = torch.zeros(self.cap, device=d)
        self.s2 = torch.zeros((self.cap, n_obs), device=d)
        self.d = torch.zeros(self.cap, device=d)
        self.size_t = torch.zeros((), dtype=torch.int64, device=d)  # fill level, exact at any capacity

    def _slots(self, n):
        """Ring slots of the next n pushes, as one or two contiguous ranges."""
        p = self.pos
        if p + n <= self.cap:
            return [(p, p + n, 0)]
        k = self.cap - p
        return [(p, self.cap, 0), (0, n - k, k)]

    def push(self, s, a, r, s2, d):
        n = s.shape[0]
        if n > self.cap:
            raise ValueError(f"push of {n} transitions exceeds the ring capacity {self.cap}")
        self._before_push(n)
        for lo, hi, off in self._slots(n):
            m = hi - lo
            self.s[lo:hi] = s[off:off + m]
            self.a[lo:hi] = a[off:off + m]
            self.r[lo:hi] = r[off:off + m].float()
            self.s2[lo:hi] = s2[off:off + m]
            self.d[lo:hi] = d[off:off + m].float()
        self.pos = (self.pos + n) % self.cap
        self.size = min(self.size + n, self.cap)
        self.size_t.fill_(self.size)

    def _before_push(self, n):
        pass

    def sample_indices(self, batch):
        # float64 uniforms: float32's 24-bit mantissa cannot reach every slot of a ring past 2^24 transitions
        # (C5 fills 32.8 M) and skews the draw well below that; the reference draws in float64 too
        u = torch.rand(batch, device=self.device, dtype=torch.float64)
        return torch.minimum((u * self.size_t).long(), self.size_t - 1)

    def sample(self, batch):
        """(s, a, r, s2, d, importance weights or None)."""
        i = self.sample_indices(batch)
        return self.s[i], self.a[i], self.r[i], self.s2[i], self.d[i], None

    def update_priorities(self, td):
        pass

    def __len__(self):
        return self.size


class PrioritizedRing(ReplayRing):
    """rl/replay/prioritized_buffer.py:6-69 on the device.

    * every slot starts at ``init_weight`` (1e8); a pushed transition gets the maximum weight over the filled
      slots, the slot's own previous weight included (the reference assigns after its size increment), so
      unseen data is drawn first;
    * sampling draws ``batch`` indices with replacement, P(i) = w_i / sum(w) over the filled slots (NaN / inf
      weights -> 0, floor 1e-6), by inverse CDF like ``np.random.choice``;
    * importance weights (learner.py:199-210): p_b = w[inds] / sum(w[inds]) over the BATCH,
      (1 / (p_b * size)) ** beta, divided by their maximum;
    * after the critic step the sampled slots' weights become clamp(|td|, 1e-6, 1e6) with td the mean of the
      two critics' absolute TD errors (learner.py:163-176)."""

    prioritized = True

    def __init__(self, capacity, n_obs=18, n_act=4, device="cuda:0", beta=0.15, init_weight=1e8):
        super().__init__(capacity, n_obs, n_act, device)
        self.beta = float(beta)
        self.w = torch.full((self.cap,), float(init_weight), device=self.device)
        self.last = torch.zeros(1, dtype=torch.long, device=self.device)
        self._slot = torch.arange(self.cap, device=self.device)

    def _before_push(self, n):
        # pushed one by one, slot k would get max(w[:size_k]); while the ring fills the fresh slot itself holds
        # init_weight, and once it is full size_k == cap: either way every slot of the push gets the maximum
        # over the slots filled after it (old weights, before the push writes them)
        wmax = self.w[:min(self.size + n, self.cap)].max()
        for lo, hi, _ in self._slots(n):
            self.w[lo:hi] = wmax

    def sample_indices(self, batch):
        valid = self._slot < self.size_t
        w = torch.nan_to_num(self.w, nan=0.0, posinf=0.0, neginf=0.0).clamp_min(1e-6) * valid
        cdf = torch.cumsum(w.double(), 0)
        u = torch.rand(batch, device=self.device, dtype=torch.float64) * cdf[-1]
        i = torch.searchsorted(cdf, u, right=True).clamp_max(self.cap - 1)
        self.last = i
        return i

    def sample(self, batch):
        i = self.sample_indices(batch)
        wb = self.w[i]
        p = wb / wb.sum()
        iw = (1.0 / (p * self.size_t)) ** self.beta
        iw = iw / iw.max()
        return self.s[i], self.a[i], self.r[i], self.s2[i], self.d[i], iw

    def update_priorities(self, td):
        """w[last] = clamp(td) with numpy's semantics for a slot drawn more than once in the batch: the LAST
        occurrence wins (prioritized_buffer.py update_priorities).  A plain device index_put leaves the winner to
        the scheduler, so every duplicate writes its group's last value instead (sort by (slot, position), the
        group end by a reversed running minimum): deterministic, graph-capturable, no host sync."""
        i = self.last
        b = i.numel()
        ar = torch.arange(b, device=i.device)
        key, perm = torch.sort(i * b + ar)
        slot = key // b
        is_last = torch.ones(b, dtype=torch.bool, device=i.device)
        is_last[:-1] = slot[1:] != slot[:-1]
        end = torch.where(is_last, ar, torch.full_like(ar, b))
        end = torch.flip(torch.cummin(torch.flip(end, [0]), 0).values, [0])
        self.w[slot] = torch.clamp(td.detach()[perm[end]], 1e-6, 1e6)


class TD3:
    def __init__(self, cfg=None, device="cuda:0", seed=0, max_total_steps=None, n_envs=1, noise_seed=None, h=256):
        self.cfg = cfg or TD3Config()
        self.device = torch.device(device)
        self.seed = seed
        torch.manual_seed(seed)
        self.actor, self.critic = Actor(h=h).to(self.device), TwinQ(h=h).to(self.device)
        self.target_actor, self.target_critic = Actor(h=h).to(self.device), TwinQ(h=h).to(self.device)
        self.target_actor.load_state_dict(self.actor.state_dict())
        self.target_critic.load_state_dict(self.critic.state_dict())
        for net in (self.target_actor, self.target_critic):
            for p in net.parameters():
                p.requires_grad_(False)
        cap = self.device.type == "cuda"
        self.opt_actor = torch.optim.Adam(self.actor.parameters(), lr=self.cfg.lr_pol, eps=1e-6,
                                          weight_decay=self.cfg.wd_pol, capturable=cap)
        self.opt_critic = torch.optim.Adam(self.critic.parameters(), lr=self.cfg.lr_q, eps=1e-6,
                                           weight_decay=self.cfg.wd_q, capturable=cap)
        self.train_step = 0
        self.total_steps = 0  # agent.get_action calls with eval_mode False (rl/td3/agent.py:198-203)
        self.max_total_steps = max_total_steps
        self.initial_noise_scale = self.current_noise_scale = self.cfg.action_noise_scale
        self.noise = make_noise(self.cfg.noise_mode, n_envs, 4, self.cfg.action_noise_scale, self.cfg.max_steps,
                                self.device, seed if noise_seed is None else noise_seed)

    # ---------------------------------------------------------------- learner (rl/td3/learner.py)
    def compute_target(self, s2, r, d):
        c = self.cfg
        with torch.no_grad():
            ta = self.target_actor(s2)
            raw = getattr(self, "_noise_override", None)  # tests: the reference's own N(0, scale) draw
            if raw is None:
                raw = torch.randn_like(ta) * c.target_action_noise_scale
            noise = torch.clamp(raw, -c.target_action_noise_clip, c.target_action_noise_clip)
            ta = torch.clamp(ta + noise, -1.0, 1.0)
            q1, q2 = self.target_critic(s2, ta)
            return r + c.gamma * (1 - d) * torch.minimum(q1, q2)

    def soft_update(self):
        with torch.no_grad():
            for tgt, src, tau in ((self.target_actor, self.actor, self.cfg.tau_actor),
                                  (self.target_critic, self.critic, self.cfg.tau_critic)):
                tp, sp = list(tgt.parameters()), list(src.parameters())
                torch._foreach_mul_(tp, 1.0 - tau)
                torch._foreach_add_(tp, sp, alpha=tau)

    def _no_fused(self, what):
        # a FusedLearner (hockey_amd.learner_hip) owns this agent's optimiser state and MFMA operand packs from the
        # moment it is attached: an eager update would split the Adam moments, and weights loaded afterwards would
        # not reach the packs -- fail loudly instead of training on stale state
        if getattr(self, "_fused_learner", None) is not None:
            raise RuntimeError(f"TD3.{what}: a fused learner is attached to this agent; update through it "
                               "(Learner(..., fused=True)) or build a new agent")

    def _update_tensors(self, s, a, r, s2, d, iw=None, ring=None, train_actor=None):
        """One learner.update on a sampled batch; returns (actor loss or None, critic loss) as 0-d tensors."""
        self._no_fused("update")
        if train_actor is None:
            self.train_step += 1
            train_actor = self.train_step % self.cfg.policy_update_freq == 0
        target = self.compute_target(s2, r, d)
        self.opt_critic.zero_grad(set_to_none=True)
        q1, q2 = self.critic(s, a)
        critic_loss = (smooth_l1(q1, target, iw) + smooth_l1(q2, target, iw)) * 0.5
        critic_loss.backward()
        self.opt_critic.step()
        if ring is not None and ring.prioritized:
            ring.update_priorities(((q1 - target).abs() + (q2 - target).abs()).detach() / 2)
        actor_loss = None
        if train_actor:
            self.opt_actor.zero_grad(set_to_none=True)
            q = self.critic.q1_only(s, self.actor(s))
            actor_loss = -q.mean()
            actor_loss.backward(inputs=list(self.actor.parameters()))  # the actor's gradients only
            self.opt_actor.step()
            self.soft_update()
        return (None if actor_loss is None else actor_loss.detach()), critic_loss.detach()

    def update(self, s, a, r, s2, d, iw=None):
        """One eager learner update (learner.py:55-72) on the given batch."""
        return self._update_tensors(s, a, r, s2, d, iw)

    # ---------------------------------------------------------------- acting (rl/td3/agent.py)
    def noise_scale(self):
        """_update_noise_scale (agent.py:247-264)."""
        c = self.cfg
        if not c.use_noise_annealing:
            return self.initial_noise_scale
        if self.max_total_steps is None:
            return self.current_noise_scale
        progress = min(self.total_steps / self.max_total_steps, 1.0)
        if c.noise_anneal_mode == "linear":
            scale = self.initial_noise_scale * (1 - progress)
        elif c.noise_anneal_mode == "exp":
            scale = self.initial_noise_scale * (0.1 ** progress)
        else:
            raise ValueError("Unknown anneal mode")
        return max(scale, c.noise_min_scale)

    def act(self, obs, noise=True, count=None):
        """get_action for a batch of arenas (one call per arena, in arena order): the agent's step count
        advances by N (or ``count``: the arenas whose episode is still running); arena i's action is uniform
        random while its step index is below start_steps, else actor + exploration noise (noise=False:
        eval_mode, no count, no noise)."""
        n = obs.shape[0]
        if not noise:
            with torch.no_grad():
                return self.actor(obs)
        first = self.total_steps + 1  # arena 0's total_steps after its increment
        self.total_steps += n if count is None else int(count)
        c = self.cfg
        if self.total_steps < c.start_steps:  # every arena of the batch is in the random phase
            return torch.rand((n, 4), device=obs.device) * 2 - 1
        with torch.no_grad():
            a = self.actor(obs)
        self.current_noise_scale = self.noise_scale()
        a = torch.clamp(a + self.noise() * (self.current_noise_scale / self.initial_noise_scale), -1, 1)
        if first < c.start_steps:  # the batch straddles the end of the random phase
            rnd = (torch.arange(n, device=obs.device) + first) < c.start_steps
            a = torch.where(rnd[:, None], torch.rand((n, 4), device=obs.device) * 2 - 1, a)
        return a

    def reset_noise(self):
        """agent.reset() at an episode start: OU state back to x0, a fresh pink block."""
        self.noise.reset()

    def checkpoint(self):
        """The reference's td3_*.pt layout (policy / critic / target_policy / target_critic); tensors are copies (the
        fused learner keeps the parameters as views of one flat buffer per network)."""
        def sd(m):
            return {k: v.detach().clone() for k, v in m.state_dict().items()}
        return {"policy": sd(self.actor), "critic": sd(self.critic), "target_policy": sd(self.target_actor),
                "target_critic": sd(self.target_critic)}

    def load(self, ck):
        """agent.load (rl/td3/agent.py:278-286): all four networks from a td3_*.pt dict (or a path, read
        weights-only); the optimiser state is left as it is (the reference's resume starts fresh Adam moments).
        Call before a fused Learner is attached: it packs its operands from these weights when built."""
        self._no_fused("load")
        if isinstance(ck, (str, bytes)) or hasattr(ck, "__fspath__"):
            ck = load_checkpoint(ck)
        with torch.no_grad():
            for key, net in (("policy", self.actor), ("critic", self.critic), ("target_policy", self.target_actor),
                             ("target_critic", self.target_critic)):
                net.load_state_dict({k: torch.as_tensor(v) for k, v in ck[key].items()})


def load_checkpoint(path):
    """A td3_*.pt (``torch.load(weights_only=True)``) or the ``<net>/<param>`` npz fixture of one
    (tests/golden/extract_resume_checkpoint.py) as the reference's {policy, critic, target_policy, target_critic}
    dict of CPU tensors."""
    import os
    path = os.fsdecode(os.fspath(path))
    if path.endswith(".npz"):
        import numpy as np
        z = np.load(path)
        out = {}
        for key in z.files:
            if "/" in key:
                net, name = key.split("/", 1)
                out.setdefault(net, {})[name] = torch.from_numpy(z[key])
        return out
    return torch.load(path, map_location="cpu", weights_only=True)


FUSED_MIN_BATCH = 256  # fused="auto": the MFMA learner for batches of 256 and up (its chunk granularity): 0.32 ms
# per update at the reference's batch 256 against 1.44 ms for the graph-captured PyTorch pair, 0.39 ms at C5's 16 384
# (profiles/r04/learner_profile*.log)


def fused_available():
    """True when the fused learner library is built (hockey_amd/_lib/libhockey_learner.so)."""
    from .learner_hip import LIB_PATH
    import os
    return os.path.exists(LIB_PATH)


class Learner:
    """Runs ``k`` learner updates (sample + learner.update) of ``agent`` on ``ring``.

    With ``graphs`` on a GPU the pair (critic update; critic + delayed actor + Polyak) is captured once as a HIP
    graph after ``warm_pairs`` eager pairs and replayed: the same updates, launched as one graph instead of a few
    hundred kernel launches.  Losses accumulate on the device (no host sync per update).

    fused: True runs every update through the fused fp32 MFMA kernels (hockey_amd.learner_hip: a handful of HIP
    kernels per update; batches that are multiples of 256, GPU only, fails loudly without the library); False
    through PyTorch ops; "auto" (default) picks fused for GPU batches of at least FUSED_MIN_BATCH (multiples of 256)
    at hidden width 256 when the library is built.  fused_rng: "device" (the batch's slots and target noise from the
    fused learner's Philox stream, one kernel) or "torch" (torch's generator, in the eager learner's order)."""

    def __init__(self, agent, ring, batch, graphs=True, warm_pairs=3, fused="auto", fused_rng="device"):
        self.agent, self.ring, self.batch = agent, ring, int(batch)
        self.use_graph = bool(graphs) and agent.device.type == "cuda" and agent.cfg.policy_update_freq == 2
        self.warm_left = int(warm_pairs)
        self.graph = None
        self.acc = torch.zeros(4, dtype=torch.float64, device=agent.device)  # sum critic, sum actor, n c, n a
        if fused == "auto":
            fused = (agent.device.type == "cuda" and self.batch >= FUSED_MIN_BATCH and self.batch % 256 == 0 and
                     agent.actor.fc1.out_features == 256 and fused_available())
        self.fused = None
        if fused:
            from .learner_hip import FusedLearner
            self.fused = FusedLearner(agent, ring, self.batch, rng=fused_rng)
            self.fused.set_loss_accumulator(self.acc)

    def _one(self, train_actor=None):
        if self.fused is not None:
            if train_actor is None:
                self.agent.train_step += 1
                train_actor = self.agent.train_step % self.agent.cfg.policy_update_freq == 0
            self.fused.update(train_actor)
            return
        s, a, r, s2, d, iw = self.ring.sample(self.batch)
        al, cl = self.agent._update_tensors(s, a, r, s2, d, iw, self.ring, train_actor)
        self.acc[0] += cl
        self.acc[2] += 1
        if al is not None:
            self.acc[1] += al
            self.acc[3] += 1

    def _pair(self):
        self._one(False)
        self._one(True)

    def run(self, k):
        ag = self.agent
        k = int(k)
        if not self.use_graph or ag.train_step % 2:
            for _ in range(k):
                self._one()
            return
        pairs, rest = divmod(k, 2)
        for _ in range(pairs):
            if self.graph is not None:
                self.graph.replay()
            elif self.warm_left > 0:  # eager warm-up pairs on a side stream (graph capture prerequisite)
                st = torch.cuda.Stream(ag.device)
                st.wait_stream(torch.cuda.current_stream(ag.device))
                with torch.cuda.stream(st):
                    self._pair()
                torch.cuda.current_stream(ag.device).wait_stream(st)
                self.warm_left -= 1
            else:
                self.graph = torch.cuda.CUDAGraph()
                ag.opt_critic.zero_grad(set_to_none=True)
                ag.opt_actor.zero_grad(set_to_none=True)
                with torch.cuda.graph(self.graph):
                    self._pair()
                self.graph.replay()  # capture records without running: this replay is the pair's update
            ag.train_step += 2
        for _ in range(rest):
            self._one()

    def take_losses(self):
        """Mean critic / actor loss since the last call (one host sync)."""
        s = self.acc.cpu().tolist()
        self.acc.zero_()
        return (s[0] / s[2] if s[2] else None), (s[1] / s[3] if s[3] else None)


def train(n_arenas=1024, rounds=10, cfg=None, device="cuda:0", seed=0, updates_per_round=None, mode=Mode.NORMAL,
          curriculum=None, use_self_play=None, self_play_interval=None, pool_size=None, reset="seeded", log=None,
          replay_capacity=None, graphs=True, eval_fn=None, learner_batch=None, timing=False, replay_ratio=None,
          env=None, on_step=None, episode_end="max_steps", fused="auto", resume_from=None):
    """Batched TD3 training (rl/training/train.py TD3Trainer.train).  Each round runs ``max_steps`` steps of
    ``n_arenas`` parallel episodes (no break on done), stores every transition, then performs the learner
    updates of those episodes at the replay ratio: ``ratio * n_arenas * max_steps / B`` updates of batch B =
    ``learner_batch`` (default ``cfg.batch_size``), ratio = ``replay_ratio`` (default ``cfg.replay_ratio``:
    ``train_iters`` per episode at the config's batch), unless ``updates_per_round`` overrides it.  Player 2 follows the curriculum's opponent mix (``hockey_amd.opponents.OpponentMix``),
    re-drawn per arena and step.

    Replay capacity: ``cfg.buffer_size``, raised to one full round of every arena (``n_arenas * max_steps``)
    when that is larger, so sampled data always spans whole episodes (65 536 arenas x 500 steps = 5.5 GB of
    HBM at C5).  reset: "seeded" places episode e (1-based, arena i of round k: e = k*N + i + 1) like
    ``reset(seed=seed + e)`` (the reference's PCG64 stream, drawn on the host: ~0.5 s per round at 65 536
    arenas); "device" uses the kernel's Philox placement (same distribution, no host work).
    eval_fn(agent, episodes_done) is called every ``cfg.eval_interval`` episodes.  timing: synchronise around each
    round's collection and updates and record their wall seconds in ``stats["round_time"]``.  Returns
    (agent, stats).  fused: the learner path (Learner).  env: a VecHockeyEnv-shaped batch of n_arenas arenas to train on (default: a new
    VecHockeyEnv on ``device``; the CPU tests pass the kernel source's host build).  on_step(obs, action,
    reward, next_obs, done, step_result) sees every stored transition (test hook).

    episode_end: "max_steps" -- the reference's current loop (rl/training/train.py:145-169): every episode runs
    max_steps steps without a break on done, every transition is stored, and the sticky done repeats the
    terminal +-10 on every post-goal step.  "done" -- an episode ends at its done step (later steps of that
    arena are neither stored nor counted): the semantics the reference's recorded runs were produced with --
    over the 47 000 episodes of pretrained/stage_{1,2,3}/metrics/metrics.json the return never exceeds 10.0,
    the +10 of a single goal, which the no-break loop (+10 per post-goal step) cannot produce.  A round ends
    when every arena's episode has ended.

    resume_from: a td3_*.pt path, its npz fixture or a checkpoint dict: rl/main.py:66-67 ``agent.load(resume_from)``
    before training (all four networks; fresh optimisers, noise schedule and replay)."""
    import time
    from .opponents import OpponentMix
    from .vec_env import VecHockeyEnv

    cfg = cfg or TD3Config()
    curriculum = cfg.curriculum_name if curriculum is None else curriculum
    use_self_play = cfg.use_self_play if use_self_play is None else use_self_play
    self_play_interval = cfg.self_play_interval if self_play_interval is None else self_play_interval
    pool_size = cfg.self_play_pool_size if pool_size is None else pool_size
    planned = rounds * cfg.max_steps * n_arenas
    agent = TD3(cfg, device, seed, max_total_steps=planned, n_envs=n_arenas)
    if resume_from is not None:
        agent.load(resume_from)
    own_env = env is None
    if own_env:
        env = VecHockeyEnv(n_arenas, mode=mode, device=device, policies=("external", "external"), auto_reset=False,
                           seed=seed)
    mix = OpponentMix(n_arenas, curriculum, use_self_play, self_play_interval, pool_size, device, seed)
    cap = replay_capacity or max(cfg.buffer_size, n_arenas * cfg.max_steps)
    ring = (PrioritizedRing(cap, device=device, beta=cfg.beta) if cfg.prioritized_replay
            else ReplayRing(cap, device=device))
    batch = int(learner_batch or cfg.batch_size)
    learner = Learner(agent, ring, batch, graphs=graphs, fused=fused)
    updates = updates_per_round if updates_per_round is not None else \
        updates_for(cfg, n_arenas, cfg.max_steps, batch, replay_ratio)
    act8 = torch.zeros((n_arenas, 8), device=device)
    stats = {"env_steps": 0, "updates": 0, "updates_per_round": updates, "batch": batch,
             "replay_ratio": updates * batch / (n_arenas * cfg.max_steps),
             "replay_capacity": cap, "critic_loss": [], "actor_loss": [], "mean_reward": [], "opponents": [],
             "pool_size": [], "evals": [], "round_time": []}
    episodes = 0
    next_eval = cfg.eval_interval
    if episode_end not in ("max_steps", "done"):
        raise ValueError("episode_end must be 'max_steps' or 'done'")
    stop_at_done = episode_end == "done"
    sync = (lambda: torch.cuda.synchronize(device)) if timing else (lambda: None)
    for rnd in range(rounds):
        sync()
        t0 = time.perf_counter()
        mix.update_schedule((episodes + 1) / (rounds * n_arenas))  # update_schedule(ep, max_episodes)
        if reset == "device":
            obs, obs2 = (t.clone() for t in env.reset())
        else:
            # episode e = rnd * N + i + 1 is the train env's e-th reset: seed + e, puck side toggling per reset
            p, _, _ = reset_params(n_arenas, seed + rnd * n_arenas + 1, mode, first_reset=rnd * n_arenas)
            env.reset_params(p)
            obs, obs2 = (t.clone() for t in env.observe())
        agent.reset_noise()
        ep_reward = torch.zeros(n_arenas, device=device)
        alive = torch.ones(n_arenas, dtype=torch.bool, device=device)  # episode_end="done": not yet done
        n_alive, round_steps = n_arenas, 0
        for _ in range(cfg.max_steps):
            a = agent.act(obs, count=n_alive)
            policy2, a2, _ = mix.select(obs2)
            act8[:, :4] = a
            if a2 is not None:
                act8[:, 4:] = a2
            res = env.step(act8, with_agent_two=True, policy2=policy2)
            o2, r, d = res.obs.clone(), res.reward.clone(), res.done.clone()
            round_steps += n_alive
            if stop_at_done:  # only the transitions of episodes that were still running are stored
                idx = torch.nonzero(alive).squeeze(1)
                ring.push(obs[idx], a[idx], r[idx], o2[idx], d[idx])
                if on_step is not None:
                    on_step(obs[idx], a[idx], r[idx], o2[idx], d[idx], res)
                mix.register_outcomes(d & alive, r)
                ep_reward += torch.where(alive, r, torch.zeros_like(r))
                alive &= d == 0
                n_alive = int(alive.sum())
                if n_alive == 0:
                    break
            else:
                ring.push(obs, a, r, o2, d)
                if on_step is not None:
                    on_step(obs, a, r, o2, d, res)
                mix.register_outcomes(d, r)
                ep_reward += r
            obs, obs2 = o2, res.obs2.clone()
        episodes += n_arenas
        stats["env_steps"] += round_steps
        stats["mean_reward"].append(float(ep_reward.mean().item()))
        stats["opponents"].append(mix.end_round(agent.actor, episodes=n_arenas))
        stats["pool_size"].append(len(mix.pool) if mix.pool is not None else 0)
        sync()
        t1 = time.perf_counter()
        if agent.total_steps > batch:  # _train_agent's guard (train.py:177-185)
            learner.run(updates)
            stats["updates"] += updates
            cl, al = learner.take_losses()
            stats["critic_loss"].append(cl)
            if al is not None:
                stats["actor_loss"].append(al)
        sync()
        if timing:
            stats["round_time"].append((t1 - t0, time.perf_counter() - t1))
        if eval_fn is not None and episodes >= next_eval:
            stats["evals"].append(eval_fn(agent, episodes))
            next_eval = (episodes // cfg.eval_interval + 1) * cfg.eval_interval
        if log:
            log(rnd, stats)
    if own_env:
        env.close()
    stats["replay_size"] = len(ring)
    stats["train_step"] = agent.train_step
    return agent, stats


REFERENCE_REPLAY_RATIO = 32 * 256 / 500  # train_iters x batch_size per max_steps-step episode (config.py defaults)


def updates_for(cfg, n_arenas, steps, batch=None, ratio=None):
    """Learner updates that follow ``steps`` collection steps of ``n_arenas`` at ``ratio`` samples per stored
    transition (default ``cfg.replay_ratio``; rounds shorter than an episode pass the reference's
    ``REFERENCE_REPLAY_RATIO``), drawn as batches of ``batch`` (default ``cfg.batch_size``): the reference's 32
    updates per 500-step episode at batch 256, proportionally fewer updates of a larger batch."""
    b = int(batch or cfg.batch_size)
    r = cfg.replay_ratio if ratio is None else float(ratio)
    return max(1, int(math.floor(r * n_arenas * steps / b + 0.5)))
