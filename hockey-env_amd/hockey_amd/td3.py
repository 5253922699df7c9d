"""GPU-resident TD3 over batched arenas (BASELINE config C5).

Mirrors the reference's learner and collection semantics on device tensors end to end:

* networks: rl/td3/networks.py -- actor 18-256-256-4 (tanh, tanh); twin Q critics 22-256-256-1 (tanh
  hidden, identity out) fed with the action unscaled to [-1, 1]; state-dict names match the reference's
  td3_*.pt checkpoints, so ``TD3.checkpoint()`` and ``evaluate.load_actor`` interoperate with them;
* update: rl/td3/learner.py:55-218 -- target policy smoothing N(0, 0.2) clipped to +-0.3, clipped double Q,
  weighted smooth-L1 critic loss (rl/utils/torch_utils.py:12-24, unit weights), delayed actor update every
  ``policy_update_freq`` critic updates with -Q1 as the actor loss, Polyak averaging rho = 1 - tau;
  Adam(lr 4e-4, eps 1e-6) for both (rl/td3/agent.py _init_optimizers);
* acting: rl/td3/agent.py:198-243 -- uniform random actions for the first ``start_steps`` agent steps,
  then actor + Gaussian noise (scale linearly annealed towards ``noise_min_scale``), clamped to [-1, 1];
* collection: rl/training/train.py:135-207 -- an episode is ``max_steps`` environment steps WITHOUT
  breaking on done (the env's done is sticky, so post-goal steps repeat the terminal reward) and every
  transition is stored with ``done``; ``train_iters`` updates follow each episode.

* opponents: rl/training/opponent_manager.py + self_play.py + curricula.py (``hockey_amd.opponents``) --
  player 2 of every arena is re-drawn every step (self-play snapshot / strong bot / weak bot) from the
  curriculum row of the training progress; the bots run fused in the kernel (``hk_step_io.policy2``), the
  step's self-play snapshot as one batched actor forward; the pool snapshots the actor every
  ``self_play_interval`` episodes.

Batched differences (by design): N episodes run side by side (one arena each) and their transitions enter
one device replay ring; updates per round scale with N through ``updates_per_round``; see
``hockey_amd.opponents`` for the opponent draws.
"""
from dataclasses import dataclass

import torch

from .constants import Mode
from .evaluate import Actor, reset_params


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

    def forward(self, state, action):
        action = ((action - self.action_low) / self.action_range) * 2 - 1.0  # TwinQNetwork._unscale_action
        x = torch.cat([state, action], dim=-1)
        return self.q1(x), self.q2(x)


def smooth_l1(x, y):
    """rl/utils/torch_utils.py weighted_smooth_l1_loss with unit weights."""
    diff = x - y
    return torch.where(diff.abs() < 1, 0.5 * diff ** 2, diff.abs() - 0.5).mean()


@dataclass
class TD3Config:  # defaults = pretrained/stage_3/config/config.json
    gamma: float = 0.99
    tau_actor: float = 0.005
    tau_critic: float = 0.005
    policy_update_freq: int = 2
    lr_q: float = 4e-4
    lr_pol: float = 4e-4
    batch_size: int = 256
    buffer_size: int = 300_000
    start_steps: int = 2000
    action_noise_scale: float = 0.2
    target_action_noise_scale: float = 0.2
    target_action_noise_clip: float = 0.3
    noise_min_scale: float = 0.07
    max_steps: int = 500
    train_iters: int = 32


class ReplayRing:
    """Device-resident FIFO replay buffer (uniform sampling)."""

    def __init__(self, capacity, n_obs=18, n_act=4, device="cuda:0"):
        self.cap, self.size, self.pos = int(capacity), 0, 0
        d = device
        self.s = torch.zeros((self.cap, n_obs), device=d)
        self.a = torch.zeros((self.cap, n_act), device=d)
        self.r = torch.zeros(self.cap, device=d)
        self.s2 = torch.zeros((self.cap, n_obs), device=d)
        self.d = torch.zeros(self.cap, device=d)

    def push(self, s, a, r, s2, d):
        n = s.shape[0]
        idx = (torch.arange(n, device=s.device) + self.pos) % self.cap
        self.s[idx], self.a[idx], self.r[idx], self.s2[idx], self.d[idx] = s, a, r.float(), s2, d.float()
        self.pos = (self.pos + n) % self.cap
        self.size = min(self.size + n, self.cap)

    def sample(self, batch, gen=None):
        i = torch.randint(0, self.size, (batch,), device=self.s.device, generator=gen)
        return self.s[i], self.a[i], self.r[i], self.s2[i], self.d[i]

    def __len__(self):
        return self.size


class TD3:
    def __init__(self, cfg=None, device="cuda:0", seed=0):
        self.cfg = cfg or TD3Config()
        self.device = torch.device(device)
        torch.manual_seed(seed)
        self.actor, self.critic = Actor().to(self.device), TwinQ().to(self.device)
        self.target_actor, self.target_critic = Actor().to(self.device), TwinQ().to(self.device)
        self.target_actor.load_state_dict(self.actor.state_dict())
        self.target_critic.load_state_dict(self.critic.state_dict())
        self.opt_actor = torch.optim.Adam(self.actor.parameters(), lr=self.cfg.lr_pol, eps=1e-6)
        self.opt_critic = torch.optim.Adam(self.critic.parameters(), lr=self.cfg.lr_q, eps=1e-6)
        self.train_step = 0

    # ---------------------------------------------------------------- learner (rl/td3/learner.py)
    def compute_target(self, s2, r, d):
        c = self.cfg
        with torch.no_grad():
            ta = self.target_actor(s2)
            noise = torch.clamp(torch.randn_like(ta) * c.target_action_noise_scale, -c.target_action_noise_clip,
                                c.target_action_noise_clip)
            ta = torch.clamp(ta + noise, -1.0, 1.0)
            q1, q2 = self.target_critic(s2, ta)
            return r + c.gamma * (1 - d) * torch.minimum(q1, q2)

    def soft_update(self):
        with torch.no_grad():
            for tgt, src, tau in ((self.target_actor, self.actor, self.cfg.tau_actor),
                                  (self.target_critic, self.critic, self.cfg.tau_critic)):
                for pt, ps in zip(tgt.parameters(), src.parameters()):
                    pt.mul_(1 - tau).add_(ps, alpha=tau)

    def update(self, s, a, r, s2, d):
        self.train_step += 1
        target = self.compute_target(s2, r, d)
        self.opt_critic.zero_grad(set_to_none=True)
        q1, q2 = self.critic(s, a)
        critic_loss = (smooth_l1(q1, target) + smooth_l1(q2, target)) * 0.5
        critic_loss.backward()
        self.opt_critic.step()
        actor_loss = None
        if self.train_step % self.cfg.policy_update_freq == 0:
            self.opt_actor.zero_grad(set_to_none=True)
            q, _ = self.critic(s, self.actor(s))
            actor_loss = -q.mean()
            actor_loss.backward()
            self.opt_actor.step()
            self.soft_update()
        return (None if actor_loss is None else actor_loss.detach()), critic_loss.detach()

    # ---------------------------------------------------------------- acting (rl/td3/agent.py)
    def act(self, obs, agent_steps, total_planned_steps, noise=True):
        c = self.cfg
        if noise and agent_steps < c.start_steps:
            return torch.rand((obs.shape[0], 4), device=obs.device) * 2 - 1
        with torch.no_grad():
            a = self.actor(obs)
        if noise:
            progress = min(agent_steps / max(total_planned_steps, 1), 1.0)
            scale = max(c.action_noise_scale * (1 - progress), c.noise_min_scale)
            a = torch.clamp(a + torch.randn_like(a) * scale, -1, 1)
        return a

    def checkpoint(self):
        """The reference's td3_*.pt layout (policy / critic / target_policy / target_critic)."""
        return {"policy": self.actor.state_dict(), "critic": self.critic.state_dict(),
                "target_policy": self.target_actor.state_dict(), "target_critic": self.target_critic.state_dict()}


def train(n_arenas=1024, rounds=10, cfg=None, device="cuda:0", seed=0, updates_per_round=None, mode=Mode.NORMAL,
          curriculum="stage3", use_self_play=True, self_play_interval=100, pool_size=40, reset="seeded", log=None):
    """Batched TD3 training: each round runs ``max_steps`` steps of ``n_arenas`` parallel episodes (no break on
    done), stores every transition, then performs ``updates_per_round`` learner updates (default: the
    reference's ``train_iters`` per episode, scaled by n_arenas / 64).  Player 2 follows the curriculum's
    opponent mix (``hockey_amd.opponents.OpponentMix``), re-drawn per arena and step.
    reset: "seeded" places episode i of a round like ``reset(seed=seed + episode)`` (the reference's PCG64
    stream, drawn on the host: ~0.5 s per round at 65 536 arenas); "device" uses the kernel's Philox placement
    (hk_reset without params; same distribution, no host work).  Returns (agent, stats)."""
    from .opponents import OpponentMix
    from .vec_env import VecHockeyEnv

    cfg = cfg or TD3Config()
    agent = TD3(cfg, device, seed)
    env = VecHockeyEnv(n_arenas, mode=mode, device=device, policies=("external", "external"), auto_reset=False,
                       seed=seed)
    mix = OpponentMix(n_arenas, curriculum, use_self_play, self_play_interval, pool_size, device, seed)
    ring = ReplayRing(min(cfg.buffer_size, n_arenas * cfg.max_steps * 4), device=device)
    updates = updates_per_round or max(1, cfg.train_iters * n_arenas // 64)
    planned = rounds * cfg.max_steps * n_arenas
    act8 = torch.zeros((n_arenas, 8), device=device)
    agent_steps = 0
    stats = {"env_steps": 0, "updates": 0, "critic_loss": [], "actor_loss": [], "mean_reward": [], "opponents": [],
             "pool_size": []}
    for rnd in range(rounds):
        mix.update_schedule(rnd / rounds)
        if reset == "device":
            obs, obs2 = (t.clone() for t in env.reset())
        else:  # episode i of this round resets with seed + round * n_arenas + i (the reference: seed + episode)
            p, _, _ = reset_params(n_arenas, seed + rnd * n_arenas, mode)
            env.reset_params(p)
            obs, obs2 = (t.clone() for t in env.observe())
        ep_reward = torch.zeros(n_arenas, device=device)
        for _ in range(cfg.max_steps):
            a = agent.act(obs, agent_steps, planned)
            agent_steps += n_arenas
            policy2, a2, _ = mix.select(obs2)
            act8[:, :4] = a
            if a2 is not None:
                act8[:, 4:] = a2
            res = env.step(act8, with_agent_two=True, policy2=policy2)
            o2, r, d = res.obs.clone(), res.reward.clone(), res.done.clone()
            ring.push(obs, a, r, o2, d)
            mix.register_outcomes(d, r)
            ep_reward += r
            obs, obs2 = o2, res.obs2.clone()
        stats["env_steps"] += cfg.max_steps * n_arenas
        stats["mean_reward"].append(float(ep_reward.mean().item()))
        stats["opponents"].append(mix.end_round(agent.actor, episodes=n_arenas))
        stats["pool_size"].append(len(mix.pool) if mix.pool is not None else 0)
        if agent_steps > cfg.batch_size:
            for _ in range(updates):
                al, cl = agent.update(*ring.sample(cfg.batch_size))
                stats["updates"] += 1
                stats["critic_loss"].append(cl)
                if al is not None:
                    stats["actor_loss"].append(al)
        if log:
            log(rnd, stats)
    env.close()
    stats["critic_loss"] = [float(x) for x in stats["critic_loss"]]
    stats["actor_loss"] = [float(x) for x in stats["actor_loss"]]
    stats["replay_size"] = len(ring)
    return agent, stats
