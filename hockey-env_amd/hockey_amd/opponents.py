"""Player-2 opponents of the batched TD3 loop (BASELINE config C5).

Batched form of the reference's opponent machinery, device-resident and free of per-step host syncs:

* ``CURRICULA`` -- the stage tables of rl/training/curricula.py: rows (progress threshold, P(strong bot),
  P(weak bot), P(self-play)); ``OpponentMix.update_schedule`` picks the first row whose threshold exceeds
  the training progress (opponent_manager.py:38-51).
* ``SelfPlayPool`` -- rl/training/self_play.py:20-68: frozen actor snapshots taken every ``interval``
  episodes, at most ``pool_size`` kept (oldest dropped), a difficulty score per snapshot (start 1.0, x1.2 on
  an outcome that is not an agent win, x0.95 on a win, clipped to [0.1, 10]) and score-weighted sampling.
* ``OpponentMix.select`` -- opponent_manager.py:62-91, per arena and per step: with probability P(self-play)
  (only once the pool holds a snapshot) the opponent is the snapshot sampled for this step, evaluated as
  ONE batched ``PolicyOpponent`` forward (hockey_env.py:908-922) over every arena's agent-two observation;
  otherwise a second draw picks the strong bot below P(strong) and the weak bot above it.  The choice goes
  to the kernel as ``hk_step_io.policy2`` (external for self-play arenas, whose actions fill
  ``actions[:, 4:8]``; the fused BasicOpponent for the bots, each bot kind with its own phase, as the
  reference's manager holds one ``BasicOpponent`` of each kind).

Batched differences (by design, documented): the draws come from a torch generator on the device instead of
the process-global ``np.random``; the snapshot is sampled once per step for all arenas (the reference samples
one per step for its single env); ``register_outcome`` counts the done steps of self-play arenas against the
snapshot they faced (the reference charges the last sampled snapshot for every done step of any opponent),
tallied per step on the device and folded into the scores step by step at the end of the round (within one
step, the non-win outcomes are applied before the wins; clipping follows every outcome as in the reference).
"""
import copy
import math

import numpy as np
import torch

from . import _native as N

# rl/training/curricula.py (threshold, strong, weak, self_play)
CURRICULA = {
    "stage1": [(1.00, 0.00, 1.00, 0.00)],
    "stage2": [(0.33, 0.55, 0.45, 0.00), (0.66, 0.45, 0.45, 0.10), (1.00, 0.50, 0.40, 0.10)],
    "stage3": [(0.15, 0.30, 0.70, 0.00), (0.70, 0.60, 0.30, 0.10), (1.00, 0.35, 0.35, 0.30)],
    "noise_study": [(1.0, 0.5, 0.5, 0.0)],
}
CURRICULA["ablation"] = CURRICULA["stage2"]

SCORE_MIN, SCORE_MAX, SCORE_LOSS, SCORE_WIN = 0.1, 10.0, 1.2, 0.95


class SelfPlayPool:
    """Frozen actor snapshots with difficulty scores (rl/training/self_play.py)."""

    def __init__(self, interval=100, pool_size=40, seed=0):
        self.interval, self.pool_size = int(interval), int(pool_size)
        self.episode_counter = 0
        self.pool, self.scores = [], []
        self.rng = np.random.default_rng(seed)

    def step(self, actor, episodes=1):
        """Count `episodes` finished training episodes; snapshot the actor when an interval boundary is crossed
        (at most one snapshot per call: a batched round crosses several boundaries with the same weights)."""
        before = self.episode_counter // self.interval
        self.episode_counter += int(episodes)
        if self.episode_counter // self.interval > before:
            self.add_snapshot(actor)

    def add_snapshot(self, actor):
        snap = copy.deepcopy(actor).eval()
        for p in snap.parameters():
            p.requires_grad_(False)
        self.pool.append(snap)
        self.scores.append(1.0)
        if len(self.pool) > self.pool_size:
            self.pool.pop(0)
            self.scores.pop(0)

    def update_difficulty(self, idx, wins, others):
        """One step's outcomes against snapshot ``idx``: ``others`` outcomes that are not agent wins (x1.2 each)
        then ``wins`` agent wins (x0.95 each), clipped to [0.1, 10] after EVERY outcome as the reference does
        (self_play.py:45-55).  Both runs are monotone, so clipping after each factor equals clipping the run's
        product once: min(10, s * 1.2^others), then max(0.1, s * 0.95^wins)."""
        s = self.scores[idx]
        if others:
            s = min(SCORE_MAX, math.exp(min(math.log(s) + others * math.log(SCORE_LOSS), 50.0)))
        if wins:
            s = max(SCORE_MIN, math.exp(math.log(s) + wins * math.log(SCORE_WIN)))
        self.scores[idx] = float(np.clip(s, SCORE_MIN, SCORE_MAX))

    def sample(self):
        """Score-weighted snapshot index (get_opponent), or None with an empty pool."""
        if not self.pool:
            return None
        w = np.asarray(self.scores, np.float64)
        return int(self.rng.choice(len(self.pool), p=w / w.sum()))

    def __len__(self):
        return len(self.pool)


class OpponentMix:
    """Per-arena, per-step opponent selection for player 2 (rl/training/opponent_manager.py)."""

    def __init__(self, n_arenas, curriculum="stage3", use_self_play=True, self_play_interval=100, pool_size=40,
                 device="cuda:0", seed=0):
        self.n = int(n_arenas)
        self.device = torch.device(device)
        self.table = CURRICULA[curriculum] if isinstance(curriculum, str) else [tuple(r) for r in curriculum]
        self.pool = SelfPlayPool(self_play_interval, pool_size, seed) if use_self_play else None
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed) + 0x5EED)
        self.p_strong, self.p_weak, self.p_self = 0.0, 1.0, 0.0
        self.update_schedule(0.0)
        self._policy2 = torch.empty(self.n, dtype=torch.uint8, device=self.device)
        self.reset_stats()

    def update_schedule(self, progress):
        for threshold, strong, weak, self_play in self.table:
            if progress < threshold:
                if strong + weak + self_play <= 0:
                    raise ValueError("Bot probabilities must sum to > 0")
                self.p_strong, self.p_weak, self.p_self = strong, weak, self_play
                return

    def reset_stats(self):
        self._counts = torch.zeros(3, dtype=torch.int64, device=self.device)  # strong, weak, self-play
        self._outcomes = []  # per step: device tensor [snapshot index, wins, others]

    def select(self, obs2):
        """(policy2 [N] uint8, player-2 actions [N,4] or None, snapshot index or None) for this step.
        obs2: [N,18] agent-two observations (device)."""
        n, dev = self.n, self.device
        idx = self.pool.sample() if self.pool is not None else None
        u_sp = torch.rand(n, device=dev, generator=self.gen)
        u_bot = torch.rand(n, device=dev, generator=self.gen)
        sp = (u_sp < self.p_self) if idx is not None else torch.zeros(n, dtype=torch.bool, device=dev)
        strong = ~sp & (u_bot < self.p_strong)
        weak = ~sp & ~strong
        p2 = self._policy2
        p2.fill_(N.POLICY_BASIC_WEAK)
        p2.masked_fill_(strong, N.POLICY_BASIC_STRONG)
        p2.masked_fill_(sp, N.POLICY_EXTERNAL)
        self._counts += torch.stack([strong.sum(), weak.sum(), sp.sum()])
        act = None
        if idx is not None:
            with torch.no_grad():
                act = self.pool.pool[idx](obs2)  # one batched PolicyOpponent forward for the step
            act = act * sp.unsqueeze(1)
        self._sp_mask, self._idx = sp, idx
        return p2, act, idx

    def register_outcomes(self, done, reward):
        """Done steps of this step's self-play arenas: agent win (reward > 0) or not (opponent_manager
        register_outcome -> update_difficulty).  Tallied per step on the device; end_round() applies the steps in
        order, clipping after every outcome."""
        if self._idx is None:
            return
        d = (done != 0) & self._sp_mask
        win = d & (reward > 0)
        self._outcomes.append(torch.stack([torch.full((), self._idx, dtype=torch.int64, device=self.device),
                                           win.sum(), (d & ~win).sum()]))

    def end_round(self, actor=None, episodes=0):
        """Fold the round's outcomes into the snapshot scores, advance the self-play episode counter (taking a
        snapshot on an interval boundary) and return the round's opponent counts."""
        counts = self._counts.cpu().tolist()
        if self.pool is not None:
            if self._outcomes:
                for idx, w, o in torch.stack(self._outcomes).cpu().tolist():
                    if idx < len(self.pool) and (w or o):
                        self.pool.update_difficulty(idx, w, o)
            if actor is not None and episodes:
                self.pool.step(actor, episodes)
        self.reset_stats()
        return {"strong": counts[0], "weak": counts[1], "self_play": counts[2]}
