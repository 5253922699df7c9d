"""Checkpoint interop and the reference's evaluation protocol on GPU arenas.

* ``load_actor(path)`` reads a TD3 checkpoint in the reference's layout (``td3_*.pt`` = dict with a
  ``policy`` state dict: fc1 256x18, fc2 256x256, fc3 4x256 + biases; rl/td3/networks.py ActorNetwork:
  tanh hidden and output activations) with ``torch.load(weights_only=True)`` -- nothing in the file is
  executed.  A bare state dict is accepted too.
* ``evaluate(policy, episodes, ...)`` runs the protocol of rl/utils/evaluator.py:10-35 and
  model_evaluation/model_evaluator.py:81-108 -- ``Hockey-One-v0`` (player 2 = BasicOpponent, strong or
  weak), reset seeds ``seed + i``, greedy actions, episode return summed up to and including the done
  step, win = ``info['winner'] == 1`` -- with one arena per episode, all episodes stepping together in
  one ``hk_step`` launch per time step.

Differences from running the reference protocol serially (documented, statistical only): the opponent's
phase increments come from the per-arena Philox stream instead of the process-global ``np.random``.  The
reference's Evaluator reuses one env -- and so one BasicOpponent -- for all its episodes and evaluations
(rl/main.py:37-51), so an episode starts wherever the opponent's phase walk (U(0, 0.2) per step) has got to:
``opponent_phase="walked"`` (default) starts every episode at a phase uniform on [0, 2 pi), "fresh" at a new
BasicOpponent's U(0, pi).  One reference env object reused across the 100 episodes toggles ``one_starts`` on
every reset; episode i therefore starts with ``one_starts = (i % 2 == 1)`` here as there (100 is even, so every
evaluation of a run starts alike).

``replicas`` = R plays each of the ``episodes`` placements R times (R x episodes arenas, placement i of every
replica from ``reset(seed=seed + i)``), each replica with its own opponent phases: the per-placement win
frequencies estimate the conditional win probability of each of the reference's fixed evaluation placements
(tests/test_gpu_checkpoints.py).
"""
import math

import numpy as np
import torch

from .constants import Mode
from .placement import np_random, placement


class Actor(torch.nn.Module):
    """rl/td3/networks.py ActorNetwork (input 18, hidden 256, output 4, tanh / tanh)."""

    def __init__(self, n_obs=18, n_act=4, h=256):
        super().__init__()
        self.fc1 = torch.nn.Linear(n_obs, h)
        self.fc2 = torch.nn.Linear(h, h)
        self.fc3 = torch.nn.Linear(h, n_act)

    def forward(self, x):
        x = torch.tanh(self.fc1(x))
        x = torch.tanh(self.fc2(x))
        return torch.tanh(self.fc3(x))


def load_actor(path_or_state, device="cuda:0"):
    """Actor from a reference TD3 checkpoint path (or an already loaded dict)."""
    state = path_or_state
    if isinstance(path_or_state, (str, bytes)) or hasattr(path_or_state, "__fspath__"):
        state = torch.load(path_or_state, map_location="cpu", weights_only=True)
    if isinstance(state, dict) and "policy" in state:
        state = state["policy"]
    if not isinstance(state, dict) or "fc1.weight" not in state:
        raise ValueError("not a TD3 actor checkpoint: expected a 'policy' state dict with fc1/fc2/fc3")
    h, n_obs = state["fc1.weight"].shape
    n_act = state["fc3.weight"].shape[0]
    actor = Actor(n_obs, n_act, h)
    actor.load_state_dict({k: v for k, v in state.items() if k.split(".")[0] in ("fc1", "fc2", "fc3")})
    return actor.to(device).eval()


def reset_params(episodes, seed, mode=Mode.NORMAL, first_reset=0):
    """Placement of episode i as ``env.reset(seed=seed + i)`` on a reused reference env whose
    ``first_reset + i``-th reset (0-based, after the constructor's) it is: ``one_starts`` toggles on every
    reset from the constructor's True, so it is False on the even ones."""
    params = np.zeros((episodes, 6), np.float32)
    one = np.zeros(episodes, bool)
    for i in range(episodes):
        rng, _ = np_random(seed + i)
        one[i] = ((first_reset + i) % 2) == 1
        params[i], max_t = placement(mode, bool(one[i]), rng)
    return params, max_t, one


@torch.no_grad()
def evaluate(policy, episodes=100, seed=42, weak_opponent=False, mode=Mode.NORMAL, device="cuda:0",
             player1=None, replicas=1, opponent_phase="walked", phase_seed=None, per_episode=False):
    """Win rate and mean return of ``policy`` (obs [N,18] tensor -> actions [N,4]) against BasicOpponent.

    ``player1`` = "strong" / "weak" evaluates the fused BasicOpponent as player 1 instead of ``policy``
    (the reference notebook's BasicOpponent-vs-BasicOpponent study).  ``replicas``, ``opponent_phase``: see the
    module docstring; ``phase_seed`` seeds the walked phases (default ``seed``).  Returns a dict with win / draw /
    loss rates, mean return and mean episode length over all replicas x episodes games; ``per_episode`` adds
    ``winner`` [replicas, episodes] (+1 / 0 / -1)."""
    from .vec_env import VecHockeyEnv

    if opponent_phase not in ("walked", "fresh"):
        raise ValueError("opponent_phase must be 'walked' or 'fresh'")
    reps = int(replicas)
    n = episodes * reps
    p1 = player1 if player1 is not None else "external"
    env = VecHockeyEnv(n, keep_mode=True, mode=mode, device=device,
                       policies=(p1, "weak" if weak_opponent else "strong"), auto_reset=False, seed=seed)
    params, max_t, _ = reset_params(episodes, seed, mode)
    env.reset_params(np.tile(params, (reps, 1)))
    if opponent_phase == "walked":
        rng = np.random.default_rng(seed if phase_seed is None else phase_seed)
        env.opponent_phase(rng.uniform(0, 2 * np.pi, (n, 2)))
    obs, _ = env.observe()
    dev = env.device
    ret = torch.zeros(n, dtype=torch.float64, device=dev)
    length = torch.zeros(n, dtype=torch.int64, device=dev)
    winner = torch.zeros(n, dtype=torch.float32, device=dev)
    live = torch.ones(n, dtype=torch.bool, device=dev)
    act = torch.zeros((n, 8), dtype=torch.float32, device=dev)
    for _ in range(max_t + 1):  # the longest episode is max_t + 1 steps (done when time >= max_t)
        if player1 is None:
            act[:, :4] = policy(obs).float()
        res = env.step(act if player1 is None else None)
        ret += torch.where(live, res.reward.double(), torch.zeros_like(ret))
        length += live.long()
        d = res.done.bool()
        winner = torch.where(live & d, res.info[:, 0], winner)
        live &= ~d
        obs = res.obs
        if not bool(live.any()):
            break
    env.close()
    w = winner.cpu().numpy()
    out = {"episodes": n, "win": float((w == 1).mean()), "draw": float((w == 0).mean()),
           "loss": float((w == -1).mean()), "mean_return": float(ret.mean().item()),
           "mean_length": float(length.double().mean().item())}
    if per_episode:
        out["winner"] = w.reshape(reps, episodes).astype(np.int8)
    return out


# Hockey-Env.ipynb:940-2154 (cells 51-57): 1000 strong-vs-strong BasicOpponent games, unseeded resets on one
# reused env, up to 500 steps with a break at done.  Recorded: 150 911 steps, winners +1/0/-1 = 319/368/313,
# sum of rewards -4360.24 (agent 1) / -4367.87 (agent 2), and the per-feature mean of every step's obs.
NOTEBOOK_STUDY = {
    "games": 1000, "steps": 150911, "win": 0.319, "draw": 0.368, "loss": 0.313,
    "reward_sum": -4360.24, "reward2_sum": -4367.87,
    "obs_mean": [-2.9737481, -0.00389052, -0.00098744, -0.06068974, 0.00053737, 0.00684031, 2.96906086,
                 0.00154943, -0.0013995, 0.0559986, -0.00210782, -0.00475535, -0.0208698, -0.0031277,
                 0.01032396, 0.00961799, 1.10906428, 1.10767273]}


@torch.no_grad()
def basic_vs_basic_study(games, seed=0, vel_ref_semantics=False, device="cuda:0"):
    """The notebook's strong-vs-strong study on ``games`` arenas (one game each, resets alternating the puck side
    like the reused reference env, opponent phases uniform mod 2 pi like its long-lived opponents), with per-game
    statistics for standard errors: winner, length, return of
    both agents and the per-game sum of obs.  Returns a dict of numpy arrays."""
    from .vec_env import VecHockeyEnv

    env = VecHockeyEnv(games, keep_mode=True, device=device, policies=("strong", "strong"), auto_reset=False,
                       seed=seed, vel_ref_semantics=vel_ref_semantics)
    params, max_t, _ = reset_params(games, seed)
    env.reset_params(params)
    # the notebook's two BasicOpponent objects live across all 1000 games, so a game starts wherever the phase
    # walk (U(0, 0.2) per step) has got to: uniform mod 2 pi, not the U(0, pi) of a fresh BasicOpponent
    env.opponent_phase(np.random.default_rng(seed).uniform(0, 2 * np.pi, (games, 2)))
    dev = env.device
    live = torch.ones(games, dtype=torch.bool, device=dev)
    ret = torch.zeros(games, dtype=torch.float64, device=dev)
    ret2 = torch.zeros(games, dtype=torch.float64, device=dev)
    length = torch.zeros(games, dtype=torch.int64, device=dev)
    winner = torch.zeros(games, dtype=torch.float32, device=dev)
    obs_sum = torch.zeros((games, 18), dtype=torch.float64, device=dev)
    for _ in range(max_t + 1):
        res = env.step(None, with_agent_two=True)
        lv = live.double()
        ret += lv * res.reward.double()
        ret2 += lv * res.reward2.double()
        obs_sum += lv[:, None] * res.obs.double()
        length += live.long()
        d = res.done.bool()
        winner = torch.where(live & d, res.info[:, 0], winner)
        live &= ~d
        if not bool(live.any()):
            break
    env.close()
    return {"winner": winner.cpu().numpy(), "length": length.cpu().numpy(), "return": ret.cpu().numpy(),
            "return2": ret2.cpu().numpy(), "obs_sum": obs_sum.cpu().numpy()}


def study_zscores(per_game, ref=NOTEBOOK_STUDY):
    """z-scores of a per-game study against the notebook's 1000 games, with the combined standard error of both
    estimates (the notebook's own error estimated from this study's between-game spread at n = 1000; obs means
    by the ratio estimator sum(obs) / sum(steps) with per-game clustering)."""
    w, L = per_game["winner"], per_game["length"].astype(np.float64)
    n, m = len(w), ref["games"]
    out = {"games": n}

    def z(est, ref_val, var1):  # var1 = variance of one game's contribution
        se = np.sqrt(var1 / n + var1 / m)
        return {"value": float(est), "notebook": float(ref_val), "se_combined": float(se),
                "z": float((est - ref_val) / se) if se > 0 else 0.0}

    for key, val in (("win", 1), ("draw", 0), ("loss", -1)):
        p = float((w == val).mean())
        out[key] = z(p, ref[key], p * (1 - p))
    out["steps_per_game"] = z(L.mean(), ref["steps"] / m, L.var())
    for key, col in (("reward_per_game", "return"), ("reward2_per_game", "return2")):
        r = per_game[col]
        out[key] = z(r.mean(), ref[key.replace("_per_game", "_sum")] / m, r.var())
    mu = per_game["obs_sum"].sum(0) / L.sum()
    resid = per_game["obs_sum"] - L[:, None] * mu[None, :]  # linearised ratio estimator
    var1 = (resid ** 2).mean(0) / L.mean() ** 2
    out["obs_mean"] = [z(mu[k], ref["obs_mean"][k], var1[k]) for k in range(18)]
    return out


def recorded_rate_z(winner, recorded):
    """z-score of a win rate the reference recorded over its fixed evaluation placements against this simulator.

    ``winner`` [R, E]: R replicas of the reference's E evaluation placements (``evaluate(..., replicas=R,
    per_episode=True)``).  Given the placements, the reference's only randomness is its opponent's phase, so the
    recorded rate is a mean of E Bernoulli(p_i), p_i = the win probability from placement i, which the replicas
    estimate (shrunk to (k_i + 1/2) / (R + 1) so that no variance is zero).  Under the hypothesis that the
    simulator is the reference's, recorded - mean(p_i) has variance sum p_i (1 - p_i) / E^2 (the recorded rate)
    + the same / R (this estimate).  Returns a dict with z = (recorded - estimate) / se and, for comparison, the
    binomial z that ignores the fixed placements."""
    w = np.asarray(winner)
    reps, e = w.shape
    k = (w == 1).sum(0).astype(np.float64)
    p_i = k / reps
    q_i = (k + 0.5) / (reps + 1.0)
    est = float(p_i.mean())
    var1 = float((q_i * (1 - q_i)).sum()) / e ** 2
    se = math.sqrt(var1 * (1.0 + 1.0 / reps))
    pb = min(max(est, 0.5 / (reps * e)), 1 - 0.5 / (reps * e))
    se_b = math.sqrt(pb * (1 - pb) / e + pb * (1 - pb) / (reps * e))
    return {"recorded": float(recorded), "estimate": est, "se": se, "z": (float(recorded) - est) / se,
            "z_binomial": (float(recorded) - est) / se_b, "replicas": reps, "placements": e}


def pin_acceptance(rows):
    """The acceptance rule of the checkpoint pins (tests/test_gpu_checkpoints.py), as a verdict instead of asserts:
    rates no selection touched need |z| < 3 each and sum z^2 below the chi-square 0.1 % point; rates behind a
    best-checkpoint selection need -3 < z < Phi^-1(1 - 0.01 / n_evals).  Returns a dict with ``passed`` and the
    statistics behind it (free chi^2 and its p-value, the violating rows)."""
    from scipy import stats

    free = [r for r in rows if not r["selected"]]
    sel = [r for r in rows if r["selected"]]
    chi2 = float(sum(r["z"] ** 2 for r in free))
    crit = float(stats.chi2.ppf(0.999, len(free))) if free else float("inf")
    bad_free = [(r["checkpoint"], r["opponent"], round(r["z"], 2)) for r in free if not abs(r["z"]) < 3]
    bad_sel = [(r["checkpoint"], r["opponent"], round(r["z"], 2)) for r in sel
               if not -3 < r["z"] < stats.norm.ppf(1 - 0.01 / r["n_evals"])]
    return {"passed": not bad_free and not bad_sel and chi2 < crit, "free_chi2": chi2, "free_dof": len(free),
            "free_chi2_crit_0.999": crit, "free_chi2_p": float(stats.chi2.sf(chi2, len(free))) if free else 1.0,
            "violations_free": bad_free, "violations_selected": bad_sel, "n_free": len(free), "n_selected": len(sel)}


def checkpoint_pins(fixture, replicas=64, device="cuda:0"):
    """Every shipped checkpoint against its recorded evaluation (tests/golden/checkpoint_actors.npz, written by
    tests/golden/extract_checkpoint_actors.py): each actor runs the reference's evaluation protocol on R =
    ``replicas`` replicas of the reference's own 100 placements (reset seeds run_seed + i) against the strong and,
    where the run evaluated it, the weak bot.  Returns one row per recorded rate with its z (recorded_rate_z), and
    whether the rate took part in the run's best-checkpoint selection: a td3_best.pt is the evaluation whose score
    beat the running best (rl/utils/model_manager.py:15-23), so the rates behind that score are maxima of a noisy
    series and sit above the policy's own rate by construction."""
    import json

    z = np.load(fixture) if isinstance(fixture, (str, bytes)) or hasattr(fixture, "__fspath__") else fixture
    meta = json.loads(str(z["meta"]))
    rows = []
    for k, ck in enumerate(meta["checkpoints"]):
        actor = Actor().to(device)
        with torch.no_grad():
            for name, p in actor.named_parameters():
                p.copy_(torch.from_numpy(z[f"{k}/{name.replace('.', '_')}"]))
        actor.eval()
        for opp, rec in (("strong", ck["wr_strong"]), ("weak", ck["wr_weak"])):
            if rec is None:
                continue
            r = evaluate(actor, episodes=ck["eval_episodes"], seed=ck["eval_seed"], weak_opponent=opp == "weak",
                         device=device, replicas=replicas, phase_seed=1000 + 2 * k + (opp == "weak"),
                         per_episode=True)
            row = recorded_rate_z(r["winner"], rec)
            score = ck["score"]
            selected = ck["kind"] == "best" and (score in ("min", "winrates") or score == opp)
            row.update(checkpoint=ck["name"], kind=ck["kind"], opponent=opp, eval_index=ck["eval_index"],
                       n_evals=ck["n_evals"], selected=selected, mean_length=r["mean_length"])
            rows.append(row)
    return rows
