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
phase increments come from the per-arena Philox stream instead of the process-global ``np.random``, and
every episode starts from a fresh BasicOpponent phase.  One reference env object reused across the 100
episodes toggles ``one_starts`` on every reset; episode i therefore starts with ``one_starts = (i % 2 ==
1)`` here as there.
"""
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


def reset_params(episodes, seed, mode=Mode.NORMAL):
    """Placement of episode i as ``env.reset(seed=seed + i)`` on a reused reference env."""
    params = np.zeros((episodes, 6), np.float32)
    one = np.zeros(episodes, bool)
    for i in range(episodes):
        rng, _ = np_random(seed + i)
        one[i] = (i % 2) == 1
        params[i], max_t = placement(mode, bool(one[i]), rng)
    return params, max_t, one


@torch.no_grad()
def evaluate(policy, episodes=100, seed=42, weak_opponent=False, mode=Mode.NORMAL, device="cuda:0",
             player1=None):
    """Win rate and mean return of ``policy`` (obs [N,18] tensor -> actions [N,4]) against BasicOpponent.

    ``player1`` = "strong" / "weak" evaluates the fused BasicOpponent as player 1 instead of ``policy``
    (the reference notebook's BasicOpponent-vs-BasicOpponent study).  Returns a dict with win / draw /
    loss rates, mean return and mean episode length."""
    from .vec_env import VecHockeyEnv

    p1 = player1 if player1 is not None else "external"
    env = VecHockeyEnv(episodes, keep_mode=True, mode=mode, device=device,
                       policies=(p1, "weak" if weak_opponent else "strong"), auto_reset=False, seed=seed)
    params, max_t, _ = reset_params(episodes, seed, mode)
    env.reset_params(params)
    obs, _ = env.observe()
    dev = env.device
    ret = torch.zeros(episodes, dtype=torch.float64, device=dev)
    length = torch.zeros(episodes, dtype=torch.int64, device=dev)
    winner = torch.zeros(episodes, dtype=torch.float32, device=dev)
    live = torch.ones(episodes, dtype=torch.bool, device=dev)
    act = torch.zeros((episodes, 8), dtype=torch.float32, device=dev)
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
    return {"episodes": episodes, "win": float((w == 1).mean()), "draw": float((w == 0).mean()),
            "loss": float((w == -1).mean()), "mean_return": float(ret.mean().item()),
            "mean_length": float(length.double().mean().item())}
