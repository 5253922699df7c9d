"""The stage-1 best checkpoint's recorded WR_strong (0.44, z = -2.91 in the checkpoint pin) under the reference's exact
evaluation protocol.  CPU oracle, test infrastructure only.

rl/utils/evaluator.py:10-35 plays ``episodes`` games in sequence on ONE Hockey-One-v0 env (rl/main.py:37-51): reset seeds
run_seed + i (420 + i for stage 1), one_starts toggling on every reset of the reused env, and one BasicOpponent whose
phase walks on across episodes (phase += U(0, 0.2) per act call, hockey_env.py:787-833) from wherever the run's earlier
evaluations left it.  The checkpoint pin (hockey_amd.evaluate.checkpoint_pins) instead gives every episode an
independent uniform phase.  Here each of M replicas replays the 100-episode sequence exactly -- the phase carried from
episode to episode, the episode order kept -- from a uniform initial phase (the 40 earlier evaluations of the run make
it uniform), and the distribution of the replicas' 100-game win rates is compared with the recorded 0.44 and with the
independent-phase model.  Also reported: the other rates of the same run and the consistency of the metrics file.

Usage: python scripts/stage1_strong_replay.py [replicas] > profiles/r05/stage1_strong_replay.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from hockey_amd.evaluate import reset_params  # noqa: E402
from pin_power_study import load_actors  # noqa: E402


@torch.no_grad()
def sequential_rates(actor, seed, episodes, replicas, strong=True, phase_seed=7):
    params, max_t, one = reset_params(episodes, seed)
    ov = O.OracleVec(replicas, policies=("external", "strong" if strong else "weak"), auto_reset=False, seed=phase_seed)
    ep = np.zeros(replicas, np.int64)  # the episode each replica is playing
    ov.reset(params=params[ep], max_t=np.full(replicas, max_t, np.int32))
    ov.phase(np.random.default_rng(phase_seed).uniform(0, 2 * np.pi, (replicas, 2)))
    wins = np.zeros(replicas, np.int64)
    length = np.zeros(replicas, np.int64)
    obs, _ = ov.observe()
    act = np.zeros((replicas, 8), np.float32)
    running = np.ones(replicas, bool)
    while running.any():
        act[:, :4] = actor(torch.from_numpy(obs)).numpy()
        out = ov.step(act)
        length += running
        d = out["done"].astype(bool) & running
        wins += (d & (out["info"][:, 0] == 1)).astype(np.int64)
        ep += d
        running &= ep < episodes
        nxt = d & running
        if nxt.any():  # the next seed's placement; the opponent's phase carries over (hkov_reset keeps it)
            ov.reset(mask=nxt.astype(np.uint8), params=params[np.minimum(ep, episodes - 1)],
                     max_t=np.full(replicas, max_t, np.int32))
            o2, _ = ov.observe()
            obs = np.where(nxt[:, None], o2, out["obs"])
        else:
            obs = out["obs"]
    ov.close()
    return wins / episodes, float(length.sum() / (episodes * replicas))


def metrics_consistency():
    """winrates_min == min(winrates_strong, winrates_weak) per evaluation, for every shipped run with both series
    (rl/utils/metrics.py log_eval writes exactly that)."""
    import glob
    out = {}
    for f in sorted(glob.glob("/root/reference/pretrained/*/metrics/metrics.json") +
                    glob.glob("/root/reference/runs/*/metrics/metrics.json")):
        m = json.load(open(f))
        s, w, mn = m.get("winrates_strong") or [], m.get("winrates_weak") or [], m.get("winrates_min") or []
        if s and w and mn:
            ok = sum(abs(c - min(a, b)) < 1e-9 for a, b, c in zip(s, w, mn))
            out[os.path.relpath(f, "/root/reference")] = {"evaluations": len(mn), "min_equals_min_of_series": ok}
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    meta, actors = load_actors()
    res = {"protocol": __doc__.split("Usage")[0].strip(), "replicas": reps, "rates": []}
    for k, ck in enumerate(meta["checkpoints"]):
        if ck["name"] != "pretrained/stage_1:best":
            continue
        for opp, rec in (("strong", ck["wr_strong"]), ("weak", ck["wr_weak"])):
            r, mean_len = sequential_rates(actors[k], ck["eval_seed"], ck["eval_episodes"], reps, opp == "strong",
                                           phase_seed=11 + k * 2 + (opp == "weak"))
            row = {"checkpoint": ck["name"], "opponent": opp, "recorded": rec, "eval_index": ck["eval_index"],
                   "replay_mean": float(r.mean()), "replay_std": float(r.std(ddof=1)),
                   "P(rate <= recorded)": float((r <= rec + 1e-9).mean()),
                   "P(rate >= recorded)": float((r >= rec - 1e-9).mean()),
                   "z_replay": float((rec - r.mean()) / r.std(ddof=1)), "mean_length": mean_len,
                   "quantiles_1_5_50_95_99": [float(np.quantile(r, q)) for q in (0.01, 0.05, 0.5, 0.95, 0.99)]}
            res["rates"].append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    if os.path.isdir("/root/reference"):
        res["metrics_file_consistency"] = metrics_consistency()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
