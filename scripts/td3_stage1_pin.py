"""Learning pin of the GPU TD3 loop: the reference's stage-1 run on batched arenas.

Reference run: pretrained/stage_1 (config/config.json, config/run_info.json: seed 420, 10 000 episodes of 500
steps, weak BasicOpponent only, buffer 100 k, batch 256, 32 updates per episode = 320 000 updates, Gaussian
noise 0.2, no self-play, no PER).  Its metrics/metrics.json records WR_weak over 100 evaluation episodes every
200 episodes, rising from 0.10 to 0.93-0.98 (first >= 0.9 at episode 6 800, ~218 k updates).

Here: ``hockey_amd.td3.train`` with the same config on ``--arenas`` parallel arenas (20: one round = 20
episodes, so the 200-episode evaluation cadence and the 32-updates-per-episode ratio land exactly), the same
evaluation protocol (rl/utils/evaluator.py: Hockey-One-v0, weak / strong bot, seeds seed + i, greedy actions)
through ``hockey_amd.evaluate.evaluate``.  Writes the curve as JSON (``--out``) after every evaluation.

Usage: python scripts/td3_stage1_pin.py [--arenas 20] [--episodes 10000] [--out gpurun_out/r03/stage1_pin.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

import torch  # noqa: E402

from hockey_amd.evaluate import evaluate  # noqa: E402
from hockey_amd.td3 import TD3Config, train, updates_for  # noqa: E402

REF_WR_WEAK = [0.1, 0.14, 0.14, 0.15, 0.08, 0.17, 0.22, 0.09, 0.32, 0.3, 0.28, 0.34, 0.38, 0.33, 0.37, 0.41, 0.4, 0.51,
               0.5, 0.42, 0.43, 0.52, 0.47, 0.46, 0.6, 0.44, 0.58, 0.43, 0.68, 0.71, 0.74, 0.86, 0.86, 0.92, 0.91,
               0.91, 0.97, 0.97, 0.98, 0.96, 0.99, 0.97, 0.99, 0.97, 0.96, 0.98, 0.97, 0.93, 0.96, 0.98]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=20)
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--eval-episodes", type=int, default=100)
    ap.add_argument("--seed", type=int, default=420)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--episode-end", choices=["done", "max_steps"], default="done",
                    help="'done': an episode ends at its goal / time limit, as in the runs behind the recorded "
                         "metrics (their returns never exceed +10); 'max_steps': the reference's current no-break "
                         "500-step loop (hockey_amd.td3.train docstring)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r03", "stage1_pin.json"))
    ap.add_argument("--checkpoint", default=None, help="save the final agent (reference td3_*.pt layout) here")
    ap.add_argument("--learner", choices=["auto", "fused", "eager"], default="auto",
                    help="hockey_amd.td3.train's learner: the fused MFMA kernels (auto: on the GPU from batch 256) "
                         "or the eager PyTorch update (r03's runs)")
    args = ap.parse_args()
    cfg = TD3Config.from_json(os.path.join(ROOT, "tests", "golden", "stage1_config.json"))
    n = args.arenas
    rounds = args.episodes // n
    dev = "cuda:0"
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    out = {"config": vars(cfg), "arenas": n, "rounds": rounds, "episodes": rounds * n, "seed": args.seed,
           "episode_end": args.episode_end, "learner": args.learner,
           "updates_per_round": updates_for(cfg, n, cfg.max_steps), "eval_episodes": args.eval_episodes,
           "reference_wr_weak": REF_WR_WEAK, "evals": []}
    t_start = time.time()
    hist = {"rounds": 0}  # per-round stats of train() since the last evaluation (diagnostics)

    def log(rnd, st):
        hist["st"] = st

    last = {"env_steps": 0, "rounds": 0, "critic": 0, "actor": 0}

    def diag():
        st = hist.get("st")
        if st is None:
            return {}
        r0, c0, a0 = last["rounds"], last["critic"], last["actor"]
        nr = len(st["mean_reward"])
        cl, al = st["critic_loss"][c0:], st["actor_loss"][a0:]
        d = {"mean_return": sum(st["mean_reward"][r0:]) / max(1, nr - r0),
             "env_steps_per_episode": (st["env_steps"] - last["env_steps"]) / max(1, (nr - r0) * n),
             "critic_loss": sum(cl) / max(1, len(cl)), "actor_loss": sum(al) / max(1, len(al))}
        last.update(env_steps=st["env_steps"], rounds=nr, critic=len(st["critic_loss"]), actor=len(st["actor_loss"]))
        return d

    def eval_fn(agent, episodes):
        agent.actor.eval()
        w = evaluate(agent.actor, episodes=args.eval_episodes, seed=agent.seed, weak_opponent=True, device=dev)
        s = evaluate(agent.actor, episodes=args.eval_episodes, seed=agent.seed, weak_opponent=False, device=dev)
        agent.actor.train()
        rec = {"episode": episodes, "updates": agent.train_step, "wr_weak": w["win"], "wr_strong": s["win"],
               "r_weak": w["mean_return"], "r_strong": s["mean_return"], "draw_weak": w["draw"],
               "len_weak": w["mean_length"], "wall_s": time.time() - t_start, "train": diag()}
        out["evals"].append(rec)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(rec), flush=True)
        return rec

    fused = {"auto": "auto", "fused": True, "eager": False}[args.learner]
    agent, st = train(n_arenas=n, rounds=rounds, cfg=cfg, device=dev, seed=args.seed, eval_fn=eval_fn,
                      graphs=not args.no_graphs, episode_end=args.episode_end, log=log, fused=fused)
    torch.cuda.synchronize()
    wr = [e["wr_weak"] for e in out["evals"]]
    first = next((e for e in out["evals"] if e["wr_weak"] >= 0.9), None)
    out.update(updates=st["updates"], env_steps=st["env_steps"], wall_s=time.time() - t_start,
               critic_loss_last=st["critic_loss"][-5:], actor_loss_last=st["actor_loss"][-5:],
               first_wr_weak_ge_0_9=first, best_wr_weak=max(wr) if wr else None,
               final5_wr_weak_mean=sum(wr[-5:]) / max(1, len(wr[-5:])))
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    if args.checkpoint:
        torch.save(agent.checkpoint(), args.checkpoint)
    print(json.dumps({k: out[k] for k in ("updates", "env_steps", "wall_s", "first_wr_weak_ge_0_9", "best_wr_weak",
                                          "final5_wr_weak_mean")}), flush=True)


if __name__ == "__main__":
    main()
