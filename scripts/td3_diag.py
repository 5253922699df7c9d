"""Diagnostics for the GPU TD3 loop's learning (hockey_amd.td3): is the graph-captured update's RNG fresh on
every replay, and does the eager learner learn where the graph-captured one does not?

Usage: python scripts/td3_diag.py [episodes] [arenas] [graphs 0/1] [eval_every_rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

import torch  # noqa: E402

from hockey_amd.evaluate import evaluate  # noqa: E402
from hockey_amd.td3 import TD3Config, train  # noqa: E402


def graph_rng_check():
    x = torch.zeros(4, device="cuda:0")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        x.copy_(torch.rand(4, device="cuda:0"))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x.copy_(torch.rand(4, device="cuda:0"))
    outs = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        outs.append(x.cpu().tolist())
    return {"replays": outs, "fresh": outs[0] != outs[1] and outs[1] != outs[2]}


def main():
    episodes = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    graphs = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
    every = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    print(json.dumps({"graph_rng": graph_rng_check()}), flush=True)
    cfg = TD3Config.from_json(os.path.join(ROOT, "tests", "golden", "stage1_config.json"), eval_interval=every * n)
    t0 = time.time()

    def eval_fn(agent, eps):
        agent.actor.eval()
        w = evaluate(agent.actor, episodes=200, seed=agent.seed, weak_opponent=True)
        agent.actor.train()
        rec = {"episode": eps, "updates": agent.train_step, "wr_weak": w["win"], "r_weak": w["mean_return"],
               "wall_s": round(time.time() - t0, 1)}
        print(json.dumps(rec), flush=True)
        return rec

    agent, st = train(n_arenas=n, rounds=episodes // n, cfg=cfg, seed=420, eval_fn=eval_fn, graphs=graphs)
    print(json.dumps({"graphs": graphs, "critic_loss": st["critic_loss"][-3:], "actor_loss": st["actor_loss"][-3:],
                      "mean_reward": st["mean_reward"][-3:]}), flush=True)


if __name__ == "__main__":
    main()
