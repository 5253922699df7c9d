"""C5 and f4 numbers on one GPU: env-steps/s of the batched TD3 collection loop at 65 536 arenas (actor
inference + fused-opponent hk_step + device replay push per step), learner updates/s, and the
BasicOpponent-vs-BasicOpponent evaluation statistics next to the reference notebook's 1000-game study."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
import torch  # noqa: E402

from hockey_amd.evaluate import evaluate  # noqa: E402
from hockey_amd.td3 import TD3Config, train  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    cfg = TD3Config(max_steps=100, start_steps=0)
    train(n_arenas=1024, rounds=1, cfg=TD3Config(max_steps=10), updates_per_round=5)  # warm-up
    torch.cuda.synchronize()
    marks = []
    t0 = time.perf_counter()
    agent, st = train(n_arenas=n, rounds=2, cfg=cfg, updates_per_round=200,
                      log=lambda r, s: (torch.cuda.synchronize(), marks.append(time.perf_counter())))
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    # separate the learner: time 200 updates alone
    t1 = time.perf_counter()
    from hockey_amd.td3 import ReplayRing
    ring = ReplayRing(100_000)
    ring.push(torch.randn(100_000, 18, device="cuda:0"), torch.rand(100_000, 4, device="cuda:0"),
              torch.randn(100_000, device="cuda:0"), torch.randn(100_000, 18, device="cuda:0"),
              torch.zeros(100_000, device="cuda:0"))
    for _ in range(200):
        agent.update(*ring.sample(cfg.batch_size))
    torch.cuda.synchronize()
    upd = 200 / (time.perf_counter() - t1)
    collect = (total - 2 * 200 / upd)
    out = {"c5_arenas": n, "c5_env_steps": st["env_steps"], "c5_wall_s": total,
           "c5_collect_env_steps_per_s": st["env_steps"] / collect, "learner_updates_per_s": upd,
           "mean_round_reward": st["mean_reward"]}
    t2 = time.perf_counter()
    ev = evaluate(None, episodes=10000, seed=0, player1="strong")
    ev["wall_s"] = time.perf_counter() - t2
    out["basic_vs_basic_10000"] = ev
    out["reference_notebook_1000"] = {"win": 0.319, "draw": 0.368, "loss": 0.313, "mean_length": 150.911}
    print(json.dumps(out, indent=1))
