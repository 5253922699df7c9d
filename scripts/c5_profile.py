"""Where the C5 collection step's time goes: one TD3 round (65 536 arenas, opponent mix) with torch's
profiler over the steps of the second round.  Usage: python scripts/c5_profile.py [arenas] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
import torch  # noqa: E402

from hockey_amd.td3 import TD3Config, train  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = TD3Config(max_steps=steps, start_steps=0)
table = [(1.0, 0.35, 0.35, 0.30)]
train(n_arenas=n, rounds=2, cfg=TD3Config(max_steps=3, start_steps=0), updates_per_round=1, curriculum=table,
      self_play_interval=n)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    t0 = time.perf_counter()
    train(n_arenas=n, rounds=2, cfg=cfg, updates_per_round=1, curriculum=table, self_play_interval=n)
    torch.cuda.synchronize()
    print("wall", time.perf_counter() - t0)
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))
