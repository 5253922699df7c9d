"""Per-phase shader-clock breakdown of the step kernel (diagnostic build, HK_LIB=..._timers.so).

Phases: 0 load+reset+policy, 1 pre-solve laws, 2 collide, 3 island solve, 4 TOI, 5 obs/outputs/store.
Prints average shader cycles per wave per step for each phase (timing shares, not wall time).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HK_LIB", os.path.join(ROOT, "hockey-env_amd", "hockey_amd", "_lib", "libhockey_hip_timers.so"))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

import torch  # noqa: E402

from hockey_amd import _native as N  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402

NAMES = ["load+policy+presolve", "collide", "isl-setup", "isl-velocity", "isl-position+sleep", "toi-events+out", "toi-scan", "toi-b2TOI"]

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    policy = sys.argv[2] if len(sys.argv) > 2 else "strong"
    steps = 200
    env = VecHockeyEnv(n, device="cuda:0", policies=(policy, policy), auto_reset=True, seed=1)
    env.reset()
    io = N.StepIO()
    io.obs = env.obs_buf.data_ptr()
    io.reward = env.reward_buf.data_ptr()
    io.done = env.done_buf.data_ptr()
    for _ in range(300):
        env.step_raw(io)
    torch.cuda.synchronize()
    env.reset_counters()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        env.step_raw(io)
    e1.record()
    torch.cuda.synchronize()
    c = env.counters()
    waves = (n + 63) // 64
    tot = sum(int(c[8 + k]) for k in range(8))
    print(f"{n} arenas, policy {policy}: {e0.elapsed_time(e1) / steps:.3f} ms/step (timer build)")
    for k, name in enumerate(NAMES):
        cyc = int(c[8 + k]) / waves / steps
        print(f"  {name:14s} {cyc:12.0f} cycles/wave-step  {100.0 * int(c[8 + k]) / max(tot, 1):5.1f}%")
