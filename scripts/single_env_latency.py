"""Single-arena step latency on the GPU, split into its parts: launch + sync per step (the facade's shape),
back-to-back launches with one sync at the end (launch gaps, no host round trip), and hk_rollout (K steps in one
launch: the kernel's own per-step time with a warm instruction cache).  Strong vs strong, auto-reset, N = 1
and N = 64 (one full wave).  Prints one JSON line per N."""
import json
import os
import sys
import time

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "hockey-env_amd")]
import torch  # noqa: E402

from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402


def measure(n, steps=2000, k=200):
    v = VecHockeyEnv(n, policies=("strong", "strong"), auto_reset=True, device="cuda:0")
    s = torch.cuda.current_stream()
    for _ in range(50):
        v.step()
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        v.step()
        s.synchronize()
    sync_us = 1e6 * (time.perf_counter() - t0) / steps
    t0 = time.perf_counter()
    for _ in range(steps):
        v.step()
    s.synchronize()
    b2b_us = 1e6 * (time.perf_counter() - t0) / steps
    v.rollout(k)
    s.synchronize()
    reps = max(1, steps // k)
    t0 = time.perf_counter()
    for _ in range(reps):
        v.rollout(k)
    s.synchronize()
    roll_us = 1e6 * (time.perf_counter() - t0) / (reps * k)
    v.close()
    return {"arenas": n, "us_step_launch_sync": sync_us, "us_step_back_to_back": b2b_us, "us_rollout_per_step": roll_us}


if __name__ == "__main__":
    for n in (1, 64):
        print(json.dumps(measure(n)), flush=True)
