"""Timing-only ablations of the step kernel (results are physically wrong under ablation).

HK_ABLATE bits: 1 = skip velocity iterations, 2 = single position iteration, 4 = skip TOI, 8 = skip collide.
Prints the average step-kernel time per configuration (65 536 arenas, strong-vs-strong, auto-reset).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

import torch  # noqa: E402

from hockey_amd import _native as N  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402


def run(ablate, n, policy, warm, steps):
    os.environ["HK_ABLATE"] = str(ablate)
    env = VecHockeyEnv(n, device="cuda:0", policies=(policy, policy), auto_reset=True, seed=1)
    env.reset()
    io = N.StepIO()
    io.obs = env.obs_buf.data_ptr()
    io.reward = env.reward_buf.data_ptr()
    io.done = env.done_buf.data_ptr()
    for _ in range(warm):
        env.step_raw(io)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        env.step_raw(io)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    env.close()
    return ms


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    policy = sys.argv[2] if len(sys.argv) > 2 else "strong"
    configs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 4, 8, 5, 7, 15]
    for ab in configs:
        t = time.time()
        ms = run(ab, n, policy, 300, 200)
        print(f"ablate={ab:2d}  {ms:8.3f} ms/step  ({n / ms * 1e3 / 1e6:7.1f} M steps/s)  [{time.time() - t:.1f}s]",
              flush=True)
