"""Per-step hk_step kernel time over a long run of the bench workload (65 536 arenas, strong-vs-strong BasicOpponent,
auto-reset): which steps of the episode cycle are heavy?  HIP events around every launch on the launch stream;
prints per-window (default 25 steps) mean kernel ms, episodes finished and TOI events, and writes the per-step
series to gpurun_out/step_profile.json.
Usage: python scripts/step_profile.py [steps] [arenas] [window]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
import torch  # noqa: E402

from hockey_amd import _native as N  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    win = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    dev = torch.device("cuda", 0)
    env = VecHockeyEnv(n, device=dev, policies=("strong", "strong"), auto_reset=True, seed=0, arena_offset=0)
    env.reset()
    io = N.StepIO()
    io.obs, io.reward, io.done, io.info = (env.obs_buf.data_ptr(), env.reward_buf.data_ptr(),
                                           env.done_buf.data_ptr(), env.info_buf.data_ptr())
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    done = torch.zeros(steps, dtype=torch.int32, device=dev)
    for k in range(steps):
        ev[k][0].record(stream)
        env.step_raw(io)
        ev[k][1].record(stream)
        done[k] = env.done_buf.sum()
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    d = done.cpu().tolist()
    out = {"arenas": n, "steps": steps, "kernel_ms": ms, "done": d}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "step_profile.json"), "w") as f:
        json.dump(out, f)
    for s in range(0, steps, win):
        w = ms[s:s + win]
        print(f"steps {s:5d}-{s + len(w) - 1:5d}: kernel {sum(w) / len(w):.4f} ms (max {max(w):.4f})  "
              f"done {sum(d[s:s + win]):7d}", flush=True)
    env.close()


if __name__ == "__main__":
    main()
