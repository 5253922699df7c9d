"""Analysis: the bench workload (65 536 arenas, strong vs strong, auto-reset) as S shard contexts stepped on S
HIP streams, for several S, under this process's GPU_MAX_HW_QUEUES.  Every shard keeps its global arena ids
(same trajectories as one context).  Prints one JSON line per S.
Usage: GPU_MAX_HW_QUEUES=<q> python scripts/stream_sweep.py [S ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hockey-env_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from hockey_amd import _native as N  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402

n, steps, warm = 65536, 300, 50
dev = "cuda:0"
pol = ("strong", "strong")
for S in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    m = n // S
    envs, ios, streams = [], [], []
    for k in range(S):
        e = VecHockeyEnv(m, device=dev, policies=pol, auto_reset=True, seed=0, arena_offset=k * m)
        e.reset()
        bench.preroll(e, 1000, N)
        io = N.StepIO()
        io.obs, io.reward, io.done, io.info = (e.obs_buf.data_ptr(), e.reward_buf.data_ptr(),
                                               e.done_buf.data_ptr(), e.info_buf.data_ptr())
        envs.append(e)
        ios.append(io)
        streams.append(torch.cuda.Stream(dev))
    torch.cuda.synchronize()

    def run(k):
        for _ in range(k):
            for e, io, st in zip(envs, ios, streams):
                with torch.cuda.stream(st):
                    e.step_raw(io)

    run(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.close()
    print(json.dumps({"hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "streams": S, "arenas_per_stream": m,
                      "M_env_steps_per_s": round(n * steps / dt / 1e6, 1), "ms_per_step": round(dt / steps * 1e3, 4)}),
          flush=True)
