"""Where the single-env facade's time goes (BASELINE C1 shape on the GPU): per-step cost of the bare
hk_step_host call (mapped zero-copy buffer, and HK_STEP_HOST_STAGED=1 with H2D / D2H copies), of an empty
launch + sync round trip, and of the full Hockey-One-v0 facade step.  Prints one JSON line.  Run under
`rocprofv3 --kernel-trace --stats` to get the N=1 step_kernel duration beside it."""
import ctypes
import json
import os
import sys
import time

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "hockey-env_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def bare(steps, staged):
    from hockey_amd import _native as N
    from hockey_amd.vec_env import VecHockeyEnv

    os.environ["HK_STEP_HOST_STAGED"] = "1" if staged else "0"
    v = VecHockeyEnv(1, keep_mode=True, mode="NORMAL", device="cuda:0", policies=("external", "strong"))
    act = np.zeros(8, np.float32)
    out = np.zeros(N.HOST_RECORD_BYTES, np.uint8)
    ap, op = act.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p)
    st = v._stream()
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (steps, 4)).astype(np.float32)
    for k in range(20):
        act[:4] = acts[k]
        N.check(v.L.hk_step_host(v._ctx, ap, None, 0, op, st), "hk_step_host")
    t0 = time.perf_counter()
    for k in range(steps):
        act[:4] = acts[k]
        N.check(v.L.hk_step_host(v._ctx, ap, None, 0, op, st), "hk_step_host")
    dt = time.perf_counter() - t0
    v.close()
    return 1e6 * dt / steps


def empty_round_trip(steps):
    x = torch.zeros(1, device="cuda:0")
    s = torch.cuda.current_stream()
    for _ in range(20):
        x.add_(1)
        s.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        x.add_(1)
        s.synchronize()
    return 1e6 * (time.perf_counter() - t0) / steps


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    import bench

    r = {"us_empty_launch_sync": empty_round_trip(steps),
         "us_hk_step_host_mapped": bare(steps, False),
         "us_hk_step_host_staged": bare(steps, True)}
    os.environ["HK_STEP_HOST_STAGED"] = "0"
    f = bench.time_facade(steps, "cuda:0")
    r["us_facade_step"] = 1e6 / f["value"]
    r["facade_steps_per_s"] = f["value"]
    print(json.dumps(r))


if __name__ == "__main__":
    main()
