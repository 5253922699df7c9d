"""Benchmark: env-steps/s of the batched hockey step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the 65 536-arena config the metric is quoted on): 65 536 arenas per
GPU, NORMAL mode, keep_mode, both players driven by the BasicOpponent heuristic (strong vs strong)
evaluated on-GPU inside the step kernel, auto-reset on done (device placement), synthetic state from
seeded device RNG.  One "step" = one hk_step launch that advances every arena by one HockeyEnv.step
(pre-solve laws + Box2D-2.3 world.Step + obs/reward/done).  --policy random gives configs[1]/[3]'s
random-vs-random rollouts.

Multi-GPU (weak scaling, no data-path collective: arenas are independent): one process per
GPU, launched by torch.distributed.run; rank r owns global arenas [r*N, (r+1)*N).  The timed region is
bracketed by barrier + synchronize on every rank and the max over ranks is reported.

Output: ONE JSON line on rank 0 with `roofline` (step kernel: algorithmic bytes / measured average
kernel duration vs 8 TB/s HBM) and `cpu_baseline` (the C oracle on host cores, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--arenas", type=int, default=65536, help="arenas per GPU")
    ap.add_argument("--policy", choices=["basic", "random"], default="basic")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rollout", type=int, default=50,
                    help="also time hk_rollout with this many steps per launch (0 = skip); reported under 'rollout'")
    ap.add_argument("--cpu-arenas", type=int, default=32768, help="CPU baseline sample: arenas per step")
    ap.add_argument("--cpu-steps", type=int, default=1000,
                    help="CPU baseline sample: steps (32768 x 1000 is ~13 s on 16 host cores)")
    ap.add_argument("--streams", type=int, default=2,
                    help="also time the same arenas as this many shards stepped on as many HIP streams (0 = skip); "
                         "reported under 'streams'")
    return ap.parse_args()


def _traffic_from_profiles(n_arenas, policy):
    """HBM bytes per step-kernel launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        key = f"{policy}_{n_arenas}"
        return d[key]["hbm_bytes_per_launch"] if key in d else None
    except Exception:  # noqa: BLE001
        return None


def cpu_baseline(policy, n_arenas, steps):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # the checker, timed as the CPU baseline (kind "port")

    O.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    total, sec = O.bench_random(n_arenas, steps, threads, 0, policy)
    return {"value": total / sec, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n_arenas} arenas x {steps} steps ({'strong-vs-strong BasicOpponent' if policy == 'basic' else 'random actions'}, "
                      f"auto-reset) on the C restatement of HockeyEnv.step (oracle/hk_oracle.c), {sec:.1f} s"}


def reduce_over_ranks(elapsed, counters, dist, device):
    """Whole-job numbers: the slowest rank's elapsed time (MAX) and the summed device counters (SUM).
    The only collectives of the bench; none on the step path (arenas are sharded)."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor(counters, dtype=torch.int64, device=device)
    dist.all_reduce(c)
    return float(t.item()), c.cpu().numpy()


def shard_offset(rank, n_per_rank):
    """Global id of this rank's first arena: rank r owns [r*N, (r+1)*N); RNG streams key on the global id."""
    return rank * n_per_rank


def _time_rollout(env, N, torch, dist, world, dev, args):
    """Same workload through hk_rollout: K steps per launch, every step's obs/reward/done/info written
    ([K, N, ...] buffers), so a launch is paced by the average wave instead of each step's slowest wave."""
    k, n = args.rollout, env.n
    launches = max(1, args.steps // k)
    obs = torch.empty((k, n, N.OBS_DIM), dtype=torch.float32, device=dev)
    rew = torch.empty((k, n), dtype=torch.float32, device=dev)
    done = torch.empty((k, n), dtype=torch.uint8, device=dev)
    info = torch.empty((k, n, N.INFO_DIM), dtype=torch.float32, device=dev)
    io = N.StepIO()
    io.obs, io.reward, io.done, io.info = obs.data_ptr(), rew.data_ptr(), done.data_ptr(), info.data_ptr()
    env.rollout_raw(k, io)  # warm
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(launches):
        env.rollout_raw(k, io)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    steps = launches * k
    return {"steps_per_launch": k, "launches": launches, "value": n * world * steps / elapsed,
            "unit": "env-steps/s", "ms_per_step": elapsed / steps * 1e3}


def _time_streams(args, N, torch, dist, world, rank, dev, pol):
    """The same N arenas as S shard contexts (global arena ids unchanged, so every arena's trajectory is
    the single-context one) stepped by hk_step on S HIP streams: each call still advances its shard by one
    step, but one shard's slowest wave no longer idles the SIMDs the other shards' steps can use."""
    from hockey_amd.vec_env import VecHockeyEnv

    S, n = args.streams, args.arenas
    if n % S:
        return None
    m = n // S
    envs, ios, streams = [], [], []
    for k in range(S):
        e = VecHockeyEnv(m, device=dev, policies=pol, auto_reset=True, seed=args.seed,
                         arena_offset=shard_offset(rank, n) + k * m)
        e.reset()
        io = N.StepIO()
        io.obs, io.reward, io.done, io.info = (e.obs_buf.data_ptr(), e.reward_buf.data_ptr(),
                                               e.done_buf.data_ptr(), e.info_buf.data_ptr())
        envs.append(e)
        ios.append(io)
        streams.append(torch.cuda.Stream(dev))
    torch.cuda.synchronize()

    def run(steps):
        for _ in range(steps):
            for e, io, st in zip(envs, ios, streams):
                with torch.cuda.stream(st):
                    e.step_raw(io)

    run(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    for e in envs:
        e.close()
    return {"streams": S, "arenas_per_stream": m, "value": n * world * args.steps / elapsed,
            "unit": "env-steps/s", "ms_per_step": elapsed / args.steps * 1e3}


def main():
    args = _args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from hockey_amd import _native as N
    from hockey_amd.vec_env import VecHockeyEnv

    n = args.arenas
    pol = ("strong", "strong") if args.policy == "basic" else ("random", "random")
    env = VecHockeyEnv(n, device=dev, policies=pol, auto_reset=True, seed=args.seed,
                       arena_offset=shard_offset(rank, n))
    env.reset()
    io = N.StepIO()
    io.obs = env.obs_buf.data_ptr()
    io.reward = env.reward_buf.data_ptr()
    io.done = env.done_buf.data_ptr()
    io.info = env.info_buf.data_ptr()

    for _ in range(args.warmup):
        env.step_raw(io)
    torch.cuda.synchronize()
    env.reset_counters()
    stream = torch.cuda.current_stream(dev)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        env.step_raw(io)
        ends[k].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps
    cnt = env.counters()
    if world > 1:
        elapsed, cnt = reduce_over_ranks(elapsed, cnt, dist, dev)
    rollout = None
    if args.rollout > 1:
        rollout = _time_rollout(env, N, torch, dist, world, dev, args)
    streams = None
    if args.streams > 1:
        streams = _time_streams(args, N, torch, dist, world, rank, dev, pol)
    total_steps = n * world * args.steps
    assert int(cnt[N.CNT_STEPS]) == total_steps, (cnt, total_steps)
    assert int(cnt[N.CNT_OVERFLOW]) == 0, cnt
    value = total_steps / elapsed

    if rank == 0:
        alg_bytes, impl_bytes = env.bytes_per_step()
        achieved = alg_bytes * n / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": "env-steps/sec at 65536 arenas per MI355X (BASELINE.json metric)",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded device RNG placement; on-GPU policy actions)",
            "config": {"workload": f"{n} arenas/GPU, NORMAL, keep_mode, "
                                   f"{'strong-vs-strong BasicOpponent on-GPU' if args.policy == 'basic' else 'random-vs-random'}"
                                   f", auto-reset", "arenas_per_gpu": n, "policy": args.policy,
                       "parallelism": f"arena-sharded x{world} (no collectives)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": _traffic_from_profiles(n, args.policy),
                         "kernel": "hk::step_kernel", "kernel_avg_ms": kern_ms,
                         "algorithmic_bytes_per_env_step": alg_bytes},
            "episodes": int(cnt[N.CNT_EPISODES]),
            "toi_events": int(cnt[N.CNT_TOI]),
        }
        if rollout is not None:
            line["rollout"] = rollout
        if streams is not None:
            line["streams"] = streams
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.policy, args.cpu_arenas, args.cpu_steps)
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
