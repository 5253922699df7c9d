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

Steady state: before the warmup every arena is pre-rolled --preroll steps (default 1000, hk_rollout launches
with no outputs, independent of --warmup), so the timed steps see desynchronised episodes at their steady
contact / TOI load; the timed region must contain finished episodes (asserted).

Output: ONE JSON line on rank 0 with `roofline` (step kernel, VALU-bound: the algorithmic fp32 FLOPs of the
workload per launch / measured average kernel duration vs the 157.3 TFLOP/s fp32 vector peak;
`roofline.hbm`: algorithmic bytes / the same duration vs 8 TB/s; `roofline.valu_issue`: issued active-lane VALU
operations from the committed SQ counters, reported beside, not as the headline) and `cpu_baseline` (the C
oracle's batched context on the same workload on host cores, plus the C1 single-env number; rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

# Hardware queues per process (HIP reads GPU_MAX_HW_QUEUES when its runtime starts; its default, and the value the
# GPU box exports, is 4).  The `streams` side leg overlaps S shard streams only while each has a queue of its own
# besides the default stream's (S < queues; profiles/r03/stream_sweep_per_process.log), so it runs
# S = min(--streams, queues - 1) and records the queue count it ran under.  The bench never changes the variable.
def hw_queues():
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "") or 4))
    except ValueError:
        return 4


ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# fp32 VALU lane-operation peak: 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz (MI355X_MICROARCH.md: 157.3 TFLOPS
# counts an FMA as 2).  One wave per SIMD (this kernel's occupancy) issues a VALU op every 4 cycles, not 2.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 vector peak (MI355X_MICROARCH.md), an FMA counted as 2


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--preroll", type=int, default=1000,
                    help="steps every arena is advanced (hk_rollout, no outputs) before the warmup, so the timed "
                         "steps run at the steady episode mix whatever --warmup is")
    ap.add_argument("--arenas", type=int, default=65536, help="arenas per GPU")
    ap.add_argument("--policy", choices=["basic", "random"], default="basic")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rollout", type=int, default=50,
                    help="also time hk_rollout with this many steps per launch (0 = skip); reported under 'rollout'")
    ap.add_argument("--cpu-arenas", type=int, default=65536, help="CPU baseline sample: arenas (C3 size)")
    ap.add_argument("--cpu-preroll", type=int, default=260, help="CPU baseline: untimed steps first (> 251)")
    ap.add_argument("--cpu-steps", type=int, default=150,
                    help="CPU baseline sample: timed steps (65536 x (260 + 150) is ~15 s on 16 host cores)")
    ap.add_argument("--facade-steps", type=int, default=2000,
                    help="also time the single-env gym facade (Hockey-One-v0) this many steps (0 = skip); "
                         "reported under 'facade_single_env' beside cpu_baseline.single_env")
    ap.add_argument("--c5-steps", type=int, default=50,
                    help="also time one C5 TD3 collection round (65 536 arenas, opponent mix) of this many steps "
                         "(0 = skip); reported under 'c5_collect'")
    ap.add_argument("--c4-steps", type=int, default=100,
                    help="also time BASELINE C4's per-GPU shard (2x --arenas, random rollouts) this many steps "
                         "(0 = skip); reported under 'c4_shard'")
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU-only rehearsal of the multi-rank path (gloo, no simulation): launcher, barrier, "
                         "max-over-ranks timing and the line format; the line carries \"rehearsal\": true")
    ap.add_argument("--streams", type=int, default=4,
                    help="also time the same arenas as up to this many shards stepped on as many HIP streams, at most "
                         "GPU_MAX_HW_QUEUES - 1 (0 = skip); reported under 'streams'")
    ap.add_argument("--rank-timeout", type=float, default=1200.0,
                    help="--gpus N launcher: wall-clock seconds after which ranks still running are killed and the "
                         "launch fails")
    ap.add_argument("--rehearse-hang-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher test hook
    return ap.parse_args()


def _profile(name, key):
    """profiles/<name>.json [key] (committed rocprofv3 summaries, scripts/pmc_reduce.py / sq_reduce.py), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            return json.load(f).get(key)
    except Exception:  # noqa: BLE001
        return None


def host_cores():
    """CPU cores this process may run on (the box's CPU share: its affinity mask, capped by OMP_NUM_THREADS)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, omp) if omp > 0 else n)


def cpu_baseline(policy, n_arenas, preroll, steps, seed):
    """The oracle's batched context (the C restatement of HockeyEnv.step, oracle/hk_oracle.c) on the same
    workload as the GPU line -- same policies, Philox streams, auto-reset -- on all host cores this process
    may use; plus BASELINE C1 (one env, one thread)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O  # the checker, timed as the CPU baseline (kind "port")
    from hockey_amd.placement import np_random, placement

    O.build()
    cores = host_cores()
    pol = ("strong", "strong") if policy == "basic" else ("random", "random")
    ov = O.OracleVec(n_arenas, policies=pol, auto_reset=True, seed=seed)
    pre = ov.time_steps(preroll, cores)
    sec = ov.time_steps(steps, cores)
    ep = int(ov.counters()[1])
    ov.close()
    # C1: BasicOpponent(weak) vs U(-1,1) from default_rng(0), np.random.seed(0) phase stream,
    # reset(seed=episode) on done, 10 000 steps, 1 thread
    c1_steps = 10_000
    p2 = np.random.default_rng(0).uniform(-1, 1, (c1_steps, 4)).astype(np.float32)
    legacy = np.random.RandomState(0)
    phase0 = legacy.uniform(0, np.pi)
    inc = legacy.uniform(0, 0.2, c1_steps)
    params, one = [], True
    for e in range(400):
        one = not one
        rng, _ = np_random(e)
        params.append(placement(0, one, rng)[0])
    _, _, c1_eps, c1_sec = O.run_c1(p2, inc, phase0, np.stack(params), record=False)
    return {"value": n_arenas * steps / sec, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n_arenas} arenas x {steps} timed steps after {preroll} untimed ({pre:.1f} s), "
                      f"{'strong-vs-strong BasicOpponent' if policy == 'basic' else 'random actions'} with the GPU "
                      f"line's Philox streams and auto-reset ({ep} episodes finished), batched C restatement of "
                      f"HockeyEnv.step (oracle/hk_oracle.c hkov_*), OpenMP over arenas, {sec:.1f} s",
            "single_env": {"value": c1_steps / c1_sec, "unit": "env-steps/s", "cores": 1,
                           "sample": f"BASELINE C1: 1 env, BasicOpponent(weak) vs U(-1,1), reset(seed=episode) on "
                                     f"done, {c1_steps} steps ({c1_eps} episodes), 1 thread, {c1_sec:.3f} s"}}


def preroll(env, steps, N):
    """Advance every arena `steps` steps with no outputs (hk_rollout launches of at most 250 steps)."""
    io = N.StepIO()
    left = steps
    while left > 0:
        k = min(250, left)
        env.rollout_raw(k, io)
        left -= k


def init_collectives(dist):
    """The bench's process group: gloo over host tensors on the GPU path too.  Arenas are sharded with no
    step-path exchange (north_star: "no RCCL collectives needed"), so the whole job needs only a
    barrier, one MAX and one SUM of host scalars; RCCL is never brought up (tests/test_distributed_gloo.py
    rehearses exactly this group)."""
    dist.init_process_group(backend="gloo")
    return dist.get_backend()


def max_over_ranks(elapsed, dist):
    """The slowest rank's elapsed time (MAX over a gloo group, host tensor)."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_over_ranks(elapsed, counters, dist, device=None):
    """Whole-job numbers: the slowest rank's elapsed time (MAX) and the summed device counters (SUM), both on
    host tensors over the gloo group.  The only collectives of the bench; none on the step path (arenas are
    sharded).  `device` is accepted for old callers and ignored: nothing is reduced on the GPU."""
    import numpy as np
    import torch

    c = torch.tensor(np.asarray(counters, dtype=np.int64), dtype=torch.int64)
    dist.all_reduce(c)
    return max_over_ranks(elapsed, dist), c.numpy()


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
        elapsed = max_over_ranks(elapsed, dist)
    steps = launches * k
    return {"steps_per_launch": k, "launches": launches, "value": n * world * steps / elapsed,
            "unit": "env-steps/s", "ms_per_step": elapsed / steps * 1e3}


def _time_streams(args, N, torch, dist, world, rank, dev, pol):
    """The same N arenas as S shard contexts (global arena ids unchanged, so every arena's trajectory is
    the single-context one) stepped by hk_step on S HIP streams: each call still advances its shard by one
    step, but one shard's slowest wave no longer idles the SIMDs the other shards' steps can use."""
    from hockey_amd.vec_env import VecHockeyEnv

    q = hw_queues()
    S, n = min(args.streams, q - 1), args.arenas
    if S < 2 or n < S:
        return None
    sizes = [n // S + (k < n % S) for k in range(S)]  # contiguous shards, sizes differing by at most one
    envs, ios, streams = [], [], []
    for k in range(S):
        e = VecHockeyEnv(sizes[k], device=dev, policies=pol, auto_reset=True, seed=args.seed,
                         arena_offset=shard_offset(rank, n) + sum(sizes[:k]))
        e.reset()
        preroll(e, args.preroll, N)
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
        elapsed = max_over_ranks(elapsed, dist)
    for e in envs:
        e.close()
    return {"streams": S, "arenas_per_stream": sizes, "hw_queues": q, "value": n * world * args.steps / elapsed,
            "unit": "env-steps/s", "ms_per_step": elapsed / args.steps * 1e3}


def time_facade(steps, dev):
    """The reference's deployment shape on the GPU: ONE env behind the gym facade (hockey_amd.make
    ("Hockey-One-v0"): one hk_step launch per env.step plus the host round trip), random agent actions."""
    import numpy as np
    import torch

    from hockey_amd import make

    env = make("Hockey-One-v0", device=dev)
    env.reset(seed=0)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (steps, 4)).astype(np.float32)
    for k in range(20):
        _, _, d, _, _ = env.step(acts[k])
    env.reset(seed=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eps = 0
    for k in range(steps):
        _, _, d, _, _ = env.step(acts[k])
        if d:
            eps += 1
            env.reset(seed=2 + eps)
    sec = time.perf_counter() - t0
    env.close()
    return {"value": steps / sec, "unit": "env-steps/s", "steps": steps, "episodes": eps,
            "sample": "1 env, Hockey-One-v0 facade (strong BasicOpponent fused), U(-1,1) agent actions, "
                      "reset(seed) on done: per step one hk_step launch + obs/reward/done/info copies to the host"}


def time_c5(n, steps, dev, batch=16384):
    """BASELINE C5: one round of the batched TD3 loop (hockey_amd.td3.train) on n arenas: device reset, actor
    forward + exploration noise, per-arena per-step opponent mix (strong / weak bot fused in the kernel,
    self-play snapshot forward), hk_step, replay push -- then the learner updates of that round at the
    reference's replay ratio (32 updates x 256 samples per 500-step episode = 16.4 samples per transition,
    rl/training/train.py:145-207) as graph-captured updates of `batch` samples.  Reports the whole round
    (collection + updates) and the collection alone; round 2 is timed (the self-play pool is populated)."""
    from hockey_amd.td3 import REFERENCE_REPLAY_RATIO as RR
    from hockey_amd.td3 import TD3Config, train, updates_for

    cfg = TD3Config(max_steps=steps, start_steps=0)
    table = [(1.0, 0.35, 0.35, 0.30)]  # stage-3's last curriculum row (self-play active from round 2)
    train(n_arenas=n, rounds=2, cfg=TD3Config(max_steps=5, start_steps=0), device=dev, curriculum=table,
          self_play_interval=n, reset="device", learner_batch=batch, replay_ratio=RR)  # warm-up
    agent, st = train(n_arenas=n, rounds=2, cfg=cfg, device=dev, curriculum=table, self_play_interval=n,
                      reset="device", learner_batch=batch, timing=True, replay_ratio=RR)
    collect, update = st["round_time"][1]
    ups = updates_for(cfg, n, steps, batch, RR)
    return {"value": n * steps / (collect + update), "unit": "env-steps/s", "arenas": n, "steps": steps,
            "collect_value": n * steps / collect, "collect_s": collect, "update_s": update,
            "updates": ups, "batch": batch, "samples_per_transition": ups * batch / (n * steps),
            "opponents": st["opponents"][1],
            "sample": f"round 2 of hockey_amd.td3.train on {n} arenas x {steps} steps (device reset, actor + noise, "
                      f"opponent mix, hk_step, replay push) + {ups} learner updates of {batch} samples "
                      f"(the reference's 16.4 samples per stored transition); value = whole round, "
                      f"collect_value = collection only"}


def time_c4(n, steps, preroll_steps, seed, dev):
    """BASELINE C4's per-GPU shard: n (131 072) arenas on one GPU, random-vs-random rollouts (U(-1,1) actions
    drawn in the kernel), auto-reset, one hk_step launch per step after a pre-roll past the first episodes.
    With twice as many waves as SIMDs, a SIMD whose first wave finishes early starts a queued one, so a
    launch is paced less by any single slow wave than at 65 536 arenas."""
    import torch

    from hockey_amd import _native as N
    from hockey_amd.vec_env import VecHockeyEnv

    env = VecHockeyEnv(n, device=dev, policies=("random", "random"), auto_reset=True, seed=seed,
                       arena_offset=0)
    env.reset()
    preroll(env, preroll_steps, N)
    io = N.StepIO()
    io.obs, io.reward, io.done, io.info = (env.obs_buf.data_ptr(), env.reward_buf.data_ptr(),
                                           env.done_buf.data_ptr(), env.info_buf.data_ptr())
    for _ in range(20):
        env.step_raw(io)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        env.step_raw(io)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    env.close()
    return {"value": n * steps / sec, "unit": "env-steps/s", "arenas": n, "steps": steps,
            "ms_per_step": sec / steps * 1e3,
            "sample": f"BASELINE C4 per-GPU shard: {n} arenas, random-vs-random (in-kernel U(-1,1)), auto-reset, "
                      f"{steps} hk_step launches after a {preroll_steps}-step pre-roll"}


def launch_ranks(args):
    """`--gpus N` without a torch.distributed launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set like torch.distributed.run) BEFORE this process touches any
    GPU, wait for all of them, and return non-zero if any rank failed.  Rank 0 prints the bench line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # wait for every rank under one wall-clock limit; a rank that fails or a rank still running at the limit ends
    # the launch, and the ranks still running (likely waiting on the lost one in a collective) are killed
    deadline = time.monotonic() + args.rank_timeout
    why = None
    while why is None:
        rcs = [p.poll() for p in procs]
        bad = [(r, rc) for r, rc in enumerate(rcs) if rc not in (None, 0)]
        if bad:
            why = f"rank(s) failed: {bad}"
        elif all(rc == 0 for rc in rcs):
            return 0
        elif time.monotonic() > deadline:
            why = f"rank(s) {[r for r, rc in enumerate(rcs) if rc is None]} still running after {args.rank_timeout:g} s"
        else:
            time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.kill()
    for p in procs:
        p.wait()
    print(f"bench.py: {why}", file=sys.stderr, flush=True)
    return 1


class RehearsalEnv:
    """--rehearse: a CPU stand-in for one rank's arena shard (no GPU, gloo collectives).  It runs the launcher,
    the barrier / max-over-ranks timing and the line format of the real bench on a CPU-only host; its
    step_raw does no simulation and the line it yields says so ("rehearsal": true)."""

    def __init__(self, n):
        self.n = n
        self.steps = 0

    def step_raw(self, io):
        self.steps += self.n

    def rollout_raw(self, k, io):
        self.steps += self.n * k

    def reset_counters(self):
        self.steps = 0

    def counters(self):
        c = [0] * 16
        c[0], c[1] = self.steps, 1
        return c

    def bytes_per_step(self):
        return 285, 0

    def close(self):
        pass


def provenance():
    """Which code the numbers describe: the library's build hash (its .srchash sidecar), the hash of the
    sources in this tree, and whether the committed counter summaries were collected at that same hash."""
    from hockey_amd._native import built_hash, source_hash

    return built_hash(), source_hash()


def main():
    args = _args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))  # before `import torch` / any GPU call in this process
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.arenas <= 0 or args.steps <= 0:
        sys.exit(f"bench.py: rank {rank}: --arenas and --steps must be positive")
    import torch
    import torch.distributed as dist

    gpu = not args.rehearse
    if world > 1:
        init_collectives(dist)  # gloo on the GPU path too: host scalars only, no RCCL bring-up
    if gpu:
        # HK_BENCH_ONE_DEVICE=<d>: every rank on device d -- a multi-rank rehearsal of the real GPU path (gloo
        # collectives, barriers, max-over-ranks timing, the line) on a one-GPU box; never set by the driver
        one = os.environ.get("HK_BENCH_ONE_DEVICE")
        if one is not None:
            local = int(one)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    else:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731

    from hockey_amd import _native as N

    n = args.arenas
    pol = ("strong", "strong") if args.policy == "basic" else ("random", "random")
    io = N.StepIO()
    if gpu:
        from hockey_amd.vec_env import VecHockeyEnv

        env = VecHockeyEnv(n, device=dev, policies=pol, auto_reset=True, seed=args.seed,
                           arena_offset=shard_offset(rank, n))
        env.reset()
        io.obs = env.obs_buf.data_ptr()
        io.reward = env.reward_buf.data_ptr()
        io.done = env.done_buf.data_ptr()
        io.info = env.info_buf.data_ptr()
    else:
        env = RehearsalEnv(n)
        if rank == args.rehearse_hang_rank:
            time.sleep(3600)  # launcher test hook: a rank that never reaches the barrier

    preroll(env, args.preroll, N)
    for _ in range(args.warmup):
        env.step_raw(io)
    sync()
    env.reset_counters()
    if gpu:
        # two HIP events on the launch stream bracket the K launches (no marker between launches: a per-launch
        # event pair adds a marker packet to every launch gap inside the timed region); their GPU time / K is the
        # kernel's average launch duration, launch gaps included
        stream = torch.cuda.current_stream(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if gpu:
        ev0.record(stream)
    for k in range(args.steps):
        env.step_raw(io)
    if gpu:
        ev1.record(stream)
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps if gpu else elapsed / args.steps * 1e3
    cnt = env.counters()
    if world > 1:
        elapsed, cnt = reduce_over_ranks(elapsed, cnt, dist)
    rollout = streams = None
    if gpu and args.rollout > 1:
        rollout = _time_rollout(env, N, torch, dist, world, dev, args)
    if gpu and args.streams > 1:
        streams = _time_streams(args, N, torch, dist, world, rank, dev, pol)
    total_steps = n * world * args.steps
    assert int(cnt[N.CNT_STEPS]) == total_steps, (cnt, total_steps)
    assert int(cnt[N.CNT_OVERFLOW]) == 0, cnt
    assert int(cnt[N.CNT_EPISODES]) > 0, "timed region holds no finished episode: not at steady state"
    value = total_steps / elapsed

    if rank == 0:
        alg_bytes, impl_bytes = env.bytes_per_step()
        hbm_gbs = alg_bytes * n / (kern_ms * 1e-3) / 1e9
        key = f"{args.policy}_{n}"
        pmc = _profile("pmc_summary.json", key) or {}
        sq = _profile("sq_summary.json", key) or {}
        lib_hash, src_hash = provenance()
        stale = (sq.get("source_hash") != lib_hash or pmc.get("source_hash") != lib_hash or lib_hash != src_hash)
        lane_ops = sq.get("valu_lane_ops_per_launch")
        flops = None
        try:  # algorithmic FLOPs per env-step of this workload (scripts/flop_count.py, host build of the kernel source)
            with open(os.path.join(ROOT, "profiles", "r04", "flop_count.json")) as f:
                flops = json.load(f)["flops_per_env_step"] if args.policy == "basic" else None
        except Exception:  # noqa: BLE001
            flops = None
        useful_tflops = flops * n / (kern_ms * 1e-3) / 1e12 if flops else None
        valu_tops = lane_ops / (kern_ms * 1e-3) / 1e12 if lane_ops else None
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
            # the headline roof is ALGORITHMIC work: Box2D's useful fp32 FLOPs per env-step of this
            # workload x arenas / the kernel's average launch duration, against the fp32 vector peak; the HBM roof
            # (285 algorithmic B per env-step) beside it; issued active-lane VALU ops (what the SIMDs actually
            # executed, from the committed SQ counters) under valu_issue, never as the headline
            "roofline": {"bound": "valu", "achieved": useful_tflops, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": useful_tflops / FP32_PEAK_TFLOPS if useful_tflops else None,
                         "basis": "algorithmic fp32 FLOPs of Box2D's arithmetic on this workload "
                                  "(profiles/r04/flop_count.json, scripts/flop_count.py) per launch / kernel_avg_ms",
                         "flops_per_env_step": flops,
                         "traffic": pmc.get("hbm_bytes_per_launch"),
                         "kernel": "hk::step_kernel", "kernel_avg_ms": kern_ms,
                         "kernel_avg_from": "HIP events bracketing the K timed launches on their stream: GPU time / K, "
                                            "launch gaps included",
                         "library_hash": lib_hash, "source_hash": src_hash,
                         "counters_hash": {"sq": sq.get("source_hash"), "pmc": pmc.get("source_hash")},
                         "counters_stale": bool(stale),
                         "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": hbm_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_env_step": alg_bytes,
                                 "traffic_bytes_per_launch": pmc.get("hbm_bytes_per_launch"),
                                 "traffic_from": pmc.get("source")},
                         "valu_issue": {"achieved": valu_tops, "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                                        "frac": valu_tops / VALU_PEAK_TOPS if valu_tops else None,
                                        "lane_ops_per_launch": lane_ops,
                                        "lane_ops_per_useful_flop": (lane_ops / (flops * n)
                                                                     if lane_ops and flops else None),
                                        "issue_util": sq.get("valu_issue_util"), "lane_util": sq.get("valu_lane_util"),
                                        "counters_from": sq.get("source"),
                                        "note": "issued active-lane VALU operations (SQ_THREAD_CYCLES_VALU), not "
                                                "algorithmic work"}},
            "preroll": args.preroll,
            "episodes": int(cnt[N.CNT_EPISODES]),
            "toi_events": int(cnt[N.CNT_TOI]),
        }
        if not gpu:
            line["rehearsal"] = True
            line["data"] = "REHEARSAL on CPU (gloo): no simulation ran; launcher / timing / line format only"
        if rollout is not None:
            line["rollout"] = rollout
        if streams is not None:
            line["streams"] = streams
        # side legs: reported beside the headline, never allowed to take the bench line down with them
        if gpu and world == 1 and args.facade_steps > 0:
            try:
                line["facade_single_env"] = time_facade(args.facade_steps, dev)
            except Exception as e:  # noqa: BLE001
                line["facade_single_env"] = {"error": repr(e)[:300]}
        if gpu and world == 1 and args.c5_steps > 0:
            try:
                line["c5_round"] = time_c5(n, args.c5_steps, dev)
            except Exception as e:  # noqa: BLE001
                line["c5_round"] = {"error": repr(e)[:300]}
        if gpu and world == 1 and args.c4_steps > 0:
            try:
                line["c4_shard"] = time_c4(2 * n, args.c4_steps, args.preroll, args.seed, dev)
            except Exception as e:  # noqa: BLE001
                line["c4_shard"] = {"error": repr(e)[:300]}
        if gpu and world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.policy, args.cpu_arenas, args.cpu_preroll, args.cpu_steps,
                                                args.seed)
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
