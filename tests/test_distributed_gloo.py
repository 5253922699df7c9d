"""World-size-2 rehearsal of the multi-GPU bench path on CPU (gloo): arenas shard by global id with no
collective on the step path; the bench's only collectives (MAX of elapsed, SUM of counters) reduce
correctly; and the two shards together are bit-identical to one process running all arenas (shard
invariance of the per-arena Philox streams).  The per-arena step is the kernel source's host build
(tests/hostcheck.py), so no GPU is needed."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N_PER_RANK, STEPS = 96, 60


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests"), root]
    import bench
    from hostcheck import HostVec

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    env = HostVec(N_PER_RANK, policies=("strong", "strong"), auto_reset=True, seed=5,
                  arena_offset=bench.shard_offset(rank, N_PER_RANK))
    for _ in range(STEPS):
        env.step(None)
    st, aux = env.get_state()
    c = env.counters().astype(np.int64)
    elapsed, total = bench.reduce_over_ranks(1.0 + rank, c, dist, torch.device("cpu"))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), st=st, aux=aux, c=c, total=total, elapsed=elapsed)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(tmp_path):
    from hostcheck import HostVec, lib

    lib()  # build the harness once, before the workers load it
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    # bench reductions: MAX elapsed, SUM counters
    assert float(r[0]["elapsed"]) == 2.0 and float(r[1]["elapsed"]) == 2.0
    assert np.array_equal(r[0]["total"], r[0]["c"] + r[1]["c"])
    assert int(r[0]["total"][0]) == 2 * N_PER_RANK * STEPS
    # shard invariance: ranks 0+1 == one process over 2N arenas
    one = HostVec(2 * N_PER_RANK, policies=("strong", "strong"), auto_reset=True, seed=5, arena_offset=0)
    for _ in range(STEPS):
        one.step(None)
    st, aux = one.get_state()
    assert np.array_equal(st, np.concatenate([r[0]["st"], r[1]["st"]]))
    assert np.array_equal(aux, np.concatenate([r[0]["aux"], r[1]["aux"]]))


def _bench(args, env_extra=None):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` (no torch.distributed launcher) starts 2 ranks itself; rank 0 prints one line whose
    n_gpus and whole-job value cover both ranks (CPU rehearsal: gloo, no simulation)."""
    rc, lines, err = _bench(["--gpus", "2", "--rehearse", "--steps", "4", "--warmup", "1", "--preroll", "0",
                             "--arenas", "64"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["rehearsal"] is True and ln["steps"] == 4
    assert abs(ln["value"] - 2 * 64 * 4 / (ln["ms_per_step"] * 4 / 1e3)) / ln["value"] < 1e-9


def test_bench_rejects_gpus_world_size_mismatch():
    rc, lines, err = _bench(["--gpus", "1", "--rehearse", "--steps", "2", "--warmup", "0", "--preroll", "0",
                             "--arenas", "64"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines
    assert "WORLD_SIZE=2" in err


def test_bench_failed_rank_fails_the_launch():
    """A rank that dies makes the launcher exit non-zero (here: an invalid arena count on every rank)."""
    rc, lines, err = _bench(["--gpus", "2", "--rehearse", "--steps", "2", "--warmup", "0", "--preroll", "0",
                             "--arenas", "0"])
    assert rc != 0


def test_bench_hung_rank_times_out_and_fails_the_launch():
    """A rank that never reaches the barrier: the launcher kills the ranks still running at --rank-timeout and
    exits non-zero, instead of waiting forever."""
    import time

    t0 = time.monotonic()
    rc, lines, err = _bench(["--gpus", "2", "--rehearse", "--steps", "2", "--warmup", "0", "--preroll", "0",
                             "--arenas", "64", "--rank-timeout", "20", "--rehearse-hang-rank", "1"])
    assert rc != 0 and not lines
    assert "still running after 20 s" in err, err[-2000:]
    assert time.monotonic() - t0 < 120


def test_bench_never_constructs_an_nccl_group(monkeypatch):
    """the multi-GPU bench needs a barrier, a MAX and a SUM of host scalars, so its GPU path
    brings up the same gloo group this file rehearses, never RCCL.  Statically: the only init_process_group call
    in bench.py is init_collectives' gloo one and no string names nccl; dynamically: init_collectives asks for
    gloo, and reduce_over_ranks reduces host tensors only."""
    import ast
    import sys

    import torch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "bench.py")).read()
    tree = ast.parse(src)
    calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call) and getattr(n.func, "attr", "") == "init_process_group"]
    assert len(calls) == 1
    kw = {k.arg: k.value.value for k in calls[0].keywords if isinstance(k.value, ast.Constant)}
    assert kw == {"backend": "gloo"}
    consts = [n.value.lower() for n in ast.walk(tree) if isinstance(n, ast.Constant) and isinstance(n.value, str)]
    assert not any("nccl" in c for c in consts)
    assert "device_id" not in src

    sys.path.insert(0, root)
    import bench

    seen = {}

    class FakeDist:
        class ReduceOp:
            MAX = "max"

        @staticmethod
        def init_process_group(backend=None, **kw):
            seen["backend"] = backend

        @staticmethod
        def get_backend():
            return seen["backend"]

        @staticmethod
        def all_reduce(t, op=None):
            seen.setdefault("devices", []).append(t.device.type)

    assert bench.init_collectives(FakeDist) == "gloo"
    el, c = bench.reduce_over_ranks(1.5, np.arange(4), FakeDist)
    assert el == 1.5 and list(c) == [0, 1, 2, 3]
    assert seen["devices"] == ["cpu", "cpu"]
