"""Where a C5 learner update's time goes: hockey_amd.td3.Learner on a ring of random transitions, batch B (default
16 384, the C5 learner batch), K updates after a warm-up, for the PyTorch path and the fused MFMA path (each eager
and graph-replayed).  Prints ms per update and the fused path's achieved fp32 FLOP/s (algorithmic FLOPs of
hockey_amd.learner_hip.update_flops); run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
Usage: python scripts/learner_profile.py [B] [K] [paths: torch,fused]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("HK_PKG_DIR") or os.path.join(ROOT, "hockey-env_amd"))  # HK_PKG_DIR: an A/B copy
import torch  # noqa: E402

from hockey_amd.td3 import TD3, Learner, ReplayRing, TD3Config  # noqa: E402

if os.environ.get("HK_BLAS"):  # "cublas" (rocBLAS on ROCm) or "cublaslt" (hipBLASLt, torch's default here)
    torch.backends.cuda.preferred_blas_library(os.environ["HK_BLAS"])
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = "cuda:0"
agent = TD3(TD3Config(), dev, seed=0)
ring = ReplayRing(1 << 20, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
n = 1 << 20
ring.push(torch.randn(n, 18, device=dev, generator=g), torch.rand(n, 4, device=dev, generator=g) * 2 - 1,
          torch.randn(n, device=dev, generator=g), torch.randn(n, 18, device=dev, generator=g),
          (torch.rand(n, device=dev, generator=g) < 0.01).float())
paths = (sys.argv[3] if len(sys.argv) > 3 else "torch,fused").split(",")
out = {"batch": B, "updates": K, "blas": str(torch.backends.cuda.preferred_blas_library())}
for path in paths:
    for graphs in (False, True):
        agent = TD3(TD3Config(), dev, seed=0)
        L = Learner(agent, ring, B, graphs=graphs, fused=(path == "fused"))
        L.run(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.run(K)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        out[f"{path}_ms_per_update_{'graphs' if graphs else 'eager'}"] = ms
        if path == "fused":
            from hockey_amd.learner_hip import update_flops
            out[f"fused_tflops_{'graphs' if graphs else 'eager'}"] = update_flops(B) / (ms * 1e-3) / 1e12
        print(json.dumps(out), flush=True)
