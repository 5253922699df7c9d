"""Where a C5 learner update's time goes: hockey_amd.td3.Learner on a ring of random transitions, batch B (default
16 384, the C5 learner batch), K updates after a warm-up.  Prints ms per update; run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.  Usage: python scripts/learner_profile.py [B] [K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
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
out = {"batch": B, "updates": K, "blas": str(torch.backends.cuda.preferred_blas_library())}
for graphs in (False, True):
    L = Learner(agent, ring, B, graphs=graphs)
    L.run(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.run(K)
    torch.cuda.synchronize()
    out["ms_per_update_graphs" if graphs else "ms_per_update_eager"] = (time.perf_counter() - t0) / K * 1e3
print(json.dumps(out))
