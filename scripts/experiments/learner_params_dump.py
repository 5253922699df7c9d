"""Dump the flat actor / critic parameters after K fused learner updates on a seeded random ring (A/B bit check of
learner-library variants: run once per HK_LEARNER_LIB, compare the .pt files)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
import torch  # noqa: E402

from hockey_amd.td3 import TD3, Learner, PrioritizedRing, ReplayRing, TD3Config  # noqa: E402

out, B, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dev = "cuda:0"
ring = (PrioritizedRing if len(sys.argv) > 4 else ReplayRing)(1 << 18, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
n = 1 << 18
ring.push(torch.randn(n, 18, device=dev, generator=g), torch.rand(n, 4, device=dev, generator=g) * 2 - 1,
          torch.randn(n, device=dev, generator=g), torch.randn(n, 18, device=dev, generator=g),
          (torch.rand(n, device=dev, generator=g) < 0.01).float())
agent = TD3(TD3Config(), dev, seed=0)
L = Learner(agent, ring, B, graphs=False, fused=True)
L.run(K)
torch.cuda.synchronize()
torch.save({k: torch.cat([p.detach().flatten() for p in getattr(agent, k).parameters()]).cpu()
            for k in ("actor", "critic", "target_actor", "target_critic")}, out)
print("dumped", out)
