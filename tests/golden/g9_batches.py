"""The seeded batch sequence of the G9 / G9b learner goldens (g9_td3_learner.npz, g9b_td3_learner_h256.npz).

Plain data generation, split out of the build-container generator so the tests that feed these batches to the
learner (tests/test_td3.py, tests/test_gpu_learner.py) import nothing that touches the reference: update k draws
its batch from torch.Generator().manual_seed(1000 + k) in the order s, a, r, s2, d."""
import torch

H, B, K = 32, 64, 30  # G9: hidden size, batch, updates


def batch(k, b=B):
    g = torch.Generator().manual_seed(1000 + k)
    s = torch.randn(b, 18, generator=g)
    a = torch.rand(b, 4, generator=g) * 2 - 1
    r = torch.randn(b, generator=g) * 3
    s2 = torch.randn(b, 18, generator=g)
    d = (torch.rand(b, generator=g) < 0.15).float()
    return s, a, r, s2, d
