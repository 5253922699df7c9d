"""§8 row f3: the GPU-resident TD3 (hockey_amd/td3.py).  CPU tests pin the learner arithmetic against the
reference formulas (rl/td3/learner.py:55-218, rl/utils/torch_utils.py:12-24); the GPU test runs the batched
collection + update loop over real arenas."""
import numpy as np
import pytest
import torch

from hockey_amd.evaluate import load_actor
from hockey_amd.td3 import TD3, ReplayRing, TD3Config, smooth_l1


def test_smooth_l1_matches_reference_formula():
    x, y = torch.tensor([0.0, 0.5, 3.0, -2.0]), torch.tensor([0.2, 0.0, 0.0, 0.0])
    d = x - y
    ref = torch.where(d.abs() < 1, 0.5 * d ** 2, d.abs() - 0.5).mean()
    assert torch.equal(smooth_l1(x, y), ref)


def test_target_and_delayed_soft_update():
    torch.manual_seed(0)
    agent = TD3(TD3Config(batch_size=8), device="cpu")
    s, a = torch.randn(8, 18), torch.rand(8, 4) * 2 - 1
    r, s2, d = torch.randn(8), torch.randn(8, 18), (torch.rand(8) < 0.3).float()
    # clipped double-Q target with smoothing noise (reference compute_target)
    torch.manual_seed(1)
    t = agent.compute_target(s2, r, d)
    torch.manual_seed(1)
    ta = agent.target_actor(s2)
    ta = torch.clamp(ta + torch.clamp(torch.randn_like(ta) * 0.2, -0.3, 0.3), -1, 1)
    q1, q2 = agent.target_critic(s2, ta)
    assert torch.allclose(t, r + 0.99 * (1 - d) * torch.minimum(q1, q2))
    # delayed actor update + Polyak averaging only every policy_update_freq-th step
    before = [p.clone() for p in agent.target_actor.parameters()]
    al, cl = agent.update(s, a, r, s2, d)
    assert al is None and torch.isfinite(cl)
    assert all(torch.equal(b, p) for b, p in zip(before, agent.target_actor.parameters()))
    al, cl = agent.update(s, a, r, s2, d)
    assert al is not None
    assert any(not torch.equal(b, p) for b, p in zip(before, agent.target_actor.parameters()))


def test_checkpoint_layout_roundtrip(tmp_path):
    agent = TD3(device="cpu")
    ck = agent.checkpoint()
    assert {"policy", "critic", "target_policy", "target_critic"} <= set(ck)
    assert {"action_low", "action_high", "action_range", "q1.fc1.weight", "q2.fc3.bias"} <= set(ck["critic"])
    torch.save(ck, tmp_path / "td3_last.pt")
    actor = load_actor(str(tmp_path / "td3_last.pt"), device="cpu")
    x = torch.randn(5, 18)
    assert torch.equal(actor(x), agent.actor(x))


def test_replay_ring_wraps():
    ring = ReplayRing(10, device="cpu")
    for k in range(3):
        ring.push(torch.full((4, 18), float(k)), torch.zeros(4, 4), torch.zeros(4), torch.zeros(4, 18),
                  torch.zeros(4))
    assert len(ring) == 10 and ring.pos == 2
    assert ring.s[0, 0] == 2 and ring.s[9, 0] == 2 and ring.s[7, 0] == 1


@pytest.mark.gpu
def test_batched_training_loop_runs():
    from hockey_amd.td3 import train

    cfg = TD3Config(max_steps=60, start_steps=256, batch_size=128)
    agent, st = train(n_arenas=256, rounds=3, cfg=cfg, updates_per_round=20, seed=3)
    assert st["env_steps"] == 3 * 60 * 256 and st["updates"] == 60
    assert all(torch.isfinite(torch.tensor(st["critic_loss"]))) and len(st["actor_loss"]) == 30
    x = torch.zeros(4, 18, device="cuda:0")
    assert torch.isfinite(agent.actor(x)).all()


@pytest.mark.gpu
def test_c5_training_loop_65536_arenas_with_opponent_mix():
    """BASELINE C5: the TD3 loop fed by 65 536 GPU arenas, player 2 re-drawn per arena and step between the
    strong bot, the weak bot and a self-play snapshot (rl/training/opponent_manager.py:62-91); the pool
    snapshots the actor every 65 536 episodes, i.e. after every round here."""
    from hockey_amd.td3 import train

    n, rounds, steps = 65536, 3, 40
    cfg = TD3Config(max_steps=steps, start_steps=0, batch_size=256)
    agent, st = train(n_arenas=n, rounds=rounds, cfg=cfg, updates_per_round=10, seed=5,
                      curriculum=[(1.0, 0.35, 0.35, 0.30)], self_play_interval=n, pool_size=2)
    assert st["env_steps"] == rounds * steps * n
    assert st["replay_size"] == min(cfg.buffer_size, n * steps * 4)
    assert st["updates"] == rounds * 10 and len(st["actor_loss"]) == rounds * 5
    assert all(np.isfinite(st["critic_loss"])) and all(np.isfinite(st["actor_loss"]))
    assert st["pool_size"] == [1, 2, 2]  # one snapshot per round, capped at pool_size
    first, *later = st["opponents"]
    assert first["self_play"] == 0 and first["strong"] + first["weak"] == steps * n  # empty pool: bots only
    for o in later:
        assert sum(o.values()) == steps * n
        assert abs(o["self_play"] / (steps * n) - 0.30) < 0.01
        assert abs(o["strong"] / (steps * n) - 0.70 * 0.35) < 0.01
    assert torch.isfinite(agent.actor(torch.zeros(4, 18, device="cuda:0"))).all()
