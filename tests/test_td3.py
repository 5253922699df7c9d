"""§8 row f3: the GPU-resident TD3 (hockey_amd/td3.py).  CPU tests pin the learner arithmetic against the
reference formulas (rl/td3/learner.py:55-218, rl/utils/torch_utils.py:12-24); the GPU test runs the batched
collection + update loop over real arenas."""
import math

import numpy as np
import pytest
import torch

import os

from hockey_amd.evaluate import load_actor
from hockey_amd.noise import GaussianNoise, OrnsteinUhlenbeckNoise, PinkNoise, UniformNoise, make_noise
from hockey_amd.td3 import (REFERENCE_REPLAY_RATIO, TD3, Learner, PrioritizedRing, ReplayRing, TD3Config, smooth_l1,
                            updates_for)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_smooth_l1_matches_reference_formula():
    x, y = torch.tensor([0.0, 0.5, 3.0, -2.0]), torch.tensor([0.2, 0.0, 0.0, 0.0])
    d = x - y
    ref = torch.where(d.abs() < 1, 0.5 * d ** 2, d.abs() - 0.5).mean()
    assert torch.equal(smooth_l1(x, y), ref)


def test_learner_matches_reference_learner_g9():
    """G9 (tests/golden/make_td3_golden.py): the reference's own TD3Learner (rl/td3/learner.py) run on a seeded
    batch sequence from the same initial weights.  hockey_amd.td3 reproduces its losses and final actor /
    critic / target parameters (float32 rounding only: Polyak averaging is fused)."""
    import sys

    sys.path.insert(0, GOLDEN)
    from g9_batches import B, H, K, batch

    g9 = np.load(os.path.join(GOLDEN, "g9_td3_learner.npz"))
    agent = TD3(TD3Config(), device="cpu", seed=0, h=H)
    for k in range(K):
        torch.manual_seed(2000 + k)
        al, cl = agent.update(*batch(k))
        assert abs(float(cl) - g9["critic_loss"][k]) <= 1e-5 * max(1.0, abs(g9["critic_loss"][k])), k
        if al is None:
            assert np.isnan(g9["actor_loss"][k])
        else:
            assert abs(float(al) - g9["actor_loss"][k]) <= 1e-5 * max(1.0, abs(g9["actor_loss"][k])), k
    for name, net in (("actor", agent.actor), ("critic", agent.critic), ("target_actor", agent.target_actor),
                      ("target_critic", agent.target_critic)):
        for key, v in net.state_dict().items():
            np.testing.assert_allclose(v.numpy(), g9[f"{name}/{key}"], rtol=0, atol=1e-6, err_msg=f"{name}/{key}")
    assert B == 64


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
    assert len(ring) == 10 and ring.pos == 2 and float(ring.size_t) == 10
    assert ring.s[0, 0] == 2 and ring.s[9, 0] == 2 and ring.s[7, 0] == 1
    i = ring.sample_indices(10_000)
    assert int(i.min()) == 0 and int(i.max()) == 9  # (rand * size).astype(int) over the filled slots


def test_uniform_sampling_reaches_every_slot_past_2_24():
    """Fill levels past 2^24 (a C5 round stores 65 536 x 500 = 32.8 M transitions): float64 uniforms and an
    exact integer fill level keep every slot reachable (float32 would draw only even slots there) and never
    index past the filled range."""
    ring = ReplayRing(4, device="cpu")
    size = 2 ** 25 + 3
    ring.size_t.fill_(size)  # sampling reads only the fill level
    torch.manual_seed(0)
    i = ring.sample_indices(1_000_000)
    assert int(i.min()) >= 0 and int(i.max()) <= size - 1
    odd = float((i % 2 == 1).double().mean())
    assert abs(odd - 0.5) < 0.005, odd
    hi = float((i >= size // 2).double().mean())
    assert abs(hi - 0.5) < 0.005, hi


class _RefPER:
    """rl/replay/prioritized_buffer.py:6-69 weight bookkeeping, restated with numpy (one push at a time)."""

    def __init__(self, cap, init_weight=1e8):
        self.cap, self.size, self.cur = cap, 0, 0
        self.weights = np.full(cap, init_weight, np.float32)

    def push(self):
        self.size = min(self.size + 1, self.cap)
        self.cur = (self.cur + 1) % self.cap
        self.weights[self.cur - 1] = np.max(self.weights[: self.size])

    def probs(self):
        w = np.maximum(np.nan_to_num(self.weights[: self.size], nan=0.0, posinf=0.0, neginf=0.0), 1e-6)
        return w / w.sum()


def test_prioritized_ring_matches_reference_bookkeeping():
    cap = 50
    ring, ref = PrioritizedRing(cap, device="cpu", beta=0.15), _RefPER(cap)
    rng = np.random.default_rng(0)
    for k in range(9):
        n = int(rng.integers(1, 17))
        ring.push(torch.randn(n, 18), torch.randn(n, 4), torch.randn(n), torch.randn(n, 18), torch.zeros(n))
        for _ in range(n):
            ref.push()
        assert np.array_equal(ring.w.numpy(), ref.weights), k
        # sample, then the sampled slots take their TD-error priorities (learner.update_critic)
        s, a, r, s2, d, iw = ring.sample(8)
        inds = ring.last.numpy()
        assert inds.max() < ref.size
        p_b = ref.weights[inds] / ref.weights[inds].sum()  # learner._compute_importance_weights
        w = (1 / (p_b * ref.size)) ** 0.15
        assert np.allclose(iw.numpy(), w / w.max(), rtol=1e-5)
        td = torch.rand(8) * 3
        ring.update_priorities(td)
        ref.weights[inds] = np.clip(td.numpy(), 1e-6, 1e6)
        assert np.array_equal(ring.w.numpy(), ref.weights)
    # sampling follows P(i) = w_i / sum(w) over the filled slots
    ring.w[:] = 1.0
    ring.w[3] = 40.0
    hits = torch.cat([ring.sample_indices(4096) for _ in range(8)])
    p = ring.w[:ring.size].double() / ring.w[:ring.size].double().sum()
    assert abs(float((hits == 3).double().mean()) - float(p[3])) < 0.02
    assert int(hits.max()) < ring.size


def test_weighted_smooth_l1():
    x, y, w = torch.tensor([0.0, 0.5, 3.0, -2.0]), torch.tensor([0.2, 0.0, 0.0, 0.0]), torch.tensor([1., 2., 3., 4.])
    d = x - y
    ref = torch.where(d.abs() < 1, 0.5 * w * d ** 2, (d.abs() - 0.5) * w).mean()
    assert torch.equal(smooth_l1(x, y, w), ref)


def test_noise_processes_match_reference_formulas():
    n, dim = 4096, 4
    g = GaussianNoise(n, dim, 0.2, "cpu", 0)
    x = g()
    assert x.shape == (n, dim) and abs(float(x.std()) - 0.2) < 0.01
    u = make_noise("uniform", n, dim, 0.2, 500, "cpu", 0)
    x = u()
    assert float(x.abs().max()) <= 0.2 * np.sqrt(3) and abs(float(x.std()) - 0.2) < 0.01
    # OU: x <- x + theta (mu - x) dt + sigma sqrt(dt) N(0,1), dt = 1.0 as the agent builds it, reset to 0
    ou = make_noise("ornstein-uhlenbeck", 3, dim, 0.2, 500, "cpu", 7)
    assert isinstance(ou, OrnsteinUhlenbeckNoise) and ou.dt == 1.0 and ou.theta == 0.15
    twin = torch.Generator()
    twin.manual_seed(7 + 0xA0)
    xr = torch.zeros(3, dim)
    for _ in range(5):
        xr = xr + 0.15 * (0.0 - xr) * 1.0 + 0.2 * 1.0 * torch.randn((3, dim), generator=twin)
        assert torch.allclose(ou(), xr)
    ou.reset()
    assert torch.equal(ou.x, torch.zeros(3, dim))
    # pink: unit-variance blocks of seq_len steps with a 1/f power spectrum, renewed when used up
    pk = make_noise("pink", 512, dim, 0.3, 256, "cpu", 1)
    assert isinstance(pk, PinkNoise)
    blk = pk.block
    assert blk.shape == (512, dim, 256)
    assert torch.allclose(blk.std(dim=-1, unbiased=False), torch.ones(512, dim, dtype=blk.dtype), atol=1e-9)
    psd = (torch.fft.rfft(blk, dim=-1).abs() ** 2).mean(dim=(0, 1))
    f = torch.fft.rfftfreq(256, dtype=torch.float64)
    slope = np.polyfit(np.log(f[2:100].numpy()), np.log(psd[2:100].numpy()), 1)[0]
    assert -1.25 < slope < -0.75  # power ~ 1/f
    first = pk()
    assert torch.allclose(first, (0.3 * blk[:, :, 0]).float())
    for _ in range(255):
        pk()
    pk()  # the 257th draw starts a new block
    assert pk.idx == 1 and not torch.equal(pk.block, blk)
    assert isinstance(make_noise("gaussian", 1, 4, 0.2, 10, "cpu"), GaussianNoise)
    assert isinstance(make_noise("uniform", 1, 4, 0.2, 10, "cpu"), UniformNoise)
    with pytest.raises(ValueError):
        make_noise("brown", 1, 4, 0.2, 10, "cpu")


def test_noise_schedule_and_random_phase():
    cfg = TD3Config(start_steps=10, use_noise_annealing=True, noise_anneal_mode="linear", noise_min_scale=0.07)
    agent = TD3(cfg, device="cpu", max_total_steps=100, n_envs=4)
    agent.total_steps = 50
    assert math.isclose(agent.noise_scale(), 0.1)
    agent.total_steps = 99
    assert agent.noise_scale() == 0.07
    agent.cfg.noise_anneal_mode = "exp"
    agent.total_steps = 20
    assert math.isclose(agent.noise_scale(), 0.2 * 0.1 ** 0.2)
    agent.cfg.use_noise_annealing = False
    assert agent.noise_scale() == 0.2
    # get_action: arena i of a batch is call total_steps + i + 1; random while that is below start_steps
    agent = TD3(TD3Config(start_steps=10, action_noise_scale=1e-12), device="cpu", n_envs=4)
    obs = torch.zeros(4, 18)
    agent.act(obs)  # calls 1..4: random
    a = agent.act(obs)  # calls 5..8: random
    assert agent.total_steps == 8
    a = agent.act(obs)  # calls 9..12: 9 random, 10..12 the (noise-free) actor
    pol = agent.actor(obs)
    assert not torch.allclose(a[0], pol[0]) and torch.allclose(a[1:], pol[1:])
    assert torch.equal(agent.act(obs, noise=False), pol) and agent.total_steps == 12


def test_stage1_config_and_replay_ratio():
    cfg = TD3Config.from_json(os.path.join(GOLDEN, "stage1_config.json"))
    assert (cfg.buffer_size, cfg.noise_min_scale, cfg.use_self_play, cfg.prioritized_replay) == (100_000, 0.1, False,
                                                                                                  False)
    assert math.isclose(cfg.replay_ratio, 32 * 256 / 500)
    assert updates_for(cfg, 1, 500) == 32  # train_iters per 500-step episode at the reference's batch
    assert updates_for(cfg, 20, 500) == 640
    assert updates_for(cfg, 65536, 50, batch=16384) == round(16.384 * 65536 * 50 / 16384)
    short = TD3Config(max_steps=50)  # a 50-step round at the reference's ratio, not 32 updates per 50 steps
    assert updates_for(short, 65536, 50, batch=16384, ratio=REFERENCE_REPLAY_RATIO) == 3277


def test_learner_eager_updates_on_cpu():
    torch.manual_seed(0)
    agent = TD3(TD3Config(batch_size=16), device="cpu")
    for ring in (ReplayRing(64, device="cpu"), PrioritizedRing(64, device="cpu")):
        ring.push(torch.randn(40, 18), torch.rand(40, 4) * 2 - 1, torch.randn(40), torch.randn(40, 18),
                  (torch.rand(40) < 0.2).float())
        lr = Learner(agent, ring, 16, graphs=True)  # no GPU: eager
        before = [p.clone() for p in agent.actor.parameters()]
        t0 = agent.train_step
        lr.run(5)
        assert agent.train_step == t0 + 5
        cl, al = lr.take_losses()
        assert np.isfinite(cl) and np.isfinite(al)
        assert any(not torch.equal(b, p) for b, p in zip(before, agent.actor.parameters()))
    assert float(ring.w[:40].max()) < 1e8  # sampled priorities were updated


@pytest.mark.gpu
def test_batched_training_loop_runs():
    from hockey_amd.td3 import train

    cfg = TD3Config(max_steps=60, start_steps=256, batch_size=128)
    agent, st = train(n_arenas=256, rounds=3, cfg=cfg, updates_per_round=20, seed=3)
    assert st["env_steps"] == 3 * 60 * 256 and st["updates"] == 60 and agent.train_step == 60
    assert all(np.isfinite(st["critic_loss"])) and len(st["actor_loss"]) == 3
    x = torch.zeros(4, 18, device="cuda:0")
    assert torch.isfinite(agent.actor(x)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("noise,per", [("ornstein-uhlenbeck", True), ("pink", False), ("uniform", True)])
def test_learner_options_on_gpu(noise, per):
    """The reference's learner options (rl/td3/agent.py:128-156 noise kinds, rl/replay/prioritized_buffer.py)
    through the batched loop: updates run (graph-captured pairs), priorities move off their initial 1e8."""
    from hockey_amd.td3 import train

    cfg = TD3Config(max_steps=40, start_steps=0, batch_size=256, noise_mode=noise, prioritized_replay=per,
                    use_self_play=False, curriculum_name="stage1")
    agent, st = train(n_arenas=128, rounds=3, cfg=cfg, seed=4)
    assert st["updates"] == 3 * updates_for(cfg, 128, 40)
    assert all(np.isfinite(st["critic_loss"])) and all(np.isfinite(st["actor_loss"]))
    assert st["opponents"][0]["weak"] == 40 * 128  # stage-1 curriculum: weak bot only


@pytest.mark.gpu
def test_graph_captured_updates_equal_eager_updates():
    """Learner: the HIP-graph replay of an update pair performs the same arithmetic as the eager updates.  With
    identical ring entries (sampling cannot matter) and no target smoothing noise, both paths are
    deterministic, so the parameters after 40 updates agree."""
    dev = "cuda:0"
    nets = []
    for graphs in (False, True):
        torch.manual_seed(0)
        cfg = TD3Config(batch_size=64, target_action_noise_scale=0.0)
        agent = TD3(cfg, device=dev, seed=0)
        ring = ReplayRing(512, device=dev)
        g = torch.Generator().manual_seed(1)
        one = [torch.randn(1, 18, generator=g), torch.rand(1, 4, generator=g) * 2 - 1, torch.randn(1, generator=g),
               torch.randn(1, 18, generator=g), torch.zeros(1)]
        ring.push(*(t.expand(512, *t.shape[1:]).contiguous().to(dev) for t in one))
        lr = Learner(agent, ring, 64, graphs=graphs, warm_pairs=2)
        for _ in range(4):
            lr.run(10)
        assert agent.train_step == 40
        assert (lr.graph is not None) == graphs
        nets.append(torch.cat([p.detach().flatten() for p in list(agent.actor.parameters()) +
                               list(agent.critic.parameters()) + list(agent.target_actor.parameters())]))
    assert torch.allclose(nets[0], nets[1], rtol=1e-5, atol=1e-6), (nets[0] - nets[1]).abs().max()


@pytest.mark.gpu
def test_c5_training_loop_65536_arenas_with_opponent_mix():
    """BASELINE C5: the TD3 loop fed by 65 536 GPU arenas, player 2 re-drawn per arena and step between the
    strong bot, the weak bot and a self-play snapshot (rl/training/opponent_manager.py:62-91); the pool
    snapshots the actor every 65 536 episodes, i.e. after every round here.  The ring holds a whole round of
    every arena; the updates run at the reference's replay ratio with a large batch."""
    from hockey_amd.td3 import train

    n, rounds, steps = 65536, 3, 40
    cfg = TD3Config(max_steps=steps, start_steps=0, batch_size=256)
    agent, st = train(n_arenas=n, rounds=rounds, cfg=cfg, seed=5, learner_batch=16384,
                      replay_ratio=REFERENCE_REPLAY_RATIO, curriculum=[(1.0, 0.35, 0.35, 0.30)],
                      self_play_interval=n, pool_size=2)
    assert st["env_steps"] == rounds * steps * n
    assert st["replay_capacity"] == n * steps and st["replay_size"] == n * steps
    ups = updates_for(cfg, n, steps, batch=16384, ratio=REFERENCE_REPLAY_RATIO)
    assert ups == round(16.384 * n * steps / 16384) and st["updates"] == rounds * ups
    assert abs(st["replay_ratio"] - 16.384) < 0.01
    assert all(np.isfinite(st["critic_loss"])) and all(np.isfinite(st["actor_loss"]))
    assert st["pool_size"] == [1, 2, 2]  # one snapshot per round, capped at pool_size
    first, *later = st["opponents"]
    assert first["self_play"] == 0 and first["strong"] + first["weak"] == steps * n  # empty pool: bots only
    for o in later:
        assert sum(o.values()) == steps * n
        assert abs(o["self_play"] / (steps * n) - 0.30) < 0.01
        assert abs(o["strong"] / (steps * n) - 0.70 * 0.35) < 0.01
    assert torch.isfinite(agent.actor(torch.zeros(4, 18, device="cuda:0"))).all()


def test_collection_loop_on_host_build_stores_what_the_kernel_applied():
    """hockey_amd.td3.train's collection on the kernel source's host build (tests/hostcheck.py): every stored
    transition's action is the one the kernel applied to player 1 (clipped to [-1, 1]), its next obs is the
    step's obs, the next transition starts from it, player 2 is the weak bot (stage-1 curriculum), and the
    ring holds exactly the stored transitions."""
    from hostcheck import HostTorchEnv

    from hockey_amd.td3 import train

    n, steps = 8, 40
    env = HostTorchEnv(n, policies=("external", "external"))
    seen = []

    def on_step(obs, a, r, o2, d, res):
        seen.append((obs.clone(), a.clone(), r.clone(), o2.clone(), d.clone(), res.actions.clone()))

    cfg = TD3Config(max_steps=steps, start_steps=100, batch_size=32, use_self_play=False,
                    curriculum_name="stage1")
    agent, st = train(n_arenas=n, rounds=2, cfg=cfg, device="cpu", seed=3, env=env, on_step=on_step,
                      graphs=False, updates_per_round=4)
    assert len(seen) == 2 * steps and st["updates"] == 8 and st["replay_size"] == 2 * steps * n
    for t, (obs, a, r, o2, d, applied) in enumerate(seen):
        assert torch.equal(applied[:, :4], torch.clamp(a, -1, 1)), t
        assert torch.all(applied[:, 4:7].abs().sum(1) > 0)  # the fused weak bot acts for player 2
        if t % steps:
            assert torch.equal(obs, seen[t - 1][3]), t  # transitions chain within an episode
    assert st["opponents"][0] == {"strong": 0, "weak": steps * n, "self_play": 0}


def test_episode_end_done_stores_only_running_episodes():
    """episode_end="done": an arena's transitions stop at its done step (the last stored one carries done=1),
    the agent's step count advances only for running episodes, and the round ends once every episode has."""
    from hostcheck import HostTorchEnv

    from hockey_amd.td3 import train

    n = 8
    env = HostTorchEnv(n, policies=("external", "external"))
    seen = []
    cfg = TD3Config(max_steps=400, start_steps=10 ** 9, batch_size=32, use_self_play=False, curriculum_name="stage1")
    agent, st = train(n_arenas=n, rounds=1, cfg=cfg, device="cpu", seed=5, env=env, graphs=False,
                      updates_per_round=0, episode_end="done",
                      on_step=lambda o, a, r, o2, d, res: seen.append((d.clone(), res.done.clone())))
    stored = sum(int(d.numel()) for d, _ in seen)
    assert st["replay_size"] == stored == st["env_steps"] == agent.total_steps
    # each stored step holds exactly the arenas not yet done; the round stops at the last done (time limit 251)
    running = n
    for d, full in seen:
        assert d.numel() == running
        running -= int(d.sum())
    assert running == 0 and len(seen) <= 251
    assert stored < n * len(seen) or len(seen) == 251


def test_resume_from_loads_all_four_networks():
    """train(resume_from=...) = rl/main.py:66-67 agent.load: policy, critic and both targets come from the checkpoint
    (tests/golden/stage1_best_full.npz, the reference's stage-1 best = the Stage II resume point); with no update the
    trained agent's checkpoint() is the fixture bit for bit, and the resumed actor acts from the first step."""
    from hostcheck import HostTorchEnv

    from hockey_amd.td3 import load_checkpoint, train

    ck = load_checkpoint(os.path.join(GOLDEN, "stage1_best_full.npz"))
    assert set(ck) == {"policy", "critic", "target_policy", "target_critic"}
    n = 4
    env = HostTorchEnv(n, policies=("external", "external"))
    cfg = TD3Config(max_steps=5, start_steps=0, batch_size=32, use_self_play=False, curriculum_name="stage2",
                    use_noise_annealing=False, action_noise_scale=1e-30)
    acts = []
    agent, st = train(n_arenas=n, rounds=1, cfg=cfg, device="cpu", seed=7, env=env, graphs=False,
                      updates_per_round=0, resume_from=ck, on_step=lambda o, a, r, o2, d, res: acts.append((o, a)))
    got = agent.checkpoint()
    for net in ck:
        assert set(got[net]) == set(ck[net]), net
        for k, v in ck[net].items():
            assert torch.equal(got[net][k], v), (net, k)
    o, a = acts[0]
    with torch.no_grad():
        assert torch.allclose(a, agent.actor(o), atol=1e-6)


def test_learner_matches_reference_learner_g9b_wide():
    """G9b (hidden 256, batch 256: the C5 network shapes; tests/golden/make_td3_golden.py --wide): the eager learner on
    the CPU reproduces the reference's TD3Learner losses and parameters (float32 rounding only)."""
    import sys

    sys.path.insert(0, GOLDEN)
    import g9_batches as M

    g = np.load(os.path.join(GOLDEN, "g9b_td3_learner_h256.npz"))
    gb = int(g["b"])
    agent = TD3(TD3Config(), device="cpu", seed=0, h=int(g["h"]))
    for k in range(len(g["critic_loss"])):
        torch.manual_seed(2000 + k)
        al, cl = agent.update(*M.batch(k, gb))
        assert abs(float(cl) - g["critic_loss"][k]) <= 1e-5 * max(1.0, abs(g["critic_loss"][k])), k
        if al is not None:
            assert abs(float(al) - g["actor_loss"][k]) <= 1e-5 * max(1.0, abs(g["actor_loss"][k])), k
    for name, net in (("actor", agent.actor), ("critic", agent.critic), ("target_actor", agent.target_actor),
                      ("target_critic", agent.target_critic)):
        for key, v in net.state_dict().items():
            np.testing.assert_allclose(v.numpy(), g[f"{name}/{key}"], rtol=0, atol=1e-6, err_msg=f"{name}/{key}")
