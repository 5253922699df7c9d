"""The GPU learner paths of hockey_amd.td3 (BASELINE C5) against the reference's own TD3Learner.

* G9 (hidden 32, batch 64; tests/golden/make_td3_golden.py) through the eager PyTorch learner on the GPU;
* G9b (hidden 256, batch 256, 10 updates: the C5 network shapes) through the fused fp32 MFMA learner
  (hockey_amd.learner_hip, csrc/hk_learner.hip) fed the reference's own batches and target noise;
* the fused learner against the eager learner on the same ring, slots and noise at a C5-like batch.

Tolerances: fp32 with a different summation order (MFMA fma chains vs the reference's BLAS): losses within
1e-4 relative, parameters within 1e-5 absolute after the sequence (Adam steps are ~lr = 4e-4 per update, so a
wrong gradient sign or scale moves a parameter by ~1e-4 per update and fails)."""
import ctypes
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hockey_amd.td3 import TD3, Learner, ReplayRing, TD3Config  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda:0"
LOSS_RTOL, PARAM_ATOL = 1e-4, 1e-5


def _golden_batches():
    sys.path.insert(0, GOLDEN)
    import g9_batches as M
    return M


def _close_params(agent, g, atol):
    bad = []
    for name, net in (("actor", agent.actor), ("critic", agent.critic), ("target_actor", agent.target_actor),
                      ("target_critic", agent.target_critic)):
        for key, v in net.state_dict().items():
            d = float(np.abs(v.detach().cpu().numpy() - g[f"{name}/{key}"]).max())
            if d > atol:
                bad.append((f"{name}/{key}", d))
    return bad


def test_eager_learner_on_gpu_matches_reference_learner_g9():
    M = _golden_batches()
    g9 = np.load(os.path.join(GOLDEN, "g9_td3_learner.npz"))
    agent = TD3(TD3Config(), device="cpu", seed=0, h=M.H)
    gpu = TD3(TD3Config(), device=DEV, seed=0, h=M.H)
    for src, dst in ((agent.actor, gpu.actor), (agent.critic, gpu.critic), (agent.target_actor, gpu.target_actor),
                     (agent.target_critic, gpu.target_critic)):
        dst.load_state_dict(src.state_dict())
    B = 64
    for k in range(M.K):
        s, a, r, s2, d = (t.to(DEV) for t in M.batch(k))
        torch.manual_seed(2000 + k)
        noise = torch.normal(0, 0.2, size=(B, 4))  # the reference's CPU draw, fed to the GPU update
        gpu._noise_override = noise.to(DEV)
        al, cl = gpu.update(s, a, r, s2, d)
        assert abs(float(cl) - g9["critic_loss"][k]) <= LOSS_RTOL * max(1.0, abs(g9["critic_loss"][k])), k
        if al is not None:
            assert abs(float(al) - g9["actor_loss"][k]) <= LOSS_RTOL * max(1.0, abs(g9["actor_loss"][k])), k
    assert not _close_params(gpu, g9, PARAM_ATOL)


def _ring_with(batches, device):
    """A ring holding the concatenated golden batches in order (slot = k * B + i)."""
    n = sum(b[0].shape[0] for b in batches)
    ring = ReplayRing(n, device=device)
    for s, a, r, s2, d in batches:
        ring.push(s.to(device), a.to(device), r.to(device), s2.to(device), d.to(device))
    return ring


def test_fused_learner_matches_reference_learner_g9b():
    """G9b: the reference's TD3Learner at hidden 256 / batch 256 over 10 updates (5 actor updates, 5 Polyak
    averagings) vs the fused MFMA learner fed the same batches (ring slots k*256 .. k*256+255) and the same
    target noise."""
    from hockey_amd.learner_hip import FusedLearner

    M = _golden_batches()
    g = np.load(os.path.join(GOLDEN, "g9b_td3_learner_h256.npz"))
    B, K = int(g["b"]), len(g["critic_loss"])
    batches = [M.batch(k, B) for k in range(K)]
    agent = TD3(TD3Config(), device=DEV, seed=0, h=256)
    init = TD3(TD3Config(), device="cpu", seed=0, h=256)  # the golden's initial weights (CPU init of seed 0)
    for src, dst in ((init.actor, agent.actor), (init.critic, agent.critic), (init.target_actor, agent.target_actor),
                     (init.target_critic, agent.target_critic)):
        dst.load_state_dict(src.state_dict())
    ring = _ring_with(batches, DEV)
    fl = FusedLearner(agent, ring, B)
    acc = torch.zeros(4, dtype=torch.float64, device=DEV)
    fl.set_loss_accumulator(acc)
    for k in range(K):
        idx = torch.arange(k * B, (k + 1) * B, device=DEV)
        train_actor = (k + 1) % 2 == 0
        before = acc.clone()
        fl.update(train_actor, idx=idx, noise=torch.from_numpy(g["noise"][k]).to(DEV))
        d = (acc - before).cpu().numpy()
        assert abs(d[0] - g["critic_loss"][k]) <= LOSS_RTOL * max(1.0, abs(g["critic_loss"][k])), (k, d[0])
        if train_actor:
            assert abs(d[1] - g["actor_loss"][k]) <= LOSS_RTOL * max(1.0, abs(g["actor_loss"][k])), (k, d[1])
    torch.cuda.synchronize()
    bad = _close_params(agent, g, PARAM_ATOL)
    assert not bad, bad[:8]


@pytest.mark.parametrize("batch,updates,per,wd", [(4096, 8, False, 0.0), (16384, 6, False, 0.0),
                                                   (4096, 6, True, 0.0), (4096, 6, False, 1e-3)],
                         ids=["b4096", "b16384_c5", "per", "weight_decay"])
def test_fused_learner_matches_eager_learner_on_ring(batch, updates, per, wd):
    """Fused vs eager (PyTorch) learner from the same weights and ring, with the same torch RNG stream (slots, then
    target noise; the fused learner's torch-RNG mode): critic and actor updates at 4096 samples, at C5's production
    batch of 16 384 (bench c5_round, train(learner_batch=16384)), with prioritized replay (importance weights, the
    weighted smooth-L1, TD-error priorities written back: rl/replay/prioritized_buffer.py, learner.py:163-210; each
    learner on its own copy of the ring, whose weights must agree too) and with Adam's L2 weight decay
    (rl/td3/agent.py:160-167 wd_q / wd_pol)."""
    from hockey_amd.td3 import PrioritizedRing

    cfg = TD3Config(prioritized_replay=per, wd_q=wd, wd_pol=wd)
    torch.manual_seed(7)
    cap = 50_000
    s, s2 = torch.randn(cap, 18, device=DEV), torch.randn(cap, 18, device=DEV)
    a = torch.rand(cap, 4, device=DEV) * 2 - 1
    r, d = torch.randn(cap, device=DEV), (torch.rand(cap, device=DEV) < 0.1).float()
    rings = []
    for _ in range(2 if per else 1):
        ring = PrioritizedRing(cap, device=DEV, beta=cfg.beta) if per else ReplayRing(cap, device=DEV)
        ring.push(s, a, r, s2, d)
        rings.append(ring)
    ring_e, ring_f = rings[0], rings[-1]
    eager, fused = TD3(cfg, device=DEV, seed=3), TD3(cfg, device=DEV, seed=3)
    le = Learner(eager, ring_e, batch, graphs=False, fused=False)
    lf = Learner(fused, ring_f, batch, graphs=False, fused=True, fused_rng="torch")
    for k in range(updates):
        torch.manual_seed(100 + k)
        le._one()
        torch.manual_seed(100 + k)
        lf._one()
    assert eager.train_step == fused.train_step == updates
    ce, ae = le.take_losses()
    cf, af = lf.take_losses()
    assert abs(ce - cf) <= LOSS_RTOL * max(1.0, abs(ce)) and abs(ae - af) <= LOSS_RTOL * max(1.0, abs(ae)), (ce, cf, ae, af)
    worst = 0.0
    for ne, nf in ((eager.actor, fused.actor), (eager.critic, fused.critic), (eager.target_actor, fused.target_actor),
                   (eager.target_critic, fused.target_critic)):
        for (kk, ve), (_, vf) in zip(ne.state_dict().items(), nf.state_dict().items()):
            worst = max(worst, float((ve - vf).abs().max()))
    assert worst <= PARAM_ATOL, worst
    if per:  # the priorities written back agree (same slots, TD errors within fp32 summation order)
        wdiff = (ring_e.w[:cap] - ring_f.w[:cap]).abs() / ring_e.w[:cap].abs().clamp_min(1.0)
        assert float(wdiff.max()) <= 1e-4, float(wdiff.max())


def test_fused_graph_replay_equals_fused_eager():
    """The fused updates captured as a HIP graph (Learner's update pairs) give the same parameters as launching them
    one by one: identical ring entries (sampling cannot matter) and no target noise make both paths deterministic,
    and the kernels reduce in fixed orders (no atomics), so the parameters are bit-identical."""
    nets = []
    for graphs in (False, True):
        torch.manual_seed(0)
        cfg = TD3Config(target_action_noise_scale=0.0)
        agent = TD3(cfg, device=DEV, seed=0)
        ring = ReplayRing(4096, device=DEV)
        g = torch.Generator().manual_seed(1)
        one = [torch.randn(1, 18, generator=g), torch.rand(1, 4, generator=g) * 2 - 1, torch.randn(1, generator=g),
               torch.randn(1, 18, generator=g), torch.zeros(1)]
        ring.push(*(t.expand(4096, *t.shape[1:]).contiguous().to(DEV) for t in one))
        lr = Learner(agent, ring, 2048, graphs=graphs, warm_pairs=1, fused=True)
        for _ in range(3):
            lr.run(8)
        assert agent.train_step == 24 and (lr.graph is not None) == graphs
        torch.cuda.synchronize()
        nets.append(torch.cat([p.detach().flatten() for p in list(agent.actor.parameters()) +
                               list(agent.critic.parameters()) + list(agent.target_actor.parameters()) +
                               list(agent.target_critic.parameters())]))
    assert torch.equal(nets[0], nets[1]), (nets[0] - nets[1]).abs().max()


def test_packs_current_after_updates_with_folded_soft_update():
    """soft_update runs inside the Adam launches (the critic's on actor updates only) and the actor and target
    packs are re-laid in one launch: after critic-only and actor updates every network's operand pack is
    bit-identical to what hkl_pack writes from its weights now, and each optimiser's step count advanced once per
    Adam step."""
    from hockey_amd import learner_hip as LH

    torch.manual_seed(5)
    cfg = TD3Config()
    agent = TD3(cfg, device=DEV, seed=5)
    cap = 8192
    ring = ReplayRing(cap, device=DEV)
    ring.push(torch.randn(cap, 18, device=DEV), torch.rand(cap, 4, device=DEV) * 2 - 1, torch.randn(cap, device=DEV),
              torch.randn(cap, 18, device=DEV), (torch.rand(cap, device=DEV) < 0.1).float())
    lr = Learner(agent, ring, 2048, graphs=False, fused=True)
    f = lr.fused
    for k in range(5):
        f.update(train_actor=k % 2 == 1)
    torch.cuda.synchronize()
    assert int(f.step["critic"]) == 5 and int(f.step["actor"]) == 2
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    for key, nb in f.nets.items():
        fresh = torch.full_like(nb.pack, float("nan"))
        net = LH.Net.from_buffer_copy(nb.net)
        net.pack = fresh.data_ptr()
        LH._check(LH.lib().hkl_pack((LH.Net * 1)(net), 1, None, st), "hkl_pack")
        torch.cuda.synchronize()
        assert torch.equal(nb.pack, fresh), (key, (nb.pack - fresh).abs().max())


def test_fused_learner_runs_without_a_caller_accumulator():
    """FusedLearner used directly (no set_loss_accumulator call) still has a device accumulator for the Adam
    launches' loss sums: two updates run, and its counts read one critic and one actor step per actor update."""
    from hockey_amd.learner_hip import FusedLearner

    cap = 4096
    ring = ReplayRing(cap, device=DEV)
    ring.push(torch.randn(cap, 18, device=DEV), torch.rand(cap, 4, device=DEV) * 2 - 1, torch.randn(cap, device=DEV),
              torch.randn(cap, 18, device=DEV), torch.zeros(cap, device=DEV))
    fl = FusedLearner(TD3(TD3Config(), device=DEV, seed=2), ring, 1024)
    fl.update(train_actor=False)
    fl.update(train_actor=True)
    torch.cuda.synchronize()
    acc = fl._acc.cpu().tolist()
    assert acc[2] == 2.0 and acc[3] == 1.0, acc


def test_fused_tanh_accuracy():
    """The fused kernels' branch-free tanh against torch.tanh over [-20, 20] and near 0: |error| < 2e-7."""
    from hockey_amd.learner_hip import tanh_probe

    x = torch.cat([torch.linspace(-20, 20, 1_000_001, device=DEV), torch.linspace(-1e-3, 1e-3, 100_001, device=DEV)])
    err = (tanh_probe(x).double() - torch.tanh(x.double())).abs().max().item()
    assert err < 2e-7, err


def test_device_sampling_distribution():
    """The fused learner's device sampling (rng="device"): slots uniform over the filled ring (odd / even and halves
    balanced at a fill level past 2^24) and target noise with the N(0, 0.2) moments, clipped to +-0.3."""
    from hockey_amd.learner_hip import FusedLearner

    cfg = TD3Config()
    agent = TD3(cfg, device=DEV, seed=1)
    ring = ReplayRing(1024, device=DEV)
    ring.push(torch.zeros(1024, 18, device=DEV), torch.zeros(1024, 4, device=DEV), torch.zeros(1024, device=DEV),
              torch.zeros(1024, 18, device=DEV), torch.zeros(1024, device=DEV))
    fl = FusedLearner(agent, ring, 16384)
    size = 2 ** 25 + 3
    ring.size_t.fill_(size)  # sampling reads only the fill level
    idx, noise = [], []
    for _ in range(16):
        fl.L.hkl_sample(__import__("ctypes").byref(fl.sio), fl._stream())
        fl.sample_counter += 1
        idx.append(fl.idx.clone())
        noise.append(fl.buf["noise"].clone())
    i, z = torch.cat(idx), torch.cat(noise)
    assert int(i.min()) >= 0 and int(i.max()) < size
    assert abs(float((i % 2 == 1).double().mean()) - 0.5) < 0.01
    assert abs(float((i >= size // 2).double().mean()) - 0.5) < 0.01
    assert len(torch.unique(idx[0])) > 16000  # consecutive counters give different batches
    assert float(z.abs().max()) <= 0.3 + 1e-7
    inner = z[z.abs() < 0.29]
    assert abs(float(inner.mean())) < 0.003
    clip_share = float((z.abs() >= 0.3 - 1e-7).double().mean())
    assert abs(clip_share - 0.1336) < 0.01, clip_share  # P(|N(0, 0.2)| > 0.3) = 2 (1 - Phi(1.5))


def test_wgrad_pair_equals_two_wgrad_launches():
    """hkl_wgrad_pair (dW2 and dW1 tiles of the critics in one launch) writes exactly the slabs -- weight and bias
    column sums -- that one hkl_wgrad call per k width writes."""
    import ctypes

    from hockey_amd.learner_hip import XP, WgJob, _p, lib

    L = lib()
    B, H = 1024, 256
    g = torch.Generator(device=DEV).manual_seed(5)
    dz2 = [torch.randn(B, H, device=DEV, generator=g) for _ in range(2)]
    h1 = [torch.randn(B, H, device=DEV, generator=g) for _ in range(2)]
    dz1 = [torch.randn(B, H, device=DEV, generator=g) for _ in range(2)]
    x0 = torch.randn(B, XP, device=DEV, generator=g)
    C, C1 = B // 512, B // 256
    outs = []
    for pair in (False, True):
        s2 = [torch.full((C, H, H), 7.0, device=DEV) for _ in range(2)]
        b2 = [torch.full((C, H), 7.0, device=DEV) for _ in range(2)]
        s1 = [torch.full((C1, H, XP), 7.0, device=DEV) for _ in range(2)]
        b1 = [torch.full((C1, H), 7.0, device=DEV) for _ in range(2)]
        wide = (WgJob * 2)(*[WgJob(_p(dz2[k]), _p(h1[k]), _p(s2[k]), _p(b2[k])) for k in range(2)])
        narrow = (WgJob * 2)(*[WgJob(_p(dz1[k]), _p(x0), _p(s1[k]), _p(b1[k])) for k in range(2)])
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if pair:
            assert L.hkl_wgrad_pair(wide, 2, narrow, 2, B, st) == 0
        else:
            assert L.hkl_wgrad(wide, 2, 256, B, st) == 0
            assert L.hkl_wgrad(narrow, 2, XP, B, st) == 0
        torch.cuda.synchronize()
        outs.append(s2 + b2 + s1 + b1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # and they are the weight gradients: chunk sums of DZ^T X
    ref = dz2[0].double().T @ h1[0].double()
    assert torch.allclose(outs[1][0].double().sum(0), ref, rtol=1e-4, atol=1e-3)
    # one k-width-256 job (the actor's) takes 256-sample chunks: B / 256 slabs, the same sums
    s2a, b2a = torch.full((B // 256, H, H), 7.0, device=DEV), torch.full((B // 256, H), 7.0, device=DEV)
    s1a, b1a = torch.full((C1, H, XP), 7.0, device=DEV), torch.full((C1, H), 7.0, device=DEV)
    wide = (WgJob * 1)(WgJob(_p(dz2[0]), _p(h1[0]), _p(s2a), _p(b2a)))
    narrow = (WgJob * 1)(WgJob(_p(dz1[0]), _p(x0), _p(s1a), _p(b1a)))
    assert L.hkl_wgrad_pair(wide, 1, narrow, 1, B, st) == 0
    torch.cuda.synchronize()
    assert torch.allclose(s2a.double().sum(0), ref, rtol=1e-4, atol=1e-3)
    assert torch.allclose(b2a.double().sum(0), dz2[0].double().sum(0), rtol=1e-4, atol=1e-3)
    assert torch.equal(s1a, outs[1][4]) and torch.equal(b1a, outs[1][6])


def _pack_reference(w1, w2, w3, n_in, n_out):
    """numpy restatement of hk_learner.hip's operand pack (f1, fp, bp, fo, wa) from torch Linear weights."""
    H = 256
    f1 = np.zeros((16, 64, 8), np.float32)
    fp = np.zeros((16, 16, 64, 4), np.float32)
    bp = np.zeros((16, 16, 64, 4), np.float32)
    fo = np.zeros((16, 64, 4), np.float32)
    wa = np.zeros((256, 4), np.float32)
    lane = np.arange(64)
    lo, hi = lane & 15, lane >> 4
    for ob in range(16):
        for s in range(6):
            c = 4 * s + hi
            ok = c < n_in
            f1[ob, ok, s] = w1[16 * ob + lo[ok], c[ok]]
        for kb in range(16):
            for r in range(4):
                fp[ob, kb, :, r] = w2[16 * ob + lo, 16 * kb + 4 * hi + r]
                bp[kb, ob, :, r] = w2[16 * ob + 4 * hi + r, 16 * kb + lo]
    for kb in range(16):
        for r in range(4):
            ok = lo < n_out
            fo[kb, ok, r] = w3[lo[ok], 16 * kb + 4 * hi[ok] + r]
    if n_in == 22:
        wa[:, :] = w1[:, 18:22]
    assert fp.size == bp.size == 16 * 16 * 64 * 4 and H == 256
    return np.concatenate([f1.ravel(), fp.ravel(), bp.ravel(), fo.ravel(), wa.ravel()])


def test_operand_pack_layout_matches_numpy_restatement():
    """hkl_pack's MFMA operand layouts (f1 / fp / bp / fo / wa, hk_learner.hip) against an independent numpy
    restatement, for an actor (18 -> 256 -> 256 -> 4) and a critic (22 -> 256 -> 256 -> 1)."""
    from hockey_amd.learner_hip import FusedLearner, PACK_FLOATS

    cap = 1024
    ring = ReplayRing(cap, device=DEV)
    ring.push(torch.randn(cap, 18, device=DEV), torch.rand(cap, 4, device=DEV) * 2 - 1, torch.randn(cap, device=DEV),
              torch.randn(cap, 18, device=DEV), torch.zeros(cap, device=DEV))
    fl = FusedLearner(TD3(TD3Config(), device=DEV, seed=9), ring, 256)
    torch.cuda.synchronize()
    for key in ("actor", "q1"):
        nb = fl.nets[key]
        f1, f2, f3 = nb.m.fc1, nb.m.fc2, nb.m.fc3
        ref = _pack_reference(f1.weight.detach().cpu().numpy(), f2.weight.detach().cpu().numpy(),
                              f3.weight.detach().cpu().numpy(), f1.in_features, f3.out_features)
        assert ref.size == PACK_FLOATS
        got = nb.pack.cpu().numpy()
        assert np.array_equal(got, ref), (key, int(np.argmax(got != ref)))


def test_eager_update_and_load_fail_loudly_with_a_fused_learner_attached():
    """a FusedLearner owns its agent's Adam moments and MFMA operand packs, so an eager agent.update()
    (split optimiser state) or agent.load() (weights the packs would not see) afterwards raises instead of training
    on stale state; a second FusedLearner on the same agent is refused too."""
    from hockey_amd.learner_hip import FusedLearner

    agent = TD3(TD3Config(), device=DEV, seed=4)
    ring = ReplayRing(4096, device=DEV)
    ring.push(torch.zeros(4096, 18, device=DEV), torch.zeros(4096, 4, device=DEV), torch.zeros(4096, device=DEV),
              torch.zeros(4096, 18, device=DEV), torch.zeros(4096, device=DEV))
    ck = agent.checkpoint()
    FusedLearner(agent, ring, 256)
    s = torch.zeros(8, 18, device=DEV)
    with pytest.raises(RuntimeError, match="fused learner"):
        agent.update(s, torch.zeros(8, 4, device=DEV), torch.zeros(8, device=DEV), s, torch.zeros(8, device=DEV))
    with pytest.raises(RuntimeError, match="fused learner"):
        agent.load(ck)
    with pytest.raises(RuntimeError, match="fused learner"):
        FusedLearner(agent, ring, 256)


def test_resume_from_stage1_best_on_the_gpu_with_the_fused_learner():
    """The Stage II resume (scripts/noise_study.py --protocol stage2): train(resume_from=stage1_best_full.npz) on GPU
    arenas with the fused learner attached.  Before any update the agent's four networks are the reference's stage-1
    best bit for bit and the fused learner's operand packs are those of these weights (its first critic / actor updates
    from the resumed weights equal the eager learner's from the same weights: fused == eager after 4 updates), and
    the resumed actor plays the weak bot like the stage-1 best checkpoint (recorded 0.99, simulated 0.967: >= 0.9 over
    200 games)."""
    from hockey_amd.evaluate import evaluate
    from hockey_amd.td3 import load_checkpoint, train

    ck = load_checkpoint(os.path.join(GOLDEN, "stage1_best_full.npz"))
    cfg = TD3Config(max_steps=20, curriculum_name="stage2", use_self_play=False, start_steps=0)
    agent, st = train(n_arenas=256, rounds=1, cfg=cfg, device=DEV, seed=11, updates_per_round=0, fused=True,
                      resume_from=ck, learner_batch=256)
    got = agent.checkpoint()
    for net in ck:
        for k, v in ck[net].items():
            assert torch.equal(got[net][k].cpu(), v), (net, k)
    agent.actor.eval()
    w = evaluate(agent.actor, episodes=200, seed=420, weak_opponent=True, device=DEV)
    assert w["win"] >= 0.9, w
    # fused from the resumed weights == eager from the same weights
    torch.manual_seed(3)
    cap = 20_000
    ring = ReplayRing(cap, device=DEV)
    ring.push(torch.randn(cap, 18, device=DEV), torch.rand(cap, 4, device=DEV) * 2 - 1, torch.randn(cap, device=DEV),
              torch.randn(cap, 18, device=DEV), (torch.rand(cap, device=DEV) < 0.1).float())
    eager, fused = TD3(TD3Config(), device=DEV, seed=1), TD3(TD3Config(), device=DEV, seed=1)
    eager.load(ck)
    fused.load(ck)
    le = Learner(eager, ring, 1024, graphs=False, fused=False)
    lf = Learner(fused, ring, 1024, graphs=False, fused=True, fused_rng="torch")
    for k in range(4):
        torch.manual_seed(50 + k)
        le._one()
        torch.manual_seed(50 + k)
        lf._one()
    worst = max(float((a - b).abs().max()) for ne, nf in ((eager.actor, fused.actor), (eager.critic, fused.critic))
                for a, b in zip(ne.state_dict().values(), nf.state_dict().values()))
    assert worst <= PARAM_ATOL, worst
