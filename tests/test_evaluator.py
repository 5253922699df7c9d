"""§8 row f4: checkpoint interop (reference TD3 checkpoint layout, weights-only loading) and the reference's
evaluation protocol (rl/utils/evaluator.py:10-35) run on GPU arenas, pinned against the reference
notebook's recorded 1000-game BasicOpponent study (Hockey-Env.ipynb:999, :2088-2154: 150.9 steps/game,
winners +1/0/-1 = 319/368/313).  The reference's own trained checkpoints are not copied into this repo;
`load_actor` reads any such file at run time."""
import numpy as np
import pytest
import torch

from hockey_amd.evaluate import Actor, load_actor, reset_params


def _fake_checkpoint(seed=0):
    g = torch.Generator().manual_seed(seed)
    actor = Actor()
    with torch.no_grad():
        for p in actor.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.2)
    critic = {"action_low": -torch.ones(4), "action_high": torch.ones(4), "q1.fc1.weight": torch.zeros(256, 22)}
    return {"policy": actor.state_dict(), "critic": critic, "target_policy": actor.state_dict(),
            "target_critic": critic}, actor


def test_load_actor_reference_layout(tmp_path):
    ck, ref = _fake_checkpoint()
    path = tmp_path / "td3_best.pt"
    torch.save(ck, path)
    actor = load_actor(str(path), device="cpu")
    x = torch.randn(64, 18)
    assert torch.equal(actor(x), ref(x))
    with pytest.raises(ValueError):
        load_actor({"critic": ck["critic"]}, device="cpu")


def test_reset_protocol_alternates_side():
    p, max_t, one = reset_params(6, 42)
    assert max_t == 250 and list(one) == [False, True, False, True, False, True]
    # puck on player 2's half when one_starts is False (hockey_env.py:381-392)
    assert all((p[i, 2] > 5.0) == (not one[i]) for i in range(6))


@pytest.mark.gpu
@pytest.mark.parametrize("vel_ref", [False, True])
def test_basic_vs_basic_matches_notebook_study(vel_ref):
    """20 000 strong-vs-strong games under either Q1 reading vs the notebook's 1000: outcome split, steps per game,
    both agents' reward per game within 3 combined standard errors, and the 18 obs means jointly (chi-square
    with 18 degrees of freedom below its 0.1 % point, 42.3).  DESIGN.md §4 records the z-scores."""
    from hockey_amd.evaluate import basic_vs_basic_study, study_zscores

    zs = study_zscores(basic_vs_basic_study(20000, seed=0, vel_ref_semantics=vel_ref))
    for key in ("win", "draw", "loss", "steps_per_game", "reward_per_game", "reward2_per_game"):
        assert abs(zs[key]["z"]) < 3.0, (key, zs[key])
    chi2 = sum(o["z"] ** 2 for o in zs["obs_mean"])
    assert chi2 < 42.3, [round(o["z"], 2) for o in zs["obs_mean"]]


@pytest.mark.gpu
def test_checkpoint_policy_evaluation_runs(tmp_path):
    from hockey_amd.evaluate import evaluate

    ck, _ = _fake_checkpoint(1)
    path = tmp_path / "td3_last.pt"
    torch.save(ck, path)
    actor = load_actor(str(path), device="cuda:0")
    r = evaluate(actor, episodes=256, seed=42, weak_opponent=True)
    assert abs(r["win"] + r["draw"] + r["loss"] - 1.0) < 1e-9
    assert 1.0 <= r["mean_length"] <= 251.0 and np.isfinite(r["mean_return"])


def test_checkpoint_fixture_matches_stage3_extraction():
    """tests/golden/checkpoint_actors.npz holds the 12 distinct shipped actors with their recorded evaluations;
    its stage-3 best actor is the one tests/golden/stage3_actor.npz extracted (same eval index, same weights)."""
    import json
    import os

    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(g, "checkpoint_actors.npz"))
    meta = json.loads(str(z["meta"]))
    cks = meta["checkpoints"]
    assert len(cks) == 12 and len(meta["skipped"]) == 1
    assert sum(c["wr_weak"] is not None for c in cks) + len(cks) == 20
    s3 = np.load(os.path.join(g, "stage3_actor.npz"))
    k = [i for i, c in enumerate(cks) if c["name"] == "pretrained/stage_3:best"][0]
    assert cks[k]["eval_index"] == int(s3["best_eval_index"]) and cks[k]["wr_strong"] == float(s3["wr_strong"])
    for name in ("fc1_weight", "fc1_bias", "fc2_weight", "fc2_bias", "fc3_weight", "fc3_bias"):
        assert np.array_equal(z[f"{k}/{name}"], s3[name])
    for c in cks:  # td3_last is the last evaluation of its run; td3_best one of them
        assert 0 <= c["eval_index"] < c["n_evals"] and (c["kind"] == "best" or c["eval_index"] == c["n_evals"] - 1)


def test_recorded_rate_z_statistic():
    from hockey_amd.evaluate import recorded_rate_z

    rng = np.random.default_rng(0)
    p = rng.uniform(0.3, 1.0, 100)
    w = (rng.uniform(size=(64, 100)) < p).astype(np.int8)
    r = recorded_rate_z(w, p.mean())
    assert abs(r["estimate"] - p.mean()) < 0.02 and abs(r["z"]) < 3
    # the conditional se is below the binomial one (placements fixed)
    assert abs(r["z"]) >= abs(r["z_binomial"]) - 1e-12
