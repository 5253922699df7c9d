"""Behavioural pin of world.Step against every checkpoint the reference ships.

Box2D is absent here, so the restated physics cannot be pinned per trajectory.  What the reference does
hold is 12 trained actors with the win rates its own evaluator recorded for them (100 episodes per opponent, reset
seeds run_seed + i, rl/utils/evaluator.py:10-35): pretrained/stage_{1,2,3}, runs/* (td3_best and td3_last each;
byte-identical copies once; the cluster run never evaluated).  Each actor is played on R replicas of the reference's
100 placements against the fused BasicOpponent (hockey_amd.evaluate.checkpoint_pins), and each recorded rate gets a
z-score against the simulator's conditional win probabilities of those placements (recorded_rate_z).

Assertions (20 recorded rates):
* rates that no selection touched -- every td3_last rate, and the stage-1 best checkpoint's strong rate (stage 1
  selected on the weak rate): |z| < 3 each, and jointly sum z^2 below the chi-square 0.1 % point;
* rates behind a best-checkpoint selection (the recorded value is the running maximum of a noisy series, so it sits
  above the policy's own rate): z > -3 (the simulator's rate may not exceed the recorded one by more than chance),
  and z below the Bonferroni bound over the run's evaluations, Phi^-1(1 - 0.01 / n_evals) (3.29 at 50, 3.54 at 125):
  a selected maximum exceeds its policy's rate by no more than the largest of n_evals noise draws.
DESIGN.md §4 lists every z (profiles/r04/checkpoint_pins.json)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
stats = pytest.importorskip("scipy.stats")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_every_shipped_checkpoint_reproduces_its_recorded_win_rates():
    from hockey_amd.evaluate import checkpoint_pins

    rows = checkpoint_pins(os.path.join(GOLDEN, "checkpoint_actors.npz"), replicas=64)
    out = os.environ.get("HK_PIN_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)
    for r in rows:
        print(f"{r['checkpoint']:62s} {r['opponent']:6s} rec {r['recorded']:.2f} sim {r['estimate']:.4f} "
              f"z {r['z']:+.2f} (binomial {r['z_binomial']:+.2f}){' selected' if r['selected'] else ''}")
    assert len(rows) == 20
    free = [r for r in rows if not r["selected"]]
    sel = [r for r in rows if r["selected"]]
    assert len(free) == 11 and len(sel) == 9
    for r in free:
        assert abs(r["z"]) < 3, r
    chi2 = sum(r["z"] ** 2 for r in free)
    assert chi2 < stats.chi2.ppf(0.999, len(free)), (chi2, len(free))
    for r in sel:
        bound = stats.norm.ppf(1 - 0.01 / r["n_evals"])
        assert -3 < r["z"] < bound, (r, bound)
    # the same rule as one verdict (hockey_amd.evaluate.pin_acceptance): the CPU power study
    # (scripts/pin_power_study.py, tests/test_pin_power.py) applies exactly this to deliberately wrong physics
    from hockey_amd.evaluate import pin_acceptance
    assert pin_acceptance(rows)["passed"]
