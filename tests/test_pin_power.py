"""Power of the behavioural pin on world.Step (SURVEY §8 rows a7 / c).  CPU only: the oracle.

profiles/r05/pin_power_r64.json is scripts/pin_power_study.py's run of the checkpoint pin (the reference's 12 shipped
actors x its 100 evaluation placements x R = 64, 20 recorded win rates) on the CPU oracle -- which the kernel equals bit
for bit -- for the pinned restatement and for variants, four of them deliberately wrong physics.  Asserted here:

* the committed verdicts are what hockey_amd.evaluate.pin_acceptance (the GPU pin's own rule) says of the committed
  rows: base passes, and wrong physics fails (SolveTOI skipped; restitution mixed by min) -- the pin has power;
* the pin's resolution: a uniform shift of the free rates by ~2-3 win-rate points fails it, while the solver-detail
  variants (iteration counts, restitution threshold, friction mixing) move the trained policies' rates by < 1 point
  on average, which no outcome statistic at the reference's 100 episodes per rate can resolve;
* live: the study's protocol code, re-run at a small size, reproduces the direction and size of the no-TOI shift.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILE = os.path.join(ROOT, "profiles", "r05", "pin_power_r64.json")


@pytest.fixture(scope="module")
def study():
    with open(PROFILE) as f:
        return json.load(f)


def test_committed_verdicts_follow_the_pin_rule(study):
    from hockey_amd.evaluate import pin_acceptance

    v = study["variants"]
    assert study["replicas"] == 64 and len(v["base"]["rows"]) == 20
    for name, rec in v.items():
        acc = pin_acceptance(rec["rows"])
        assert acc["passed"] == rec["acceptance"]["passed"], name
        assert abs(acc["free_chi2"] - rec["acceptance"]["free_chi2"]) < 1e-2, name  # rows are stored to 5 digits
    assert v["base"]["acceptance"]["passed"]
    failed_wrong = [n for n, r in v.items() if r["wrong_physics"] and not r["acceptance"]["passed"]]
    assert "no_toi" in failed_wrong and "rest_min" in failed_wrong, failed_wrong


def test_pin_resolution_against_solver_detail_variants(study):
    s = study["summary"]
    res = s["_pin_resolution_pts"]
    assert res["up"] < 4 and res["down"] < 4  # a few points of systematic shift fail the pin
    for name in ("iters_8_3", "rest_thresh0", "arith_fric", "reverse", "no_block", "no_sleep", "live_q1"):
        assert abs(s[name]["shift_mean_pts"]) < 1.0, (name, s[name])  # below the resolution: invisible to any pin
    assert s["no_toi"]["shift_mean_pts"] < -10 and s["rest_min"]["shift_mean_pts"] < -50


def test_live_protocol_reproduces_the_no_toi_shift():
    sys.path[:0] = [os.path.join(ROOT, "scripts"), os.path.join(ROOT, "oracle")]
    import oracle as O
    import pin_power_study as P

    meta, actors = P.load_actors()
    k = next(i for i, c in enumerate(meta["checkpoints"]) if c["name"] == "pretrained/stage_3:best")
    ck = meta["checkpoints"][k]
    rates = {}
    for name in ("base", "no_toi"):
        O.set_variant(P.VARIANTS[name][0])
        try:
            w, _ = P.oracle_eval(actors[k], ck["eval_episodes"], ck["eval_seed"], False, 4, 1000 + 2 * k)
        finally:
            O.set_variant(0)
        rates[name] = float((w == 1).mean())
    committed = {r["checkpoint"] + r["opponent"]: r for r in
                 json.load(open(PROFILE))["variants"]["base"]["rows"]}["pretrained/stage_3:beststrong"]
    assert abs(rates["base"] - committed["estimate"]) < 0.08  # R = 4 of the committed R = 64
    assert rates["no_toi"] < rates["base"] - 0.05, rates
