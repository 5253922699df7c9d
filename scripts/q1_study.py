"""SURVEY App. B Q1 study: the notebook's strong-vs-strong BasicOpponent statistics (Hockey-Env.ipynb:940-2154)
under both readings of pybox2d's velocity getter in _check_boundaries (copy = default, live reference), with
z-scores against the notebook's 1000 games.  Usage: python scripts/q1_study.py [games] > profiles/r02/q1_study.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

from hockey_amd.evaluate import basic_vs_basic_study, study_zscores  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
out = {}
for name, ref in (("copy", False), ("live_reference", True)):
    zs = study_zscores(basic_vs_basic_study(games, seed=0, vel_ref_semantics=ref))
    obs_z = [o["z"] for o in zs["obs_mean"]]
    zs["obs_mean_max_abs_z"] = max(abs(x) for x in obs_z)
    zs["obs_mean_chi2_18"] = sum(x * x for x in obs_z)
    out[name] = zs
    print(name, {k: (round(v["value"], 4), round(v["z"], 2)) for k, v in zs.items() if isinstance(v, dict)},
          "obs max|z|", round(zs["obs_mean_max_abs_z"], 2), "chi2", round(zs["obs_mean_chi2_18"], 1), file=sys.stderr)
print(json.dumps(out, indent=1))
