"""The committed learning-parity summaries regenerate from the committed per-run records (no GPU).

profiles/r05/noise_study_summary.json and the reference-loop comparisons are what DESIGN.md §7 f3 quotes; each is
the output of a script over per-run JSON files that are committed beside it (profiles/r05/noise_runs/,
profiles/r05/reference_loop_*/).  Re-running the scripts must give the committed files, so a quoted number can be
traced to the runs that produced it.  Also checks the records' own invariants: every run's best checkpoint is the
first evaluation that beat the previous best by more than 0.01 (rl/utils/model_manager.py:15-23)."""
import glob
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

R05 = os.path.join(ROOT, "profiles", "r05")


def _run(script, *args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script), *args], cwd=ROOT, check=True,
                         capture_output=True, text=True).stdout
    return json.loads(out)


def test_noise_study_summary_regenerates():
    """r06's summary (profiles/r06/noise_study_summary_t.json: r05's plus the Welch-Satterthwaite df and t-based p per
    cell) regenerates from r05's run records, and every number r05's committed summary holds is unchanged."""
    got = _run("noise_study_summary.py", os.path.join("profiles", "r05", "noise_runs"))
    want = json.load(open(os.path.join(ROOT, "profiles", "r06", "noise_study_summary_t.json")))
    assert got == want
    old = json.load(open(os.path.join(R05, "noise_study_summary.json")))
    for proto, cells in old["protocols"].items():
        for cell, row in cells.items():
            for key, v in row.items():
                if isinstance(v, dict):
                    assert {k: got["protocols"][proto][cell][key][k] for k in v} == v, (proto, cell, key)
                else:
                    assert got["protocols"][proto][cell][key] == v, (proto, cell, key)
    for proto, cells in got["protocols"].items():
        for cell, row in cells.items():
            for key in ("wr_weak", "wr_strong"):
                assert row[key]["welch_df"] is None or row[key]["welch_df"] > 1.0
                assert row[key]["welch_p"] is None or 0.0 <= row[key]["welch_p"] <= 1.0


@pytest.mark.parametrize("ref", ["stage1", "stage2", "sp_per", "scratch_ou"])
def test_reference_loop_comparison_regenerates(ref):
    got = _run("reference_loop_compare.py", "--gpu", os.path.join("profiles", "r05", "noise_runs"),
               "--ref", os.path.join("profiles", "r05", f"reference_loop_{ref}"))
    want = json.load(open(os.path.join(R05, f"reference_loop_{ref}_comparison.json")))
    assert got == want


def test_best_checkpoint_rule_holds_in_every_record():
    files = sorted(glob.glob(os.path.join(R05, "noise_runs", "*_s*.json")))
    files += sorted(glob.glob(os.path.join(R05, "reference_loop_*", "*.json")))
    assert len(files) > 100
    for f in files:
        r = json.load(open(f))
        best, pick = float("-inf"), None
        for e in r["evals"]:
            if e["score"] > best + 0.01:
                best, pick = e["score"], e
        if pick is None:
            continue
        assert r["best"]["episode"] == pick["episode"] and r["best"]["score"] == pick["score"], f
        if "final_eval" in r:
            assert 0.0 <= r["final_eval"]["wr_weak"] <= 1.0 and 0.0 <= r["final_eval"]["wr_strong"] <= 1.0, f
