"""Behavioural fixture: every TD3 actor the reference ships, with the evaluation the reference
recorded for it.  Build container only (reads /root/reference; the GPU box uses the committed .npz).

Checkpoints: ``pretrained/stage_{1,2,3}``, the five ``runs/*`` and ``rl/cluster_runs/*``, ``models/td3_{best,last}.pt``.
Each is read with ``torch.load(weights_only=True)`` (nothing in the file is executed) and only its ``policy`` tensors
are kept (rl/td3/networks.py ActorNetwork: fc1 256x18, fc2 256x256, fc3 4x256 + biases).  Byte-identical files
(``runs/20260216_005033_*`` is ``pretrained/stage_2``, ``runs/20260216_113921_*`` is ``pretrained/stage_3``) are kept
once.  The cluster run stopped after 20 episodes, before its first evaluation: it has no recorded rate and is
listed as skipped.

Which evaluation produced each checkpoint:

* ``td3_last.pt`` is written in ``finally`` after the loop (rl/training/train.py:118-131, 270-281).  Every run
  completed its planned episodes (``run_info.json`` run_result), a multiple of ``eval_interval``, and the last
  episode's evaluation runs after its updates with nothing in between: td3_last is the policy of the LAST recorded
  evaluation.
* ``td3_best.pt`` is written by ModelManager.update (rl/utils/model_manager.py:15-23) whenever the evaluation's score
  exceeds the running best by more than ``min_delta`` = 0.01 (rl/training/train.py:228-248): it is the policy of the
  last evaluation at which that happened.  The rule is replayed here in float64 exactly as Python evaluates it.
  The score is ``min(WR_strong, WR_weak)`` in the current code (train.py:225); runs made by earlier code versions
  scored differently, so each run's score series is the candidate -- min, weak, strong, or the single ``winrates``
  series of the strong-only runs -- whose replayed best equals the ``best_winrate`` its ``run_info.json`` records.
  pretrained/stage_1 matches only the weak series (its saved ``winrates_min`` is not min(strong, weak) either: an
  earlier code version).

Writes tests/golden/checkpoint_actors.npz: ``k/fc1_weight`` ... per checkpoint k, and ``meta`` (JSON): name, file,
kind, evaluation index, recorded WR_strong / WR_weak (null where the run did not evaluate that opponent), the
reference evaluator's seed (the run seed: agent.seed + i, rl/utils/evaluator.py:18) and episodes, the number of
evaluations the run made and the score used for the best-checkpoint selection.

Usage:  python tests/golden/extract_checkpoint_actors.py     (needs /root/reference)
"""
import glob
import hashlib
import json
import os

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checkpoint_actors.npz")


def replay_model_manager(score, min_delta=0.01):
    """(best index, best score) of rl/utils/model_manager.py:15-23 over a score series."""
    best, idx = float("-inf"), None
    for i, s in enumerate(score):
        if s > best + min_delta:
            best, idx = s, i
    return idx, best


def run_series(m):
    """Candidate score series of a run's metrics.json."""
    ws, ww = m.get("winrates_strong") or [], m.get("winrates_weak") or []
    cand = {}
    if ws and ww:
        cand["min"] = [min(a, b) for a, b in zip(ws, ww)]
        cand["weak"] = list(ww)
        cand["strong"] = list(ws)
    if m.get("winrates"):
        cand["winrates"] = list(m["winrates"])
    return ws, ww, cand


def main():
    runs = sorted(glob.glob(f"{REF}/pretrained/*")) + sorted(glob.glob(f"{REF}/runs/*")) + \
        sorted(glob.glob(f"{REF}/rl/cluster_runs/*"))
    arrays, meta, skipped, seen = {}, [], [], {}
    for d in runs:
        rel = os.path.relpath(d, REF)
        m = json.load(open(os.path.join(d, "metrics", "metrics.json")))
        info = json.load(open(os.path.join(d, "config", "run_info.json")))
        cfg = json.load(open(os.path.join(d, "config", "config.json")))
        ws, ww, cand = run_series(m)
        n_eval = max(len(ws), len(m.get("winrates") or []))
        if n_eval == 0:
            skipped.append({"run": rel, "reason": f"no evaluation recorded ({len(m.get('episode_rewards', []))} episodes)"})
            continue
        rr = info["run_result"]
        assert rr["episodes_completed"] == n_eval * cfg["eval_interval"] and not rr["early_stopped"], rel
        score_name = [k for k, s in cand.items() if replay_model_manager(s)[1] == rr["best_winrate"]]
        assert score_name, (rel, rr["best_winrate"])
        score_name = score_name[0]
        best_idx, _ = replay_model_manager(cand[score_name])
        for kind, idx in (("best", best_idx), ("last", n_eval - 1)):
            path = os.path.join(d, "models", f"td3_{kind}.pt")
            digest = hashlib.md5(open(path, "rb").read()).hexdigest()
            if digest in seen:
                seen[digest]["aliases"].append(f"{rel}/models/td3_{kind}.pt")
                continue
            pol = torch.load(path, map_location="cpu", weights_only=True)["policy"]
            k = len(meta)
            for key, v in pol.items():
                if key.split(".")[0] in ("fc1", "fc2", "fc3"):
                    arrays[f"{k}/{key.replace('.', '_')}"] = v.detach().cpu().numpy().astype(np.float32)
            assert arrays[f"{k}/fc1_weight"].shape == (256, 18) and arrays[f"{k}/fc3_weight"].shape == (4, 256)
            rec = {"name": f"{rel}:{kind}", "file": f"{rel}/models/td3_{kind}.pt", "md5": digest, "kind": kind,
                   "eval_index": idx, "episode": (idx + 1) * cfg["eval_interval"], "n_evals": n_eval,
                   "score": score_name, "eval_episodes": cfg["eval_episodes"],
                   "eval_seed": info["run_settings"]["seed"],
                   "eval_opponent": info["environment"].get("eval_opponent"),
                   "wr_strong": ws[idx] if ws else m["winrates"][idx],
                   "wr_weak": ww[idx] if ww else None, "aliases": []}
            seen[digest] = rec
            meta.append(rec)
    arrays["meta"] = np.array(json.dumps({"checkpoints": meta, "skipped": skipped}))
    np.savez_compressed(OUT, **arrays)
    for r in meta:
        print(f"{r['name']:70s} eval {r['eval_index']:3d}/{r['n_evals']} score={r['score']:8s} "
              f"WR_strong={r['wr_strong']} WR_weak={r['wr_weak']} seed={r['eval_seed']} aliases={r['aliases']}")
    print("skipped:", skipped)
    print(f"{OUT}: {os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
