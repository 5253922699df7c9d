"""Learning parity of the GPU TD3 loop against the reference's exploration-noise study.

Reference: latex/report/template.tex:238-279 (Table "Exploration noise ablation", mean +- std over three seeds of the
best checkpoint of each run, re-evaluated: WR weak / strong, return weak / strong) and rl/experiment/definitions.py.
Two readings of "the protocol" exist in the reference and both are run here:

* ``--protocol scratch`` -- the code's ``noise_study(seed)`` (definitions.py:10-31): 10 000 episodes from scratch
  (``resume_from=None``), curriculum ``noise_study`` (50 % strong / 50 % weak bot, curricula.py NOISE_STUDY), no PER,
  no self-play, annealed noise, every other field at rl/td3/config.py's defaults (lr 4e-4, buffer 300 k).
* ``--protocol stage2`` -- the report's text: "For controlled comparisons, we use the Stage II setup and vary only the
  component under study" and "All variants use the Stage II curriculum" (template.tex:160-161, 239).  The Stage II
  setup is definitions.py:93-114 ``stage2``: resume from the stage-1 best checkpoint (all four networks,
  tests/golden/stage1_best_full.npz), curriculum ``stage2``, lr 3e-4, noise_min_scale 0.06, no PER, no self-play;
  10 000 episodes as in ``noise_study``.

Both: ``hockey_amd.td3.train`` on ``--arenas`` arenas (20: a round is 20 episodes, so the 200-episode evaluation lands
exactly), an episode ends at its done step (the recorded runs' semantics, td3.train docstring), 32 updates of 256 per
episode.  Every 200 episodes: 100 greedy games against each bot, reset seeds seed + i (rl/utils/evaluator.py:10-35);
score min(WR_strong, WR_weak) and the best-checkpoint rule of rl/utils/model_manager.py:15-23 (score > best + 0.01).
At the end the best checkpoint is re-evaluated on ``--final-games`` fresh placements per bot (seeds 100 000 + i).

Writes <out>/<protocol>_<noise>_s<seed>.json after every evaluation and the best actor's weights (reference td3
``policy`` layout) as <...>_best_actor.pt whenever it changes.

Usage: python scripts/noise_study.py --protocol stage2 --noise gaussian --seed 42 --out gpurun_out/r05/noise
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))

import torch  # noqa: E402

from hockey_amd.evaluate import Actor, evaluate  # noqa: E402
from hockey_amd.td3 import TD3Config, train  # noqa: E402

NOISES = {"gaussian": "gaussian", "ou": "ornstein-uhlenbeck", "pink": "pink", "uniform": "uniform"}
RESUME = os.path.join(ROOT, "tests", "golden", "stage1_best_full.npz")

# template.tex:244-272, mean +- std over three seeds (percent for the win rates)
REFERENCE = {"gaussian": {"wr_weak": (92.50, 4.48), "wr_strong": (81.00, 0.47), "r_weak": (8.22, 0.80),
                          "r_strong": (5.69, 0.10)},
             "ou": {"wr_weak": (94.67, 0.58), "wr_strong": (89.00, 2.65), "r_weak": (8.56, 0.13),
                    "r_strong": (7.06, 0.46)},
             "pink": {"wr_weak": (92.56, 4.30), "wr_strong": (86.11, 2.84), "r_weak": (8.17, 0.57),
                      "r_strong": (6.40, 0.34)},
             "uniform": {"wr_weak": (91.22, 2.84), "wr_strong": (80.22, 8.39), "r_weak": (8.10, 0.55),
                         "r_strong": (5.51, 1.51)}}


# template.tex:313-345 (Table "Final evaluation results", mean +- std over three seeds, percent / return)
REFERENCE_SP_PER = {(False, False): {"wr_weak": (93.07, 3.75), "wr_strong": (78.27, 3.07), "r_weak": (8.33, 0.66),
                                     "r_strong": (5.00, 0.70)},
                    (False, True): {"wr_weak": (90.73, 5.90), "wr_strong": (72.60, 7.63), "r_weak": (7.62, 1.26),
                                    "r_strong": (4.06, 1.56)},
                    (True, False): {"wr_weak": (75.80, 9.18), "wr_strong": (66.07, 4.69), "r_weak": (4.22, 2.00),
                                    "r_strong": (1.99, 1.04)},
                    (True, True): {"wr_weak": (78.27, 2.23), "wr_strong": (65.33, 5.14), "r_weak": (4.71, 0.54),
                                   "r_strong": (1.78, 1.01)}}


def config(protocol, noise, per=False, sp=False):
    common = dict(noise_mode=NOISES[noise], prioritized_replay=False, use_self_play=False, use_noise_annealing=True)
    if protocol == "scratch":
        return TD3Config(curriculum_name="noise_study", **common), None
    if protocol == "stage1":
        # definitions.py:70-90 stage1: from scratch, curriculum stage1 (the weak bot only), annealed noise (Gaussian
        # there; --noise here), lr 4e-4, no PER, no self-play; compared with the reference's own loop
        # (scripts/reference_loop_study.py --protocol stage1), the report has no multi-seed stage-1 table
        return TD3Config(curriculum_name="stage1", lr_q=4e-4, lr_pol=4e-4, **common), None
    if protocol == "sp_per":
        # definitions.py:34-66 prioritized_selfplay_study: resume from weak_10k/td3_best.pt (= pretrained/stage_1 best,
        # pretrained/stage_2/config/run_info.json), curriculum "ablation" (= STAGE_2), OU noise, annealing, PER and
        # self-play switched, every other field at config.py's defaults (lr 4e-4, self-play interval 250, pool 12)
        return TD3Config(curriculum_name="ablation", noise_mode="ornstein-uhlenbeck", use_noise_annealing=True,
                         prioritized_replay=per, use_self_play=sp), RESUME
    return TD3Config(curriculum_name="stage2", lr_q=3e-4, lr_pol=3e-4, noise_min_scale=0.06, **common), RESUME


# episodes of each protocol's Experiment in rl/experiment/definitions.py (noise study :16-18, PER / self-play
# study :53-55, stage1 :72-74, stage2 :97-99)
DEFINITION_EPISODES = {"scratch": 10_000, "sp_per": 10_000, "stage1": 10_000, "stage2": 15_000}


def deviations(protocol, episodes):
    """Explicit deviations of this run from the reference's Experiment definition (recorded in the run
    JSON, not only in a docstring)."""
    want = DEFINITION_EPISODES[protocol]
    if episodes == want:
        return []
    return [{"what": "noise-study length", "episodes": episodes, "definition_episodes": want,
             "why": "the report's Stage II table is compared at the noise study's 10 000 episodes; pass --episodes "
                    f"{want} for the definition's length"}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--protocol", choices=["scratch", "stage1", "stage2", "sp_per"], required=True)
    ap.add_argument("--per", type=int, default=0, help="sp_per: prioritized replay on (1) / off (0)")
    ap.add_argument("--sp", type=int, default=0, help="sp_per: self-play on (1) / off (0)")
    ap.add_argument("--noise", choices=sorted(NOISES), required=True)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--arenas", type=int, default=20)
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--eval-episodes", type=int, default=100)
    ap.add_argument("--final-games", type=int, default=1000)
    ap.add_argument("--learner", choices=["auto", "fused", "eager"], default="auto")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "noise_study"))
    args = ap.parse_args()
    cfg, resume = config(args.protocol, args.noise, bool(args.per), bool(args.sp))
    n = args.arenas
    rounds = args.episodes // n
    dev = "cuda:0"
    os.makedirs(args.out, exist_ok=True)
    name = f"{args.protocol}_{args.noise}" if args.protocol != "sp_per" else f"sp_per_p{args.per}_sp{args.sp}"
    stem = os.path.join(args.out, f"{name}_s{args.seed}")
    ref = (REFERENCE_SP_PER[(bool(args.per), bool(args.sp))] if args.protocol == "sp_per"
           else None if args.protocol == "stage1" else REFERENCE[args.noise])
    out = {"protocol": args.protocol, "noise": args.noise if args.protocol != "sp_per" else "ou", "seed": args.seed,
           "per": bool(cfg.prioritized_replay), "self_play": bool(cfg.use_self_play), "config": vars(cfg),
           "resume_from": None if resume is None else os.path.relpath(resume, ROOT), "arenas": n,
           "episodes": rounds * n, "eval_episodes": args.eval_episodes, "reference": ref, "evals": [], "best": None,
           "deviations": deviations(args.protocol, rounds * n)}
    t0 = time.time()
    best = {"score": float("-inf")}

    def dump():
        with open(stem + ".json", "w") as f:
            json.dump(out, f, indent=1)

    def eval_fn(agent, episodes):
        agent.actor.eval()
        s = evaluate(agent.actor, episodes=args.eval_episodes, seed=agent.seed, weak_opponent=False, device=dev)
        w = evaluate(agent.actor, episodes=args.eval_episodes, seed=agent.seed, weak_opponent=True, device=dev)
        agent.actor.train()
        score = min(s["win"], w["win"])  # rl/training/train.py:228
        rec = {"episode": episodes, "updates": agent.train_step, "wr_strong": s["win"], "wr_weak": w["win"],
               "r_strong": s["mean_return"], "r_weak": w["mean_return"], "score": score,
               "noise_scale": agent.current_noise_scale, "wall_s": round(time.time() - t0, 1)}
        if score > best["score"] + 0.01:  # rl/utils/model_manager.py:15-23
            best.update(score=score, state={k: v.detach().clone() for k, v in agent.actor.state_dict().items()})
            out["best"] = dict(rec)
            torch.save({"policy": {k: v.cpu() for k, v in best["state"].items()}}, stem + "_best_actor.pt")
            rec["new_best"] = True
        out["evals"].append(rec)
        dump()
        print(json.dumps(rec), flush=True)
        return rec

    fused = {"auto": "auto", "fused": True, "eager": False}[args.learner]
    agent, st = train(n_arenas=n, rounds=rounds, cfg=cfg, device=dev, seed=args.seed, eval_fn=eval_fn,
                      episode_end="done", fused=fused, resume_from=resume)
    torch.cuda.synchronize()
    out.update(updates=st["updates"], env_steps=st["env_steps"], train_wall_s=round(time.time() - t0, 1))
    if "state" in best:
        actor = Actor().to(dev)
        actor.load_state_dict(best["state"])
        actor.eval()
        fin = {}
        for opp in ("strong", "weak"):
            r = evaluate(actor, episodes=args.final_games, seed=100_000, weak_opponent=opp == "weak", device=dev)
            fin[f"wr_{opp}"], fin[f"r_{opp}"] = r["win"], r["mean_return"]
            fin[f"draw_{opp}"], fin[f"len_{opp}"] = r["draw"], r["mean_length"]
        fin["games"] = args.final_games
        out["final_eval"] = fin
    out["wall_s"] = round(time.time() - t0, 1)
    dump()
    print(json.dumps({k: out.get(k) for k in ("protocol", "noise", "seed", "best", "final_eval", "wall_s")}),
          flush=True)


if __name__ == "__main__":
    main()
