"""Behavioural fixture ("Behavioural"): the reference's stage-3 TD3 actor and its recorded
evaluation, extracted in the build container only.

Reads /root/reference/pretrained/stage_3/models/td3_best.pt with ``torch.load(weights_only=True)`` (nothing in the
file is executed) and keeps only the ``policy`` tensors (rl/td3/networks.py ActorNetwork: fc1 256x18, fc2 256x256,
fc3 4x256 + biases); the recorded evaluation comes from pretrained/stage_3/metrics/metrics.json (plain JSON).
The best checkpoint is the evaluation with the highest min(WR_strong, WR_weak) (rl/training/train.py:228-245).
Writes tests/golden/stage3_actor.npz.

Usage:  python tests/golden/extract_stage3_actor.py     (needs /root/reference)
"""
import json
import os

import numpy as np
import torch

REF = "/root/reference/pretrained/stage_3"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stage3_actor.npz")


def main():
    ck = torch.load(os.path.join(REF, "models", "td3_best.pt"), map_location="cpu", weights_only=True)
    pol = ck["policy"]
    arrays = {k.replace(".", "_"): v.detach().cpu().numpy().astype(np.float32) for k, v in pol.items()
              if k.split(".")[0] in ("fc1", "fc2", "fc3")}
    m = json.load(open(os.path.join(REF, "metrics", "metrics.json")))
    ws, ww = np.array(m["winrates_strong"]), np.array(m["winrates_weak"])
    best = int(np.argmax(np.minimum(ws, ww)))
    cfg = json.load(open(os.path.join(REF, "config", "config.json")))
    arrays.update(best_eval_index=np.array(best), wr_strong=np.array(ws[best]), wr_weak=np.array(ww[best]),
                  reward_strong=np.array(m["reward_strong"][best]), reward_weak=np.array(m["reward_weak"][best]),
                  eval_episodes=np.array(cfg["eval_episodes"]), eval_seed=np.array(42))
    np.savez_compressed(OUT, **arrays)
    print({k: (v.shape if v.ndim else v.item()) for k, v in arrays.items()})


if __name__ == "__main__":
    main()
