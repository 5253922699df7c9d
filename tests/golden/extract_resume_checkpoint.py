"""Resume point of the reference's "Stage II setup" (VERDICT r04 item 2).  Build container only (reads /root/reference;
the GPU box uses the committed .npz).

The reference's report compares its exploration noises "under identical training conditions. All variants use the
Stage II curriculum" and "For controlled comparisons, we use the Stage II setup" (latex/report/template.tex:160-161,
238-239).  The Stage II setup resumes from the stage-1 best checkpoint (rl/experiment/definitions.py:93-114 stage2:
``resume_from=pretrained/stage_1/models/td3_best.pt``; pretrained/stage_2/config/run_info.json: pretrained_path
``weak_10k/models/td3_best.pt``), and ``agent.load`` restores all four networks (rl/td3/agent.py:278-286) while the
optimisers start fresh.

Reads pretrained/stage_1/models/td3_best.pt with ``torch.load(weights_only=True)`` (nothing in the file is executed)
and writes tests/golden/stage1_best_full.npz: ``<net>/<param>`` for net in policy / critic / target_policy /
target_critic, float32, the reference's state-dict names with '.' kept.  Data only.

Usage:  python tests/golden/extract_resume_checkpoint.py     (needs /root/reference)
"""
import hashlib
import json
import os

import numpy as np
import torch

REF = "/root/reference"
SRC = "pretrained/stage_1/models/td3_best.pt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stage1_best_full.npz")


def main():
    path = os.path.join(REF, SRC)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    arrays = {}
    for net in ("policy", "critic", "target_policy", "target_critic"):
        for k, v in ck[net].items():
            arrays[f"{net}/{k}"] = v.detach().cpu().numpy().astype(np.float32)
    assert arrays["policy/fc1.weight"].shape == (256, 18) and arrays["critic/q1.fc1.weight"].shape == (256, 22)
    meta = {"source": SRC, "md5": hashlib.md5(open(path, "rb").read()).hexdigest()}
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(OUT, **arrays)
    print(f"{OUT}: {len(arrays) - 1} tensors, {os.path.getsize(OUT) / 1e6:.2f} MB, {meta}")


if __name__ == "__main__":
    main()
