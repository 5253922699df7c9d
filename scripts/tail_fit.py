"""Per-iteration cost of the step kernel's solver loops (diagnostics build libhockey_hip_timers.so): per wave,
the island velocity-phase cycles divided by the wave's longest island solve (iterations), grouped by the
largest island (contacts) of the wave; the same for the TOI event slot (lane-0 view) against the longest TOI
solve.  Usage: python scripts/tail_fit.py [arenas] [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HK_LIB", os.path.join(ROOT, "hockey-env_amd", "hockey_amd", "_lib", "libhockey_hip_timers.so"))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
import torch  # noqa: E402

from hockey_amd import _native as N  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
env = VecHockeyEnv(n, device="cuda:0", policies=("strong", "strong"), auto_reset=True, seed=1)
env.reset()
dbg = torch.zeros((n, 24), dtype=torch.float32, device="cuda:0")
io = N.StepIO()
io.obs = env.obs_buf.data_ptr()
io.reward = env.reward_buf.data_ptr()
io.done = env.done_buf.data_ptr()
for _ in range(600):
    env.step_raw(io)
io.debug = dbg.data_ptr()
rows = []
for s in range(steps):
    env.step_raw(io)
    torch.cuda.synchronize()
    rows.append(dbg.cpu().numpy().copy())
D = np.stack(rows).reshape(steps, n // 64, 64, 24)
L = D[:, :, :, 1:8]  # ntoi, vit_isl, vit_toi, pit, toi_calls, nc_max, nbig
P = D[:, :, 0, 8:21]  # lane-0 phase cycles
W = D[:, :, 0, 0]
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "tail_fit.npz"), lanes=L.astype(np.int16), phases=P,
                    wave=W)
ncm = L[..., 5].max(2)
vim = L[..., 1].max(2)
vtm = L[..., 2].max(2)
ptm = L[..., 3].max(2)
print(f"waves {W.size}: cycles mean {W.mean():.0f}, per-step max mean {W.max(1).mean():.0f}")
print("island velocity: cycles per iteration of the wave's longest solve, by wave max contacts")
for c in range(1, 6):
    m = (ncm == c) & (vim > 0)
    if m.sum():
        cyc = P[..., 3][m]
        it = vim[m]
        long = m & (vim >= 180)
        print(f"  nc_max {c}: waves {m.sum():6d}  cyc/it {np.mean(cyc / it):7.0f}  "
              f"180-it waves {long.sum():5d} mean cyc {P[..., 3][long].mean() if long.sum() else 0:8.0f}")
print("island position: cycles per pass by wave max contacts")
for c in range(1, 6):
    m = (ncm == c) & (ptm > 0)
    if m.sum():
        print(f"  nc_max {c}: cyc/pass {np.mean(P[..., 4][m] / ptm[m]):7.0f}")
print("TOI events (lane-0 slot 5 + 8..11) vs longest TOI velocity solve")
tslot = P[..., 5] + P[..., 8:12].sum(-1)
for lo, hi in ((0, 1), (1, 20), (20, 100), (100, 400)):
    m = (vtm >= lo) & (vtm < hi)
    if m.sum():
        print(f"  vit_toi [{lo},{hi}): waves {m.sum():6d} toi-event cycles {tslot[m].mean():8.0f}  "
              f"ntoi max {L[..., 0].max(2)[m].mean():.2f}")
sl = W.argmax(1)
print("slowest wave per step: mean phases", np.round(P[np.arange(steps), sl].mean(0)).astype(int).tolist())
print("slowest wave: nc_max", np.bincount(ncm[np.arange(steps), sl].astype(int)).tolist(),
      " vit_isl>=180 share", float((vim[np.arange(steps), sl] >= 180).mean()),
      " vit_toi>=180 share", float((vtm[np.arange(steps), sl] >= 180).mean()))
