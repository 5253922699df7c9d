"""Tail analysis (diagnostics build libhockey_hip_timers.so): per-wave step cycles and the per-lane work that
drives the slowest waves.  Usage: python scripts/tail_stats.py [arenas] [steps]"""
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
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
env = VecHockeyEnv(n, device="cuda:0", policies=("strong", "strong"), auto_reset=True, seed=1)
env.reset()
dbg = torch.zeros((n, 24), dtype=torch.float32, device="cuda:0")
io = N.StepIO()
io.obs = env.obs_buf.data_ptr()
io.reward = env.reward_buf.data_ptr()
io.done = env.done_buf.data_ptr()
for _ in range(300):
    env.step_raw(io)
io.debug = dbg.data_ptr()
names = ["wave_cyc", "ntoi", "vit_isl", "vit_toi", "pit", "toi_calls", "nc_max", "nbig"]
rows = []
for s in range(steps):
    env.step_raw(io)
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().copy()
    rows.append(d)
D = np.stack(rows)  # [steps, n, 24]: 0 wave cycles, 1-7 lane work, 8-19 wave phase cycles
wave = D[:, ::64, 0]  # [steps, waves]
print(f"wave cycles per step: mean {wave.mean():.0f}  median {np.median(wave):.0f}  p99 {np.percentile(wave, 99):.0f}  "
      f"max-per-step mean {wave.max(1).mean():.0f}")
lanes = D.reshape(steps, n // 64, 64, 24)
for q in (50, 90, 99):
    print(f"per-lane p{q}:", {nm: float(np.percentile(D[:, :, k], q)) for k, nm in enumerate(names) if k})
print("per-lane max:", {nm: float(D[:, :, k].max()) for k, nm in enumerate(names) if k})
PH = ["load+policy+presolve", "collide", "isl-setup", "isl-velocity", "isl-position+sleep", "toi-min",
      "toi-scan", "toi-b2TOI", "toi-event-update", "toi-island-build", "toi-position", "toi-velocity", "outputs"]
ph = D[:, ::64, 8:21]  # [steps, waves, 13]
slow = ph[np.arange(steps), wave.argmax(1)]  # the slowest wave of each step
print("phase cycles: mean wave vs slowest wave of each step (mean over steps)")
for k, nm in enumerate(PH):
    print(f"  {nm:22s} {ph[:, :, k].mean():10.0f} {slow[:, k].mean():10.0f}")
# slowest waves: max-lane stats
flat = wave.reshape(-1)
idx = np.argsort(flat)[-10:]
for i in idx[::-1]:
    st, wv = divmod(int(i), n // 64)
    L = lanes[st, wv]
    print(f"step {st} wave {wv} cycles {flat[i]:.0f} | lane max:",
          {nm: float(L[:, k].max()) for k, nm in enumerate(names) if k},
          "| lane sum ntoi", float(L[:, 1].sum()), "vit_isl sum", float(L[:, 2].sum()))
# correlation of wave cycles with wave-max stats
for k, nm in enumerate(names):
    if k:
        m = lanes[:, :, :, k].max(2).reshape(-1)
        c = np.corrcoef(m, flat)[0, 1] if m.std() > 0 else 0
        print(f"corr(wave cycles, wave-max {nm}) = {c:.2f}")
# island velocity cycles of a wave against its slowest lane's island solve (iterations, contacts)
vel = ph[:, :, 3].reshape(-1)
W = lanes.reshape(-1, 64, 24)
vmax = W[:, :, 2].max(1)
print("isl-velocity cycles per wave by the wave's longest island solve:")
for lo, hi in ((0, 9), (9, 17), (17, 100), (100, 179), (180, 181)):
    m = (vmax >= lo) & (vmax < hi)
    if m.any():
        print(f"  max vit_isl [{lo},{hi}): waves {m.mean() * 100:6.2f}%  cycles mean {vel[m].mean():9.0f}  "
              f"p90 {np.percentile(vel[m], 90):9.0f}  max {vel[m].max():9.0f}")
full = W[:, :, 2] >= 180
ncl = np.where(full, W[:, :, 6], -1).max(1)  # contacts of the lanes that ran 180 iterations
for c in range(1, 5):
    m = ncl == c
    if m.any():
        print(f"  waves whose 180-iteration lanes have at most {c} contacts: {m.sum():6d}  cycles mean {vel[m].mean():9.0f}"
              f"  per iteration {vel[m].mean() / 180:7.0f}")
nfull = full.sum(1)
for c in (1, 2, 3):
    m = nfull == c
    if m.any():
        print(f"  waves with {c} lanes at 180: {m.sum():6d}  cycles mean {vel[m].mean():9.0f}")
# velocity-loop family cycles (d[21..23], island + TOI solves) in the slowest wave of each step vs the mean wave
fam = D[:, ::64, 21:24]
sf = fam[np.arange(steps), wave.argmax(1)]
print("velocity families (general / two / one), cycles: mean wave", fam.mean((0, 1)).round(0).tolist(),
      " slowest wave", sf.mean(0).round(0).tolist())
# TOI events seen from the lanes that had them: each lane's timers hold its own event phases (lane 0's slot 5
# "toi-min" also absorbs the events of other lanes, which it waits out exec-masked)
ev = D[:, :, 1] >= 1
if ev.any():
    E = D[:, :, 8:21][ev]
    print(f"lanes with >= 1 TOI event: {ev.mean() * 100:.2f}% of lane-steps; their own phase cycles (mean):")
    for k in (5, 6, 7, 8, 9, 10, 11):
        print(f"  {PH[k]:22s} {E[:, k].mean():10.0f}")
# what bounds the launch (r05): the per-step maximum over waves, recomputed with each class of wave removed -- the most
# a faster loop for that class could save (its waves would still cost something).  Classes: the contact count of the
# wave's 180-iteration island lanes (0: none), a lane with >= 30 position passes, a lane with a 180-iteration TOI solve.
wave_cyc = wave  # [steps, waves]
ncl_sw = ncl.reshape(steps, n // 64)
pit_sw = W[:, :, 4].max(1).reshape(steps, n // 64)
vtoi_sw = W[:, :, 3].max(1).reshape(steps, n // 64)
base = wave_cyc.max(1).mean()
print(f"launch bound (mean over steps of the slowest wave): {base:.0f} cycles")
classes = {f"180-iteration island with {c} contacts": ncl_sw == c for c in (1, 2, 3, 4)}
classes["any 180-iteration island lane"] = ncl_sw >= 1
classes["position loop >= 30 passes"] = pit_sw >= 30
classes["TOI solve >= 100 iterations"] = vtoi_sw >= 100
for nm, m in classes.items():
    rest = np.where(m, 0, wave_cyc).max(1).mean()
    share = m[np.arange(steps), wave_cyc.argmax(1)].mean()
    print(f"  {nm:40s} waves/step {m.sum(1).mean():7.1f}  owns the slowest wave in {share * 100:5.1f}% of steps  "
          f"max without them {rest:9.0f} ({(1 - rest / base) * 100:4.1f}% lower)")
sw = wave_cyc.argmax(1)
print("slowest wave of each step: phase cycles by its 180-iteration contact class")
for c in (0, 1, 2, 3, 4):
    m = ncl_sw[np.arange(steps), sw] == c
    if m.any():
        print(f"  class {c}: {m.sum():3d} steps  total {wave_cyc[np.arange(steps), sw][m].mean():9.0f}  " +
              " ".join(f"{PH[k].split('+')[0]} {slow[m, k].mean():7.0f}" for k in (1, 3, 4, 5, 7, 11)))
# the velocity-family split of those slowest waves (d[21..23]: general + S3 / two-contact / one-contact loop cycles,
# island and TOI solves together; r06: written by the timers build since the debug-slot fix in hk_kernels.hip)
sfam = np.stack([D[t, sw[t] * 64:(sw[t] + 1) * 64, 21:24].max(0) for t in range(steps)])  # max over the wave's lanes
for c in (0, 1, 2, 3, 4):
    m = ncl_sw[np.arange(steps), sw] == c
    if m.any():
        g, t2, o = sfam[m].mean(0)
        print(f"  class {c}: velocity families  general+S3 {g:9.0f}  two {t2:9.0f}  one {o:9.0f}")
