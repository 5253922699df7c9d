"""Debug: step GPU arenas and the host build of the same kernel source in lockstep; report the first
divergence (step, arena, state before/after).  Usage: python scripts/debug_lockstep.py MODE SEED N STEPS"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hockey-env_amd"), ROOT]
from hostcheck import HostVec  # noqa: E402
from hockey_amd.placement import np_random, placement  # noqa: E402
from hockey_amd.vec_env import VecHockeyEnv  # noqa: E402

import torch  # noqa: E402

mode, seed, n, steps = (int(x) for x in sys.argv[1:5])
pol = sys.argv[5] if len(sys.argv) > 5 else "external"
auto = pol != "external"
g = VecHockeyEnv(n, keep_mode=True, mode=mode, device="cuda:0", policies=(pol, pol), auto_reset=auto, seed=seed)
h = HostVec(n, keep_mode=True, mode=mode, policies=(pol, pol), auto_reset=auto, seed=seed)
TR = 13 + 24 * 4 + 128 if os.environ.get("HK_TRACE") else 13
dbg = torch.zeros((n, TR), dtype=torch.float32, device="cuda:0")
params = np.zeros((n, 6), np.float32)
for i in range(n):
    rng, _ = np_random(seed * 100_000 + i)
    params[i], max_t = placement(mode, bool(i % 2), rng)
g.reset_params(params)
h.reset_params(params)
rng = np.random.default_rng(seed)
prev = None
for t in range(steps):
    acts = rng.uniform(-1, 1, (n, 8)).astype(np.float32) if not auto else None
    rg = g.step(acts, with_agent_two=True, debug=dbg)
    rh = h.step(acts, with_agent_two=True, debug=TR)
    sg, ag = (x.cpu().numpy() for x in g.get_state())
    sh, ah = h.get_state()
    bad = np.where((sg.view(np.uint32) != sh.view(np.uint32)).any(1) | (ag != ah).any(1))[0]
    if len(bad):
        np.set_printoptions(precision=9, linewidth=200)
        for i in bad[:3]:
            print(f"step {t} arena {i}")
            print(" gpu  state", sg[i], ag[i])
            print(" host state", sh[i], ah[i])
            print(" diff idx", np.where(sg[i].view(np.uint32) != sh[i].view(np.uint32))[0])
            print(" prev state", None if prev is None else (prev[0][i], prev[1][i]))
            print(" action", None if acts is None else acts[i])
            dg, dh = dbg.cpu().numpy()[i], rh.debug[i]
            print(" dbg gpu", dg[:13])
            print(" dbg host", dh[:13])
            for k in range(4 if TR > 13 else 0):
                tg, th = dg[13 + 24 * k:37 + 24 * k], dh[13 + 24 * k:37 + 24 * k]
                ig, ih = tg.view(np.int32), th.view(np.int32)
                print(f" phase {k}: equal={np.array_equal(ig, ih)}")
                print("   gpu ", tg[:18], "touch %07x en %07x awake %d ntoi %g nbig %g cisl %07x" % (ig[18], ig[19], ig[20], tg[21], tg[22], ig[23]))
                print("   host", th[:18], "touch %07x en %07x awake %d ntoi %g nbig %g cisl %07x" % (ih[18], ih[19], ih[20], th[21], th[22], ih[23]))
        print("counters gpu", g.counters()[:7], "host", h.counters()[:7])
        sys.exit(0)
    prev = (sh, ah)
print("no divergence", "counters gpu", g.counters()[:7], "host", h.counters()[:7])
