"""Lockstep comparison of a batched implementation (the gfx950 kernel through the C ABI, or its host
build) with the oracle's batched context (oracle/hk_oracle.c hkov_*), which restates the hk_step contract
of include/hockey.h: fused policies, Philox randomness keyed by global arena id, device auto-reset.

Test infrastructure only.  Every compared field is bit-exact (float32 bit patterns, uint8 done).
"""
import numpy as np

FIELDS = ("obs", "obs2", "reward", "reward2", "done", "info", "info2", "actions", "final_obs")


def first_mismatch(step, got, want, fields=None):
    """Return a description of the first differing field / arena, or None.

    fields: the fields to compare (default: every field the oracle produced).  A requested field that either
    side lacks is itself a mismatch, so an output the implementation silently dropped cannot pass."""
    for f in (tuple(want) if fields is None else fields):
        if f not in want or got.get(f) is None:
            return {"step": step, "field": f, "missing": "oracle" if f not in want else "implementation"}
        g = np.asarray(got[f]).reshape(want[f].shape[0], -1)
        w = want[f].reshape(want[f].shape[0], -1)
        if g.shape != w.shape or g.dtype.itemsize != w.dtype.itemsize:
            return {"step": step, "field": f, "shape": [g.shape, w.shape], "dtype": [str(g.dtype), str(w.dtype)]}
        ok = np.all(g.view(np.uint8) == w.view(np.uint8), axis=1) if g.dtype == np.uint8 else \
            np.all(g.view(np.uint32) == w.view(np.uint32), axis=1)
        if not ok.all():
            i = int(np.nonzero(~ok)[0][0])
            return {"step": step, "field": f, "arena": i, "got": g[i].tolist(), "want": w[i].tolist()}
    return None


def oracle_steps(ov, steps, actions=None, opp_inc=None):
    """Run the oracle context for `steps` steps; yield each step's output dict."""
    for t in range(steps):
        yield ov.step(None if actions is None else actions[t], None if opp_inc is None else opp_inc[t],
                      with_agent_two=True, final_obs=True)
