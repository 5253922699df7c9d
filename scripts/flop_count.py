"""Algorithmic FLOPs of an env-step (SURVEY §8(d) "count exact FLOPs from the kernel source").

The host build of the kernel's own per-arena source (tests/hostcheck.py: hk_step.h and below compiled for the CPU,
bit-identical to the GPU binary) counts the events of the bench workload -- BASELINE C3: strong-vs-strong
BasicOpponent, NORMAL mode, auto-reset, Philox placement -- and each event is priced at the arithmetic its source
performs (adds, subtracts, multiplies, divides, square roots, min / max of a clamp; no compares, selects, moves or
integer work).  The velocity and position rows, the constraint set-up, the warm start and b2Rot::Set are counted
operation by operation from hk_solver.h / hk_core.h (the "exact" classes); the narrow phase, GJK and the TOI root
finder are priced per call or iteration from their typical path (hk_geom.h; "est").  These are the FLOPs Box2D's
algorithm needs, NOT the instructions the kernel issues (no snapshot compares, select chains, packing or exec-mask
work), so FLOP/s over the kernel time is the useful-work roofline beside the counter-based VALU one.

Writes profiles/r04/flop_count.json.  Usage: python scripts/flop_count.py [arenas] [steps] [preroll]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hostcheck  # noqa: E402

# (event, FLOPs per event, how the price was obtained); order = hk_core.h EV_* enum
EVENTS = [
    ("vel_row_1pt", 78, "exact: fslot_solve_velocity_p, one point: tangent row 40 (relative velocity 10, dot 4, "
                        "lambda 1, max friction 1, clamp 3, delta 1, impulse 2, vA 4, wA 5, vB 4, wB 5) + normal row 38"),
    ("vel_row_2pt", 158, "exact: two tangent rows 80 + block solver 78 (two relative velocities 20, dots 6, bias 2, "
                         "b - K a 8, -N b 6, impulse apply 36; Box2D's first case)"),
    ("pos_point", 88, "exact: fslot_solve_position per point (transforms 16, plane / clip / normal 22, separation 7, "
                      "arms 4, clamp 5, K 13, impulse 3, body updates 18), b2Rot::Set counted separately"),
    ("init_contact", 82, "exact: fslot_init_velocity per contact (body transforms 16, world manifold 66)"),
    ("init_point", 46, "exact: per velocity point (arms 4, normal / tangent masses 30, relative velocity 13 - bias)"),
    ("init_block", 45, "exact: 2-point block solver set-up (K 21, condition 5, inverse 4 + crosses 12 + det 3)"),
    ("warm_point", 24, "exact: fslot_warm_start per point"),
    ("collide_poly_circle", 75, "est: b2CollidePolygonAndCircle (transforms 16, 7 edge separations 35, regions 24)"),
    ("collide_polygons", 830, "est: b2CollidePolygons (2 x b2FindMaxSeparation over 7 x 7 = 714, incident edge 33, "
                              "clipping 80)"),
    ("gjk_call", 45, "est: b2Distance set-up, witness points and distance"),
    ("gjk_iteration", 100, "est: one b2Distance iteration (solve2 / solve3, search direction, two supports over 7 "
                           "vertices, two transforms)"),
    ("rot_set", 24, "exact: hk_core.h rot_set (Cody-Waite reduction 7, z 1, sine 7, cosine 9)"),
    ("toi_call", 10, "est: b2TimeOfImpact set-up (sweep normalisation, target, tolerance)"),
    ("toi_sep_find_min", 55, "est: b2SeparationFunction::FindMinSeparation without its b2Rot::Set"),
    ("toi_sep_eval", 25, "est: b2SeparationFunction::Evaluate without its b2Rot::Set"),
    ("env_step_fixed", 600, "est: per arena-step work outside the above (force laws, integration, broad-phase tests "
                            "of 27 pairs, obs / obs2, info / reward in double, two BasicOpponent controllers)"),
]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    pre = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    L = hostcheck.lib()
    import ctypes
    L.hkh_flop_events.argtypes = [ctypes.c_void_p]
    L.hkh_flop_events.restype = None
    assert L.hkh_flop_event_count() == len(EVENTS)
    ev = np.zeros(len(EVENTS), np.uint64)
    env = hostcheck.HostVec(n, policies=("strong", "strong"), auto_reset=True, seed=0)
    for _ in range(pre):
        env.step()
    L.hkh_flop_events(ev.ctypes.data)  # discard the pre-roll's counts
    for _ in range(steps):
        env.step()
    L.hkh_flop_events(ev.ctypes.data)
    env.close()
    env_steps = int(ev[-1])
    assert env_steps == n * steps, (env_steps, n * steps)
    rows, exact, total = [], 0.0, 0.0
    for (name, f, how), c in zip(EVENTS, ev):
        per = float(c) / env_steps if name != "env_step_fixed" else 1.0
        fl = per * f
        total += fl
        if how.startswith("exact"):
            exact += fl
        rows.append({"event": name, "per_env_step": per, "flops_per_event": f, "flops_per_env_step": fl, "price": how})
    vel = sum(r["flops_per_env_step"] for r in rows if r["event"].startswith("vel_row"))
    out = {"workload": f"BASELINE C3 (strong-vs-strong BasicOpponent, NORMAL, auto-reset), {n} arenas x {steps} "
                       f"counted steps after {pre}, host build of the kernel source (tests/hostcheck.py)",
           "flops_per_env_step": total, "exact_flops_per_env_step": exact,
           "velocity_row_flops_per_env_step": vel, "events": rows}
    os.makedirs(os.path.join(ROOT, "profiles", "r04"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r04", "flop_count.json"), "w") as f:
        json.dump(out, f, indent=1)
    for r in rows:
        print(f"{r['event']:22s} {r['per_env_step']:10.3f} x {r['flops_per_event']:5d} = {r['flops_per_env_step']:9.1f}")
    print(f"FLOPs per env-step: {total:.0f} (exact classes {exact:.0f}, velocity rows {vel:.0f})")


if __name__ == "__main__":
    main()
