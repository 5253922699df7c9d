"""The collide broad phase (hk_arena.h pair_far_collide) rejects a polygon pair once a lower bound on the core
distance exceeds 2 x total radius + kFarMargin.  Box2D's b2CollidePolygons emits contact points only within
about sqrt(2) x total radius of the cores for these shapes; this test hill-climbs the worst touching
configuration with the oracle's restatement (tests/native/contact_bound.c) and requires it to stay well
inside the bound (measured: 1.38 x total radius)."""
import os
import re
import subprocess

from conftest import ROOT


def test_polygon_contacts_stay_inside_the_broadphase_bound(tmp_path):
    exe = str(tmp_path / "contact_bound")
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-DRESTARTS=40", "-ffp-contract=off",
                           "-fno-fast-math", "-fopenmp", "-w", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "contact_bound.c"), "-lm"])
    out = subprocess.check_output([exe]).decode()
    worst = float(re.search(r"overall ([0-9.]+)", out).group(1))
    assert 0.9 < worst < 1.6, out
