"""The kernels' compile-time scene (hockey-env_amd/csrc/hk_scene_data.inc) is exactly what the host scene
builder (hk_scene.cpp build_scene: Box2D 2.3 hulls, normals, mass data) computes: regenerate it with
hk_scene_gen.cpp and compare the text, then check it against the golden geometry through the oracle
(tests/test_oracle_golden.py pins the oracle's geometry to G6)."""
import os
import re
import subprocess

import numpy as np

from conftest import ROOT

CSRC = os.path.join(ROOT, "hockey-env_amd", "csrc")


def test_compiled_scene_is_the_builder_output(tmp_path):
    exe = str(tmp_path / "hk_scene_gen")
    subprocess.check_call(["g++", "-O0", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-o", exe, "hk_scene_gen.cpp"], cwd=CSRC)
    fresh = subprocess.check_output([exe]).decode()
    with open(os.path.join(CSRC, "hk_scene_data.inc")) as f:
        assert fresh == f.read()


def test_compiled_scene_masses_match_oracle(oracle):
    """Dynamic-body mass / inverse mass / inertia literals equal the oracle's scene constants."""
    with open(os.path.join(CSRC, "hk_scene_data.inc")) as f:
        text = f.read()
    rows = [r for r in text.split("\n") if r.startswith("{") and "," in r and "0x" in r and r.count(",") == 3]
    vals = [[float.fromhex(v.strip().rstrip("f")) for v in r.strip("{},").split(",")] for r in rows[:4]]
    mass, inv_mass, inertia, inv_inertia = (np.array(v, np.float32) for v in vals)
    assert np.allclose(mass[:2], 58.0, rtol=1e-6) and abs(mass[2] - 1.0323623) < 1e-6
    assert np.array_equal(inv_mass, (np.float32(1.0) / mass).astype(np.float32))
    assert np.array_equal(inv_inertia, (np.float32(1.0) / inertia).astype(np.float32))
