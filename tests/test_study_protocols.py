"""The learning-parity studies run the reference's experiment definitions (rl/experiment/definitions.py) field for
field: scripts/noise_study.py's protocol configs against the overrides written there (restated here with their
lines), on top of rl/td3/config.py's defaults as hockey_amd.td3.TD3Config restates them.  No GPU."""
import importlib.util
import os

import pytest

from conftest import ROOT


def _study():
    spec = importlib.util.spec_from_file_location("noise_study", os.path.join(ROOT, "scripts", "noise_study.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# rl/experiment/definitions.py: the override dicts of each experiment (noise_mode / PER / self-play where switched)
DEFINITIONS = {
    "scratch": dict(curriculum_name="noise_study", prioritized_replay=False, use_self_play=False,
                    use_noise_annealing=True),                                                     # :10-31
    "stage1": dict(curriculum_name="stage1", use_self_play=False, prioritized_replay=False, use_noise_annealing=True,
                   lr_q=4e-4, lr_pol=4e-4),                                                       # :70-90
    "stage2": dict(curriculum_name="stage2", use_self_play=False, prioritized_replay=False, lr_q=3e-4, lr_pol=3e-4,
                   noise_min_scale=0.06),                                                          # :93-114
    "sp_per": dict(curriculum_name="ablation", noise_mode="ornstein-uhlenbeck", use_noise_annealing=True),  # :34-66
}


@pytest.mark.parametrize("protocol", sorted(DEFINITIONS))
def test_protocol_configs_follow_the_definitions(protocol):
    from hockey_amd.td3 import TD3Config

    ns = _study()
    cfg, resume = ns.config(protocol, "ou" if protocol == "sp_per" else "gaussian", per=False, sp=False)
    base = TD3Config()
    for k, v in DEFINITIONS[protocol].items():
        assert getattr(cfg, k) == v, (protocol, k)
    overridden = set(DEFINITIONS[protocol]) | {"noise_mode", "prioritized_replay", "use_self_play", "use_noise_annealing"}
    for k, v in vars(base).items():  # everything else at config.py's defaults
        if k not in overridden:
            assert getattr(cfg, k) == v, (protocol, k)
    # resume: stage 2 and the PER / self-play study start from the stage-1 best (definitions.py:35, :94), the others
    # from scratch
    assert (resume is not None) == (protocol in ("stage2", "sp_per"))
    if resume is not None:
        assert os.path.exists(resume)


def test_sp_per_switches_and_report_rows():
    ns = _study()
    for per in (False, True):
        for sp in (False, True):
            cfg, _ = ns.config("sp_per", "ou", per=per, sp=sp)
            assert cfg.prioritized_replay == per and cfg.use_self_play == sp
            assert (per, sp) in ns.REFERENCE_SP_PER
    assert set(ns.REFERENCE) == {"gaussian", "ou", "pink", "uniform"}
