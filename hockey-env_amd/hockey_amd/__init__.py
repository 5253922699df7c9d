"""hockey_amd -- MI355X-native batched air-hockey simulator (drop-in for julilili42/hockey-env's hot path).

Public surface:
  VecHockeyEnv                      N arenas on one GPU, torch tensors in/out (hockey_amd.vec_env)
  HockeyEnv, HockeyEnv_BasicOpponent, BasicOpponent, Mode, make
                                    the reference's single-env API (hockey_amd.hockey_env)
The compute path is libhockey_hip.so (csrc/, C ABI in include/hockey.h); torch only provides device
memory and streams.
"""
from .constants import Mode  # noqa: F401


def __getattr__(name):
    if name == "VecHockeyEnv":
        from .vec_env import VecHockeyEnv
        return VecHockeyEnv
    if name in ("HockeyEnv", "HockeyEnv_BasicOpponent", "BasicOpponent", "make", "register_envs"):
        from . import hockey_env
        return getattr(hockey_env, name)
    raise AttributeError(name)
