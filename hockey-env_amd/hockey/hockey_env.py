"""Drop-in module path of the reference (hockey/hockey_env.py) backed by hockey_amd."""
from hockey_amd.constants import *  # noqa: F401,F403
from hockey_amd.hockey_env import (BasicOpponent, HockeyEnv, HockeyEnv_BasicOpponent, Mode,  # noqa: F401
                                   make, register_envs)
