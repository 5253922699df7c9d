"""Scene constants and the game-mode enum (hockey/hockey_env.py:17-37, 78-81)."""
import math
from enum import Enum

FPS = 50
SCALE = 60.0
VIEWPORT_W = 600
VIEWPORT_H = 480
W = VIEWPORT_W / SCALE
H = VIEWPORT_H / SCALE
CENTER_X = W / 2
CENTER_Y = H / 2
ZONE = W / 20
MAX_ANGLE = math.pi / 3
MAX_TIME_KEEP_PUCK = 15
GOAL_SIZE = 75
RACKETPOLY = [(-10, 20), (+5, 20), (+5, -20), (-10, -20), (-18, -10), (-21, 0), (-18, 10)]
RACKETFACTOR = 1.2
FORCEMULTIPLIER = 6000
SHOOTFORCEMULTIPLIER = 60
TORQUEMULTIPLIER = 400
MAX_PUCK_SPEED = 25

# float32 Box2D mass of the puck: density 7 * b2_pi * r * r with r = 13/SCALE (b2CircleShape::ComputeMass)
PUCK_MASS = 1.0323623418807983

OBS_DIM = 18
ACT_DIM = 8  # joint action, 4 per player (keep_mode)


class Mode(Enum):
    NORMAL = 0
    TRAIN_SHOOTING = 1
    TRAIN_DEFENSE = 2


def parse_mode(value):
    """HockeyEnv.mode setter semantics (hockey_env.py:758-779)."""
    if isinstance(value, Mode):
        return value
    if isinstance(value, str):
        try:
            return Mode[value]
        except KeyError:
            raise ValueError(f"{value} is not a valid name for {Mode.__name__}") from None
    if isinstance(value, int):
        try:
            return Mode(value)
        except ValueError:
            raise ValueError(f"{value} is not a valid value for {Mode.__name__}") from None
    raise TypeError("Input value must be an Enum, name (str), or value (int)")
