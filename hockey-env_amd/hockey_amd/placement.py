"""Reset placement: the reference's RNG draws for HockeyEnv.reset, host side.

Mirrors ``hockey/hockey_env.py:345-418`` (``reset``) with ``r_uniform`` (``:180-181``) drawing from
``gymnasium.utils.seeding.np_random(seed)`` == ``Generator(PCG64(SeedSequence(seed)))``.  The draws are
float64 (numpy), positions are rounded to float32 when the body is created, and the TRAIN_DEFENSE
initial shot uses pybox2d float32 ``b2Vec2`` arithmetic (``:407-411``).  Output per arena:
``params = [p2x, p2y, puckx, pucky, puck_fx, puck_fy]`` (float32) + ``max_timesteps``; the device reset
kernel consumes exactly this vector, so explicit-seed resets are bit-identical to the reference.
"""
import numpy as np

from .constants import CENTER_Y, GOAL_SIZE, H, PUCK_MASS, SCALE, SHOOTFORCEMULTIPLIER, W, Mode

_f32 = np.float32


def np_random(seed=None):
    """gymnasium.utils.seeding.np_random (returns the Generator and the seed entropy)."""
    ss = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(ss)), ss.entropy


def _r(rng, lo, hi):
    return rng.uniform(lo, hi, 1)[0]


def placement(mode, one_starts, rng):
    """Return (params6 float32, max_timesteps) for one reset (hockey_env.py:357-411)."""
    mode = Mode(mode)
    max_t = 250 if mode == Mode.NORMAL else 80
    if mode != Mode.NORMAL:
        p2x = 4 * W / 5 + _r(rng, -W / 3, W / 6)
        p2y = H / 2 + _r(rng, -H / 4, H / 4)
    else:
        p2x, p2y = 4 * W / 5, H / 2
    fx = fy = _f32(0.0)
    if mode == Mode.NORMAL or mode == Mode.TRAIN_SHOOTING:
        if one_starts or mode == Mode.TRAIN_SHOOTING:
            px = W / 2 - _r(rng, H / 8, H / 4)
            py = H / 2 + _r(rng, -H / 8, H / 8)
        else:
            px = W / 2 + _r(rng, H / 8, H / 4)
            py = H / 2 + _r(rng, -H / 8, H / 8)
    else:  # TRAIN_DEFENSE
        px = W / 2 + _r(rng, 0, W / 3)
        py = H / 2 + 0.8 * _r(rng, -H / 2, H / 2)
        aim = _f32(H / 2 + .6 * _r(rng, -GOAL_SIZE / SCALE, GOAL_SIZE / SCALE))
        # direction = puck.position - (0, aim) ; direction /= direction.length  (float32 b2Vec2)
        dx = _f32(_f32(px) - _f32(0.0))
        dy = _f32(_f32(py) - aim)
        ln = np.sqrt(_f32(_f32(dx * dx) + _f32(dy * dy)), dtype=np.float32)
        dx, dy = _f32(dx / ln), _f32(dy / ln)
        # force = -direction * SHOOTFORCEMULTIPLIER * puck.mass / timeStep
        m = _f32(PUCK_MASS)
        dt = _f32(1.0 / 50)
        fx = _f32(_f32(_f32(-dx * _f32(SHOOTFORCEMULTIPLIER)) * m) / dt)
        fy = _f32(_f32(_f32(-dy * _f32(SHOOTFORCEMULTIPLIER)) * m) / dt)
    return np.array([p2x, p2y, px, py, fx, fy], np.float32), max_t


__all__ = ["np_random", "placement", "CENTER_Y"]
