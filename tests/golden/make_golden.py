"""Golden-vector generator for the hockey hot path (runs ONLY in the build container).

This script imports the real reference module ``/root/reference/hockey/hockey_env.py`` with stub
``Box2D`` / ``gymnasium`` modules (neither is installed here) and drives the
reference's own pure-Python code with a fake ``b2World`` that reproduces the *pybox2d* value
semantics the reference relies on:

* every body quantity is stored as float32 (Box2D ``float32``),
* vector getters (``position``, ``linearVelocity``) return float32 *copies* (SURVEY Appendix B Q1,
  default "copy"),
* ``b2Vec2`` arithmetic (``-``, ``+``, unary ``-``, ``* s``, ``/ s``, ``.length``) is float32,
* ``ApplyForceToCenter`` / ``ApplyTorque`` accumulate float32 forces / torques,
* ``world.Step`` is a recorded no-op: the Box2D solve itself cannot run here (F1), so these vectors
  pin everything *around* the solve -- reset placement (G1), the pre-solve force laws, hold/shoot and
  the obs/reward/info/done emission (G2/G3), ``BasicOpponent`` (G4), discrete map + mode parsing (G5),
  G2 under the live-reference velocity getter (G2R), ``ContactDetector.BeginContact`` on
  fake contacts (G7) and ``set_state`` (G8).

Mass properties (G6) come from a float32 restatement of Box2D 2.3 ``b2PolygonShape::Set`` /
``ComputeMass`` / ``b2Body::ResetMassData`` written here with numpy float32 scalars; the reference
tree does not contain Box2D, so G6 is *our* restatement, not a reference output (documented in
DESIGN.md).  The C oracle recomputes G6 independently and the tests check the two agree.

Outputs: ``tests/golden/*.npz`` (plain arrays, loadable with ``allow_pickle=False``).
The reference source never leaves this container; only the generated arrays are committed.

Usage:  python tests/golden/make_golden.py     (needs /root/reference)
"""
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
f32 = np.float32

# --------------------------------------------------------------------------------------------
# pybox2d value-semantics fakes
# --------------------------------------------------------------------------------------------


def _seq2(o):
    if isinstance(o, FakeVec):
        return o.x, o.y
    return f32(o[0]), f32(o[1])


class FakeVec:
    """float32 b2Vec2 with pybox2d operator semantics."""

    __slots__ = ("x", "y")

    def __init__(self, x=0.0, y=0.0):
        self.x = f32(x)
        self.y = f32(y)

    def __getitem__(self, i):
        if i == 0 or i == -2:
            return float(self.x)
        if i == 1 or i == -1:
            return float(self.y)
        raise IndexError(i)

    def __setitem__(self, i, v):  # writes into the (copied) vector only
        if i == 0:
            self.x = f32(v)
        else:
            self.y = f32(v)

    def __len__(self):
        return 2

    def __iter__(self):
        yield float(self.x)
        yield float(self.y)

    def __sub__(self, o):
        ox, oy = _seq2(o)
        return FakeVec(self.x - ox, self.y - oy)

    def __add__(self, o):
        ox, oy = _seq2(o)
        return FakeVec(self.x + ox, self.y + oy)

    def __neg__(self):
        return FakeVec(-self.x, -self.y)

    def __mul__(self, s):
        s = f32(s)
        return FakeVec(self.x * s, self.y * s)

    __rmul__ = __mul__

    def __truediv__(self, s):
        s = f32(s)
        return FakeVec(self.x / s, self.y / s)

    @property
    def length(self):
        return float(np.sqrt(f32(self.x * self.x + self.y * self.y), dtype=np.float32))

    def copy(self):
        return FakeVec(self.x, self.y)

    def tuple(self):
        return float(self.x), float(self.y)


class FakeBody:
    def __init__(self, position, angle, kind, mass=0.0):
        self._p = FakeVec(*_seq2(position))
        self._a = f32(angle)
        self._v = FakeVec(0.0, 0.0)
        self._w = f32(0.0)
        self.kind = kind
        self._mass = f32(mass)
        self._ld = f32(0.0)
        self._ad = f32(0.0)
        self.force = FakeVec(0.0, 0.0)
        self.torque = f32(0.0)
        self.n_force_calls = 0

    # --- getters return copies (Q1: copy semantics) ---
    position = property(lambda s: s._p.copy(), lambda s, v: setattr(s, "_p", FakeVec(*_seq2(v))))
    linearVelocity = property(lambda s: s._v.copy(), lambda s, v: setattr(s, "_v", FakeVec(*_seq2(v))))
    angle = property(lambda s: float(s._a), lambda s, v: setattr(s, "_a", f32(v)))
    angularVelocity = property(lambda s: float(s._w), lambda s, v: setattr(s, "_w", f32(v)))
    mass = property(lambda s: float(s._mass))
    linearDamping = property(lambda s: float(s._ld), lambda s, v: setattr(s, "_ld", f32(v)))
    angularDamping = property(lambda s: float(s._ad), lambda s, v: setattr(s, "_ad", f32(v)))

    def ApplyForceToCenter(self, f, wake):
        fx, fy = _seq2(f)
        self.force = FakeVec(self.force.x + fx, self.force.y + fy)
        self.n_force_calls += 1

    def ApplyTorque(self, t, wake):
        self.torque = f32(self.torque + f32(t))


# masses are filled in after the float32 Box2D mass restatement below
MASS = {}


class FakeWorld:
    def __init__(self, *a, **k):
        self.steps = 0
        self._dyn = 0

    def CreateDynamicBody(self, position, angle, fixtures):
        kind = ("player1", "player2", "puck")[self._dyn % 3]
        self._dyn += 1
        return FakeBody(position, angle, kind, MASS[kind])

    def CreateStaticBody(self, position, angle, fixtures):
        return FakeBody(position, angle, "static")

    def DestroyBody(self, b):
        pass

    def Step(self, dt, vi, pi):
        self.steps += 1
        self.last_step = (dt, vi, pi)


def install_stubs():
    B = types.ModuleType("Box2D")
    b2 = types.ModuleType("Box2D.b2")

    class _Any:
        def __init__(self, *a, **k):
            self.kw = k

    for n in ["edgeShape", "circleShape", "fixtureDef", "polygonShape", "revoluteJointDef"]:
        setattr(b2, n, _Any)

    class contactListener:
        def __init__(self, *a, **k):
            pass

    b2.contactListener = contactListener
    B.b2 = b2
    B.b2World = FakeWorld
    B.b2Vec2 = FakeVec
    sys.modules["Box2D"] = B
    sys.modules["Box2D.b2"] = b2

    g = types.ModuleType("gymnasium")
    sp = types.ModuleType("gymnasium.spaces")
    er = types.ModuleType("gymnasium.error")
    ut = types.ModuleType("gymnasium.utils")
    en = types.ModuleType("gymnasium.envs")
    rg = types.ModuleType("gymnasium.envs.registration")

    class Box:
        def __init__(self, low, high, shape=None, dtype=None):
            self.shape = shape
            self.dtype = dtype
            self.low = np.full(shape, low, dtype)
            self.high = np.full(shape, high, dtype)

    class Discrete:
        def __init__(self, n):
            self.n = n

    class seeding:  # gymnasium.utils.seeding.np_random semantics
        @staticmethod
        def np_random(seed=None):
            ss = np.random.SeedSequence(seed)
            return np.random.Generator(np.random.PCG64(ss)), ss.entropy

    class EzPickle:
        def __init__(self, *a, **k):
            pass

    class Env:
        pass

    sp.Box, sp.Discrete = Box, Discrete
    er.DependencyNotInstalled = Exception
    ut.seeding, ut.EzPickle = seeding, EzPickle
    rg.register = lambda **k: None
    g.Env, g.spaces, g.error, g.utils, g.envs = Env, sp, er, ut, en
    en.registration = rg
    g.logger = None
    for k, v in {"gymnasium": g, "gymnasium.spaces": sp, "gymnasium.error": er, "gymnasium.utils": ut,
                 "gymnasium.envs": en, "gymnasium.envs.registration": rg}.items():
        sys.modules[k] = v


# --------------------------------------------------------------------------------------------
# float32 restatement of Box2D 2.3 polygon hull / mass (G6)
# --------------------------------------------------------------------------------------------
LINEAR_SLOP = f32(0.005)


def b2_polygon_set(verts):
    """b2PolygonShape::Set (welding + gift-wrap hull + normals), float32."""
    ps = []
    for v in verts:
        v = (f32(v[0]), f32(v[1]))
        uniq = True
        for p in ps:
            dx, dy = f32(v[0] - p[0]), f32(v[1] - p[1])
            if f32(dx * dx + dy * dy) < f32(f32(0.5) * LINEAR_SLOP):
                uniq = False
                break
        if uniq:
            ps.append(v)
    n = len(ps)
    i0, x0 = 0, ps[0][0]
    for i in range(1, n):
        x = ps[i][0]
        if x > x0 or (x == x0 and ps[i][1] < ps[i0][1]):
            i0, x0 = i, x
    hull = []
    ih = i0
    while True:
        hull.append(ih)
        ie = 0
        for j in range(1, n):
            if ie == ih:
                ie = j
                continue
            m = hull[-1]
            rx, ry = f32(ps[ie][0] - ps[m][0]), f32(ps[ie][1] - ps[m][1])
            vx, vy = f32(ps[j][0] - ps[m][0]), f32(ps[j][1] - ps[m][1])
            c = f32(rx * vy - ry * vx)
            if c < 0:
                ie = j
            if c == 0 and f32(vx * vx + vy * vy) > f32(rx * rx + ry * ry):
                ie = j
        ih = ie
        if ie == i0:
            break
    V = [ps[i] for i in hull]
    N = []
    m = len(V)
    for i in range(m):
        j = i + 1 if i + 1 < m else 0
        ex, ey = f32(V[j][0] - V[i][0]), f32(V[j][1] - V[i][1])
        nx, ny = f32(f32(1.0) * ey), f32(-f32(1.0) * ex)  # b2Cross(edge, 1)
        ln = np.sqrt(f32(nx * nx + ny * ny), dtype=np.float32)
        inv = f32(f32(1.0) / ln)
        N.append((f32(nx * inv), f32(ny * inv)))
    return V, N


def b2_polygon_mass(V, density):
    density = f32(density)
    m = len(V)
    sx, sy = f32(0), f32(0)
    for v in V:
        sx, sy = f32(sx + v[0]), f32(sy + v[1])
    inv_n = f32(f32(1.0) / f32(m))
    sx, sy = f32(sx * inv_n), f32(sy * inv_n)
    k_inv3 = f32(f32(1.0) / f32(3.0))
    cx, cy, area, I = f32(0), f32(0), f32(0), f32(0)
    for i in range(m):
        e1x, e1y = f32(V[i][0] - sx), f32(V[i][1] - sy)
        j = i + 1 if i + 1 < m else 0
        e2x, e2y = f32(V[j][0] - sx), f32(V[j][1] - sy)
        D = f32(e1x * e2y - e1y * e2x)
        tri = f32(f32(0.5) * D)
        area = f32(area + tri)
        w = f32(tri * k_inv3)
        cx, cy = f32(cx + f32(w * f32(e1x + e2x))), f32(cy + f32(w * f32(e1y + e2y)))
        intx2 = f32(f32(f32(e1x * e1x) + f32(e2x * e1x)) + f32(e2x * e2x))
        inty2 = f32(f32(f32(e1y * e1y) + f32(e2y * e1y)) + f32(e2y * e2y))
        I = f32(I + f32(f32(f32(f32(0.25) * k_inv3) * D) * f32(intx2 + inty2)))
    mass = f32(density * area)
    inv_area = f32(f32(1.0) / area)
    cx, cy = f32(cx * inv_area), f32(cy * inv_area)
    mcx, mcy = f32(cx + sx), f32(cy + sy)
    Im = f32(density * I)
    Im = f32(Im + f32(mass * f32(f32(f32(mcx * mcx) + f32(mcy * mcy)) - f32(f32(cx * cx) + f32(cy * cy)))))
    return mass, (mcx, mcy), Im


def b2_body_mass(mass, center, I):
    """b2Body::ResetMassData for a single fixture."""
    m = f32(f32(0) + mass)
    lcx, lcy = f32(f32(0) + f32(mass * center[0])), f32(f32(0) + f32(mass * center[1]))
    Ib = f32(f32(0) + I)
    inv_m = f32(f32(1.0) / m)
    lcx, lcy = f32(lcx * inv_m), f32(lcy * inv_m)
    Ib = f32(Ib - f32(m * f32(f32(lcx * lcx) + f32(lcy * lcy))))
    inv_I = f32(f32(1.0) / Ib)
    return m, inv_m, (lcx, lcy), Ib, inv_I


def geometry(he):
    S, RF = he.SCALE, he.RACKETFACTOR
    out = {}
    for name, p2 in (("player1", False), ("player2", True)):
        verts = [(-x / S * RF if p2 else x / S * RF, y / S * RF) for x, y in he.RACKETPOLY]
        V, N = b2_polygon_set(verts)
        mass, c, I = b2_polygon_mass(V, 200.0 / RF)
        m, im, lc, Ib, iI = b2_body_mass(mass, c, I)
        out[name + "_verts"] = np.array(V, np.float32)
        out[name + "_normals"] = np.array(N, np.float32)
        out[name + "_mass"] = np.array([m, im, lc[0], lc[1], Ib, iI], np.float32)
    r = f32(13 / S)
    pi_f = f32(3.14159265359)
    cm = f32(f32(f32(f32(7.0) * pi_f) * r) * r)
    cI = f32(cm * f32(f32(f32(f32(0.5) * r) * r) + f32(0)))
    m, im, lc, Ib, iI = b2_body_mass(cm, (f32(0), f32(0)), cI)
    out["puck_mass"] = np.array([m, im, lc[0], lc[1], Ib, iI, r], np.float32)
    return out


# --------------------------------------------------------------------------------------------
# golden generation
# --------------------------------------------------------------------------------------------

def load_reference():
    install_stubs()
    sys.path.insert(0, REF)
    import hockey.hockey_env as he  # noqa: E402  (the real reference module)
    return he


def body_state(b):
    return [b._p.x, b._p.y, b._a, b._v.x, b._v.y, b._w]


def set_body(b, s):
    b._p = FakeVec(s[0], s[1])
    b._a = f32(s[2])
    b._v = FakeVec(s[3], s[4])
    b._w = f32(s[5])
    b.force = FakeVec(0.0, 0.0)
    b.torque = f32(0.0)
    b.n_force_calls = 0


MODE_IDS = {"NORMAL": 0, "TRAIN_SHOOTING": 1, "TRAIN_DEFENSE": 2}


def gen_g1(he):
    """reset(): placement, initial puck force, obs/info for seeds x modes x one_starts."""
    rows = {k: [] for k in ["mode", "seed", "one_starts", "state", "puck_force", "max_t", "obs", "info"]}

    def rec(env, seed):
        rows["mode"].append(env.mode.value)
        rows["seed"].append(seed)
        rows["one_starts"].append(int(env.one_starts))
        rows["state"].append(body_state(env.player1) + body_state(env.player2) + body_state(env.puck))
        rows["puck_force"].append([env.puck.force.x, env.puck.force.y])
        rows["max_t"].append(env.max_timesteps)

    for mode in (0, 1, 2):
        for seed in range(256):
            env = he.HockeyEnv(mode=mode)
            for call in range(3):
                if call == 2:
                    obs, info = env.reset(one_starting=True, seed=seed)
                else:
                    obs, info = env.reset(seed=seed)
                rec(env, seed)
                rows["obs"].append(np.asarray(obs, np.float64))
                rows["info"].append([info["winner"], info["reward_closeness_to_puck"], info["reward_touch_puck"],
                                     info["reward_puck_direction"]])
    np.savez_compressed(os.path.join(OUT, "g1_reset.npz"),
                        mode=np.array(rows["mode"], np.int32), seed=np.array(rows["seed"], np.int64),
                        one_starts=np.array(rows["one_starts"], np.int32),
                        state=np.array(rows["state"], np.float32), puck_force=np.array(rows["puck_force"], np.float32),
                        max_t=np.array(rows["max_t"], np.int32), obs=np.array(rows["obs"], np.float64),
                        info=np.array(rows["info"], np.float64))
    return len(rows["seed"])


def _sample_case(rng):
    """Random (state, aux, action) covering every branch of hockey_env.py:420-483,610-633,668-680."""
    def pos_player(one):
        r = rng.random()
        if r < 0.25:
            x = rng.uniform(4.3, 5.7)  # centre zone / side limits
        elif r < 0.4:
            x = rng.uniform(0.8, 1.8) if one else rng.uniform(8.2, 9.2)
        elif r < 0.5:
            x = rng.uniform(4.8, 9.0) if one else rng.uniform(1.0, 5.2)  # wrong half
        else:
            x = rng.uniform(1.0, 9.0)
        y = rng.choice([rng.uniform(0.8, 1.4), rng.uniform(6.6, 7.2), rng.uniform(1.0, 7.0)])
        return x, y

    def vel(scale):
        if rng.random() < 0.15:
            return 0.0, 0.0
        if rng.random() < 0.3:
            return rng.uniform(-scale * 1.6, scale * 1.6), rng.uniform(-scale, scale)
        return rng.uniform(-scale * 0.5, scale * 0.5), rng.uniform(-scale * 0.5, scale * 0.5)

    st = []
    for one in (True, False):
        x, y = pos_player(one)
        ang = rng.choice([rng.uniform(-0.9, 0.9), rng.uniform(-2.0, 2.0)])
        vx, vy = vel(12.0)
        w = rng.choice([0.0, rng.uniform(-6, 6)])
        st += [x, y, ang, vx, vy, w]
    px, py = rng.uniform(0.3, 9.7), rng.uniform(0.5, 7.5)
    pvx, pvy = vel(35.0)
    st += [px, py, rng.uniform(-50, 50), pvx, pvy, rng.uniform(-20, 20)]
    st = np.array(st, np.float32)
    h1 = int(rng.choice([0, 0, 0, 1, 2, 3, 7, 14, 15]))
    h2 = int(rng.choice([0, 0, 0, 1, 2, 3, 7, 14, 15]))
    t = int(rng.choice([0, 1, 79, 80, 81, 120, 249, 250, 251, int(rng.integers(0, 300))]))
    done = int(rng.random() < 0.2)
    winner = int(rng.choice([0, 0, 1, -1]))
    act = rng.uniform(-1.4, 1.4, 8)
    for k in (3, 7):
        act[k] = rng.choice([rng.uniform(-1, 1), 0.6, 0.5, 0.4])
    if rng.random() < 0.1:
        act[:] = 0.0
    return st, np.array([h1, h2, t, done, winner], np.int32), act.astype(np.float32)


def gen_g2(he, n=6000, seed=1234):
    """step() with the solve as a no-op: pre-solve laws, hold/shoot, obs/obs2/info/info2/reward/done."""
    rng = np.random.default_rng(seed)
    keys = ["mode", "keep_mode", "state", "aux", "action", "force", "torque", "ldamp", "adamp", "state_after",
            "has_after", "obs", "obs2", "reward", "reward2", "done", "info", "info2", "nforce"]
    rows = {k: [] for k in keys}
    envs = {}
    for mode in (0, 1, 2):
        for keep in (True, False):
            envs[(mode, keep)] = he.HockeyEnv(keep_mode=keep, mode=mode)
    for i in range(n):
        mode = int(rng.choice([0, 0, 0, 1, 2]))
        keep = bool(rng.random() < 0.85)
        env = envs[(mode, keep)]
        st, aux, act = _sample_case(rng)
        set_body(env.player1, st[0:6])
        set_body(env.player2, st[6:12])
        set_body(env.puck, st[12:18])
        env.player1_has_puck, env.player2_has_puck = int(aux[0]), int(aux[1])
        env.time, env.done, env.winner = int(aux[2]), bool(aux[3]), int(aux[4])
        a = act if keep else np.concatenate([act[0:3], act[4:7]])
        obs, r, d, _t, info = env.step(a.copy())
        obs2 = env.obs_agent_two()
        info2 = env.get_info_agent_two()
        r2 = env.get_reward_agent_two(info2)
        rows["mode"].append(mode)
        rows["keep_mode"].append(int(keep))
        rows["state"].append(st)
        rows["aux"].append(aux)
        rows["action"].append(act)
        bs = (env.player1, env.player2, env.puck)
        rows["force"].append([b.force.x for b in bs] + [b.force.y for b in bs])
        rows["nforce"].append([b.n_force_calls for b in bs])
        rows["torque"].append([env.player1.torque, env.player2.torque])
        rows["ldamp"].append([b._ld for b in bs])
        rows["adamp"].append([env.player1._ad, env.player2._ad])
        rows["state_after"].append(body_state(env.player1) + body_state(env.player2) + body_state(env.puck))
        rows["has_after"].append([env.player1_has_puck, env.player2_has_puck, env.time])
        rows["obs"].append(np.asarray(obs, np.float64) if keep else np.concatenate([obs, [0, 0]]))
        rows["obs2"].append(np.asarray(obs2, np.float64) if keep else np.concatenate([obs2, [0, 0]]))
        rows["reward"].append(r)
        rows["reward2"].append(r2)
        rows["done"].append(int(d))
        rows["info"].append([info["winner"], info["reward_closeness_to_puck"], info["reward_touch_puck"],
                             info["reward_puck_direction"]])
        rows["info2"].append([info2["winner"], info2["reward_closeness_to_puck"], info2["reward_touch_puck"],
                              info2["reward_puck_direction"]])
    # force / torque / damping re-ordering: force = [p1x,p2x,pkx,p1y,p2y,pky] -> [[x,y] per body]
    force = np.array(rows["force"], np.float32).reshape(n, 2, 3).transpose(0, 2, 1)
    np.savez_compressed(os.path.join(OUT, "g2_step_presolve.npz"),
                        mode=np.array(rows["mode"], np.int32), keep_mode=np.array(rows["keep_mode"], np.int32),
                        state=np.array(rows["state"], np.float32), aux=np.array(rows["aux"], np.int32),
                        action=np.array(rows["action"], np.float32), force=force,
                        nforce=np.array(rows["nforce"], np.int32),
                        torque=np.array(rows["torque"], np.float32), ldamp=np.array(rows["ldamp"], np.float32),
                        adamp=np.array(rows["adamp"], np.float32),
                        state_after=np.array(rows["state_after"], np.float32),
                        has_after=np.array(rows["has_after"], np.int32), obs=np.array(rows["obs"], np.float64),
                        obs2=np.array(rows["obs2"], np.float64), reward=np.array(rows["reward"], np.float64),
                        reward2=np.array(rows["reward2"], np.float64), done=np.array(rows["done"], np.int32),
                        info=np.array(rows["info"], np.float64), info2=np.array(rows["info2"], np.float64))
    return n


def gen_g4(he, n_seeds=64, n_acts=40):
    """BasicOpponent.act with the global np.random phase stream recorded (hockey_env.py:781-833)."""
    rng = np.random.default_rng(99)
    rows = {k: [] for k in ["weak", "keep", "phase0", "inc", "obs", "act", "phase"]}
    for s in range(n_seeds):
        for weak in (True, False):
            keep = bool(s % 5 != 4)
            np.random.seed(s)
            bo = he.BasicOpponent(weak=weak, keep_mode=keep)
            mirror = np.random.RandomState()
            mirror.seed(s)
            ph0 = mirror.uniform(0, np.pi)
            assert ph0 == bo.phase
            for k in range(n_acts):
                o = np.zeros(18)
                o[0:2] = rng.uniform([-4.5, -3.5], [0.5, 3.5])
                o[2] = rng.uniform(-1.2, 1.2)
                o[3:6] = rng.uniform(-8, 8, 3) * (rng.random() < 0.8)
                o[6:12] = rng.uniform(-4, 4, 6)
                o[12:14] = rng.uniform([-4.8, -3.8], [4.8, 3.8])
                o[14:16] = rng.choice([rng.uniform(-20, 20, 2), rng.uniform(-1, 1, 2)])
                if rng.random() < 0.3:  # behind the puck, in the kick window
                    o[12] = o[0] + rng.uniform(0.01, 2.0)
                    o[13] = o[1] + rng.uniform(-0.45, 0.45)
                o[16:18] = rng.choice([0, 0, 1, 3, 6, 7, 8, 15], 2)
                o = o.astype(np.float32).astype(np.float64)  # obs values are float32 in the env
                inc = mirror.uniform(0, 0.2)
                a = bo.act(o)
                rows["weak"].append(int(weak))
                rows["keep"].append(int(keep))
                rows["phase0"].append(ph0 if k == 0 else rows["phase"][-1])
                rows["inc"].append(inc)
                rows["obs"].append(o)
                rows["act"].append(np.concatenate([a, [0.0]]) if not keep else a)
                rows["phase"].append(bo.phase)
    np.savez_compressed(os.path.join(OUT, "g4_basic_opponent.npz"),
                        weak=np.array(rows["weak"], np.int32), keep=np.array(rows["keep"], np.int32),
                        phase0=np.array(rows["phase0"]), inc=np.array(rows["inc"]), obs=np.array(rows["obs"]),
                        act=np.array(rows["act"]), phase=np.array(rows["phase"]))
    return len(rows["act"])


def gen_g5(he):
    env = he.HockeyEnv()
    envn = he.HockeyEnv(keep_mode=False)
    disc = np.array([env.discrete_to_continous_action(i) for i in range(8)], np.float64)
    discn = np.array([envn.discrete_to_continous_action(i) for i in range(8)], np.float64)
    modes_in = ["NORMAL", "TRAIN_SHOOTING", "TRAIN_DEFENSE", "0", 0, 1, 2, 3, "BOGUS", 1.5]
    outcome = []
    for m in modes_in:
        try:
            e = he.HockeyEnv(mode=m)
            outcome.append(("ok", e.mode.value))
        except ValueError:
            outcome.append(("ValueError", -1))
        except TypeError:
            outcome.append(("TypeError", -1))
        except Exception as ex:  # noqa: BLE001
            outcome.append((type(ex).__name__, -1))
    try:
        env.reset(mode=1)
        reset_mode = "ok"
    except TypeError:
        reset_mode = "TypeError"
    np.savez_compressed(os.path.join(OUT, "g5_discrete_modes.npz"), disc=disc, disc_nokeep=discn,
                        mode_in=np.array([str(m) + ":" + type(m).__name__ for m in modes_in]),
                        mode_kind=np.array([o[0] for o in outcome]), mode_val=np.array([o[1] for o in outcome]),
                        reset_mode=np.array(reset_mode), discrete_n=np.array(env.discrete_action_space.n),
                        obs_shape=np.array(env.observation_space.shape), act_shape=np.array(env.action_space.shape),
                        act_shape_nokeep=np.array(envn.action_space.shape))


def gen_g2r(he, n=3000, seed=1234):
    """G2 under the Q1 "live reference" reading of pybox2d's velocity getter: the vector
    ``player.linearVelocity`` returns writes through to the body, so _check_boundaries' ``[i] = 0`` zeroes the
    velocity and the force becomes -0.  Same sampled cases as G2 (same seed), fewer of them."""
    orig = FakeBody.linearVelocity
    FakeBody.linearVelocity = property(lambda s: s._v, orig.fset)  # live vector: __setitem__ hits the body
    try:
        out = os.path.join(OUT, "g2_step_presolve.npz")
        tmp = os.path.join(OUT, "_g2r_tmp.npz")
        os.replace(out, out + ".keep")
        try:
            gen_g2(he, n=n, seed=seed)
            os.replace(out, tmp)
        finally:
            os.replace(out + ".keep", out)
        os.replace(tmp, os.path.join(OUT, "g2r_step_presolve_live.npz"))
    finally:
        FakeBody.linearVelocity = orig
    return n


# body ids of the oracle / kernel scene (oracle/hk_oracle.c enum B_*): p1, p2, puck, top wall, goal 1, goal 2
G7_BODIES = {"player1": 0, "player2": 1, "puck": 2, "wall": 3, "goal_player_1": 9, "goal_player_2": 10}


def gen_g7(he):
    """ContactDetector.BeginContact (hockey_env.py:44-76) on fake contacts: every ordered body pair x puck vx
    around the +-0.1 thresholds x has_puck x keep_mode x prior done / winner."""
    from types import SimpleNamespace as NS

    rows = {k: [] for k in ["keep", "body_a", "body_b", "puck_vx", "has_in", "dw_in", "has_out", "dw_out"]}
    vxs = [-5.0, -0.2, -0.1, float(f32(-0.1)), -0.0999, 0.0, 0.0999, 0.1, float(f32(0.1)), 0.1001, 0.2, 5.0]
    for keep in (True, False):
        env = he.HockeyEnv(keep_mode=keep)
        cd = he.ContactDetector(env)
        bodies = {"player1": env.player1, "player2": env.player2, "puck": env.puck, "wall": env.world_objects[-1],
                  "goal_player_1": env.goal_player_1, "goal_player_2": env.goal_player_2}
        for na, ba in bodies.items():
            for nb, bb in bodies.items():
                if na == nb:
                    continue
                for vx in vxs:
                    for h1, h2 in ((0, 0), (0, 7), (5, 0), (15, 15)):
                        for d0, w0 in ((0, 0), (1, -1), (1, 1)):
                            env.puck._v = FakeVec(vx, 0.3)
                            env.player1_has_puck, env.player2_has_puck = h1, h2
                            env.done, env.winner = bool(d0), w0
                            cd.BeginContact(NS(fixtureA=NS(body=ba), fixtureB=NS(body=bb)))
                            rows["keep"].append(int(keep))
                            rows["body_a"].append(G7_BODIES[na])
                            rows["body_b"].append(G7_BODIES[nb])
                            rows["puck_vx"].append(f32(vx))
                            rows["has_in"].append([h1, h2])
                            rows["dw_in"].append([d0, w0])
                            rows["has_out"].append([int(env.player1_has_puck), int(env.player2_has_puck)])
                            rows["dw_out"].append([int(env.done), int(env.winner)])
    np.savez_compressed(os.path.join(OUT, "g7_begin_contact.npz"),
                        **{k: np.array(v, np.float32 if k == "puck_vx" else np.int32) for k, v in rows.items()})
    return len(rows["keep"])


def gen_g8(he, n=400, seed=77):
    """HockeyEnv.set_state (hockey_env.py:594-608) on an obs-format vector: the bodies' float32 setter results,
    has_puck, and the observation that follows."""
    rng = np.random.default_rng(seed)
    rows = {k: [] for k in ["keep", "state", "raw_after", "has_after", "obs_after", "raw_before"]}
    for i in range(n):
        keep = bool(i % 4 != 3)
        env = he.HockeyEnv(keep_mode=keep)
        env.puck._a, env.puck._w = f32(rng.uniform(-3, 3)), f32(rng.uniform(-9, 9))  # untouched by set_state
        before = body_state(env.player1) + body_state(env.player2) + body_state(env.puck)
        st = np.zeros(18)
        st[0:2] = rng.uniform([-4.2, -3.2], [4.2, 3.2])
        st[2] = rng.uniform(-1.5, 1.5)
        st[3:6] = rng.uniform(-12, 12, 3)
        st[6:8] = rng.uniform([-4.2, -3.2], [4.2, 3.2])
        st[8] = rng.uniform(-1.5, 1.5)
        st[9:12] = rng.uniform(-12, 12, 3)
        st[12:14] = rng.uniform([-4.7, -3.7], [4.7, 3.7])
        st[14:16] = rng.uniform(-30, 30, 2)
        st[16:18] = rng.choice([0, 0, 3, 14, 15], 2)
        if rng.random() < 0.2:
            st[:16] = np.round(st[:16], 1)  # decimal inputs: the float64 -> float32 rounding paths
        env.set_state(st if keep else st.copy())
        rows["keep"].append(int(keep))
        rows["state"].append(st)
        rows["raw_before"].append(before)
        rows["raw_after"].append(body_state(env.player1) + body_state(env.player2) + body_state(env.puck))
        rows["has_after"].append([float(env.player1_has_puck), float(env.player2_has_puck)])
        obs = np.asarray(env._get_obs(), np.float64)
        rows["obs_after"].append(obs if keep else np.concatenate([obs, [0, 0]]))
    np.savez_compressed(os.path.join(OUT, "g8_set_state.npz"), keep=np.array(rows["keep"], np.int32),
                        state=np.array(rows["state"], np.float64), raw_before=np.array(rows["raw_before"], np.float32),
                        raw_after=np.array(rows["raw_after"], np.float32),
                        has_after=np.array(rows["has_after"], np.float64),
                        obs_after=np.array(rows["obs_after"], np.float64))
    return n


def main():
    he = load_reference()
    geo = geometry(he)
    MASS["player1"] = float(geo["player1_mass"][0])
    MASS["player2"] = float(geo["player2_mass"][0])
    MASS["puck"] = float(geo["puck_mass"][0])
    np.savez_compressed(os.path.join(OUT, "g6_geometry.npz"), **geo)
    print("G6 masses player", geo["player1_mass"], "puck", geo["puck_mass"])
    print("G1 rows", gen_g1(he))
    print("G2 rows", gen_g2(he))
    print("G4 rows", gen_g4(he))
    gen_g5(he)
    print("G2R rows", gen_g2r(he))
    print("G7 rows", gen_g7(he))
    print("G8 rows", gen_g8(he))
    print("done ->", OUT)


if __name__ == "__main__":
    main()
