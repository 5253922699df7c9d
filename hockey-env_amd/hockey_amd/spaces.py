"""gymnasium.spaces when importable, else a minimal Box/Discrete with the same attributes.

gymnasium is not installed in this image; callers of the reference only read
``shape``, ``low``, ``high``, ``dtype`` and ``n`` (rl/td3/agent.py:51-56,122-125, rl/common/scaler.py:12-32).
"""
import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    from gymnasium import spaces as _gs
    Box = _gs.Box
    Discrete = _gs.Discrete
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    HAVE_GYMNASIUM = False

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, self.dtype)
            self.high = np.full(self.shape, high, self.dtype)

        def sample(self, rng=None):
            rng = rng or np.random.default_rng()
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Discrete:
        def __init__(self, n):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.dtype(np.int64)

        def sample(self, rng=None):
            rng = rng or np.random.default_rng()
            return int(rng.integers(self.n))

        def contains(self, x):
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"
