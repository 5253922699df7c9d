"""Exploration noise of the reference's TD3 agent, batched over N arenas on the device (rl/common/noise.py:4-113,
selected by rl/td3/agent.py:128-156 ``_init_noise``).

Each generator returns an [N, dim] draw per call (one independent process per arena) and ``reset()`` restarts
every arena's process, as ``agent.reset()`` does at an episode start (rl/td3/agent.py:185-187):

* ``gaussian`` -- N(0, scale) per component (GaussianNoise);
* ``ornstein-uhlenbeck`` -- x <- x + theta (mu - x) dt + sigma sqrt(dt) N(0, 1), theta 0.15, mu 0, sigma = scale,
  dt 1.0 as the agent constructs it; reset to x0 = 0 (OrnsteinUhlenbeckNoise);
* ``pink`` -- a block of ``seq_len`` steps per arena and component: complex N(0,1) + i N(0,1) coefficients
  scaled by 1/sqrt(f) on the rfft grid (f[0] := f[1]), DC made real, inverse rfft, normalised to unit
  (population) standard deviation along time, times scale; a new block when a block is used up or on reset
  (PinkNoise);
* ``uniform`` -- U(-s, s) with s = scale * sqrt(3), the agent's choice (same variance as the Gaussian).

The draws come from a seeded torch generator on the device instead of the process-global ``np.random`` /
``np.random.default_rng()`` the reference uses (a batched difference; the distributions are the same).
"""
import math

import torch


class _Noise:
    def __init__(self, n, dim, scale, device, seed):
        self.n, self.dim, self.scale = int(n), int(dim), float(scale)
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed) + 0xA0)

    def _randn(self, *shape):
        return torch.randn(shape, device=self.device, generator=self.gen)

    def reset(self):
        pass


class GaussianNoise(_Noise):
    def __call__(self):
        return self._randn(self.n, self.dim) * self.scale


class UniformNoise(_Noise):
    """``scale`` is the half-width (the agent passes action_noise_scale * sqrt(3))."""

    def __call__(self):
        u = torch.rand((self.n, self.dim), device=self.device, generator=self.gen)
        return (2 * u - 1) * self.scale


class OrnsteinUhlenbeckNoise(_Noise):
    def __init__(self, n, dim, scale, device, seed, theta=0.15, dt=1.0, mean=0.0):
        super().__init__(n, dim, scale, device, seed)
        self.theta, self.dt, self.mean = float(theta), float(dt), float(mean)
        self.reset()

    def __call__(self):
        x = (self.x + self.theta * (self.mean - self.x) * self.dt
             + self.scale * math.sqrt(self.dt) * self._randn(self.n, self.dim))
        self.x = x
        return x

    def reset(self):
        self.x = torch.zeros((self.n, self.dim), device=self.device)


def pink_block(n, dim, seq_len, device, gen):
    """[n, dim, seq_len] unit-variance pink noise (PinkNoise._generate_pink_block, per arena)."""
    m = seq_len // 2 + 1
    freqs = torch.fft.rfftfreq(seq_len, device=device, dtype=torch.float64)
    if m > 1:
        freqs[0] = freqs[1]
    else:
        freqs[0] = 1.0
    scaling = 1.0 / torch.sqrt(freqs)
    real = torch.randn((n, dim, m), device=device, generator=gen, dtype=torch.float64)
    imag = torch.randn((n, dim, m), device=device, generator=gen, dtype=torch.float64)
    spec = torch.complex(real, imag) * scaling
    spec[..., 0] = torch.complex(spec[..., 0].real, torch.zeros_like(spec[..., 0].real))
    x = torch.fft.irfft(spec, n=seq_len, dim=-1)
    return x / x.std(dim=-1, unbiased=False, keepdim=True)


class PinkNoise(_Noise):
    def __init__(self, n, dim, scale, device, seed, seq_len=1024):
        super().__init__(n, dim, scale, device, seed)
        self.seq_len = int(seq_len)
        self.reset()

    def __call__(self):
        if self.idx >= self.seq_len:
            self.reset()
        x = self.block[:, :, self.idx]
        self.idx += 1
        return (self.scale * x).float()

    def reset(self):
        self.block = pink_block(self.n, self.dim, self.seq_len, self.device, self.gen)
        self.idx = 0


def make_noise(mode, n, dim, scale, seq_len, device, seed=0):
    """rl/td3/agent.py _init_noise: the generator for ``noise_mode``."""
    if mode == "ornstein-uhlenbeck":
        return OrnsteinUhlenbeckNoise(n, dim, scale, device, seed, dt=1.0)
    if mode == "gaussian":
        return GaussianNoise(n, dim, scale, device, seed)
    if mode == "pink":
        return PinkNoise(n, dim, scale, device, seed, seq_len=seq_len)
    if mode == "uniform":
        return UniformNoise(n, dim, scale * math.sqrt(3), device, seed)
    raise ValueError(f"Unknown noise mode: {mode}")
