"""Observation / action spaces.

Uses gymnasium.spaces when gymnasium is importable (the reference's
dependency, env.py:18-19); otherwise small duck-typed stand-ins with the same
attributes SB3 reads (shape, dtype, n, nvec, spaces, sample, contains)."""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gymnasium absent in this image
    import gymnasium as _gym
    from gymnasium import spaces as _spaces
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    _gym = None
    _spaces = None
    HAVE_GYMNASIUM = False


class _Space:
    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    @property
    def np_random(self):
        if getattr(self, "_rng", None) is None:
            self._rng = np.random.default_rng()
        return self._rng


class Box(_Space):
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self.np_random.integers(self.low, self.high + 1, self.shape).astype(self.dtype)
        return self.np_random.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


class Discrete(_Space):
    def __init__(self, n):
        self.n, self.shape, self.dtype = int(n), (), np.dtype(np.int64)

    def sample(self):
        return int(self.np_random.integers(0, self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class MultiDiscrete(_Space):
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, np.int64)
        self.shape, self.dtype = self.nvec.shape, np.dtype(np.int64)

    def sample(self):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(np.int64)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((0 <= x) & (x < self.nvec)))


class Dict(_Space):
    def __init__(self, spaces):
        self.spaces = dict(spaces)
        self.shape, self.dtype = None, None

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def contains(self, x):
        return isinstance(x, dict) and set(x) == set(self.spaces) and \
            all(s.contains(x[k]) for k, s in self.spaces.items())

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k}: {s!r}" for k, s in self.spaces.items()) + ")"


if HAVE_GYMNASIUM:  # pragma: no cover
    Box, Discrete, MultiDiscrete, Dict = _spaces.Box, _spaces.Discrete, _spaces.MultiDiscrete, _spaces.Dict
    EnvBase = _gym.Env
else:
    class EnvBase:  # minimal gymnasium.Env surface
        metadata = {"render_modes": []}
        render_mode = None
        spec = None

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass
