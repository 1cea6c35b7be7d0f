"""Capture-time stub of gymnasium.spaces (see package docstring).

`Box.sample` records every draw in `RECORDER` so that golden vectors can store the
exact uniform roll the reference's WindyForestFire consumed (ca_windy.py:57-60).
"""
import numpy as np

from .utils import seeding

RECORDER = []  # list of np.ndarray draws made by Box.sample, in order


class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self._shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._np_random = None
        if seed is not None:
            self.seed(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    @property
    def shape(self):
        return self._shape

    def seed(self, seed=None):
        self._np_random, s = seeding.np_random(seed)
        return [s]

    def sample(self):
        raise NotImplementedError

    def contains(self, x):
        raise NotImplementedError

    def __contains__(self, x):
        return self.contains(x)


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
        shape = tuple(shape)
        self.low = np.full(shape, low, dtype=np.float64).astype(dtype) if np.ndim(low) == 0 else np.asarray(low, dtype=dtype)
        self.high = np.full(shape, high, dtype=np.float64).astype(dtype) if np.ndim(high) == 0 else np.asarray(high, dtype=dtype)
        super().__init__(shape, dtype, seed)

    def sample(self):
        if np.issubdtype(self.dtype, np.floating):
            finite = np.isfinite(self.low) & np.isfinite(self.high)
            out = np.where(
                finite,
                self.np_random.uniform(low=np.where(finite, self.low, 0.0), high=np.where(finite, self.high, 1.0), size=self.shape),
                self.low + self.np_random.exponential(size=self.shape),
            ).astype(self.dtype)
        else:
            out = self.np_random.integers(self.low, self.high, endpoint=True, size=self.shape).astype(self.dtype)
        RECORDER.append(np.array(out, copy=True))
        return out

    def contains(self, x):
        x = np.asarray(x)
        return bool(x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high))

    def __eq__(self, other):
        return isinstance(other, Box) and self.shape == other.shape and np.allclose(self.low, other.low) and np.allclose(self.high, other.high)


class Discrete(Space):
    def __init__(self, n, seed=None, start=0):
        self.n = int(n)
        self.start = int(start)
        super().__init__((), np.int64, seed)

    def sample(self):
        return np.int64(self.start + self.np_random.integers(self.n))

    def contains(self, x):
        try:
            x = int(x)
        except Exception:
            return False
        return self.start <= x < self.start + self.n

    def __eq__(self, other):
        return isinstance(other, Discrete) and self.n == other.n and self.start == other.start


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec, dtype=dtype)
        super().__init__(self.nvec.shape, dtype, seed)

    def sample(self):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return bool(x.shape == self.shape and np.all(x >= 0) and np.all(x < self.nvec))

    def __eq__(self, other):
        return isinstance(other, MultiDiscrete) and np.all(self.nvec == other.nvec)


class Tuple(Space):
    def __init__(self, spaces, seed=None):
        self.spaces = tuple(spaces)
        super().__init__(None, None, seed)

    def seed(self, seed=None):
        out = super().seed(seed)
        for s in getattr(self, "spaces", ()):
            s.seed(None if seed is None else int(self.np_random.integers(2**31)))
        return out

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def contains(self, x):
        if isinstance(x, np.ndarray):
            x = tuple(x)
        return isinstance(x, tuple) and len(x) == len(self.spaces) and all(s.contains(v) for s, v in zip(self.spaces, x))

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)


class Dict(Space):
    def __init__(self, spaces=None, seed=None, **kw):
        self.spaces = dict(spaces or {}, **kw)
        super().__init__(None, None, seed)

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def contains(self, x):
        return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

    def __getitem__(self, k):
        return self.spaces[k]
