"""Minimal stand-in for the `gymnasium` API, used ONLY by tests/golden/make_golden.py.

gymnasium is not installed in this image. The reference's NumPy operators import a
handful of names from it (Space/Box/Discrete/MultiDiscrete/Tuple/Dict, Env, logger,
utils.seeding). This stub restates just enough of those public APIs for the
reference modules to import and run while golden vectors are captured. It never
ships to the GPU box as product code and is not used by the product package.
"""
import numpy as np

from . import error, logger, spaces  # noqa: F401
from .utils import seeding


class Env:
    _np_random = None
    spec = None
    metadata = {}

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = seeding.np_random(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = seeding.np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def render(self):
        return None

    def close(self):
        pass
