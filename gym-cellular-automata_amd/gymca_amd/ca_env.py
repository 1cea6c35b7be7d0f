"""CAEnv ABC — Gymnasium step/reset contract of the reference (ca_env.py:10-99)."""
import warnings
from abc import ABC, abstractmethod
from collections import Counter
from typing import Optional

import numpy as np

try:  # pragma: no cover
    import gymnasium as _gym

    _EnvBase = _gym.Env
except ImportError:

    class _EnvBase:
        """Minimal gymnasium.Env stand-in: reset(seed) seeds `self.np_random`."""

        _np_random = None
        metadata = {}
        spec = None

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = np.random.default_rng(seed)

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.default_rng()
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        def render(self):
            return None

        def close(self):
            pass


class CAEnv(ABC, _EnvBase):
    @property
    @abstractmethod
    def MDP(self):
        raise NotImplementedError

    @property
    @abstractmethod
    def initial_state(self):
        self._resample_initial = False

    def __init__(self, nrows, ncols, debug=False, **kwargs):
        self.nrows, self.ncols = nrows, ncols
        self._debug = debug

    def step(self, action):
        if not self.done:
            self.state = self.grid, self.context = self.MDP(self.grid, action, self.context)
            self._is_done()
            obs = self.state
            reward = self._award()
            terminated = self.done
            truncated = False
            info = self._report()
            self.steps_elapsed += 1
            self.reward_accumulated += reward
            return obs, reward, terminated, truncated, info
        if self.steps_beyond_done == 0:
            warnings.warn(
                "You are calling 'step()' even though this environment has already returned done = True. "
                "You should always call 'reset()' once you receive 'done = True' -- any further steps are "
                "undefined behavior."
            )
        self.steps_beyond_done += 1
        return self.state, 0.0, True, False, self._report()

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
        super().reset(seed=seed)
        self.done = False
        self.steps_elapsed = 0
        self.reward_accumulated = 0.0
        self.steps_beyond_done = 0
        self._resample_initial = True
        obs = self.state = self.grid, self.context = self.initial_state
        return obs, self._report()

    def status(self):
        return {"steps_elapsed": self.steps_elapsed, "reward_accumulated": self.reward_accumulated}

    @abstractmethod
    def _award(self):
        raise NotImplementedError

    @abstractmethod
    def _is_done(self):
        raise NotImplementedError

    @abstractmethod
    def _report(self):
        raise NotImplementedError

    def count_cells(self, grid=None):
        """Dict of cell counts (ca_env.py:94-99). A device tensor is counted where it lives (torch.unique on the
        GPU, only the per-value totals come back); a host grid as in the reference. The forest-fire envs
        override this with the fused gca_count_cells kernel."""
        grid = self.grid if grid is None else grid
        if hasattr(grid, "is_cuda") and grid.is_cuda:
            import torch

            values, counts = torch.unique(grid, return_counts=True)
            return Counter(dict(zip(values.cpu().tolist(), counts.cpu().tolist())))
        return Counter(np.asarray(grid).ravel().tolist())
