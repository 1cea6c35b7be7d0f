"""Operator ABC — the drop-in boundary of the reference (operator.py:10-75).

Same contract: class flags, spaces, `update(grid, action, context) -> (grid, context)`,
`__call__ = update`, `seed(seed) -> [seed]` creating `self.np_random`.
Operators of this package additionally keep a Philox key (`self.philox_seed`) for
their device-side draws; `seed(s)` derives it from `s`.
"""
from abc import ABC, abstractmethod
from copy import copy
from typing import Any, Optional, Tuple

import numpy as np

from .spaces import Space


class Operator(ABC):
    suboperators: Tuple = tuple()

    grid_dependant: Optional[bool] = None
    action_dependant: Optional[bool] = None
    context_dependant: Optional[bool] = None

    deterministic: Optional[bool] = None

    @abstractmethod
    def __init__(
        self,
        grid_space: Optional[Space] = None,
        action_space: Optional[Space] = None,
        context_space: Optional[Space] = None,
    ) -> None:
        self.grid_space = grid_space
        self.action_space = action_space
        self.context_space = context_space
        self.seed()

    @abstractmethod
    def update(self, grid: np.ndarray, action: Any, context: Any) -> Tuple[np.ndarray, Any]:
        """Update a CA lattice with an action and a context; return (new_grid, new_context)."""
        return copy(grid), copy(context)

    def __call__(self, *args, **kwargs):
        return self.update(*args, **kwargs)

    def seed(self, seed=None):
        self._seed = seed
        self.np_random = np.random.default_rng(seed)
        # 64-bit Philox key for device draws, reproducible from `seed`
        self.philox_seed = int(np.random.default_rng(seed).integers(0, 2**63 - 1))
        return [seed]
