"""GridSpace: the space of CA lattices over a finite set of integer cell states.

Drop-in for the reference's GridSpace (gym_cellular_automata/grid_space.py:11-90): the same constructor
(`n` states 0..n-1, or an explicit `values` set; `shape`; optional per-state `probs`; `dtype`; `seed`), the
same sampling law (`np_random.choice` over the sorted unique states, so a seeded space draws the reference's
grids), membership, equality and repr. Invalid arguments fail with AssertionError / ValueError where the
reference does.
"""
import math
from typing import Optional, Sequence

import numpy as np

from ._config import TYPE_INT
from .spaces import Space


class GridSpace(Space):
    """Lattices of `shape` whose cells take one of a finite set of integer states.

        GridSpace(n=3, shape=(2, 2))                 # states 0, 1, 2
        GridSpace(values=[-1, 0, 1], shape=(2, 2))   # explicit states
    """

    def __init__(self, n: Optional[int] = None, values: Optional[Sequence[int]] = None, shape: tuple = tuple(),
                 probs: Optional[Sequence[float]] = None, dtype=TYPE_INT, seed: Optional[int] = None):
        super().__init__(shape, dtype, seed)
        assert shape, "Shape must be a non-empty tuple."
        self._from_values = values is not None
        if self._from_values:
            states = np.unique(np.asarray(values, dtype=dtype))  # sorted, duplicates dropped
        elif n is not None:
            assert n > 0, "'n' must be a positive integer."
            states = np.arange(n, dtype=dtype)
        else:
            raise ValueError("'n' or 'values' must be provided.")
        self.values = states
        self.n = int(states.size)
        self.probs = np.full(self.n, 1.0 / self.n) if probs is None else probs
        assert len(self.probs) == self.n, "Unique values do NOT MATCH with assigned probabilities."
        self.size = math.prod(self.shape)

    def sample(self) -> np.ndarray:
        """One lattice, cells drawn iid from `values` with `probs` (one choice() call, reference order)."""
        flat = self.np_random.choice(a=self.values, size=self.size, p=self.probs)
        return flat.reshape(self.shape)

    def contains(self, x) -> bool:
        arr = np.asarray(np.array(x, dtype=self.dtype) if isinstance(x, list) else x)
        if arr.shape != self.shape:
            return False
        return bool(np.isin(np.unique(arr), self.values).all())

    def __repr__(self):
        return (f"GridSpace(values={self.values}, shape={self.shape})" if self._from_values
                else f"GridSpace(n={self.n}, shape={self.shape})")

    def __eq__(self, other):
        if not isinstance(other, GridSpace) or self.shape != other.shape:
            return False
        return self.values.shape == other.values.shape and bool(np.all(self.values == other.values))

    @property
    def is_np_flattenable(self):
        return True
