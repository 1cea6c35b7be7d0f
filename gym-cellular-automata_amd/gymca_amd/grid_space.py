"""GridSpace — integer lattice space (reference grid_space.py:11-90)."""
from functools import reduce
from operator import mul
from typing import Optional, Sequence

import numpy as np

from ._config import TYPE_INT
from .spaces import Space


class GridSpace(Space):
    """A Space for CA lattices; arbitrary integers can be cell states.

    >>> GridSpace(n=3, shape=(2, 2))
    >>> GridSpace(values=[-1, 0, 1], shape=(2, 2))
    """

    def __init__(
        self,
        n: Optional[int] = None,
        values: Optional[Sequence[int]] = None,
        shape: tuple = tuple(),
        probs: Optional[Sequence[float]] = None,
        dtype=TYPE_INT,
        seed: int = None,
    ):
        super().__init__(shape, dtype, seed)
        assert shape, "Shape must be a non-empty tuple."
        if values is not None:
            self._from_values = True
            self.values = np.unique(np.array(values, dtype=dtype))
            self.n = len(self.values)
        elif n is not None:
            self._from_values = False
            assert n is not None and n > 0, "'n' must be a positive integer."
            self.n = n
            self.values = np.arange(self.n, dtype=dtype)
        else:
            raise ValueError("'n' or 'values' must be provided.")
        self.probs = np.repeat(1.0, self.n) / self.n if probs is None else probs
        assert len(self.values) == len(self.probs), "Unique values do NOT MATCH with assigned probabilities."
        self.size = reduce(mul, self.shape)

    def sample(self) -> np.ndarray:
        return self.np_random.choice(a=self.values, size=self.size, p=self.probs).reshape(self.shape)

    def contains(self, x) -> bool:
        if isinstance(x, list):
            x = np.array(x, dtype=self.dtype)
        x = np.asarray(x)
        return set(np.unique(x)).issubset(set(self.values)) and self.shape == x.shape

    def __repr__(self):
        if self._from_values:
            return f"GridSpace(values={self.values}, shape={self.shape})"
        return f"GridSpace(n={self.n}, shape={self.shape})"

    def __eq__(self, other):
        return isinstance(other, GridSpace) and (self.shape == other.shape) and np.all(self.values == other.values)

    @property
    def is_np_flattenable(self):
        return True
