"""RepeatCA: advance a CA by whole units of accumulated time (drop-in for repeat_ca.py:11-45).

Each call adds the time of the action plus the time of the state to the carried fraction and runs the
wrapped CA once per whole unit reached; the remainder is carried in the context as a float64 0-d array.
Host control logic only (it calls user-supplied timing callables); the CA it drives runs on the device.
The batched envs do the same bookkeeping per env in gca_bulldozer_pre (one lane per env).
"""
import math
from typing import Callable

import numpy as np

from ..._config import TYPE_BOX
from ...operator import Operator


class RepeatCA(Operator):
    grid_dependant = True
    action_dependant = True
    context_dependant = True

    def __init__(self, cellular_automaton, t_acting: Callable, t_perception: Callable, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.ca = cellular_automaton
        self.t_acting, self.t_perception = t_acting, t_perception
        self.suboperators = (cellular_automaton,)
        self.deterministic = cellular_automaton.deterministic

    def update(self, grid, action, context):
        ca_params, carried = context
        # (action time + state time) first, then onto the carried fraction: the reference's f64 rounding order
        elapsed = self.t_acting(action) + self.t_perception((grid, context))
        fraction, whole = math.modf(carried + elapsed)
        for _ in range(int(whole)):
            grid, ca_params = self.ca(grid, action, ca_params)
        return grid, (ca_params, np.array(fraction, dtype=TYPE_BOX))
