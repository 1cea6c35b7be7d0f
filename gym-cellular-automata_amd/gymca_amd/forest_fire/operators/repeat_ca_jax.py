"""RepeatCAJax — drop-in for the reference's repeat_ca_jax.py:12-71.

Contract (different from RepeatCA, repeat_ca.py): ``update(grid, action, per_env_context, shared_context,
accu_time)`` adds ``t_acting(action) + t_perception((grid, per_env_context, shared_context))`` to ``accu_time``,
keeps the fractional part (``jnp.modf``), and runs the wrapped CA EXACTLY ONCE, whatever the whole part is: the
reference's ``lax.fori_loop`` over the repeats is commented out (:61-69). The CA is called with four arguments,
``ca(grid, action, per_env_context, shared_context) -> (grid, per_env_context, shared_context)``
(PartiallyObservableForestFireJax, whose step is the device kernel). Returns ``(grid, (per_env_context,
fractional_time))``.

The time arithmetic keeps the inputs' precision like jnp does (float32 for the Advanced env's f32 timings and
f32 accumulated time; the batched env does the same per env in gca_advenv_post, repeat_ca_jax.py:35-40):
numpy scalars / arrays through np.modf, device tensors through x - trunc(x) (the fractional part of a float is
exact, so both agree bit for bit).
"""
from typing import Callable

import numpy as np

from ... import _device as dev
from ...operator import Operator


def _modf(x):
    if dev.is_device_tensor(x):
        import torch

        whole = torch.trunc(x)
        return x - whole, whole
    frac, whole = np.modf(x)
    return frac, whole


class RepeatCAJax(Operator):
    grid_dependant = True
    action_dependant = True
    context_dependant = True

    def __init__(self, cellular_automaton, t_acting: Callable, t_perception: Callable, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.t_acting = t_acting
        self.t_perception = t_perception
        self.ca = cellular_automaton
        self.suboperators = (self.ca,)
        self.deterministic = self.ca.deterministic

    def update(self, grid, action, per_env_context, shared_context, accu_time):
        time_action = self.t_acting(action)
        time_state = self.t_perception((grid, per_env_context, shared_context))
        time_taken = time_action + time_state
        new_accu_time = accu_time + time_taken
        modf_accu_time, _repeats = _modf(new_accu_time)
        # exactly one CA step (repeat_ca_jax.py:61-63; the repeat loop :64-69 is commented out in the reference)
        grid, new_per_env, _ = self.ca(grid, action, per_env_context, shared_context)
        return grid, (new_per_env, modf_accu_time)
