"""MoveJax / ModifyJax / MoveModifyJax — drop-ins for the reference's JAX operators (move_modify_jax.py:11-157).

They differ from the NumPy Move / Modify family (move_modify.py) in their contract, not only their array library:

* ``MoveJax.update(grid, action, context)`` — the same Move (:39-62): the four direction sets tested against the
  bounds of the starting position; returns ``(grid, new_position)``.
* ``ModifyJax.update(grid, action, context, per_env_context)`` — NOT the grid: when ``action == 1`` it sets
  ``per_env_context["dousing_count"][row, col] = 1`` (a functional ``.at[].set``: a new array stored into the
  dict the caller passed, the old array untouched) and returns ``(grid, context, per_env_context)`` (:102-114).
  Its ``effects`` are stored and unused, as in the reference.
* ``MoveModifyJax.update(grid, subactions, position, per_env_context)`` — Move then ModifyJax at the new
  position; returns ``(grid, position, per_env_context)`` (:148-157).

Every call also takes a leading env axis (the reference vmaps them, advanced_bulldozer.py:351-368): position
(E, 2), action (E,), dousing_count (E, H, W). The arithmetic is gca_move_modify (include/gca.h): the kernel for
device tensors, the host build (libgca_cpu.so) for host arrays — O(1) per env either way: ModifyJax runs it with
an "every value -> 1" effect table on the dousing layer.
"""
import numpy as np

from ... import _backend
from ... import _device as dev
from ..._lib import call, call_cpu
from ...operator import Operator
from ...spaces import Tuple
from .move_modify import Move, make_params

_DOUSE = make_params(None, {v: 1 for v in range(256)})  # Modify with every cell value -> 1


def _positions(position):
    """(E, 2) int array of the position(s) and whether the input was a single env."""
    if dev.is_device_tensor(position):
        p = position
        single = p.dim() == 1
        return (p.reshape(1, 2) if single else p), single
    p = np.asarray(position)
    single = p.ndim == 1
    return (p.reshape(1, 2) if single else p), single


def _per_env(x, E):
    """Scalar or (E,) action values -> python ints per env."""
    a = x.reshape(-1).tolist() if (dev.is_device_tensor(x) or isinstance(x, np.ndarray)) else [x]
    if len(a) == 1 and E > 1:
        a = a * E
    if len(a) != E:
        raise ValueError(f"expected {E} actions, got {len(a)}")
    return [int(v) for v in a]


class MoveJax(Move):
    """move_modify_jax.py:11-62: Move with the reference JAX operator's name; also takes position (E, 2) and
    action (E,) with grid (E, H, W) (the vmapped form)."""

    def update(self, grid, action, context):
        pos, single = _positions(context)
        if single:
            return super().update(grid, action, context)
        import torch

        E = pos.shape[0]
        H, W = tuple(grid.shape)[-2:]
        acts = _per_env(action, E)
        if dev.is_device_tensor(pos) or dev.is_device_tensor(grid):
            device = dev.require_device()
            a = torch.tensor([[m, 0] for m in acts], dtype=torch.int32, device=device)
            p = dev.to_device(pos, torch.int32, device).clone()
            call("gca_move_modify", self._params, dev.ptr(a), dev.ptr(p), None, H, W, None, E, dev.stream_ptr(device))
            return grid, p.to(pos.dtype) if dev.is_device_tensor(pos) else p.cpu().numpy().astype(np.int64)
        a = np.array([[m, 0] for m in acts], dtype=np.int32)
        p = np.ascontiguousarray(pos, dtype=np.int32).copy()
        call_cpu("gca_move_modify", self._params, a.ctypes.data, p.ctypes.data, None, H, W, None, E, None)
        return grid, p.astype(np.int64)


class ModifyJax(Operator):
    hit = False

    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, effects: dict, *args, backend=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.effects = effects  # stored like the reference's effect_keys / effect_values; the update ignores them
        self.backend = backend

    def update(self, grid, action, context, per_env_context):
        pos, single = _positions(context)
        E = pos.shape[0]
        d = per_env_context["dousing_count"]
        shots = _per_env(action, E)
        if _backend.choose(self.backend, dev.is_device_tensor(d), 0, o1=True) == "cpu":
            new = np.array(d, copy=True)  # functional: the caller's array stays as it was
            view = new.reshape((1,) + new.shape) if single else new
            from .move_modify import _run_host

            for e in range(E):
                if shots[e] == 1:
                    _run_host(_DOUSE, view[e], (31, 1), pos[e], with_grid=True)
        else:
            import torch

            device = dev.require_device()
            if dev.is_device_tensor(d) and d.dtype != torch.uint8 and d.numel() and \
                    bool(((d < 0) | (d > 255)).any()):
                raise ValueError("dousing_count values must fit the u8 layout (0..255)")
            new = dev.to_device(d, torch.uint8, device).clone()
            H, W = tuple(new.shape)[-2:]
            a = torch.tensor([[31, 1 if s == 1 else 0] for s in shots], dtype=torch.int32, device=device)
            p = dev.to_device(pos, torch.int32, device).clone()
            call("gca_move_modify", _DOUSE, dev.ptr(a), dev.ptr(p), dev.ptr(new), H, W, None, E, dev.stream_ptr(device))
            if not dev.is_device_tensor(d):
                new = new.cpu().numpy().astype(np.asarray(d).dtype)
            elif d.dtype != torch.uint8:
                new = new.to(d.dtype)
        per_env_context["dousing_count"] = new  # the reference stores the new array into the dict it was given
        return grid, context, per_env_context


class MoveModifyJax(Operator):
    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, move, modify, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.suboperators = move, modify
        self.move = move
        self.modify = modify
        if self.action_space is None:
            if self.move.action_space is not None and self.move.action_space is not None:
                self.action_space = Tuple((self.move.action_space, self.move.action_space))
        if self.context_space is None:
            if self.move.context_space is not None and self.modify.context_space is not None:
                assert self.move.context_space == self.modify.context_space
                self.context_space = self.move.context_space

    def update(self, grid, subactions, position, per_env_context):
        move_action, modify_action = subactions[0], subactions[1]
        grid, position = self.move(grid, move_action, position)
        grid, position, per_env_context = self.modify(grid, modify_action, position, per_env_context)
        return grid, position, per_env_context
