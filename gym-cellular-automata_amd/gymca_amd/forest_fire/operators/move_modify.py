"""Move / Modify / MoveModify — drop-ins for the reference operators (move_modify.py:10-134).

The arithmetic runs in the device kernel gca_move_modify (one lane per env), so the
same code path serves the single-env drop-in here and the batched envs. Semantics:
Move applies the four direction sets in order with bounds checks (:37-67); Modify
substitutes `effects[grid[row, col]]` IN PLACE and sets `self.hit` (:84-94).
"""
import numpy as np

from ... import _device as dev
from ..._lib import BulldozerParams, call
from ...operator import Operator
from ...spaces import Tuple


def _mask(s):
    m = 0
    for a in s:
        a = int(a)
        if not 0 <= a < 31:
            raise ValueError("action ids must be in [0, 31)")
        m |= 1 << a
    return m


def make_params(directions_sets=None, effects=None):
    """Fill gca_bulldozer_params' move/modify fields."""
    p = BulldozerParams()
    if directions_sets is not None:
        p.up_mask = _mask(directions_sets["up"])
        p.down_mask = _mask(directions_sets["down"])
        p.left_mask = _mask(directions_sets["left"])
        p.right_mask = _mask(directions_sets["right"])
    for v in range(256):
        p.effect[v] = -1
    for k, v in (effects or {}).items():
        k, v = int(k), int(v)
        if not (0 <= k <= 255 and 0 <= v <= 255):
            raise ValueError("effects must map u8 cell codes to u8 cell codes")
        p.effect[k] = v
    return p


def _run(params, grid, action_pair, position, with_grid):
    """One env through gca_move_modify. Returns (new_position, hit, grid_out)."""
    import torch

    device = dev.require_device()
    on_device = dev.is_device_tensor(grid)
    shape = tuple(grid.shape)
    H, W = shape[-2:]
    act = torch.tensor([[int(action_pair[0]), int(bool(action_pair[1]))]], dtype=torch.int32, device=device)
    pos = torch.tensor([[int(position[0]), int(position[1])]], dtype=torch.int32, device=device)
    hit = torch.zeros(1, dtype=torch.uint8, device=device)
    g = None
    if with_grid:
        if on_device:
            if grid.dtype != torch.uint8 or not grid.is_contiguous():
                raise ValueError("device grids must be contiguous uint8 tensors")
            g = grid
        else:
            arr = np.asarray(grid)
            if arr.size and (arr.min() < 0 or arr.max() > 255):
                raise ValueError("cell values must fit the u8 device layout (0..255)")
            g = dev.to_device(arr.astype(np.uint8), torch.uint8, device)
    call("gca_move_modify", params, dev.ptr(act), dev.ptr(pos), dev.ptr(g), H, W, dev.ptr(hit), 1,
         dev.stream_ptr(device))
    new_pos = pos.cpu().numpy()[0].astype(np.int64)
    h = bool(hit.item())
    if with_grid and not on_device:
        np.copyto(grid, g.cpu().numpy().astype(np.asarray(grid).dtype), casting="unsafe")  # in place, like :91
    return new_pos, h


class Move(Operator):
    grid_dependant = False
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, directions_sets, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.up_set = directions_sets["up"]
        self.down_set = directions_sets["down"]
        self.left_set = directions_sets["left"]
        self.right_set = directions_sets["right"]
        self.not_move_set = directions_sets["not_move"]
        self.movement_set = self.up_set | self.down_set | self.left_set | self.right_set | self.not_move_set
        self._params = make_params(directions_sets)

    def update(self, grid, action, context):
        new_pos, _ = _run(self._params, grid, (int(action), 0), context, with_grid=False)
        return grid, new_pos


class Modify(Operator):
    hit = False

    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, effects, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.effects = effects
        self._params = make_params(None, effects)

    def update(self, grid, action, context):
        self.hit = False
        if action:
            _, self.hit = _run(self._params, grid, (31, 1), context, with_grid=True)  # 31: no movement bit set
        return grid, context


class MoveModify(Operator):
    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, move, modify, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.suboperators = move, modify
        self.move = move
        self.modify = modify
        self._fused = None
        if self.action_space is None:
            if self.move.action_space is not None and self.move.action_space is not None:
                self.action_space = Tuple((self.move.action_space, self.move.action_space))
        if self.context_space is None:
            if self.move.context_space is not None and self.modify.context_space is not None:
                assert self.move.context_space == self.modify.context_space
                self.context_space = self.move.context_space

    def update(self, grid, subactions, position):
        move_action, modify_action = subactions
        if type(self.move) is Move and type(self.modify) is Modify:
            # both are this package's device operators: Move then Modify in ONE gca_move_modify launch
            # (the kernel moves first and modifies at the new position, move_modify.py:128-134)
            if self._fused is None:
                d = {"up": self.move.up_set, "down": self.move.down_set, "left": self.move.left_set,
                     "right": self.move.right_set}
                self._fused = make_params(d, self.modify.effects)
            shoot = bool(modify_action)
            position, hit = _run(self._fused, grid, (int(move_action), int(shoot)), position, with_grid=shoot)
            self.modify.hit = hit
            return grid, position
        grid, position = self.move(grid, move_action, position)
        grid, position = self.modify(grid, modify_action, position)
        return grid, position
