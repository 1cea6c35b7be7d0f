"""Move / Modify / MoveModify — drop-ins for the reference operators (move_modify.py:10-134).

The arithmetic is gca_move_modify (include/gca.h): the device kernel (one lane per env) for device tensors, the
host build of the same symbol (libgca_cpu.so) for host arrays — the work is O(1) per env, so a device round
trip would cost far more than the call (backend="hip" forces the kernel, see gymca_amd/_backend.py). Semantics:
Move applies the four direction sets in order with bounds checks (:37-67); Modify
substitutes `effects[grid[row, col]]` IN PLACE and sets `self.hit` (:84-94).
"""
import numpy as np

from ... import _backend
from ... import _device as dev
from ..._lib import BulldozerParams, GCAError, call, call_cpu
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


_SCRATCH = _backend.Scratch()


def _run_host(params, grid, action_pair, position, with_grid):
    """One env through the host build of gca_move_modify (O(1): only the target cell is touched); the grid is
    modified in place."""
    arr = grid if isinstance(grid, np.ndarray) else np.asarray(grid)
    H, W = arr.shape[-2:]
    act, p_act = _SCRATCH.get("act", (1, 2), np.int32)
    pos, p_pos = _SCRATCH.get("pos", (1, 2), np.int32)
    hit, p_hit = _SCRATCH.get("hit", (1,), np.uint8)
    act[0, 0], act[0, 1] = int(action_pair[0]), int(bool(action_pair[1]))
    pos[0, 0], pos[0, 1] = int(position[0]), int(position[1])
    hit[0] = 0
    if with_grid and arr is grid and arr.dtype == np.uint8 and arr.flags["C_CONTIGUOUS"]:
        call_cpu("gca_move_modify", params, p_act, p_pos, arr.ctypes.data, H, W, p_hit, 1, None)
        return pos[0].astype(np.int64), bool(hit[0])
    if with_grid and arr.ndim == 2 and H * W <= _backend.HOST_MAX_CELLS:  # small grid: one call on a u8 copy
        g8, p_g8 = _SCRATCH.get("grid", (H, W), np.uint8)
        if arr.size and (arr.min() < 0 or arr.max() > 255):
            raise ValueError("cell values must fit the u8 layout (0..255)")
        np.copyto(g8, arr, casting="unsafe")
        call_cpu("gca_move_modify", params, p_act, p_pos, p_g8, H, W, p_hit, 1, None)
        if hit[0]:
            r, c = int(pos[0, 0]), int(pos[0, 1])
            grid[r, c] = g8[r, c]
        return pos[0].astype(np.int64), bool(hit[0])
    call_cpu("gca_move_modify", params, p_act, p_pos, None, H, W, None, 1, None)  # Move
    if with_grid:  # Modify of the one cell under the new position (move_modify.py:84-94), written back in place
        r, c = int(pos[0, 0]), int(pos[0, 1])
        if arr.ndim != 2 or not (0 <= r < H and 0 <= c < W):  # numpy would wrap a negative index: refuse like the C path
            raise GCAError(f"gca_move_modify (host backend) failed: argument: move_modify: position ({r}, {c}) "
                           f"outside the {H}x{W} grid" if arr.ndim == 2 else
                           "gca_move_modify (host backend) failed: argument: the grid must be 2-D (one env)")
        v = int(arr[r, c])
        if not 0 <= v <= 255:
            raise ValueError("cell values must fit the u8 layout (0..255)")
        cell, p_cell = _SCRATCH.get("cell", (1, 1), np.uint8)
        act1, p_act1 = _SCRATCH.get("act1", (1, 2), np.int32)
        pos1, p_pos1 = _SCRATCH.get("pos1", (1, 2), np.int32)
        cell[0, 0] = v
        act1[0, 0], act1[0, 1] = 31, 1  # 31: no movement bit set
        pos1[0, 0] = pos1[0, 1] = 0
        call_cpu("gca_move_modify", params, p_act1, p_pos1, p_cell, 1, 1, p_hit, 1, None)
        if hit[0]:
            grid[r, c] = cell[0, 0]
    return pos[0].astype(np.int64), bool(hit[0])


def _run(params, grid, action_pair, position, with_grid, backend=None):
    """One env through gca_move_modify. Returns (new_position, hit); the grid is modified in place."""
    import torch

    on_device = dev.is_device_tensor(grid)
    if _backend.choose(backend, on_device, 0, o1=True) == "cpu":
        return _run_host(params, grid, action_pair, position, with_grid)
    device = dev.require_device()
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

    def __init__(self, directions_sets, *args, backend=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.backend = backend
        self.up_set = directions_sets["up"]
        self.down_set = directions_sets["down"]
        self.left_set = directions_sets["left"]
        self.right_set = directions_sets["right"]
        self.not_move_set = directions_sets["not_move"]
        self.movement_set = self.up_set | self.down_set | self.left_set | self.right_set | self.not_move_set
        self._params = make_params(directions_sets)

    def update(self, grid, action, context):
        new_pos, _ = _run(self._params, grid, (int(action), 0), context, with_grid=False, backend=self.backend)
        return grid, new_pos


class Modify(Operator):
    hit = False

    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = True

    def __init__(self, effects, *args, backend=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.backend = backend
        self.effects = effects
        self._params = make_params(None, effects)

    def update(self, grid, action, context):
        self.hit = False
        if action:
            _, self.hit = _run(self._params, grid, (31, 1), context, with_grid=True,  # 31: no movement bit set
                               backend=self.backend)
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
            backend = self.move.backend if self.move.backend == self.modify.backend else None
            position, hit = _run(self._fused, grid, (int(move_action), int(shoot)), position, with_grid=shoot,
                                 backend=backend)
            self.modify.hit = hit
            return grid, position
        grid, position = self.move(grid, move_action, position)
        grid, position = self.modify(grid, modify_action, position)
        return grid, position
