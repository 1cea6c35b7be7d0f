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


class DeviceIO:
    """One env's Move / Modify operands and results, staged through pinned host memory: int32[8] =
    [move, shoot, row, col, hit (u8 in the low byte), n_empty, n_tree, n_fire] on the device, one pinned copy each
    way. A call costs one H2D copy, the launch, one D2H copy and ONE synchronisation (the eager version cost two
    pageable uploads and two synchronising reads). `pending` defers even that synchronisation: the bulldozer env
    reads the position and hit back together with its cell count and observation (bulldozer.py, _step_counts)."""

    def __init__(self, device):
        import torch

        self.device = device
        self.h_in = torch.zeros(8, dtype=torch.int32, pin_memory=True)
        self.h_out = torch.zeros(8, dtype=torch.int32, pin_memory=True)
        self.d = torch.zeros(8, dtype=torch.int32, device=device)
        self.n_in, self.n_out = self.h_in.numpy(), self.h_out.numpy()
        base = self.d.data_ptr()
        self.p_act, self.p_pos, self.p_hit, self.p_counts = base, base + 8, base + 16, base + 20
        self.in_flight = False  # h_in has been handed to a copy that no synchronisation has covered yet
        self.pending = None  # (position array to fill, Modify whose hit to set) of a deferred call

    def stage(self, a0, a1, row, col):
        if self.in_flight:  # the previous call's upload must have run before its pinned source is rewritten
            self.sync_read()
        self.n_in[:] = (a0, a1, row, col, 0, 0, 0, 0)
        self.d.copy_(self.h_in, non_blocking=True)
        self.in_flight = True

    def sync_read(self, extra=()):
        """D2H of the results (+ `extra` (pinned dst, device src) pairs), one synchronisation, deferred results
        filled in. Returns the host int32[8]."""
        import torch

        self.h_out.copy_(self.d, non_blocking=True)
        for dst, src in extra:
            dst.copy_(src, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        self.in_flight = False
        if self.pending is not None:
            pos, modify = self.pending
            self.pending = None
            pos[0], pos[1] = int(self.n_out[2]), int(self.n_out[3])
            if modify is not None:
                modify.hit = bool(self.n_out[4])
        return self.n_out


def _moved(params, a, row, col, H, W):
    """Move's arithmetic (move_modify.py:37-67) on the host, for validating a position before a device Modify."""
    if 0 <= a < 32:
        vu, vd, vl, vr = row > 0, row < H - 1, col > 0, col < W - 1
        row -= 1 if (params.up_mask >> a) & 1 and vu else 0
        row += 1 if (params.down_mask >> a) & 1 and vd else 0
        col -= 1 if (params.left_mask >> a) & 1 and vl else 0
        col += 1 if (params.right_mask >> a) & 1 and vr else 0
    return row, col


def _run(params, grid, action_pair, position, with_grid, backend=None, io=None, defer=None):
    """One env through gca_move_modify. Returns (new_position, hit); the grid is modified in place.
    `io` (DeviceIO) stages a device grid's call through pinned memory; with `defer` = the Modify to update, the
    synchronisation is left to the caller's next io.sync_read(): the returned position array is filled, and
    defer.hit set, then (hit is returned as None)."""
    import torch

    on_device = dev.is_device_tensor(grid)
    if _backend.choose(backend, on_device, 0, o1=True) == "cpu":
        return _run_host(params, grid, action_pair, position, with_grid)
    device = dev.require_device()
    shape = tuple(grid.shape)
    H, W = shape[-2:]
    if on_device and io is not None:
        r, c = int(position[0]), int(position[1])
        if with_grid:
            if grid.dtype != torch.uint8 or not grid.is_contiguous():
                raise ValueError("device grids must be contiguous uint8 tensors")
            if not (0 <= r < H and 0 <= c < W):  # a caller's own out-of-grid start: refused, like the host build,
                mr, mc = _moved(params, int(action_pair[0]), r, c, H, W)  # unless the move brings it inside
                if not (0 <= mr < H and 0 <= mc < W):
                    raise GCAError(f"move_modify: position ({mr}, {mc}) outside the {H}x{W} grid")
        io.stage(int(action_pair[0]), int(bool(action_pair[1])), r, c)
        call("gca_move_modify", params, io.p_act, io.p_pos, dev.ptr(grid) if with_grid else None, H, W, io.p_hit, 1,
             dev.stream_ptr(device))
        if defer is not None:
            new_pos = np.empty(2, dtype=np.int64)
            io.pending = (new_pos, defer)
            return new_pos, None
        out = io.sync_read()
        return out[2:4].astype(np.int64), bool(out[4])
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
        self._io = None  # DeviceIO of the fused device call, made on first use
        # set by an env that reads the results back itself (ForestFireBulldozerEnv.step): the returned position is
        # filled, and modify.hit set, by that env's next self._io.sync_read()
        self.defer_sync = False
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
            io = None
            if dev.is_device_tensor(grid):
                if self._io is None or self._io.device != grid.device:
                    self._io = DeviceIO(grid.device)
                io = self._io
            defer = self.modify if (self.defer_sync and io is not None) else None
            position, hit = _run(self._fused, grid, (int(move_action), int(shoot)), position, with_grid=shoot,
                                 backend=backend, io=io, defer=defer)
            if defer is None:
                self.modify.hit = hit
            return grid, position
        grid, position = self.move(grid, move_action, position)
        grid, position = self.modify(grid, modify_action, position)
        return grid, position
