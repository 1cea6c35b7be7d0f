"""ForestFireBulldozerEnv — single-env drop-in (reference bulldozer.py:21-400).

Same constructor, spaces, operator graph (MDP = RepeatCA(WindyForestFire) then
MoveModify) and Gymnasium step/reset. The grid stays resident on the GPU between
steps: the CA passes, Move/Modify (one fused launch) and ONE cell count per step (shared
by _is_done and _award) run there; only the observation copy goes to the host
(numpy int64 like the reference's obs; `obs_device=True` returns the device u8 grid
instead and skips that copy). The batched version of the same MDP is
`BatchedForestFireBulldozerEnv` (batched.py); that is the performance path.

Deliberate difference: the reference crashes on its first CA step
because the context carries {"wind": W}; WindyForestFire here unwraps that dict.
"""
from typing import Optional, Tuple

import numpy as np

from ... import _device as dev
from ..._config import TYPE_BOX, TYPE_INT
from ..._lib import call
from ...ca_env import CAEnv
from ...grid_space import GridSpace
from ...operator import Operator
from ...spaces import Box, Discrete, MultiDiscrete
from ...spaces import Tuple as TupleSpace
from ..operators import Modify, Move, MoveModify, RepeatCA, WindyForestFire

DEFAULT_WIND = {
    "up_left": 0.48,
    "up": 0.64,
    "up_right": 0.98,
    "left": 0.12,
    "right": 0.64,
    "down_left": 0.06,
    "down": 0.12,
    "down_right": 0.48,
}


def parse_wind(windD: dict) -> np.ndarray:
    """bulldozer.py:299-316."""
    wind = np.array(
        [
            [windD["up_left"], windD["up"], windD["up_right"]],
            [windD["left"], 0.0, windD["right"]],
            [windD["down_left"], windD["down"], windD["down_right"]],
        ],
        dtype=TYPE_BOX,
    )
    assert Box(0.0, 1.0, shape=(3, 3), dtype=TYPE_BOX).contains(wind), "Bad Wind Data, check ranges [0.0, 1.0]"
    return wind


def bulldozer_timings(nrows, ncols, speed_move=0.12, speed_act=0.03, t_move=None, t_shoot=None, t_any=0.001):
    """Scale-dependent action times (bulldozer.py:111-135)."""
    scale = (nrows + ncols) // 2
    t_act_move = (1 / (speed_move * scale)) - t_any if t_move is None else t_move
    t_act_shoot = (1 / (speed_act * scale)) - t_act_move if t_shoot is None else t_shoot
    return t_act_move, t_act_shoot


MOVES = dict(up_left=0, up=1, up_right=2, left=3, not_move=4, right=5, down_left=6, down=7, down_right=8)
ACTION_SETS = {
    "up": {0, 1, 2},
    "down": {6, 7, 8},
    "left": {0, 3, 6},
    "right": {2, 5, 8},
    "not_move": {4},
}


class ForestFireBulldozerEnv(CAEnv):
    metadata = {"render_modes": ["human"], "render_mode": "rgb_array"}

    @property
    def MDP(self):
        return self._MDP

    @property
    def initial_state(self):
        if self._resample_initial:
            self.grid = self._initial_grid_distribution()
            self.context = self._initial_context_distribution()
            self._initial_state = self.grid, self.context
        self._resample_initial = False
        return self._initial_state

    def __init__(
        self,
        nrows,
        ncols,
        speed_move=0.12,
        speed_act=0.03,
        pos_bull: Optional[Tuple] = None,
        pos_fire: Optional[Tuple] = None,
        t_move: Optional[float] = None,
        t_shoot: Optional[float] = None,
        t_any=0.001,
        p_tree=0.90,
        p_empty=0.10,
        wind=DEFAULT_WIND,
        obs_device=False,
        **kwargs,
    ):
        super().__init__(nrows, ncols, **kwargs)
        self.obs_device = bool(obs_device)
        self._counts = None  # this step's device count (Counter), shared by _is_done and _award
        self._obs_host = None  # this step's observation, read back with the count
        self._obs_pinned = None
        self.title = "ForestFireBulldozer" + str(nrows) + "x" + str(ncols)
        self._shoots = {"shoot": 1, "none": 0}
        self._empty, self._tree, self._fire = 0, 3, 25
        self._pos_bull = pos_bull
        self._pos_fire = pos_fire
        self._p_tree = p_tree
        self._p_empty = p_empty
        self._wind = parse_wind(wind)
        self._effects = {self._tree: self._empty}
        self._t_env_any = t_any
        self._t_act_none = 0.0
        self._t_act_move, self._t_act_shoot = bulldozer_timings(nrows, ncols, speed_move, speed_act, t_move, t_shoot,
                                                                t_any)
        self._moves = dict(MOVES)
        self._action_sets = {k: set(v) for k, v in ACTION_SETS.items()}
        self._set_spaces()
        self._init_time_mappings()
        self.ca = WindyForestFire(self._empty, self._tree, self._fire, **self.ca_space)
        self.move = Move(self._action_sets, **self.move_space)
        self.modify = Modify(self._effects, **self.modify_space)
        self.move_modify = MoveModify(self.move, self.modify, **self.move_modify_space)
        self.repeater = RepeatCA(self.ca, self.time_per_action, self.time_per_state, **self.repeater_space)
        self._MDP = MDP(self.repeater, self.move_modify, **self.MDP_space)

    def render(self, mode="human"):  # rendering is out of scope
        return None

    # ------------------------------------------------------------------ device-resident state
    def _to_device_grid(self):
        """The env's grid as the device u8 tensor it lives in (a host array set by the caller is adopted)."""
        import torch

        if not dev.is_device_tensor(self.grid):
            arr = np.asarray(self.grid)
            if arr.size and (arr.min() < 0 or arr.max() > 255):
                raise ValueError("cell values must fit the u8 device layout (0..255)")
            self.grid = dev.to_device(arr.astype(np.uint8), torch.uint8, dev.require_device())
        return self.grid

    def _host_obs(self, obs):
        grid, ctx = obs
        if self.obs_device or not dev.is_device_tensor(grid):
            return obs
        if self._obs_host is not None:  # read back with this step's count (_step_counts)
            host, self._obs_host = self._obs_host, None
            return host, ctx
        return grid.cpu().numpy().astype(TYPE_INT), ctx

    def step(self, action):
        self._to_device_grid()
        self.state = self.grid, self.context
        self._counts = None  # Modify edits the grid in place: the count is per step, not per grid object
        self._obs_host = None
        # Move / Modify leave their read-back to this step's one synchronisation (_step_counts)
        self.move_modify.defer_sync = True
        try:
            obs, reward, terminated, truncated, info = super().step(action)
        finally:
            self.move_modify.defer_sync = False
            io = self.move_modify._io
            if io is not None and io.pending is not None:  # a step that never counted (done on entry, an error)
                io.sync_read()
        return self._host_obs(obs), reward, terminated, truncated, info

    def reset(self, *, seed=None, options=None):
        _, info = super().reset(seed=seed, options=options)
        self._to_device_grid()
        self.state = self.grid, self.context
        return self._host_obs(self.state), info

    def _award(self):
        """-(f / (t + f)) (bulldozer.py:180-213) from the step's one device count."""
        counts = self._step_counts()
        t = counts[self._tree]
        f = counts[self._fire]
        return -(f / (t + f))

    def _is_done(self):
        self.done = not bool(self._step_counts()[self._fire])

    def _step_counts(self):
        """One gca_count_cells per step: _is_done and then _award read the same count of the same grid. On the
        device the count, Move / Modify's position and hit and (unless obs_device) the observation come back in
        ONE synchronisation, through the MoveModify operator's pinned DeviceIO."""
        if self._counts is None:
            io = self.move_modify._io
            g = self.grid
            if (io is not None and getattr(self, "one_readback", True) and dev.is_device_tensor(g) and g.device == io.device
                    and g.is_contiguous()):
                self._counts = self._count_with(io, g)
            else:
                self._counts = self.count_cells(self.grid)
                if io is not None and io.pending is not None:  # resolve Move / Modify's hit and position now: _report
                    io.sync_read()                              # reads them before step() ends
        return self._counts

    def _count_with(self, io, g):
        import torch
        from collections import Counter

        H, W = g.shape[-2:]
        call("gca_count_cells", dev.ptr(g), 1, H, W, self._empty, self._tree, self._fire, io.p_counts,
             dev.stream_ptr(io.device))
        extra = ()
        if not self.obs_device:
            if self._obs_pinned is None or tuple(self._obs_pinned.shape) != tuple(g.shape):
                self._obs_pinned = torch.empty(tuple(g.shape), dtype=torch.uint8, pin_memory=True)
            extra = ((self._obs_pinned, g),)
        out = io.sync_read(extra)
        if extra:
            self._obs_host = self._obs_pinned.numpy().astype(TYPE_INT)
        c = out[5:8].tolist()
        return Counter({v: n for v, n in zip((self._empty, self._tree, self._fire), c) if n})

    def _report(self):
        return {"hit": self.modify.hit}

    def count_cells(self, grid=None):
        """Counts of EMPTY/TREE/FIRE computed by gca_count_cells on the device (host grids are uploaded)."""
        import torch
        from collections import Counter

        grid = self.grid if grid is None else grid
        device = dev.require_device()
        g = grid if dev.is_device_tensor(grid) else dev.to_device(np.asarray(grid).astype(np.uint8), torch.uint8,
                                                                   device)
        H, W = g.shape[-2:]
        g = g.contiguous()  # keep the operand referenced until the count has run
        counts = torch.empty(3, dtype=torch.int32, device=device)
        call("gca_count_cells", dev.ptr(g), 1, H, W, self._empty, self._tree, self._fire,
             dev.ptr(counts), dev.stream_ptr(device))
        c = counts.cpu().numpy().tolist()
        return Counter({v: n for v, n in zip((self._empty, self._tree, self._fire), c) if n})

    def _noise(self, ax_len):
        upper = int(ax_len * (1 / 12))
        if upper > 0:
            return self.np_random.choice(range(upper), size=1).item(0)
        return 0

    def _initial_grid_distribution(self):
        grid_space = GridSpace(
            values=[self._empty, self._tree, self._fire],
            probs=[self._p_empty, self._p_tree, 0.0],
            shape=(self.nrows, self.ncols),
        )
        grid = grid_space.sample()
        if self._pos_fire is None:
            r, c = (3 * self.nrows // 4), (1 * self.ncols // 4)
            self._pos_fire = r + self._noise(self.nrows), c + self._noise(self.ncols)
        r, c = self._pos_fire
        grid[r, c] = self._fire
        return grid

    def _initial_context_distribution(self):
        init_time = np.array(0.0)
        if self._pos_bull is None:
            r, c = (1 * self.nrows // 4), (3 * self.ncols // 4)
            r = r + self._noise(self.nrows)
            c = c + self._noise(self.ncols)
            self._pos_bull = r, c
        init_position = np.array(self._pos_bull)
        return ({"wind": self._wind}, init_position, np.array(init_time, dtype=TYPE_BOX))

    def _init_time_mappings(self):
        self._movement_timings = {move: self._t_act_move for move in self._moves.values()}
        self._shooting_timings = {shoot: self._t_act_shoot for shoot in self._shoots.values()}
        self._movement_timings[self._moves["not_move"]] = self._t_act_none
        self._shooting_timings[self._shoots["none"]] = self._t_act_none

        def time_per_action(action):
            move, shoot = action
            return self._movement_timings[int(move)] + self._shooting_timings[int(shoot)]

        self.time_per_action = time_per_action
        self.time_per_state = lambda s: self._t_env_any

    def _set_spaces(self):
        self.grid_space = GridSpace(values=[self._empty, self._tree, self._fire], shape=(self.nrows, self.ncols))
        self.ca_params_space = Box(0.0, 1.0, shape=(3, 3), dtype=TYPE_BOX)
        self.position_space = MultiDiscrete([self.nrows, self.ncols], dtype=TYPE_INT)
        self.time_space = Box(0.0, float("inf"), shape=tuple(), dtype=TYPE_BOX)
        self.context_space = TupleSpace((self.ca_params_space, self.position_space, self.time_space))
        m, n = len(self._moves), len(self._shoots)
        self.action_space = MultiDiscrete([m, n], dtype=TYPE_INT)
        self.observation_space = TupleSpace((self.grid_space, self.context_space))
        self.ca_space = {"grid_space": self.grid_space, "action_space": self.action_space,
                         "context_space": self.ca_params_space}
        self.move_space = {"grid_space": self.grid_space, "action_space": Discrete(m),
                           "context_space": self.position_space}
        self.modify_space = {"grid_space": self.grid_space, "action_space": Discrete(n),
                             "context_space": self.position_space}
        self.move_modify_space = {"grid_space": self.grid_space, "action_space": self.action_space,
                                  "context_space": self.position_space}
        self.repeater_space = {"grid_space": self.grid_space, "action_space": self.action_space,
                               "context_space": TupleSpace((self.ca_params_space, self.time_space))}
        self.MDP_space = {"grid_space": self.grid_space, "action_space": self.action_space,
                          "context_space": self.context_space}


class MDP(Operator):
    """bulldozer.py:378-400: RepeatCA then MoveModify."""

    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = False

    def __init__(self, repeat_ca, move_modify, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.repeat_ca = repeat_ca
        self.move_modify = move_modify
        self.suboperators = self.repeat_ca, self.move_modify

    def update(self, grid, action, context):
        ca_params, position, time = context
        grid, (ca_params, time) = self.repeat_ca(grid, action, (ca_params, time))
        grid, position = self.move_modify(grid, action, position)
        return grid, (ca_params, position, time)
