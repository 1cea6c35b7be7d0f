"""BatchedForestFireBulldozerEnv — E ForestFireBulldozer envs resident in HBM.

The batched form of bulldozer.py's MDP (reference bulldozer.py:378-400 +
ca_env.py:27-62), one env per lane of the env kernels and one strip of rows per
wave of the CA kernel:

    gca_bulldozer_pre        RepeatCA time bookkeeping (repeat_ca.py:32-45), dir mask (ca_windy.py:53-77)
    gca_windy_step  x P      the CA passes (P = max repeats any action can trigger)
    gca_bulldozer_interpass  between passes (parity flip + next roll)
    gca_bulldozer_post       Move/Modify (move_modify.py:128-134), reward/done (bulldozer.py:180-216)

or, when every action takes less than one time unit (one CA pass at most per env step) and W is 256 or 512 (the
bench configs 2 and 5), the same step in ONE launch (gca_bulldozer_step_fused: a workgroup per env; envs without a CA
step this env step leave after their O(1) work). `fused=None` picks it whenever it applies; the two paths are
checked to give identical envs (tests/test_gpu_windy.py).

Grids live in two buffers; env e's current grid is buf[parity[e]][e], so envs whose
RepeatCA yields 0 repeats this step (most of them: ~1 CA step per 13 env steps at
256^2 with random actions) move no bytes at all. Cell counts are
fused into the CA kernel and patched by Modify, so reward/done are O(1) per env.
"""
import math

import numpy as np

from ... import _device as dev
from ..._lib import SLOT, BoundCall, call
from ..operators.move_modify import make_params
from .bulldozer import ACTION_SETS, DEFAULT_WIND, bulldozer_timings, parse_wind


# state the pre-bound calls hold by address (step, step_random, sample_actions): assigning one of these attributes
# validates the replacement and drops the bound calls (rebind), so the next step binds the new tensor
_BOUND_STATE = frozenset({"buf", "parity", "accu", "steps", "dir_mask", "counts", "pos", "rng_step", "done", "hit",
                          "reward", "wind", "steps_elapsed", "params", "_meet", "_act_buf"})


class BatchedForestFireBulldozerEnv:
    def __setattr__(self, name, value):
        d = self.__dict__
        if name in _BOUND_STATE and "_fused_call" in d and d.get(name) is not value:
            old = d.get(name)
            if name == "params":
                if type(value) is not type(old):
                    raise TypeError(f"params must stay a {type(old).__name__}")
            elif name == "_meet" and value is None:
                pass
            elif not (dev.is_device_tensor(value) and value.dtype == old.dtype and value.shape == old.shape
                      and value.device == old.device and value.is_contiguous()):
                raise ValueError(f"env.{name}: the replacement must be a contiguous {old.dtype} tensor of shape "
                                 f"{tuple(old.shape)} on {old.device} (or update the tensor in place)")
            object.__setattr__(self, name, value)
            self.rebind()
            return
        object.__setattr__(self, name, value)

    def __init__(self, num_envs, nrows, ncols, device=None, seed=0, env_offset=0, speed_move=0.12, speed_act=0.03,
                 t_move=None, t_shoot=None, t_any=0.001, p_tree=0.90, p_empty=0.10, wind=DEFAULT_WIND,
                 materialize_obs=True, fused=None):
        import torch

        self.device = dev.require_device(device)
        self.num_envs, self.nrows, self.ncols = E, H, W = int(num_envs), int(nrows), int(ncols)
        self.seed_value = int(seed)
        self.env_offset = int(env_offset)
        self.materialize_obs = materialize_obs
        self._empty, self._tree, self._fire = 0, 3, 25
        self._p_tree, self._p_empty = p_tree, p_empty
        t_act_move, t_act_shoot = bulldozer_timings(H, W, speed_move, speed_act, t_move, t_shoot, t_any)
        self.t_act_move, self.t_act_shoot, self.t_any = t_act_move, t_act_shoot, t_any
        p = make_params(ACTION_SETS, {self._tree: self._empty})
        for a in range(9):
            p.t_move[a] = 0.0 if a == 4 else t_act_move  # not_move costs _t_act_none (bulldozer.py:285)
        p.t_shoot[0], p.t_shoot[1] = 0.0, t_act_shoot
        p.t_any = t_any
        p.seed = self.seed_value & (2**64 - 1)
        p.env_offset = self.env_offset
        p.empty, p.tree, p.fire = self._empty, self._tree, self._fire
        self.params = p
        max_t = max(p.t_move[a] for a in range(9)) + max(p.t_shoot[0], p.t_shoot[1]) + t_any
        self.max_passes = int(math.floor(1.0 + max_t))  # accu < 1 before the step
        # gca_bulldozer_step_fused's contract: W = 256 / 512, one pass at most, empty == 0 < tree < fire (the closed-form
        # rule's code ordering); anything else takes the three-kernel step
        fusable = (self.max_passes == 1 and W in (256, 512) and self._empty == 0
                   and self._empty < self._tree < self._fire)
        if fused and not fusable:
            raise ValueError("fused=True needs W in (256, 512), at most one CA pass per env step and codes "
                             "empty = 0 < tree < fire")
        self.fused = fusable if fused is None else bool(fused)
        kw = dict(device=self.device)
        self.buf = torch.zeros((2, E, H, W), dtype=torch.uint8, **kw)
        self.parity = torch.zeros(E, dtype=torch.uint8, **kw)
        self.accu = torch.zeros(E, dtype=torch.float64, **kw)
        self.steps = torch.zeros(E, dtype=torch.int32, **kw)
        self.dir_mask = torch.zeros(E, dtype=torch.uint8, **kw)
        self.counts = torch.zeros((E, 3), dtype=torch.int32, **kw)
        self.pos = torch.zeros((E, 2), dtype=torch.int32, **kw)
        self.rng_step = torch.zeros(E, dtype=torch.int32, **kw)  # uint32 bits
        self.done = torch.zeros(E, dtype=torch.uint8, **kw)
        self.hit = torch.zeros(E, dtype=torch.uint8, **kw)
        self.reward = torch.zeros(E, dtype=torch.float64, **kw)
        w = parse_wind(wind) if isinstance(wind, dict) else np.asarray(wind, dtype=np.float64)
        self.wind = dev.to_device(np.broadcast_to(w.reshape(-1, 9), (E, 9)), torch.float64, self.device)
        self.steps_elapsed = torch.zeros(E, dtype=torch.int64, **kw)
        # the fused step's per-env meeting slots (gca_bulldozer_step_fused: several workgroups per env), kept zero
        self._meet = torch.zeros(E, dtype=torch.int64, **kw)
        self._truncated = torch.zeros(E, dtype=torch.bool, **kw)
        # the eager step's host path: persistent outputs and pre-bound C-ABI calls, so a step is
        # one action check, one raw-stream read and one prepared ctypes call
        self._dev_index = dev.device_index(self.device)
        self._act_buf = torch.zeros((E, 2), dtype=torch.int32, **kw)
        self._act_shape = self._act_buf.shape
        self._done_bool = self.done.view(torch.bool)
        self._info = {"hit": self.hit, "ca_steps": self.steps}
        self._ctx = {"wind": self.wind, "position": self.pos, "time": self.accu}
        self._fused_call = self._bound_meet = None
        self._sample_call = None
        self._random_call = self._bound_meet_r = None

    # ------------------------------------------------------------------ state
    def grids(self):
        """(E, H, W) uint8 view of every env's current grid (one gather pass)."""
        import torch

        return torch.where(self.parity.bool()[:, None, None], self.buf[1], self.buf[0])

    def reset(self, seed=None, grids=None, positions=None):
        """Reset all envs. Initial distribution of bulldozer.py:233-275: the grid from Philox per cell, the fire /
        bulldozer noise from per-env draws keyed by the global env id (_seeding), so a sharded env reproduces the
        unsharded one env for env."""
        import torch

        from ..._seeding import env_integers

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        s = self.seed_value if seed is None else int(seed)
        noise = lambda tag, n: env_integers(s, self.env_offset, E, tag, 0, max(1, int(n / 12)))
        if grids is not None:
            self.buf[0].copy_(dev.to_device(np.asarray(grids).reshape(E, H, W).astype(np.uint8), torch.uint8,
                                            self.device))
        else:
            cdf = torch.tensor([self._p_empty, self._p_empty + self._p_tree, 1.0], dtype=torch.float32,
                               device=self.device)
            vals = torch.tensor([self._empty, self._tree, self._fire], dtype=torch.uint8, device=self.device)
            call("gca_fill_categorical", dev.ptr(self.buf[0]), H * W, E, self.env_offset,
                 (self.seed_value if seed is None else int(seed)) & (2**64 - 1), dev.ptr(cdf), dev.ptr(vals), 3, st)
            # one FIRE around the lower-left quadrant, noise in [0, N/12) (bulldozer.py:221-253)
            fr = 3 * H // 4 + noise(1, H)
            fc = W // 4 + noise(2, W)
            idx = torch.arange(E, device=self.device)
            self.buf[0][idx, torch.as_tensor(fr, device=self.device), torch.as_tensor(fc, device=self.device)] = \
                self._fire
        if positions is not None:
            pos = np.asarray(positions).reshape(E, 2)
            if not ((pos[:, 0] >= 0) & (pos[:, 0] < H) & (pos[:, 1] >= 0) & (pos[:, 1] < W)).all():
                raise ValueError(f"reset: every position must lie inside the {H}x{W} grid")
        else:
            pos = np.stack([H // 4 + noise(3, H), 3 * W // 4 + noise(4, W)], axis=1)
        self.pos.copy_(torch.as_tensor(pos.astype(np.int32), device=self.device))
        self.parity.zero_()
        self.accu.zero_()
        self.done.zero_()
        self.hit.zero_()
        self.rng_step.zero_()
        self.steps_elapsed.zero_()
        call("gca_count_cells", dev.ptr(self.buf[0]), E, H, W, self._empty, self._tree, self._fire,
             dev.ptr(self.counts), st)
        return self._obs(), {"hit": self.hit}

    def _obs(self):
        return (self.grids() if self.materialize_obs else None), self._ctx

    def _action(self, action):
        """action as a contiguous int32 (E, 2) device tensor: the caller's own tensor when it is one (checked on every
        call: a tensor retyped or reshaped in place since the last step is converted, not misread), else converted
        into the env's action buffer."""
        import torch

        if (type(action) is torch.Tensor and action.dtype is torch.int32 and action.get_device() == self._dev_index
                and action.shape == self._act_shape and action.is_contiguous()):
            return action
        src = action if dev.is_device_tensor(action) else torch.as_tensor(np.asarray(action))
        self._act_buf.copy_(src.reshape(self.num_envs, 2))
        return self._act_buf

    def rebind(self):
        """Drop the pre-bound step calls. The env's state tensors (buf, accu, steps, done, wind, rng_step, parity, pos,
        counts, hit, reward, steps_elapsed) and params are bound by address on the first fused step; every method here
        updates them in place. Assigning a new tensor to one of them (env.wind = w) calls this by itself
        (__setattr__, which also checks the replacement's dtype / shape / device); the bound calls hold references to
        what they bound, so nothing they address is ever freed under them."""
        import torch

        self._fused_call = self._bound_meet = None
        self._sample_call = None
        self._random_call = self._bound_meet_r = None
        self._done_bool = self.done.view(torch.bool)
        self._info = {"hit": self.hit, "ca_steps": self.steps}
        self._ctx = {"wind": self.wind, "position": self.pos, "time": self.accu}

    def _bound_tensors(self):
        return (self.params, self.accu, self.steps, self.done, self.wind, self.rng_step, self.parity, self.buf,
                self.pos, self.counts, self.hit, self.reward, self.steps_elapsed, self._meet)

    def _bind_fused(self):
        E, H, W = self.num_envs, self.nrows, self.ncols
        meet = self._meet
        self._fused_call = BoundCall(
            "gca_bulldozer_step_fused", self.params, SLOT, dev.ptr(self.accu), dev.ptr(self.steps), dev.ptr(self.done),
            dev.ptr(self.wind), 9, dev.ptr(self.rng_step), dev.ptr(self.parity), dev.ptr(self.buf[0]),
            dev.ptr(self.buf[1]), H, W, dev.ptr(self.pos), dev.ptr(self.counts), dev.ptr(self.hit),
            dev.ptr(self.reward), dev.ptr(self.steps_elapsed), dev.ptr(meet) if meet is not None else None, E, SLOT,
            keep=self._bound_tensors())
        self._bound_meet = meet
        return self._fused_call

    def step_random(self, seed=9, action_out=None):
        """One env step of every env under a uniform random policy, the action drawn INSIDE the fused step
        (gca_bulldozer_step_fused_random) exactly as sample_actions(out, tag=seed) draws it before step(out): the two
        launches in one, bit for bit. The drawn actions go to `action_out` (a contiguous int32 (E, 2) device tensor,
        default the env's action buffer). Fused step only (W = 256 / 512, one CA pass at most per env step)."""
        if not self.fused:
            raise ValueError("step_random needs the fused step (W in (256, 512), at most one CA pass per env step)")
        import torch

        out = self._act_buf if action_out is None else action_out
        if not (type(out) is torch.Tensor and out.dtype is torch.int32 and out.get_device() == self._dev_index
                and out.shape == self._act_shape and out.is_contiguous()):
            raise ValueError("step_random: action_out must be a contiguous int32 (E, 2) tensor on the env's device")
        key = (seed, out.data_ptr())
        rc = self._random_call
        if rc is None or rc[0] != key or rc[1] is not out or self._bound_meet_r is not self._meet:
            E, H, W = self.num_envs, self.nrows, self.ncols
            meet = self._meet
            self._random_call = (key, out, BoundCall(
                "gca_bulldozer_step_fused_random", self.params, int(seed) & (2**64 - 1), dev.ptr(out),
                dev.ptr(self.accu), dev.ptr(self.steps), dev.ptr(self.done), dev.ptr(self.wind), 9,
                dev.ptr(self.rng_step), dev.ptr(self.parity), dev.ptr(self.buf[0]), dev.ptr(self.buf[1]), H, W,
                dev.ptr(self.pos), dev.ptr(self.counts), dev.ptr(self.hit), dev.ptr(self.reward),
                dev.ptr(self.steps_elapsed), dev.ptr(meet) if meet is not None else None, E, SLOT,
                keep=self._bound_tensors() + (out,)))
            self._bound_meet_r = meet
        self._random_call[2](dev.raw_stream(self._dev_index))
        return self._obs(), self.reward, self._done_bool, self._truncated, self._info

    def rollout_random(self, K, seed=9, action_out=None, reward_out=None, done_out=None):
        """K env steps of every env in ONE launch under the random policy of step_random (gca_bulldozer_rollout_random):
        bit for bit K calls of step_random(seed), the env's state kept in registers across the steps. Optional per-step
        records, device tensors: action_out int32 (K, E, 2), reward_out float64 (K, E), done_out uint8 (K, E). Returns
        (reward_out, done_out). Fused step only (W = 256 / 512, one CA pass at most per env step)."""
        import torch

        if not self.fused:
            raise ValueError("rollout_random needs the fused step (W in (256, 512), at most one CA pass per env step)")
        K, E = int(K), self.num_envs
        if K < 0:
            raise ValueError("rollout_random: K >= 0")
        for name, t, dt, shape in (("action_out", action_out, torch.int32, (K, E, 2)),
                                   ("reward_out", reward_out, torch.float64, (K, E)),
                                   ("done_out", done_out, torch.uint8, (K, E))):
            if t is not None and not (type(t) is torch.Tensor and t.dtype == dt and tuple(t.shape) == shape
                                      and t.device == self.device and t.is_contiguous()):
                raise ValueError(f"rollout_random: {name} must be a contiguous {dt} {shape} tensor on the env's device")
        H, W = self.nrows, self.ncols
        call("gca_bulldozer_rollout_random", self.params, int(seed) & (2**64 - 1), K, dev.ptr(action_out),
             dev.ptr(reward_out), dev.ptr(done_out), dev.ptr(self.accu), dev.ptr(self.steps), dev.ptr(self.done),
             dev.ptr(self.wind), 9, dev.ptr(self.rng_step), dev.ptr(self.parity), dev.ptr(self.buf[0]),
             dev.ptr(self.buf[1]), H, W, dev.ptr(self.pos), dev.ptr(self.counts), dev.ptr(self.hit), dev.ptr(self.reward),
             dev.ptr(self.steps_elapsed), E, dev.stream_ptr(self.device))
        return reward_out, done_out

    def sample_actions(self, out=None, tag=9):
        """Uniform random actions for every env on the device -- the batched `action_space.sample()` (move in [0, 9),
        shoot in {0, 1}; Philox keyed by (tag, global env id, the env's rng_step)) -- into `out` (a contiguous int32
        (E, 2) device tensor) or the env's action buffer. Returns the tensor."""
        import torch

        out = self._act_buf if out is None else out
        if not (type(out) is torch.Tensor and out.dtype is torch.int32 and out.get_device() == self._dev_index
                and out.shape == self._act_shape and out.is_contiguous()):
            raise ValueError("sample_actions: out must be a contiguous int32 (E, 2) tensor on the env's device")
        sc = self._sample_call
        if sc is None or sc[0] is not out or sc[1] != tag or sc[2] != out.data_ptr():
            self._sample_call = (out, tag, out.data_ptr(),
                                 BoundCall("gca_random_actions", dev.ptr(out), self.num_envs, self.env_offset, tag,
                                           dev.ptr(self.rng_step), SLOT, keep=(out, self.rng_step)))
        self._sample_call[3](dev.raw_stream(self._dev_index))
        return out

    # ------------------------------------------------------------------ step
    def step(self, action):
        """action: (E, 2) int (move in [0,9), shoot in {0,1}); device tensor or numpy. Returns (obs, reward,
        terminated, truncated, info) as device tensors that the next step overwrites in place (terminated is a bool
        view of `done`, truncated a persistent all-False tensor, info one persistent dict: no kernel launch and no
        allocation per step); clone to keep them. A contiguous int32 (E, 2) device action is used as it is."""
        a = self._action(action)
        if self.fused:
            fc = self._fused_call if self._bound_meet is self._meet else None
            if fc is None:
                fc = self._bind_fused()
            fc(a.data_ptr(), dev.raw_stream(self._dev_index))
            # done is 0 / 1 bytes: a bool view, no kernel; truncated is a persistent all-False tensor
            return self._obs(), self.reward, self._done_bool, self._truncated, self._info
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        p = self.params
        call("gca_bulldozer_pre", p, dev.ptr(a), dev.ptr(self.accu), dev.ptr(self.steps), dev.ptr(self.done),
             dev.ptr(self.wind), 9, dev.ptr(self.rng_step), dev.ptr(self.dir_mask), dev.ptr(self.counts), E, st)
        P = self.max_passes
        for pss in range(P):
            call("gca_windy_step", dev.ptr(self.buf[0]), dev.ptr(self.buf[1]), dev.ptr(self.parity),
                 dev.ptr(self.steps), pss, dev.ptr(self.dir_mask), E, H, W, self._empty, self._tree, self._fire, 0,
                 dev.ptr(self.counts), st)
            if pss < P - 1:
                call("gca_bulldozer_interpass", p, pss, dev.ptr(self.steps), dev.ptr(self.parity),
                     dev.ptr(self.wind), 9, dev.ptr(self.rng_step), dev.ptr(self.dir_mask), dev.ptr(self.counts), E,
                     st)
        call("gca_bulldozer_post", p, P - 1, dev.ptr(a), dev.ptr(self.steps), dev.ptr(self.parity),
             dev.ptr(self.buf[0]), dev.ptr(self.buf[1]), H, W, dev.ptr(self.pos), dev.ptr(self.counts),
             dev.ptr(self.rng_step), dev.ptr(self.done), dev.ptr(self.hit), dev.ptr(self.reward), E, st)
        self.steps_elapsed += (self.steps >= 0).to(torch.int64)
        return self._obs(), self.reward, self._done_bool, self._truncated, self._info

    def ca_step_all(self, dir_mask=None):
        """One forced WindyForestFire step of every env (bench 'CA-only' mode, steps[E] = 1)."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        call("gca_windy_step", dev.ptr(self.buf[0]), dev.ptr(self.buf[1]), dev.ptr(self.parity), None, 0,
             dev.ptr(self.dir_mask if dir_mask is None else dir_mask), E, H, W, self._empty, self._tree, self._fire,
             0, None, st)
        self.parity ^= 1
