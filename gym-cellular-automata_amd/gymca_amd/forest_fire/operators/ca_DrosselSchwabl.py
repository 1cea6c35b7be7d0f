"""Drossel–Schwabl forest fire on the GPU — drop-in for ForestFire (ca_DrosselSchwabl.py:11-66).

Exact-stream semantics: the reference draws one f64 uniform from `self.np_random` per
TREE-without-burning-neighbour and per EMPTY cell, in row-major order
(Generator.choice with p: one random() per call). Here the device counts those cells
(gca_ds_count_draws), the SAME number of uniforms is drawn from `self.np_random`, and
gca_ds_step consumes them in the same order — so a seeded operator reproduces the
reference cell for cell (tests/golden/drossel.npz).

Grids of at most HOST_MAX_CELLS cells on host arrays (BASELINE config 1, the 5x5 helicopter) run the host build of
the same two entry points (libgca_cpu.so, gymca_amd/_backend.py); device tensors and larger grids the kernels.
"""
import numpy as np

from ... import _backend
from ... import _device as dev
from ..._config import TYPE_BOX
from ..._lib import call, call_cpu
from ...operator import Operator
from ...spaces import Box


def normalize_p(p):
    p = np.asarray(p).astype("float64")
    return p / np.sum(p)


def choice_threshold(p):
    """cdf[0] of Generator.choice([True, False], p=normalize_p([p, 1 - p])): True iff u < cdf[0]."""
    cdf = normalize_p([p, 1 - p]).cumsum()
    cdf /= cdf[-1]
    return float(cdf[0])


class ForestFire(Operator):
    grid_dependant = True
    action_dependant = False
    context_dependant = True

    deterministic = False

    def __init__(self, empty, tree, fire, *args, backend=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.backend = backend
        self._thr_cache = (None, None)
        self._scratch = _backend.Scratch()
        self.empty, self.tree, self.fire = empty, tree, fire
        dev.check_u8_codes((empty, tree, fire))
        if self.context_space is None:
            self.context_space = Box(0.0, 1.0, shape=(2,), dtype=TYPE_BOX)

    def _thresholds(self, p_fire, p_tree):
        key = (float(p_fire), float(p_tree))
        if self._thr_cache[0] != key:
            self._thr_cache = (key, np.array([choice_threshold(p_fire), choice_threshold(p_tree)]))
        return self._thr_cache[1]

    def _update_host(self, g, H, W):
        sc = self._scratch
        gin, p_in = sc.get("in", (H, W), np.uint8)
        gout, p_out = sc.get("out", (H, W), np.uint8)
        n, p_n = sc.get("n", (1,), np.int32)
        off, p_off = sc.get("off", (1,), np.int64)
        thr, p_thr = sc.get("thr", (2,), np.float64)
        np.copyto(gin, g, casting="unsafe")
        thr[:] = self._thr
        call_cpu("gca_ds_count_draws", p_in, 1, H, W, self.empty, self.tree, self.fire, p_n, None)
        u = self.np_random.random(max(int(n[0]), 1))
        call_cpu("gca_ds_step", p_in, p_out, 1, H, W, self.empty, self.tree, self.fire, p_thr, u.ctypes.data, p_off,
                 0, None, 0, None, None)
        return gout.astype(g.dtype)

    def update(self, grid, action, context):
        import torch

        p_fire, p_tree = context
        g = np.asarray(grid)
        H, W = g.shape
        self._thr = self._thresholds(p_fire, p_tree)
        if _backend.choose(self.backend, False, H * W) == "cpu":
            if g.size and (g.min() < 0 or g.max() > 255):
                raise ValueError("cell values must fit the u8 layout (0..255)")
            return self._update_host(g, H, W), context
        device = dev.require_device()
        gin = dev.to_device(g.astype(np.uint8).reshape(1, H, W), torch.uint8, device)
        gout = torch.empty_like(gin)
        st = dev.stream_ptr(device)
        n = torch.zeros(1, dtype=torch.int32, device=device)
        call("gca_ds_count_draws", dev.ptr(gin), 1, H, W, self.empty, self.tree, self.fire, dev.ptr(n), st)
        n_draws = int(n.item())
        u = dev.to_device(self.np_random.random(max(n_draws, 1)), torch.float64, device)
        thr = dev.to_device(self._thr, torch.float64, device)
        off = torch.zeros(1, dtype=torch.int64, device=device)
        call("gca_ds_step", dev.ptr(gin), dev.ptr(gout), 1, H, W, self.empty, self.tree, self.fire, dev.ptr(thr),
             dev.ptr(u), dev.ptr(off), 0, None, 0, None, st)
        return gout.cpu().numpy().reshape(H, W).astype(g.dtype), context
