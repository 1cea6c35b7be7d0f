"""Drossel–Schwabl forest fire on the GPU — drop-in for ForestFire (ca_DrosselSchwabl.py:11-66).

Exact-stream semantics: the reference draws one f64 uniform from `self.np_random` per
TREE-without-burning-neighbour and per EMPTY cell, in row-major order
(Generator.choice with p: one random() per call). Here the device counts those cells
(gca_ds_count_draws), the SAME number of uniforms is drawn from `self.np_random`, and
gca_ds_step consumes them in the same order — so a seeded operator reproduces the
reference cell for cell (tests/golden/drossel.npz).
"""
import numpy as np

from ... import _device as dev
from ..._config import TYPE_BOX
from ..._lib import call
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

    def __init__(self, empty, tree, fire, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.empty, self.tree, self.fire = empty, tree, fire
        dev.check_u8_codes((empty, tree, fire))
        if self.context_space is None:
            self.context_space = Box(0.0, 1.0, shape=(2,), dtype=TYPE_BOX)

    def update(self, grid, action, context):
        import torch

        device = dev.require_device()
        p_fire, p_tree = context
        g = np.asarray(grid)
        H, W = g.shape
        gin = dev.to_device(g.astype(np.uint8).reshape(1, H, W), torch.uint8, device)
        gout = torch.empty_like(gin)
        st = dev.stream_ptr(device)
        n = torch.zeros(1, dtype=torch.int32, device=device)
        call("gca_ds_count_draws", dev.ptr(gin), 1, H, W, self.empty, self.tree, self.fire, dev.ptr(n), st)
        n_draws = int(n.item())
        u = dev.to_device(self.np_random.random(max(n_draws, 1)), torch.float64, device)
        thr = dev.to_device(np.array([choice_threshold(p_fire), choice_threshold(p_tree)]), torch.float64, device)
        off = torch.zeros(1, dtype=torch.int64, device=device)
        call("gca_ds_step", dev.ptr(gin), dev.ptr(gout), 1, H, W, self.empty, self.tree, self.fire, dev.ptr(thr),
             dev.ptr(u), dev.ptr(off), 0, None, 0, None, st)
        return gout.cpu().numpy().reshape(H, W).astype(g.dtype), context
