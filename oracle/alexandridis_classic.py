"""Restatement of the classic PartiallyObservableForestFire.update (reference
ca_alexandridis.py:71-111, 135-183, 212-220) as a per-cell Python loop in float64, with the random
draws injected in array form. Test infrastructure only.

The reference module cannot run (it imports `jax.numpy as np` at :1 and calls `np.random` at :189),
so this restatement is pinned by its line-for-line correspondence and by the rule's invariants;
pinecone spotting (:184-210) is left out, like the device operator.

Draw arrays (one env): burn (H, W, 3, 3) uniforms — the `self.np_random.uniform(0, 1, (3, 3))` of
:104 for each cell visited; grow (H, W) — growth iff u < p_tree (`choice([True, False], p=[p_tree,
1 - p_tree])`, :173-175); age (H, W) ints in [4, 11) (:111); wind_u, wind_k — the wind change (:212-219).
"""
import math

import numpy as np

P_VEG = {1: -0.3, 2: 0.0, 3: 0.3, 4: 0.6, 5: 1.0}  # :92
P_DEN = {1: -0.4, 2: 0, 3: 0.3, 4: 0.6, 5: 1.0}  # :93
P_H = 0.58  # :94
A = 0.078  # :95


def neighbours(grid, r, c, invariant):
    """3x3 neighbourhood with constant padding (neighbors.py:6-184, invariant = EMPTY)."""
    H, W = grid.shape
    out = np.full((3, 3), invariant, dtype=grid.dtype)
    for i in range(3):
        for j in range(3):
            rr, cc = r + i - 1, c + j - 1
            if 0 <= rr < H and 0 <= cc < W:
                out[i, j] = grid[rr, cc]
    return out


def burn_probability(r, c, wind_matrix, density, vegetation, slope):
    """p_burn (3, 3) of :92-99 in float64."""
    p_veg = P_VEG[int(vegetation[r][c])]
    p_den = P_DEN[int(density[r][c])]
    p_slope = np.exp(A * np.asarray(slope[r][c], dtype=np.float64))
    return P_H * (1 + p_veg) * (1 + p_den) * np.asarray(wind_matrix, dtype=np.float64) * p_slope


def update(grid, context, draws, empty, tree, fire):
    """One step; returns (new_grid, new_fire_age, new_wind_index, probs (H, W, 3, 3) of tree cells)."""
    grid = np.asarray(grid)
    H, W = grid.shape
    wind_matrix = np.asarray(context["winds"])[int(context["wind_index"])][0]
    new_grid = grid.copy()
    fire_age = np.array(context["fire_age"], dtype=np.int64, copy=True)
    p_tree = float(context["p_tree"])
    probs = np.zeros((H, W, 3, 3))
    for r in range(H):
        for c in range(W):
            cell = grid[r, c]
            nb = neighbours(grid, r, c, empty)
            if cell == tree and (nb == fire).any():
                p_burn = burn_probability(r, c, wind_matrix, context["density"], context["vegetation"],
                                          context["slope"])
                probs[r, c] = p_burn
                burn = p_burn > np.asarray(draws["burn"][r, c], dtype=np.float64)
                if np.any((nb == fire) & burn):
                    new_grid[r, c] = fire
                    fire_age[r, c] = int(draws["age"][r, c])
            elif cell == empty:
                growth = float(draws["grow"][r, c]) < p_tree
                new_grid[r, c] = tree if growth else cell
            elif cell == fire:
                fire_age[r, c] -= 1
                if fire_age[r, c] == 0:
                    new_grid[r, c] = empty
    widx = int(context["wind_index"])
    if "wind_u" in draws and float(draws["wind_u"]) < float(context["p_wind_change"]):
        widx = (widx + int(draws["wind_k"])) % len(context["winds"])
    return new_grid, fire_age, widx, probs


def random_context(rng, H, W, n_winds=8, fire_frac=0.15, p_tree=0.1, p_wind_change=0.3):
    """A random classic context (winds as (n, 2, 3, 3) = (wind_matrix, ft), init_utils.py:225-244)."""
    grid = rng.choice(np.array([0, 1, 2], np.uint8), size=(H, W), p=[0.2, 1 - 0.2 - fire_frac, fire_frac])
    thetas = np.arange(n_winds) * (2 * math.pi / n_winds)
    winds = np.zeros((n_winds, 2, 3, 3))
    for k, th in enumerate(thetas):
        for i in range(3):
            for j in range(3):
                if (i, j) == (1, 1):
                    continue
                ang = math.atan2(1 - i, j - 1)
                ft = math.exp(1.31 * (math.cos(ang - th) - 1))
                winds[k, 0, i, j] = math.exp(0.45) * ft
                winds[k, 1, i, j] = ft
    return {
        "grid": grid,
        "winds": winds.astype(np.float32),
        "wind_index": int(rng.integers(0, n_winds)),
        "density": rng.integers(1, 6, (H, W)),
        "vegetation": rng.integers(1, 6, (H, W)),
        "slope": rng.uniform(-20, 20, (H, W, 3, 3)).astype(np.float32),
        "altitude": np.zeros((H, W)),
        "p_tree": p_tree,
        "p_wind_change": p_wind_change,
        "fire_age": np.where(grid == 2, rng.integers(-1, 6, (H, W)), 0),
    }


def random_draws(rng, H, W):
    return {"burn": rng.random((H, W, 3, 3)).astype(np.float32), "grow": rng.random((H, W)).astype(np.float32),
            "age": rng.integers(4, 11, (H, W)), "wind_u": np.float32(rng.random()), "wind_k": int(rng.integers(1, 8))}
