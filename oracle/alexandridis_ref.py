"""Restatement of PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424)
as written — neighbourhood tensors, weighted sums, f32 arithmetic — in numpy, with the
random arrays injected. Test infrastructure only.

Pinned (r06) to the reference EXECUTING: tests/golden/alexandridis_jax.npz holds consecutive `update`
calls of ca_alexandridis_jax.py run as published under a numpy stand-in for jnp / jit / vmap / lax /
random (tests/golden/_jax_standin.py; jax itself is not installed), with every random array the rule
consumed and the burn probabilities it computed; tests/test_alexandridis_jax_golden.py checks this
restatement and the C oracle against it. Also checked against `burn_probability_f64`, an independent
float64 evaluation of the probability formula.
"""
import math

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

VEG = np.array([-999, -0.1, 0.2, 0.5, 0.8, 1.2], dtype=np.float32)
DEN = np.array([-999, -0.2, 0.2, 0.5, 0.8, 1.2], dtype=np.float32)


def constants(grid_size):
    """Reference constructor constants (:54-160), f32 like jnp.array."""
    S = grid_size + grid_size // 2
    age_min, age_max = S * 1.5, S * 1.75
    R = math.ceil(math.log2(grid_size)) - 2
    total, remaining, lw = 0.065, 0.065, []
    for i in range(R):
        cells = (i * 2 + 3) ** 2 - (i * 2 + 1) ** 2 + (1 if i == 0 else 0)
        if i == R - 1:
            lw.append(remaining / cells)
        else:
            lw.append(remaining * 0.60 / cells)
            remaining *= 0.40
    K = np.zeros((2 * R + 1, 2 * R + 1), dtype=np.float32)
    c = R
    K[c, c] = lw[0]
    for i in range(R):
        ring = i + 1
        s, e = c - ring, c + ring + 1
        K[s:e, s] = lw[i]
        K[s:e, e - 1] = lw[i]
        K[s, s:e] = lw[i]
        K[e - 1, s:e] = lw[i]
    bw, iw = 0.0007 * age_max * 0.50, 0.006 * age_max * 0.50
    Wd = np.array([[bw] * 5, [bw, iw, iw, iw, bw], [bw, iw, iw, iw, bw], [bw, iw, iw, iw, bw], [bw] * 5],
                  dtype=np.float32)
    return dict(R=R, K=K, Wd=Wd, age_lo=int(np.int32(age_min)), age_hi=int(np.int32(age_max)), lw=lw,
                age_min=age_min, age_max=age_max)


def _nbhd(a, n):
    return sliding_window_view(np.pad(a, n, mode="constant", constant_values=0), (2 * n + 1, 2 * n + 1))


def burn_probability(grid, veg, den, wind, slope, dousing, C, fire=2):
    """_compute_burn_probability (:164-206) + heat/dousing sums (:345-349), all f32."""
    grid = np.asarray(grid, dtype=np.float32)
    dous = (_nbhd(np.asarray(dousing, dtype=np.float32), 2) * C["Wd"]).sum(axis=(-1, -2), dtype=np.float32)
    heat = ((_nbhd(grid, C["R"]) == fire) * C["K"]).sum(axis=(-1, -2), dtype=np.float32)
    p_veg = VEG[np.clip(veg, 1, 5)]
    p_den = DEN[np.clip(den, 1, 5)]
    p_h = (heat - dous).astype(np.float32)
    p_slope = np.exp(np.float32(0.078) * np.asarray(slope, dtype=np.float32)).astype(np.float32)
    one = np.float32(1)
    return (p_h[..., None, None] * (one + p_veg)[..., None, None] * (one + p_den)[..., None, None]
            * np.asarray(wind, dtype=np.float32) * p_slope).astype(np.float32)


def burn_probability_f64(grid, veg, den, wind, slope, dousing, C, fire=2):
    """Independent float64 evaluation of the same formula (the 1e-6 tolerance yardstick)."""
    grid = np.asarray(grid, dtype=np.float64)
    dous = (_nbhd(np.asarray(dousing, np.float64), 2) * C["Wd"].astype(np.float64)).sum(axis=(-1, -2))
    heat = ((_nbhd(grid, C["R"]) == fire) * C["K"].astype(np.float64)).sum(axis=(-1, -2))
    p_veg = VEG.astype(np.float64)[np.clip(veg, 1, 5)]
    p_den = DEN.astype(np.float64)[np.clip(den, 1, 5)]
    return ((heat - dous)[..., None, None] * (1 + p_veg)[..., None, None] * (1 + p_den)[..., None, None]
            * np.asarray(wind, np.float64) * np.exp(0.078 * np.asarray(slope, np.float32).astype(np.float64)))


def wind_change(wind_index, n_winds, p_wind_change, u, k):
    """update's wind change (:443-451) with the injected uniform u and offset k in [1, 8)."""
    return (int(wind_index) + int(k)) % int(n_winds) if np.float32(u) < np.float32(p_wind_change) else int(wind_index)


def update_grid(grid, fire_age, veg, den, slope, dousing, wind, p_tree, u_burn, u_grow, new_ages, C,
                empty=0, tree=1, fire=2):
    """_update_grid (:321-424) with injected random_values_burn/grow and new_fire_ages."""
    grid = np.asarray(grid, dtype=np.float32)
    fire_age = np.asarray(fire_age, dtype=np.float32)
    tree_mask, fire_mask, empty_mask = grid == tree, grid == fire, grid == empty
    nb = _nbhd(grid, 1)
    probs = burn_probability(grid, veg, den, wind, slope, dousing, C, fire)
    ignite = tree_mask & ((nb == fire) & (np.asarray(u_burn, np.float32) < probs)).any(axis=(-1, -2))
    new_grid = np.where(ignite, fire,
                        np.where(empty_mask & (np.asarray(u_grow, np.float32) < np.float32(p_tree)), tree,
                                 np.where(fire_mask & (fire_age <= 1), empty, grid)))
    new_fire_age = np.where((new_grid == fire) & (grid != fire), np.asarray(new_ages, np.float32), fire_age)
    new_fire_age = np.where(fire_mask, new_fire_age - 1, new_fire_age)
    return new_grid.astype(np.float32), new_fire_age.astype(np.float32), probs
