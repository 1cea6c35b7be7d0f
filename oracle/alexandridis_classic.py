"""Restatement of the classic PartiallyObservableForestFire.update (reference
ca_alexandridis.py:71-111, 135-183, 212-220) as a per-cell Python loop in float64, with the random
draws injected in array form. Test infrastructure only.

The reference module cannot run (it imports `jax.numpy as np` at :1 and calls `np.random` at :189),
so this restatement is pinned by its line-for-line correspondence and by the rule's invariants.
Pinecone spotting (:184-210, sampling :35-69, ignition :113-133) is restated with its skip list when
`pine` draws are given (`decode_pinecone_draws` turns the device's Philox convention into them).

Draw arrays (one env): burn (H, W, 3, 3) uniforms — the `self.np_random.uniform(0, 1, (3, 3))` of
:104 for each cell visited; grow (H, W) — growth iff u < p_tree (`choice([True, False], p=[p_tree,
1 - p_tree])`, :173-175); age (H, W) ints in [4, 11) (:111); wind_u, wind_k — the wind change (:212-219).
Pinecone draws `pine` (one env): n (H, W) — N_p of the cell (:37); dirs (H, W, M) in [0, 8) (:47);
thrust (H, W, M) — pinecone_thrust after :189-190 (3 N(0,1) ft[lookup[d]]); u (H, W, M) — the uniform of
_set_fire_pinecone (:127); age (H, W) — the integers(4, 11) an ignition of that target draws (:131).
"""
import math

import numpy as np

P_VEG = {1: -0.3, 2: 0.0, 3: 0.3, 4: 0.6, 5: 1.0}  # :92
P_DEN = {1: -0.4, 2: 0, 3: 0.3, 4: 0.6, 5: 1.0}  # :93
P_H = 0.58  # :94
A = 0.078  # :95
PINE_VEG = {1: 0.0, 2: 0.8, 3: 1.6, 4: 2.0, 5: 2.5}  # :122
PINE_DEN = {1: 0.0, 2: 0.6, 3: 1.2, 4: 1.5, 5: 2.0}  # :123
DX = [1, 1, 0, -1, -1, -1, 0, 1]  # :63
DY = [0, 1, 1, 1, 0, -1, -1, -1]  # :64


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


def set_fire_pinecone(row, col, new_grid, density, vegetation, fire_age, u, age, fire):
    """_set_fire_pinecone (:113-133) with its uniform and age injected."""
    p_veg = PINE_VEG[int(vegetation[row][col])]
    p_den = PINE_DEN[int(density[row][col])]
    p_burn = P_H * (1 + p_veg) * (1 + p_den)
    if p_burn > u:
        new_grid[row][col] = fire
        fire_age[row][col] = age
        return True
    return False


def update(grid, context, draws, empty, tree, fire, pine=None):
    """One step; returns (new_grid, new_fire_age, new_wind_index, probs (H, W, 3, 3) of tree cells).
    With `pine`, also the number of FIRE cells the skip list kept from throwing (5th value)."""
    grid = np.asarray(grid)
    H, W = grid.shape
    wind_matrix = np.asarray(context["winds"])[int(context["wind_index"])][0]
    new_grid = grid.copy()
    fire_age = np.array(context["fire_age"], dtype=np.int64, copy=True)
    p_tree = float(context["p_tree"])
    probs = np.zeros((H, W, 3, 3))
    skipped_indices = set()  # :147 (a set instead of the list: same membership test)
    skipped_fire = 0
    for r in range(H):
        for c in range(W):
            if (r, c) in skipped_indices:  # :151-152
                skipped_fire += int(grid[r, c] == fire)
                continue
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
                if pine is None:
                    continue
                number_pinecones = int(pine["n"][r, c])  # :184-186
                if number_pinecones == 0:
                    continue
                for i in range(number_pinecones):  # :191-210
                    d = int(pine["dirs"][r, c, i])
                    thrust = float(pine["thrust"][r, c, i])
                    new_row = round(r + DX[d] * thrust)
                    new_col = round(c + DY[d] * thrust)
                    if 0 <= new_row < H and 0 <= new_col < W and (new_row, new_col) != (r, c):
                        did_burn = set_fire_pinecone(new_row, new_col, new_grid, context["density"],
                                                     context["vegetation"], fire_age, float(pine["u"][r, c, i]),
                                                     int(pine["age"][new_row, new_col]), fire)
                        if did_burn:
                            skipped_indices.add((new_row, new_col))
    widx = int(context["wind_index"])
    if "wind_u" in draws and float(draws["wind_u"]) < float(context["p_wind_change"]):
        widx = (widx + int(draws["wind_k"])) % len(context["winds"])
    if pine is not None:
        return new_grid, fire_age, widx, probs, skipped_fire
    return new_grid, fire_age, widx, probs


def decode_pinecone_draws(H, W, seed, env_id, step, s_table, n_cdf, age_lo, age_hi, M=16):
    """The device's classic pinecone draws (gca_pine.hip: Philox (lin, env, step, PCL + 0 / 1 + m), target age
    (lin, env, step, PCLA)) as `pine` arrays; s_table (8, 48) = the env wind's thrust tables. The integer thrust
    s enters as pinecone_thrust = s, so round(r + dx * s) = r + dx * s."""
    from .philox import philox4x32_10, randint_ms, seed_key

    tag, tag_age = 0x50434C00, 0x50434C41
    key = seed_key(seed)
    lin = np.arange(H * W, dtype=np.uint64)
    ctr = lambda t: np.stack([lin, np.full_like(lin, env_id), np.full_like(lin, step), np.full_like(lin, t)], -1)
    b0 = philox4x32_10(ctr(tag), key)
    n = (b0[:, 0:1] >= np.asarray(n_cdf, np.uint32)[None, :]).sum(-1)
    dirs, thrust, u = np.zeros((H * W, M), np.int64), np.zeros((H * W, M)), np.zeros((H * W, M))
    for m in range(M):
        x = philox4x32_10(ctr(tag + 1 + m), key)
        d = (x[:, 2] >> np.uint32(29)).astype(np.int64)
        t = np.asarray(s_table, np.uint32)[d]
        K2 = t[:, 0].astype(np.int64)
        cnt = ((x[:, 0:1] >= t[:, 1:]) & (np.arange(t.shape[1] - 1)[None, :] < K2[:, None])).sum(-1)
        dirs[:, m], thrust[:, m] = d, (cnt - K2 // 2).astype(np.float64)
        u[:, m] = (x[:, 1] >> np.uint32(8)).astype(np.float64) * 2.0 ** -24
    ages = randint_ms(philox4x32_10(ctr(tag_age), key)[:, 0], age_lo, age_hi)
    return {"n": n.reshape(H, W), "dirs": dirs.reshape(H, W, M), "thrust": thrust.reshape(H, W, M),
            "u": u.reshape(H, W, M), "age": ages.reshape(H, W)}


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
