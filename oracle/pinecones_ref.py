"""Literal numpy restatement of the reference's pinecone spotting. TEST INFRASTRUCTURE ONLY.

PartiallyObservableForestFireJax._handle_pinecone_spread (ca_alexandridis_jax.py:229-319) and
_compute_pinecone_burn_probability (:208-227) line by line, with the JAX random arrays injected
(n_pinecones, directions, normal thrusts, uniforms), plus the scatter of _update_grid (:400-420,
commented out in the reference) with the duplicate rule our device kernel defines: a target ignites iff
any pinecone landing on it burns (the reference's .at[].set leaves duplicate order unspecified); its age
comes from `target_ages`. Pinned (r06) to the reference executing: tests/golden/pinecones_jax.npz holds
_handle_pinecone_spread run as published under a numpy stand-in for jax (tests/golden/_jax_standin.py), and
tests/test_pinecones_oracle.py checks the landings and burn mask bit for bit (the scatter :400-420 stays disabled in
the reference, so its duplicate rule is ours).

`decode_draws` turns the device's Philox convention (gca_pine.hip) into these arrays, so the C oracle /
device result can be checked against the literal restatement on identical draws.
"""
import numpy as np

from .philox import philox4x32_10, randint_ms, seed_key, u01_f32

TAG_PINE = 0x50494E45
TAG_PINE_AGE = 0x50494E41
DX = np.array([1, 1, 0, -1, -1, -1, 0, 1])  # :259
DY = np.array([0, 1, 1, 1, 0, -1, -1, -1])  # :260
FT_LOOKUP = np.array([(0, 0), (0, 1), (0, 2), (1, 0), (1, 2), (2, 0), (2, 1), (2, 2)])  # :261-272


def pinecone_burn_probability(vegetation, density):
    """:208-227, f32."""
    veg_probs = np.array([-999, -0.1, 0.2, 0.5, 0.8, 1.2], dtype=np.float32)
    den_probs = np.array([-999, -0.2, 0.2, 0.5, 0.8, 1.2], dtype=np.float32)
    p_veg = veg_probs[np.clip(vegetation, 1, 5)]
    p_den = den_probs[np.clip(density, 1, 5)]
    one = np.float32(1)
    return (np.float32(0.48) * (one + p_veg)) * (one + p_den)


def handle_pinecone_spread(grid, fire_mask, n_pinecones, directions, normal, uniforms, vegetation, density, ft,
                           tree, max_pinecones=5):
    """:229-319 with injected draws: n_pinecones (H, W) Poisson counts, directions (H, W, M) in [0, 8),
    normal (H, W, M) N(0, 1) thrusts, uniforms (H, W, M). grid is the step's new grid. Returns the flat
    (new_rows, new_cols, burn_mask)."""
    H, W = grid.shape
    M = directions.shape[-1]
    n = np.minimum(n_pinecones, max_pinecones)  # :245-247
    row_indices = FT_LOOKUP[directions][..., 0]  # :273
    col_indices = FT_LOOKUP[directions][..., 1]  # :274
    thrust = (np.asarray(normal, np.float32) * np.asarray(ft, np.float32)[row_indices, col_indices]).astype(np.float32)
    rows = np.arange(H, dtype=np.float32)[:, None, None]  # int32 + f32 -> f32 in JAX
    cols = np.arange(W, dtype=np.float32)[None, :, None]
    new_rows = np.clip(np.round(rows + DX.astype(np.float32)[directions] * thrust), 0, H - 1).astype(np.int32)  # :285-287
    new_cols = np.clip(np.round(cols + DY.astype(np.float32)[directions] * thrust), 0, W - 1).astype(np.int32)  # :289-291
    pinecone_mask = fire_mask[:, :, None] & (np.arange(M)[None, None, :] < n[:, :, None])  # :294-296
    probs = pinecone_burn_probability(vegetation, density)  # :299-301
    landing_mask = (grid[new_rows, new_cols] == tree) & pinecone_mask  # :309
    burn_mask = landing_mask & (np.asarray(uniforms, np.float32) < probs[new_rows, new_cols])  # :310-312
    return new_rows.reshape(-1), new_cols.reshape(-1), burn_mask.reshape(-1)


def apply_pinecones(new_grid, new_age, rows, cols, burn, target_ages, fire):
    """The scatter (:413-420) with the any-pinecone rule; returns copies."""
    g, a = new_grid.copy(), new_age.copy()
    hit = np.zeros(g.shape, dtype=bool)
    hit[rows[burn], cols[burn]] = True
    g[hit] = fire
    a[hit] = target_ages[hit]
    return g, a


def decode_draws(H, W, seed, env_id, step, s_table, n_cdf, age_lo, age_hi, M=5):
    """The device's draws as the reference's arrays: n (H, W), directions / s / uniforms (H, W, M) and the
    per-target ages (H, W); s_table (8, 17) = the env wind's thrust tables (t[0] = 2K, thresholds)."""
    key = seed_key(seed)
    lin = np.arange(H * W, dtype=np.uint64)
    ctr = lambda tag: np.stack([lin, np.full_like(lin, env_id), np.full_like(lin, step), np.full_like(lin, tag)], -1)
    b0 = philox4x32_10(ctr(TAG_PINE), key)
    n = (b0[:, 0:1] >= np.asarray(n_cdf, np.uint32)[None, :]).sum(-1)
    dirs, s, u = (np.zeros((H * W, M), np.int64), np.zeros((H * W, M), np.int64), np.zeros((H * W, M), np.float32))
    for m in range(M):
        x = philox4x32_10(ctr(TAG_PINE + 1 + m), key)
        d = (x[:, 2] >> np.uint32(29)).astype(np.int64)
        t = np.asarray(s_table, np.uint32)[d]  # (HW, 17)
        K2 = t[:, 0].astype(np.int64)
        cnt = ((x[:, 0:1] >= t[:, 1:]) & (np.arange(t.shape[1] - 1)[None, :] < K2[:, None])).sum(-1)
        dirs[:, m], s[:, m], u[:, m] = d, cnt - K2 // 2, u01_f32(x[:, 1])
    ages = randint_ms(philox4x32_10(ctr(TAG_PINE_AGE), key)[:, 0], age_lo, age_hi)
    return (n.reshape(H, W), dirs.reshape(H, W, M), s.reshape(H, W, M), u.reshape(H, W, M), ages.reshape(H, W))
