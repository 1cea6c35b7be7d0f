"""Classic pinecone spotting (PartiallyObservableForestFire, ca_alexandridis.py:35-69, 113-133, 184-210):
the C oracle's sequential pass (oracle_alex_pinecones_classic) against the literal per-cell restatement of the
reference loop with its skip list (oracle/alexandridis_classic.update(pine=...)) on the device's decoded draws,
and the host tables against their exact laws. CPU only."""
import math

import numpy as np
import pytest

from oracle import alex_c
from oracle import alexandridis_classic as cl


def _tables(ctx, seed):
    from gymca_amd.forest_fire.operators.pinecones import classic_thrust_tables, make_classic_pine_params

    pp = make_classic_pine_params(seed, 0, 1, 2)
    return pp, classic_thrust_tables(ctx["winds"])


def _dense_context(rng, H, W, fire_frac):
    ctx = cl.random_context(rng, H, W, fire_frac=fire_frac, p_tree=0.2)
    ctx["vegetation"] = rng.integers(1, 6, (H, W))
    ctx["density"] = rng.integers(1, 6, (H, W))
    return ctx


@pytest.mark.parametrize("H,W,seed,fire_frac", [(16, 16, 0, 0.3), (24, 31, 1, 0.5), (40, 40, 2, 0.6),
                                                (9, 57, 3, 0.45)])
def test_c_sequential_pass_matches_literal_skip_list_loop(H, W, seed, fire_frac):
    rng = np.random.default_rng(seed)
    ctx = _dense_context(rng, H, W, fire_frac)
    dr = cl.random_draws(rng, H, W)
    pp, tabs = _tables(ctx, 1000 + seed)
    step = 7
    pine = cl.decode_pinecone_draws(H, W, pp.seed, 0, step, tabs[ctx["wind_index"]], list(pp.n_cdf), pp.age_lo,
                                    pp.age_hi)
    base_g, base_a, _, _ = cl.update(ctx["grid"], ctx, dr, 0, 1, 2)
    want_g, want_a, _, _, want_skipped = cl.update(ctx["grid"], ctx, dr, 0, 1, 2, pine=pine)
    counts = np.stack([np.bincount(base_g.ravel(), minlength=3)]).astype(np.int32)
    g, a, c, skipped = alex_c.pinecones_classic(pp, ctx["grid"][None], base_g[None], base_a.astype(np.int16)[None],
                                                ctx["vegetation"][None], ctx["density"][None],
                                                np.array([ctx["wind_index"]]), tabs, np.array([step]), counts)
    assert np.array_equal(g[0], want_g)
    assert np.array_equal(a[0], want_a.astype(np.int16))
    assert np.array_equal(c[0], np.bincount(want_g.ravel(), minlength=3))
    assert skipped[0] == want_skipped
    assert (want_g != base_g).sum() > 0


def test_skip_list_changes_the_outcome():
    """On dense fires the skip list suppresses sources: the result differs from 'every FIRE cell throws'."""
    rng = np.random.default_rng(11)
    H = W = 32
    ctx = _dense_context(rng, H, W, 0.7)
    dr = cl.random_draws(rng, H, W)
    pp, tabs = _tables(ctx, 5)
    pine = cl.decode_pinecone_draws(H, W, pp.seed, 0, 0, tabs[ctx["wind_index"]], list(pp.n_cdf), pp.age_lo,
                                    pp.age_hi)
    g, a, _, _, skipped = cl.update(ctx["grid"], ctx, dr, 0, 1, 2, pine=pine)
    assert skipped > 0
    # every FIRE cell throwing (no skip list): visit with an empty skip set by throwing from a copy of the grid
    base_g, base_a, _, _ = cl.update(ctx["grid"], ctx, dr, 0, 1, 2)
    g2 = base_g.copy()
    for r in range(H):
        for c in range(W):
            if ctx["grid"][r, c] != 2:
                continue
            for i in range(int(pine["n"][r, c])):
                d = int(pine["dirs"][r, c, i])
                nr, nc = round(r + cl.DX[d] * pine["thrust"][r, c, i]), round(c + cl.DY[d] * pine["thrust"][r, c, i])
                if 0 <= nr < H and 0 <= nc < W and (nr, nc) != (r, c):
                    cl.set_fire_pinecone(nr, nc, g2, ctx["density"], ctx["vegetation"], base_a.copy(),
                                         pine["u"][r, c, i], 5, 2)
    assert not np.array_equal(g, g2)


def test_classic_tables_follow_their_laws():
    from gymca_amd.forest_fire.operators.pinecones import (classic_burn_probability, classic_burn_thresholds,
                                                           poisson_thresholds, thrust_law, thrust_table)

    thr = classic_burn_thresholds()
    for v in range(1, 6):
        for d in range(1, 6):
            p = classic_burn_probability(v, d)
            ks = np.arange(2 ** 24, dtype=np.float64)
            # u = k / 2^24 burns iff p > u (:127)
            want = int(np.sum(p > ks * 2.0 ** -24))
            assert thr[v, d] == want, (v, d)
    n = poisson_thresholds(1.0, 16).astype(np.float64) / 2 ** 32
    cdf = np.cumsum([math.exp(-1) / math.factorial(j) for j in range(16)])
    assert np.all(np.abs(n - np.minimum(cdf, 1.0)) <= 2 ** -32)
    for f in (0.05, 0.8, 1.7, 3.0):
        t = thrust_table(f, 48, 3.0)
        K = int(t[0]) // 2
        ks, law = thrust_law(f, K)
        pk = np.diff(np.concatenate([[0.0], t[1:1 + 2 * K].astype(np.float64) / 2 ** 32, [1.0]]))
        assert np.all(np.abs(pk - law) <= 2 ** -31)


def _classic_fixture_steps(d):
    """(context, grid, draws, pine draws, expected grid / age / wind, pinecone-ignited mask) per captured step."""
    for ci in range(int(d["n"])):
        base = {k: d[f"c{ci}_{k}"] for k in ("winds", "density", "vegetation", "slope")}
        p_tree, p_wc = d[f"c{ci}_p"]
        for t in range(int(d[f"c{ci}_steps"])):
            pre = f"c{ci}_s{t}_"
            ctx = dict(base, wind_index=int(d[pre + "wind"]), fire_age=d[pre + "age"].copy(), p_tree=float(p_tree),
                       p_wind_change=float(p_wc), altitude=np.zeros(d[pre + "grid"].shape))
            draws = {"burn": d[pre + "burn"], "grow": d[pre + "grow"], "age": d[pre + "draw_age"],
                     "wind_u": d[pre + "wind_u"], "wind_k": int(d[pre + "wind_k"])}
            pine = {"n": d[pre + "pine_n"], "dirs": d[pre + "pine_dirs"], "thrust": d[pre + "pine_thrust"],
                    "u": d[pre + "pine_u"], "age": d[pre + "pine_age"]}
            yield (ci, t), ctx, d[pre + "grid"], draws, pine, (d[pre + "out_grid"], d[pre + "out_age"],
                                                               int(d[pre + "out_wind"])), d[pre + "pine_hits"]


def test_classic_oracle_matches_the_reference_run(golden):
    """oracle/alexandridis_classic.update == the reference's own PartiallyObservableForestFire.update loop
    (ca_alexandridis.py:135-221, run with jax.numpy -> numpy by tests/golden/make_golden.py, every draw recorded):
    grid, fire ages and wind index bit for bit over 38 consecutive steps of 4 cases (16x16 .. 32x32), with
    thousands of pinecone ignitions and skip-list events (:151-152, :209-210)."""
    d = golden("alexandridis_classic")
    steps = skips = hits = 0
    for key, ctx, grid, draws, pine, (eg, ea, ew), pine_hits in _classic_fixture_steps(d):
        ng, na, nw, _, sk = cl.update(grid, ctx, draws, 0, 1, 2, pine=pine)
        assert np.array_equal(ng, eg), key
        assert np.array_equal(na, ea), key
        assert nw == ew, key
        steps, skips, hits = steps + 1, skips + sk, hits + int(pine_hits.sum())
    assert steps == 38 and skips > 100 and hits > 1000
