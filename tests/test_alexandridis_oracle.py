"""CPU: the C restatement (kernel evaluation order) against the numpy restatement of the
reference as written, the f64 probability formula, constants and the reference's invariants."""
import numpy as np
import pytest

from alex_cases import make_case, winds
from oracle import alex_c
from oracle import alexandridis_ref as ref


def params(H, p_tree, seed=7):
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params

    p, _ = make_alex_params(H, 0, 1, 2, winds(), p_tree, seed)
    return p


@pytest.mark.parametrize("H", [5, 8, 16, 33, 64, 256, 512, 1024])
def test_constants_match_reference_constructor(H):
    from gymca_amd.forest_fire.operators.ca_alexandridis import alex_constants

    c, r = alex_constants(H), ref.constants(H)
    assert c["R"] == r["R"]
    assert np.array_equal(c["burn_kernel"], r["K"])
    assert np.array_equal(c["dousing_weights"], r["Wd"])
    assert (c["age_lo"], c["age_hi"]) == (r["age_lo"], r["age_hi"])
    # heat_dw telescopes back to the ring weights
    assert np.allclose(np.cumsum(c["heat_dw"][::-1])[::-1][1:], [r["K"][r["R"], r["R"] + k] for k in range(1, r["R"] + 1)],
                       rtol=1e-6, atol=0)


@pytest.mark.parametrize("E,H,W,seed", [(2, 16, 16, 1), (1, 37, 45, 2), (2, 64, 64, 3), (1, 8, 8, 4),
                                        (2, 256, 256, 5), (2, 512, 512, 6)])  # BASELINE sizes: R = 6 and 7
def test_c_oracle_injected_matches_reference_restatement(E, H, W, seed):
    case = make_case(E, H, W, seed, p_tree=0.3)
    p = params(H, case["p_tree"])
    ps = alex_c.prepare_slope(case["slope"])
    ub, ug, ua = case["draws"]
    go, ao, counts, probs = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                             case["widx"], inj=(ub.reshape(E, H, W, 9), ug, ua), want_probs=True)
    W8 = winds()[:, 0]
    for e in range(E):
        ng, na, rp = ref.update_grid(case["grid"][e], case["age"][e], case["veg"][e].astype(np.int64),
                                     case["den"][e].astype(np.int64), case["slope"][e], case["dous"][e],
                                     W8[case["widx"][e]], case["p_tree"], ub[e], ug[e], ua[e], case["C"])
        rp8 = rp.reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
        # probabilities: the two f32 evaluations agree within 1e-6 (absolute for p <= 1, relative
        # above: p is a probability, values > 1 only saturate); they differ in summation order only
        assert np.max(np.abs(probs[e] - rp8) / np.maximum(np.abs(rp8), 1.0)) < 1e-6
        # integer states agree everywhere except where a uniform lies within rounding of p
        diff = go[e] != ng
        if diff.any():
            close = np.abs(ub[e].reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]] - rp8).min(axis=-1) < 1e-6
            assert np.all(close[diff])
        assert np.array_equal(ao[e][~diff], na.astype(np.int16)[~diff])
        assert tuple(counts[e]) == tuple(int(np.sum(go[e] == v)) for v in (0, 1, 2))


@pytest.mark.parametrize("H", [64, 256, 512])  # 256 / 512: BASELINE sizes (R = 6 / 7)
def test_probabilities_within_1e6_of_float64(H):
    E, W = 2, H
    case = make_case(E, H, W, 11)
    p = params(H, 0.0)
    ps = alex_c.prepare_slope(case["slope"])
    _, _, _, probs = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                      case["widx"], want_probs=True)
    W8 = winds()[:, 0]
    for e in range(E):
        p64 = ref.burn_probability_f64(case["grid"][e], case["veg"][e].astype(np.int64),
                                       case["den"][e].astype(np.int64), W8[case["widx"][e]], case["slope"][e],
                                       case["dous"][e], case["C"]).reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
        assert np.max(np.abs(probs[e] - p64) / np.maximum(np.abs(p64), 1.0)) < 1e-6  # TOL = 1e-6


def test_reference_invariants_philox_mode():
    """Reference rule invariants (:379-423): EMPTY stays EMPTY at p_tree = 0, TREE without a FIRE
    neighbour stays TREE, FIRE with age <= 1 burns out, old fires age by one."""
    E, H, W = 3, 48, 40
    case = make_case(E, H, W, 5)
    p = params(H, 0.0)
    ps = alex_c.prepare_slope(case["slope"])
    go, ao, _, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                    case["widx"], rng_step=np.full(E, 3, np.uint32))
    g, a = case["grid"], case["age"].astype(np.int32)
    pad = np.pad(g, ((0, 0), (1, 1), (1, 1)))
    nbfire = np.zeros_like(g, dtype=bool)
    for dr in (-1, 0, 1):
        for dc in (-1, 0, 1):
            if (dr, dc) != (0, 0):
                nbfire |= pad[:, 1 + dr:1 + dr + H, 1 + dc:1 + dc + W] == 2
    assert np.all(go[g == 0] == 0)
    assert np.all(go[(g == 1) & ~nbfire] == 1)
    assert np.all(go[(g == 2) & (a <= 1)] == 0) and np.all(go[(g == 2) & (a > 1)] == 2)
    assert np.array_equal(ao[g == 2], a[g == 2] - 1)
    new = (g == 1) & (go == 2)
    assert new.any() and np.all((ao[new] >= case["C"]["age_lo"]) & (ao[new] < case["C"]["age_hi"]))


def test_burn_law_matches_independent_directions():
    """Philox mode draws one uniform per cell against 1 - prod(1 - p_d); that is the law of the
    reference's independent per-direction draws. Monte-Carlo check of the burn frequency."""
    E, H, W = 64, 16, 16
    rng = np.random.default_rng(9)
    grid = np.ones((E, H, W), np.uint8)
    grid[:, 7, 7] = 2
    grid[:, 9, 8] = 2
    case = make_case(E, H, W, 9)
    p = params(H, 0.0)
    ps = alex_c.prepare_slope(np.zeros((E, H, W, 3, 3), np.float32))
    veg = np.full((E, H, W), 3, np.uint8)
    burned = np.zeros((H, W))
    steps = 40
    for s in range(steps):
        go, _, _, probs = alex_c.alex_step(p, grid, np.full((E, H, W), 600, np.int16), veg, veg,
                                           np.zeros((E, H, W), np.uint8), ps, np.zeros(E, np.int32),
                                           rng_step=np.full(E, s, np.uint32), want_probs=True)
        burned += (go == 2).sum(axis=0)
    # cell (8, 8) has fire neighbours at (7,7) [d=0] and (9,8) [d=6]
    pd = probs[0, 8, 8]
    law = 1 - (1 - np.clip(pd[0], 0, 1)) * (1 - np.clip(pd[6], 0, 1))
    freq = burned[8, 8] / (E * steps)
    assert abs(freq - law) < 4 * np.sqrt(law * (1 - law) / (E * steps)) + 1e-3


# ------------------------------------------------------------------ classic variant (row a8)
def _classic_inputs(ctx):
    H, W = ctx["grid"].shape
    age = ctx["fire_age"].astype(np.int16)[None]
    slope = np.asarray(ctx["slope"], np.float32).reshape(1, H, W, 9)
    return (ctx["grid"][None], age, ctx["vegetation"].astype(np.uint8)[None], ctx["density"].astype(np.uint8)[None],
            np.zeros((1, H, W), np.uint8), alex_c.prepare_slope(slope), np.array([ctx["wind_index"]], np.int32))


@pytest.mark.parametrize("H,W,seed", [(12, 12, 0), (17, 23, 1), (32, 32, 2)])
def test_c_oracle_classic_matches_classic_restatement(H, W, seed):
    """The kernel's evaluation order with the classic parameters (heat0 = p_h, classic tables,
    ages [4, 11), burn-out at age 0) against the per-cell float64 restatement of
    ca_alexandridis.py:71-183 with the same injected draws."""
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_classic_params
    from oracle import alexandridis_classic as cl

    rng = np.random.default_rng(seed)
    ctx = cl.random_context(rng, H, W)
    dr = cl.random_draws(rng, H, W)
    ng, na, _, rp = cl.update(ctx["grid"], ctx, dr, 0, 1, 2)
    p = make_classic_params(0, 1, 2, ctx["winds"], ctx["p_tree"], 5)
    grid, age, veg, den, dous, ps, widx = _classic_inputs(ctx)
    go, ao, counts, probs = alex_c.alex_step(p, grid, age, veg, den, dous, ps, widx,
                                             inj=(dr["burn"].reshape(1, H, W, 9), dr["grow"][None], dr["age"][None]),
                                             want_probs=True)
    rp8 = rp.reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
    burning_nb = np.any(rp8 != 0, axis=-1)  # where the restatement evaluated p_burn
    rel = np.abs(probs[0] - rp8) / np.maximum(np.abs(rp8), 1.0)
    assert np.max(rel[burning_nb]) < 1e-6  # f32 kernel vs f64 reference arithmetic
    diff = go[0] != ng
    if diff.any():  # only where a uniform lies within rounding of p
        close = np.abs(dr["burn"].reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]] - rp8).min(axis=-1) < 1e-6
        assert np.all(close[diff])
    assert np.array_equal(ao[0][~diff], na.astype(np.int16)[~diff])
    # classic burn-out: a FIRE with age 0 or -1 keeps burning (age -> -1 / -2), age 1 burns out
    fire = ctx["grid"] == 2
    assert np.all(go[0][fire & (ctx["fire_age"] <= 0)] == 2)
    assert np.all(go[0][fire & (ctx["fire_age"] == 1)] == 0)


def test_group_draw_convention_restated_in_numpy():
    """The C oracle's Philox-mode draws (r05, include/gca.h GCA_TAG_ALEX_CELL / _AGE) restated in numpy from the
    spec: group (r, c // 4) -> block X = Philox(r * ceil(W/4) + c // 4, env, step, ALXC); cell c tests word c % 4
    (EMPTY -> TREE iff (word >> 8) < p_tree * 2^24 exactly; TREE -> FIRE iff (word >> 8) < (1 - q) * 2^24, checked
    away from the threshold against the float64 law of the oracle's own p_d); the group's new fires in column order take
    randint of the spare word (the four low bytes) and then of words 0, 1, 2 of Philox(same counter, ALXA). A hot state
    at an odd width (partial last groups) so every rank occurs."""
    from oracle.philox import philox4x32_10, randint_ms, seed_key

    E, H, W, step = 2, 23, 45, 17
    case = make_case(E, H, W, 31, fire_p=0.45, dousing_p=0.0, p_tree=0.2)
    case["veg"][:] = 5
    case["den"][:] = 5
    p = params(H, 0.2)
    ps = alex_c.prepare_slope(case["slope"])
    go, ao, _, probs = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                        case["widx"], rng_step=np.full(E, step, np.uint32), want_probs=True)
    key = seed_key(p.seed)
    GW4 = (W + 3) // 4
    g = case["grid"]
    pad = np.pad(g, ((0, 0), (1, 1), (1, 1)))
    checked_burn = ranks_seen = 0
    seen = set()
    for e in range(E):
        env_id = int(p.env_offset) + e
        for r in range(H):
            grp = r * GW4 + np.arange(GW4)
            ctr = lambda tag: np.stack([grp, np.full(GW4, env_id), np.full(GW4, step), np.full(GW4, tag)], -1)
            X = philox4x32_10(ctr(0x414C5843), key)
            Y = philox4x32_10(ctr(0x414C5841), key)
            spare = ((X[:, 0] & 0xFF) | ((X[:, 1] & 0xFF) << 8) | ((X[:, 2] & 0xFF) << 16) |
                     ((X[:, 3] & 0xFF) << 24)).astype(np.uint32)
            for c in range(W):
                u24 = int(X[c // 4, c % 4]) >> 8
                x = int(g[e, r, c])
                if x == 0:
                    assert (go[e, r, c] == 1) == (np.float32(u24) < np.float32(p.p_tree) * np.float32(2 ** 24))
                elif x == 1:
                    nb = pad[e, r:r + 3, c:c + 3].reshape(9)[[0, 1, 2, 3, 5, 6, 7, 8]] == 2
                    law = 1.0 - np.prod(np.where(nb, 1.0 - np.clip(probs[e, r, c].astype(np.float64), 0, 1), 1.0))
                    if abs(u24 - law * 2 ** 24) > 4:
                        assert (go[e, r, c] == 2) == (u24 < law * 2 ** 24), (e, r, c)
                        checked_burn += 1
            for gi in range(GW4):
                cols = [c for c in range(4 * gi, min(4 * gi + 4, W)) if g[e, r, c] == 1 and go[e, r, c] == 2]
                for k, c in enumerate(cols):
                    word = spare[gi] if k == 0 else Y[gi, k - 1]
                    assert int(ao[e, r, c]) == int(randint_ms(np.uint32(word), p.age_lo, p.age_hi)), (e, r, c, k)
                    seen.add(k)
    assert checked_burn > 500 and seen == {0, 1, 2, 3}, (checked_burn, seen)
