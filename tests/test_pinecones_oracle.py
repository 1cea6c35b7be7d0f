"""Pinecone spotting (ca_alexandridis_jax.py:229-319, disabled in the reference): the host thrust / count
tables against their exact laws, and the C oracle's pass (oracle_alex_pinecones, the device's draw
convention) against the literal numpy restatement of _handle_pinecone_spread on the same decoded draws.
Parity unpinned at the reference level (jax absent, the code commented out there)."""
import math

import numpy as np
import pytest

from alex_cases import make_case, winds
from oracle import alex_c
from oracle import pinecones_ref as ref


def _tables():
    from gymca_amd.forest_fire.operators import pinecones

    return pinecones


@pytest.mark.parametrize("f", [0.0728, 0.2, 0.5, 0.8312, 1.0])
def test_thrust_table_matches_exact_law(f):
    pc = _tables()
    t = pc.thrust_table(f)
    K2 = int(t[0])
    thr = t[1:1 + K2].astype(np.float64)
    assert np.all(np.diff(thr) >= 0)
    probs = np.diff(np.concatenate([[0.0], thr, [2.0 ** 32]])) / 2.0 ** 32  # P(s = -K .. K) from the thresholds
    ks, law = pc.thrust_law(f, K2 // 2)
    assert np.allclose(probs, law, atol=2 * 2.0 ** -32, rtol=0)
    assert abs(law.sum() - 1) < 1e-12
    # tails beyond K fold in with < 2^-32 mass: P(|Z| > (K + 1/2) / f) tiny
    assert math.erfc((K2 // 2 + 0.5) / f / math.sqrt(2)) < 2.0 ** -31


def test_poisson_thresholds():
    pc = _tables()
    t = pc.poisson_thresholds().astype(np.float64) / 2.0 ** 32
    pmf = np.array([math.exp(-1) / math.factorial(j) for j in range(len(t))])
    assert np.allclose(t, np.cumsum(pmf), atol=2.0 ** -32)


def test_s_tables_follow_ft_lookup():
    pc = _tables()
    w = winds()
    tab = pc.s_cdf_tables(w)
    assert tab.shape == (8, 8, 17) and tab.dtype == np.uint32
    for i in (0, 5):
        for d, (a, b) in enumerate(pc.FT_LOOKUP):
            assert np.array_equal(tab[i, d], pc.thrust_table(w[i, 1][a, b]))


@pytest.mark.parametrize("E,H,W,seed", [(2, 24, 24, 1), (1, 40, 33, 2), (2, 64, 64, 3)])
def test_oracle_pass_matches_literal_restatement(E, H, W, seed):
    """C oracle (device convention) == _handle_pinecone_spread + scatter on the decoded draws."""
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params

    pc = _tables()
    case = make_case(E, H, W, seed, fire_p=0.12)
    p, _ = make_alex_params(H, 0, 1, 2, winds(), 0.0, 77 + seed)
    ps = alex_c.prepare_slope(case["slope"])
    rs = np.full(E, 3, np.uint32)
    g1, a1, c1, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                     case["widx"], rng_step=rs)
    pp = pc.make_pine_params(99 + seed, 0, 1, 2)
    tabs = pc.s_cdf_tables(winds())
    go, ao, co = alex_c.pinecones(pp, case["grid"], g1, a1, case["veg"], case["den"], case["widx"], tabs, rs, c1)
    ignited = 0
    for e in range(E):
        n, dirs, s, u, ages = ref.decode_draws(H, W, 99 + seed, e, 3, tabs[case["widx"][e]], pc.poisson_thresholds(),
                                               *pc.PINE_AGE)
        ft = winds()[case["widx"][e], 1]
        f = ft[ref.FT_LOOKUP[dirs][..., 0], ref.FT_LOOKUP[dirs][..., 1]]
        normal = (s / f.astype(np.float64)).astype(np.float32)  # thrust = normal * ft rounds back to s
        rows, cols, burn = ref.handle_pinecone_spread(g1[e], case["grid"][e] == 2, n, dirs, normal, u, case["veg"][e],
                                                      case["den"][e], ft, 1)
        want_g, want_a = ref.apply_pinecones(g1[e], a1[e], rows, cols, burn, ages, 2)
        assert np.array_equal(go[e], want_g)
        assert np.array_equal(ao[e], want_a)
        ignited += int((want_g != g1[e]).sum())
        assert co[e, 2] - c1[e, 2] == int((want_g != g1[e]).sum()) == c1[e, 1] - co[e, 1]
    assert ignited > 0


def test_restatement_reproduces_reference_run(golden):
    """oracle.pinecones_ref.handle_pinecone_spread against the reference's own _handle_pinecone_spread executed under
    the jax stand-in (tests/golden/pinecones_jax.npz, make_golden.py::gen_pinecones_jax): the same landings (rows,
    columns) and burn mask, bit for bit, from the draws the reference consumed."""
    d = golden("pinecones_jax")
    landed = burned = 0
    for ci in range(int(d["n"])):
        p = f"c{ci}_"
        rows, cols, burn = ref.handle_pinecone_spread(
            d[p + "new"].astype(np.int64), d[p + "old"] == 2, d[p + "n"], d[p + "dirs"].astype(np.int64), d[p + "normal"],
            d[p + "u"], d[p + "veg"].astype(np.int64), d[p + "den"].astype(np.int64), d[p + "ft"], tree=1)
        assert np.array_equal(rows, d[p + "rows"]) and np.array_equal(cols, d[p + "cols"]), ci
        assert np.array_equal(burn.astype(np.uint8), d[p + "burn"]), ci
        landed += int((d[p + "old"] == 2).sum())
        burned += int(d[p + "burn"].sum())
    assert landed > 50 and burned > 5
