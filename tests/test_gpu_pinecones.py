"""GPU parity of pinecone spotting (gca_alex_pinecones, ca_alexandridis_jax.py:229-319 + the scatter of
:400-420): bit-exact against the C oracle (itself checked against the literal restatement of
_handle_pinecone_spread in tests/test_pinecones_oracle.py), and the env / operator wiring."""
import numpy as np
import pytest

from alex_cases import make_case, winds
from oracle import alex_c

pytestmark = pytest.mark.gpu


def _t(x, dtype, device):
    import torch

    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


@pytest.mark.parametrize("E,H,W,seed", [(2, 24, 24, 1), (1, 40, 36, 2), (2, 64, 64, 3), (1, 256, 256, 4),
                                        (3, 48, 512, 5)])
def test_pinecones_bit_exact_vs_oracle(device, E, H, W, seed):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params
    from gymca_amd.forest_fire.operators.pinecones import make_pine_params, s_cdf_tables

    case = make_case(E, H, W, seed, fire_p=0.15)
    p, _ = make_alex_params(H, 0, 1, 2, winds(), 0.0, 5 + seed)
    rs = np.full(E, 11, np.uint32)
    g1, a1, c1, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"],
                                     alex_c.prepare_slope(case["slope"]), case["widx"], rng_step=rs)
    pp = make_pine_params(1234 + seed, 0, 1, 2, env_offset=3)
    tabs = s_cdf_tables(winds())
    want_g, want_a, want_c = alex_c.pinecones(pp, case["grid"], g1, a1, case["veg"], case["den"], case["widx"], tabs,
                                              rs, c1)
    gi = _t(case["grid"], torch.uint8, device)
    go, ao = _t(g1, torch.uint8, device), _t(a1, torch.int16, device)
    veg, den = _t(case["veg"], torch.uint8, device), _t(case["den"], torch.uint8, device)
    wi = _t(case["widx"], torch.int32, device)
    tb = _t(tabs.view(np.int32), torch.int32, device)
    rsd = _t(rs.view(np.int32), torch.int32, device)
    counts = _t(c1, torch.int32, device)
    call("gca_alex_pinecones", pp, E, H, W, dev.ptr(gi), dev.ptr(go), dev.ptr(ao), dev.ptr(veg), dev.ptr(den),
         dev.ptr(wi), dev.ptr(tb), dev.ptr(rsd), dev.ptr(counts), None, dev.stream_ptr())
    assert np.array_equal(go.cpu().numpy(), want_g)
    assert np.array_equal(ao.cpu().numpy(), want_a)
    assert np.array_equal(counts.cpu().numpy(), want_c)
    assert (want_g != g1).sum() > 0


def test_env_pinecones_ignite_only_trees(device):
    """pinecones=True: the same step as pinecones=False plus ignitions of TREE cells; fused counts stay the
    grid's counts."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 2, 256
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=9, num_envs=E, use_hidden=False, device=device, pinecones=pc,
                                           observation="grid")
            for pc in (True, False)]
    case = make_case(E, N, N, 41, hidden=False)
    for env in envs:
        env.reset()
        env.set_state(grid=case["grid"], fire_age=case["age"], wind_index=case["widx"])
    act = np.zeros((E, 2), np.int64)
    g = [env.step(act)[0][0].cpu().numpy() for env in envs]
    diff = g[0] != g[1]
    assert diff.sum() > 0 and np.all(g[1][diff] == 1) and np.all(g[0][diff] == 2)
    cnt = torch.zeros((E, 3), dtype=torch.int32, device=device)
    call("gca_count_cells", dev.ptr(envs[0].grid[envs[0].cur]), E, N, N, 0, 1, 2, dev.ptr(cnt), dev.stream_ptr())
    assert torch.equal(cnt, envs[0].counts)


# ------------------------------------------------------------------ classic operator (row a8)
def _classic_case(E, H, W, seed, fire_frac):
    rng = np.random.default_rng(seed)
    from oracle import alexandridis_classic as cl

    ctx = cl.random_context(rng, H, W)
    p3 = [0.3, 1 - 0.3 - fire_frac, fire_frac]
    grid_in = rng.choice(np.array([0, 1, 2], np.uint8), size=(E, H, W), p=p3)
    grid_out = rng.choice(np.array([0, 1, 2], np.uint8), size=(E, H, W), p=p3)
    age_out = rng.integers(-2, 12, (E, H, W)).astype(np.int16)
    veg = rng.integers(1, 6, (E, H, W)).astype(np.uint8)
    den = rng.integers(1, 6, (E, H, W)).astype(np.uint8)
    widx = rng.integers(0, len(ctx["winds"]), E).astype(np.int32)
    return ctx["winds"], grid_in, grid_out, age_out, veg, den, widx


@pytest.mark.parametrize("E,H,W,seed,fire_frac", [(3, 24, 24, 1, 0.4), (2, 37, 45, 2, 0.6), (2, 64, 64, 3, 0.5),
                                                  (1, 256, 256, 4, 0.3), (2, 512, 512, 5, 0.15),
                                                  (1, 600, 580, 6, 0.35), (1, 640, 512, 7, 0.2)])  # 640x512: just above the LDS limit
def test_classic_pinecones_bit_exact_vs_sequential_oracle(device, E, H, W, seed, fire_frac):
    """gca_alex_pinecones_classic (parallel fixed point of the skip list, LDS bitmaps up to 512^2, the scratch
    path at 600 x 580) == the C oracle's literal sequential loop: grid, ages, counts."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import GCA_PINEC_LDS_MAX_HW, call
    from gymca_amd.forest_fire.operators.pinecones import classic_thrust_tables, make_classic_pine_params

    winds, gi, go, ao, veg, den, widx = _classic_case(E, H, W, seed, fire_frac)
    pp = make_classic_pine_params(4321 + seed, 0, 1, 2, env_offset=2)
    tabs = classic_thrust_tables(winds)
    rs = np.full(E, 3 + seed, np.uint32)
    counts = np.stack([np.bincount(go[e].ravel(), minlength=3) for e in range(E)]).astype(np.int32)
    want_g, want_a, want_c, skipped = alex_c.pinecones_classic(pp, gi, go, ao, veg, den, widx, tabs, rs, counts)
    g_d, a_d, c_d = _t(go, torch.uint8, device), _t(ao, torch.int16, device), _t(counts, torch.int32, device)
    scratch = None if H * W <= GCA_PINEC_LDS_MAX_HW else torch.empty(E * 4 * ((H * W + 31) // 32), dtype=torch.int32,
                                                                     device=device)
    # every operand stays referenced until the kernel has run (a temporary's memory may be reused at once)
    gi_d, v_d, d_d = _t(gi, torch.uint8, device), _t(veg, torch.uint8, device), _t(den, torch.uint8, device)
    w_d, t_d = _t(widx, torch.int32, device), _t(tabs.view(np.int32), torch.int32, device)
    r_d = _t(rs.view(np.int32), torch.int32, device)
    call("gca_alex_pinecones_classic", pp, E, H, W, dev.ptr(gi_d), dev.ptr(g_d), dev.ptr(a_d), dev.ptr(v_d),
         dev.ptr(d_d), dev.ptr(w_d), dev.ptr(t_d), dev.ptr(r_d), dev.ptr(c_d), dev.ptr(scratch), dev.stream_ptr())
    torch.cuda.synchronize(device)
    assert np.array_equal(g_d.cpu().numpy(), want_g)
    assert np.array_equal(a_d.cpu().numpy(), want_a)
    assert np.array_equal(c_d.cpu().numpy(), want_c)
    assert (want_g != go).sum() > 0 and skipped.sum() > 0  # ignitions and skip-list suppressions exercised


@pytest.mark.parametrize("H,W,seed", [(24, 24, 0), (31, 40, 1)])
def test_classic_dropin_with_pinecones_matches_literal_loop(device, H, W, seed):
    """PartiallyObservableForestFire (pinecones on, the default) with the step's draws injected == the literal
    restatement of update (:135-221, skip list included) on the device's decoded pinecone draws, 2 calls."""
    from gymca_amd.forest_fire.operators import PartiallyObservableForestFire
    from gymca_amd.forest_fire.operators.pinecones import classic_thrust_tables, make_classic_pine_params
    from oracle import alexandridis_classic as cl

    rng = np.random.default_rng(700 + seed)
    ctx = cl.random_context(rng, H, W, fire_frac=0.45)
    op = PartiallyObservableForestFire(0, 1, 2)
    pp = make_classic_pine_params(op.philox_seed, 0, 1, 2)
    tabs = classic_thrust_tables(ctx["winds"])
    grid, total_skipped = ctx["grid"], 0
    for step in range(2):
        dr = cl.random_draws(rng, H, W)
        pine = cl.decode_pinecone_draws(H, W, pp.seed, 0, step, tabs[int(ctx["wind_index"])], list(pp.n_cdf),
                                        pp.age_lo, pp.age_hi)
        want_g, want_a, want_w, _, skipped = cl.update(grid, ctx, dr, 0, 1, 2, pine=pine)
        total_skipped += skipped
        new_grid, ctx = op(grid, None, ctx, draws=dr)
        assert np.array_equal(new_grid, want_g), f"step {step}"
        assert np.array_equal(ctx["fire_age"], want_a), f"step {step}"
        assert int(ctx["wind_index"]) == want_w
        grid = new_grid
    assert total_skipped > 0
