"""GPU parity of the edge-slope step (gca_alex_step_es, 16 B of slope per cell) and of the fire-sparsity
skip: bit-identical to gca_alex_step on the 8-plane p_slope built from the same altitude, and to the
C oracle; sparse-fire states (a few burning cells) through both layouts."""
import numpy as np
import pytest

from alex_cases import make_case, winds
from oracle import alex_c
from oracle import edge_slope

pytestmark = pytest.mark.gpu


def _t(x, dtype, device):
    import torch

    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


def altitude(E, H, W, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(0, 5, (E, H, W)) + rng.normal(0, 20, (E, H, W)) * (rng.random((E, H, W)) < 0.3)


def slopes(device, alt):
    """(edge (E,4,H,W), planes (E,8,H,W)) built on the device from the same altitude."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = alt.shape
    a = _t(alt, torch.float64, device)
    es = torch.empty((E, 4, H, W), dtype=torch.float32, device=device)
    ps = torch.empty((E, 8, H, W), dtype=torch.float32, device=device)
    call("gca_alex_edge_slope_from_altitude", dev.ptr(a), dev.ptr(es), E, H, W, dev.stream_ptr())
    call("gca_alex_slope_from_altitude", dev.ptr(a), dev.ptr(ps), None, E, H, W, dev.stream_ptr())
    return es, ps


def step(device, fn, p, case, slope, rng_step=None, inj=None, probs=False):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = case["grid"].shape
    g, a = _t(case["grid"], torch.uint8, device), _t(case["age"], torch.int16, device)
    veg, den, dous = (_t(case[k], torch.uint8, device) for k in ("veg", "den", "dous"))
    wi = _t(case["widx"], torch.int32, device)
    rs = None if rng_step is None else _t(np.asarray(rng_step, np.uint32).view(np.int32), torch.int32, device)
    go, ao = torch.empty_like(g), torch.empty_like(a)
    counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
    ij = [None] * 3
    if inj is not None:
        ij = [_t(inj[0].reshape(E, H, W, 9), torch.float32, device), _t(inj[1], torch.float32, device),
              _t(inj[2], torch.int32, device)]
    po = torch.empty((E, H, W, 8), dtype=torch.float32, device=device) if probs else None
    call(fn, p, E, H, W, dev.ptr(g), dev.ptr(go), dev.ptr(a), dev.ptr(ao), dev.ptr(veg), dev.ptr(den),
         dev.ptr(dous), dev.ptr(slope), dev.ptr(wi), dev.ptr(rs), dev.ptr(ij[0]), dev.ptr(ij[1]), dev.ptr(ij[2]),
         dev.ptr(po), dev.ptr(counts), dev.stream_ptr())
    return go.cpu().numpy(), ao.cpu().numpy(), counts.cpu().numpy(), None if po is None else po.cpu().numpy()


def params(H, p_tree=0.0, seed=1234):
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params

    p, _ = make_alex_params(H, 0, 1, 2, winds(), p_tree, seed)
    return p


# W = 512 / 300 / 1024: several tiles per row (the lane-15 / lane-0 edge loads cross tiles);
# H % 16 != 0 and odd W: the bounds-checked variant
SIZES = [(2, 5, 7, 1), (2, 16, 16, 2), (3, 37, 45, 3), (2, 64, 64, 4), (1, 100, 300, 5), (2, 256, 256, 6),
         (1, 48, 512, 7), (1, 512, 512, 8), (1, 130, 33, 9), (1, 32, 1024, 10)]


@pytest.mark.parametrize("E,H,W,seed", SIZES)
def test_edge_device_layout_matches_restatement(device, E, H, W, seed):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    alt = altitude(E, H, W, seed)
    es, ps = slopes(device, alt)
    es = es.cpu().numpy()
    # the device's own f32 slopes (get_slope with its border zeroing) -> the oracle's edge values: equal
    # bit for bit on interior cells (the same f32 slope, exp_f32 and sign rule)
    a = _t(alt, torch.float64, device)
    s9 = torch.empty((E, H, W, 3, 3), dtype=torch.float32, device=device)
    tmp = torch.empty((E, 8, H, W), dtype=torch.float32, device=device)
    call("gca_alex_slope_from_altitude", dev.ptr(a), dev.ptr(tmp), dev.ptr(s9), E, H, W, dev.stream_ptr())
    s9 = s9.cpu().numpy()
    own = np.stack([s9[:, :, :, 0, 0], s9[:, :, :, 0, 1], s9[:, :, :, 0, 2], s9[:, :, :, 1, 0]], axis=1)
    if H > 2 and W > 2:
        want = edge_slope.edge_values(own)
        assert np.array_equal(es[:, :, 1:-1, 1:-1], want[:, :, 1:-1, 1:-1])
    # all cells (borders too) against the host restatement, to the ulp of numpy's vs the device's atan
    host = edge_slope.edge_values(edge_slope.edge_from_altitude(alt))
    assert np.allclose(es, host, rtol=3e-6, atol=0)


def test_edge_factor_reciprocal_exhaustive(device):
    """The kernel's v_rcp_f32 + Newton reciprocal equals IEEE division for EVERY f32 in [1, 1121] (the range of
    exp_f32(|0.078 slope|), |slope| < 90), both signs, own and neighbour directions."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    lo = np.float32(1.0).view(np.uint32)
    hi = np.float32(1121.0).view(np.uint32)
    chunk = 1 << 24
    for start in range(int(lo), int(hi) + 1, chunk):
        bits = np.arange(start, min(start + chunk, int(hi) + 1), dtype=np.uint32)
        x = bits.view(np.float32)
        for v in (x, -x):
            vd = torch.as_tensor(v, device=device)
            own, nbr = torch.empty_like(vd), torch.empty_like(vd)
            call("gca_alex_edge_factors", dev.ptr(vd), dev.ptr(own), dev.ptr(nbr), v.size, dev.stream_ptr())
            inv = (np.float32(1) / x).astype(np.float32)
            want_own, want_nbr = (x, inv) if v[0] > 0 else (inv, x)
            assert np.array_equal(own.cpu().numpy(), want_own)
            assert np.array_equal(nbr.cpu().numpy(), want_nbr)


@pytest.mark.parametrize("E,H,W,seed", SIZES)
def test_edge_step_bit_exact_vs_planes_and_oracle(device, E, H, W, seed):
    case = make_case(E, H, W, seed, p_tree=0.01)
    p = params(H, 0.01, seed=seed * 31)
    es, ps = slopes(device, altitude(E, H, W, seed))
    ps_np = ps.cpu().numpy()
    for s in range(3):
        rs = np.full(E, 7 * s + 2, np.uint32)
        g1, a1, c1, _ = step(device, "gca_alex_step_es", p, case, es, rng_step=rs)
        g0, a0, c0, _ = step(device, "gca_alex_step", p, case, ps, rng_step=rs)
        assert np.array_equal(g1, g0), f"step {s}: {np.argwhere(g1 != g0)[:5]}"
        assert np.array_equal(a1, a0) and np.array_equal(c1, c0)
        if s == 0:
            eg, ea, ec, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"],
                                             ps_np, case["widx"], rng_step=rs)
            assert np.array_equal(g1, eg) and np.array_equal(a1, ea) and np.array_equal(c1, ec)
        case["grid"], case["age"] = g1, a1


@pytest.mark.parametrize("E,H,W,seed", [(2, 37, 45, 11), (1, 64, 512, 12), (2, 256, 256, 13)])
def test_edge_probabilities_and_injected_mode(device, E, H, W, seed):
    case = make_case(E, H, W, seed, p_tree=0.2)
    p = params(H, 0.2)
    es, ps = slopes(device, altitude(E, H, W, seed))
    _, _, _, po1 = step(device, "gca_alex_step_es", p, case, es, rng_step=np.zeros(E, np.uint32), probs=True)
    _, _, _, po0 = step(device, "gca_alex_step", p, case, ps, rng_step=np.zeros(E, np.uint32), probs=True)
    assert np.array_equal(po1.view(np.uint32), po0.view(np.uint32))
    inj = case["draws"]
    r1 = step(device, "gca_alex_step_es", p, case, es, inj=inj, probs=True)
    r0 = step(device, "gca_alex_step", p, case, ps, inj=inj, probs=True)
    for x, y in zip(r1, r0):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


@pytest.mark.parametrize("layout", ["es", "planes"])
@pytest.mark.parametrize("E,H,W,seed", [(3, 256, 256, 21), (2, 64, 512, 22), (2, 45, 37, 23)])
def test_sparse_fire_skip_bit_exact(device, layout, E, H, W, seed):
    """A few burning cells (a real episode's fire front): most waves / workgroups skip the heat and
    direction phases; the grid, ages and counts still equal the C oracle's over several steps."""
    case = make_case(E, H, W, seed, p_tree=0.0)
    rng = np.random.default_rng(seed)
    g = np.where(rng.random((E, H, W)) < 0.15, 0, 1).astype(np.uint8)
    for e in range(E):  # a small fire cluster and one isolated fire per env, one on the border
        r, c = rng.integers(1, H - 3), rng.integers(1, W - 3)
        g[e, r:r + 2, c:c + 2] = 2
        g[e, 0, rng.integers(0, W)] = 2
    case["grid"] = g
    case["age"] = np.where(g == 2, rng.integers(2, 50, (E, H, W)), 0).astype(np.int16)
    p = params(H, 0.0, seed=seed)
    es, ps = slopes(device, altitude(E, H, W, seed))
    ps_np = ps.cpu().numpy()
    for s in range(6):
        rs = np.full(E, s, np.uint32)
        got = step(device, "gca_alex_step_es" if layout == "es" else "gca_alex_step", p, case,
                   es if layout == "es" else ps, rng_step=rs)
        eg, ea, ec, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps_np,
                                         case["widx"], rng_step=rs)
        assert np.array_equal(got[0], eg), f"step {s}"
        assert np.array_equal(got[1], ea) and np.array_equal(got[2], ec)
        case["grid"], case["age"] = got[0], got[1]
    assert (case["grid"] == 2).any()


def test_env_edge_and_planes_layouts_agree(device):
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 3, 64
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=5, num_envs=E, use_hidden=True, device=device,
                                           hidden_rng=np.random.RandomState(3), slope_layout=lay)
            for lay in ("edge", "planes")]
    case = make_case(E, N, N, 9)
    for env in envs:
        env.reset()
        env.set_state(grid=case["grid"], fire_age=case["age"], wind_index=case["widx"])
    assert np.array_equal(envs[0].p_slope_planes().cpu().numpy(), envs[1].p_slope_planes().cpu().numpy())
    rng = np.random.default_rng(1)
    for _ in range(10):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        outs = [env.step(act) for env in envs]
        assert np.array_equal(outs[0][0][0].cpu().numpy(), outs[1][0][0].cpu().numpy())
        assert np.array_equal(outs[0][1].cpu().numpy(), outs[1][1].cpu().numpy())


def packed_step(device, p, case, es, rng_step):
    """gca_alex_step_packed on the packed layers built by the library from the case's u8 layers."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = case["grid"].shape
    g, a = _t(case["grid"], torch.uint8, device), _t(case["age"], torch.int16, device)
    veg, den, dous = (_t(case[k], torch.uint8, device) for k in ("veg", "den", "dous"))
    vd = torch.empty_like(veg)
    bits = torch.empty((E, H * W // 16), dtype=torch.int16, device=device)
    call("gca_alex_pack_layers", dev.ptr(veg), dev.ptr(den), dev.ptr(dous), dev.ptr(vd), dev.ptr(bits), E, H, W,
         dev.stream_ptr())
    coal = torch.empty_like(es)
    call("gca_alex_edge_slope_coalesce", dev.ptr(es), dev.ptr(coal), E, H, W, dev.stream_ptr())
    wi = _t(case["widx"], torch.int32, device)
    rs = _t(np.asarray(rng_step, np.uint32).view(np.int32), torch.int32, device)
    go, ao = torch.empty_like(g), torch.empty_like(a)
    counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
    call("gca_alex_step_packed", p, E, H, W, dev.ptr(g), dev.ptr(go), dev.ptr(a), dev.ptr(ao), dev.ptr(vd),
         dev.ptr(bits), dev.ptr(coal), dev.ptr(wi), dev.ptr(rs), dev.ptr(counts), None, None, dev.stream_ptr())
    return go.cpu().numpy(), ao.cpu().numpy(), counts.cpu().numpy(), coal.cpu().numpy(), bits.cpu().numpy()


@pytest.mark.parametrize("E,H,W,seed", [(2, 256, 256, 31), (1, 48, 512, 32), (1, 32, 1024, 33), (1, 512, 512, 34)])
def test_packed_step_bit_exact_vs_edge(device, E, H, W, seed):
    """The packed env layout (vd byte, dousing bits, coalesced edge slopes) reproduces gca_alex_step_es bit for
    bit over several steps, and the layout builders match their definitions."""
    case = make_case(E, H, W, seed, p_tree=0.01, dousing_p=0.2)
    p = params(H, 0.01, seed=seed * 7)
    es, _ = slopes(device, altitude(E, H, W, seed))
    es_np = es.cpu().numpy()
    for s in range(3):
        rs = np.full(E, 5 * s + 1, np.uint32)
        g1, a1, c1, coal, bits = packed_step(device, p, case, es, rs)
        g0, a0, c0, _ = step(device, "gca_alex_step_es", p, case, es, rng_step=rs)
        assert np.array_equal(g1, g0), f"step {s}: {np.argwhere(g1 != g0)[:5]}"
        assert np.array_equal(a1, a0) and np.array_equal(c1, c0)
        if s == 0:
            c = np.arange(W) % 256
            pos = (np.arange(W) // 256) * 256 + 64 * ((c >> 2) & 3) + 4 * (c >> 4) + (c & 3)
            want = np.empty_like(es_np)
            want[..., pos] = es_np
            assert np.array_equal(coal, want)
            d = case["dous"].reshape(E, H * W // 16, 16).astype(np.uint32)
            assert np.array_equal(bits.view(np.uint16), (d << np.arange(16, dtype=np.uint32)).sum(-1).astype(np.uint16))
        case["grid"], case["age"] = g1, a1


def test_env_packed_and_edge_layouts_agree(device):
    """The env on the packed layout (the default at W % 256 == 0) and on the plain edge layout: identical
    grids, rewards, dousing and positions over steps with shooting (dousing bits set by gca_advenv_post) and a
    conditional reset (bits zeroed by gca_reset_where)."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 3, 256
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=5, num_envs=E, use_hidden=True, device=device,
                                           hidden_rng=np.random.RandomState(3), slope_layout=lay)
            for lay in ("auto", "edge")]
    assert envs[0].slope_layout == "packed"
    case = make_case(E, N, N, 19, hidden=False)
    for env in envs:
        env.reset()
        env.set_state(grid=case["grid"], fire_age=case["age"], wind_index=case["widx"])
        env.pos[:, 0], env.pos[:, 1] = 100, 100  # shoot into the fire region
    rng = np.random.default_rng(2)
    for t in range(14):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        outs = [env.step(act) for env in envs]
        assert np.array_equal(outs[0][0][0].cpu().numpy(), outs[1][0][0].cpu().numpy()), f"step {t}"
        assert np.array_equal(outs[0][1].cpu().numpy(), outs[1][1].cpu().numpy())
        assert np.array_equal(envs[0].dousing.cpu().numpy(), envs[1].dousing.cpu().numpy())
        if t == 8:
            for env in envs:
                env.done[1] = 1
                env.conditional_reset()
    assert int(envs[0].dousing.sum()) > 0


@pytest.mark.parametrize("pinecones", [False, True])
def test_tile_skip_matches_full_step(device, pinecones):
    """The tiled packed step's tile activity map (tiles with no fire in their 3 x 3 tile neighbourhood are copied,
    not stepped) changes nothing: env trajectories from the reset state (two fires per env: most tiles skip)
    and from a mid-episode state equal the default env's (the marching step, which finds quiet tiles from the grid
    itself and keeps no map even with tile_skip=True), grid, ages, rewards and done, over steps with shooting,
    pinecones (which ignite tiles far from the fire front) and a conditional reset."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 3, 256
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=21, num_envs=E, use_hidden=True, device=device,
                                           hidden_rng=np.random.RandomState(4), pinecones=pinecones, tile_skip=ts,
                                           step_kernel=sk)
            for ts, sk in ((True, "tiled"), (True, "auto"))]
    assert envs[0].act is not None and not envs[0].march and envs[1].act is None and envs[1].march
    rng = np.random.default_rng(3)
    for phase in range(2):
        for env in envs:
            env.reset()
            if phase == 1:
                case = make_case(E, N, N, 30, fire_p=0.02, hidden=False)
                env.set_state(grid=case["grid"], fire_age=case["age"], wind_index=case["widx"])
        for t in range(30):
            act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
            outs = [env.step(act) for env in envs]
            for k in (0,):
                assert np.array_equal(outs[0][0][k].cpu().numpy(), outs[1][0][k].cpu().numpy()), f"{phase} {t}"
            assert np.array_equal(envs[0].age[envs[0].cur].cpu().numpy(), envs[1].age[envs[1].cur].cpu().numpy())
            assert np.array_equal(outs[0][1].cpu().numpy(), outs[1][1].cpu().numpy())
            assert np.array_equal(outs[0][2].cpu().numpy(), outs[1][2].cpu().numpy())
            if t == 20:
                for env in envs:
                    env.done[0] = 1
                    env.conditional_reset()
        # the map is exact: a tile is marked iff it holds a FIRE
        g = envs[0].grid[envs[0].cur].cpu().numpy()
        fire_tiles = (g == 2).reshape(E, N // 16, 16, N // 256, 256).any(axis=(2, 4)).reshape(E, -1)
        assert np.array_equal(envs[0].act[envs[0].cur].cpu().numpy().astype(bool), fire_tiles)
