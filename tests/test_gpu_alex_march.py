"""GPU parity of the marching Alexandridis step (gca_alex_step_march / _rgb, gca_alex_march.hip): bit-identical to the
tiled packed step (gca_alex_step_packed / _rgb) on the same state for every burn radius, with and without growth, over
several steps, through the tile activity map and the fused frame, and to the C oracle on the unpacked state."""
import ctypes

import numpy as np
import pytest

from alex_cases import make_case
from oracle import alex_c
from test_gpu_edge_slope import _t, altitude, params, slopes

pytestmark = pytest.mark.gpu


def _layers(device, case):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = case["grid"].shape
    veg, den, dous = (_t(case[k], torch.uint8, device) for k in ("veg", "den", "dous"))
    vd = torch.empty_like(veg)
    bits = torch.empty((E, H * W // 16), dtype=torch.int16, device=device)
    call("gca_alex_pack_layers", dev.ptr(veg), dev.ptr(den), dev.ptr(dous), dev.ptr(vd), dev.ptr(bits), E, H, W,
         dev.stream_ptr())
    return vd, bits


def _run(device, fn, p, case, slope, rng_step, vd, bits, act_in=None, rgb=None, night=None):
    """One step through `fn` (packed or march, plain or _rgb); returns the host copies of its outputs."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = case["grid"].shape
    g, a = _t(case["grid"], torch.uint8, device), _t(case["age"], torch.int16, device)
    wi = _t(case["widx"], torch.int32, device)
    rs = _t(np.asarray(rng_step, np.uint32).view(np.int32), torch.int32, device)
    go, ao = torch.empty_like(g), torch.empty_like(a)
    counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
    tiles = (H // 16) * (W // 256)
    ain = None if act_in is None else _t(act_in, torch.uint8, device)
    aout = torch.full((E, tiles), 7, dtype=torch.uint8, device=device)
    args = [p, E, H, W, dev.ptr(g), dev.ptr(go), dev.ptr(a), dev.ptr(ao), dev.ptr(vd), dev.ptr(bits), dev.ptr(slope),
            dev.ptr(wi), dev.ptr(rs), dev.ptr(counts), dev.ptr(ain), dev.ptr(aout)]
    out_rgb = None
    if rgb is not None:
        col, nt = rgb
        out_rgb = torch.full((E, H, W, 3), -1.0, dtype=torch.float32, device=device)
        args += [dev.ptr(col), dev.ptr(nt), dev.ptr(out_rgb)]
    call(fn, *args, dev.stream_ptr())
    torch.cuda.synchronize()
    return (go.cpu().numpy(), ao.cpu().numpy(), counts.cpu().numpy(), aout.cpu().numpy(),
            None if out_rgb is None else out_rgb.cpu().numpy())


def _coalesced(device, es):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, _, H, W = es.shape
    coal = torch.empty_like(es)
    call("gca_alex_edge_slope_coalesce", dev.ptr(es), dev.ptr(coal), E, H, W, dev.stream_ptr())
    return coal


def _with_radius(p, R):
    q = type(p)()
    ctypes.memmove(ctypes.addressof(q), ctypes.addressof(p), ctypes.sizeof(q))
    q.R = R
    return q


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("E,H,W,seed,p_tree", [(2, 256, 256, 41, 0.0), (3, 48, 256, 42, 0.01), (2, 16, 256, 43, 0.0),
                                               (2, 64, 512, 44, 0.0), (3, 32, 512, 45, 0.01), (1, 48, 1024, 46, 0.0)])
def test_march_matches_packed(device, R, E, H, W, seed, p_tree):
    """Grid, ages, counts and the activity map out of the marching step equal the tiled step's, three steps on; at W =
    512 / 1024 the segment waves of a strip exchange their edge values (every radius crosses the boundaries)."""
    case = make_case(E, H, W, seed, p_tree=p_tree, dousing_p=0.2, fire_p=0.05)
    p = _with_radius(params(H, p_tree, seed=seed * 5), R)
    es, _ = slopes(device, altitude(E, H, W, seed))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    for s in range(3):
        rs = np.full(E, 7 * s + 2, np.uint32)
        g0, a0, c0, t0, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        g1, a1, c1, t1, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        assert np.array_equal(g1, g0), f"R={R} step {s}: {np.argwhere(g1 != g0)[:5]}"
        assert np.array_equal(a1, a0), f"R={R} step {s}: ages {np.argwhere(a1 != a0)[:5]}"
        assert np.array_equal(c1, c0)
        assert np.array_equal(t1, t0)
        case["grid"], case["age"] = g1, a1


def test_march_tile_skip_and_frame(device):
    """act_in with fire-free tiles (copied) and the fused RGB frame: equal to the tiled kernel's, both night and
    day, and the skipped tiles' frame equals the frame of the full step."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    E, H, W = 3, 128, 256
    case = make_case(E, H, W, 51, p_tree=0.0, dousing_p=0.2, fire_p=0.0)
    # fire only in tile rows 2 and 6 of env 0, tile row 4 of env 2; env 1 has none
    case["grid"][0, 40, 10:20] = 2
    case["grid"][0, 100, 200] = 2
    case["grid"][2, 70, 0:256:9] = 2
    case["age"][case["grid"] == 2] = 3
    p = params(H, 0.0, seed=9)
    es, _ = slopes(device, altitude(E, H, W, 51))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    tiles = H // 16
    act = np.zeros((E, tiles), np.uint8)
    for e in range(E):
        for t in range(tiles):
            act[e, t] = int((case["grid"][e, 16 * t:16 * t + 16] == 2).any())
    op = make_obs_params(0, 1, 2, False, False, 8)
    col = torch.zeros((12, 4), dtype=torch.float32, device=device)
    call("gca_obs_color_table", op, dev.ptr(col), dev.stream_ptr())
    night = torch.as_tensor(np.array([0, 1, 1], np.int32), device=device)
    rs = np.full(E, 3, np.uint32)
    ref = _run(device, "gca_alex_step_packed_rgb", p, case, coal, rs, vd, bits, act_in=act, rgb=(col, night))
    got = _run(device, "gca_alex_step_march_rgb", p, case, es, rs, vd, bits, act_in=act, rgb=(col, night))
    full = _run(device, "gca_alex_step_march_rgb", p, case, es, rs, vd, bits, act_in=None, rgb=(col, night))
    for k in range(4):
        assert np.array_equal(got[k], ref[k]), k
        assert np.array_equal(full[k][:3], ref[k][:3]) if k < 3 else True
    assert np.array_equal(got[4], ref[4])
    assert np.array_equal(full[4], ref[4])
    assert (got[3][1] == 0).all() and got[3][0].any()


@pytest.mark.parametrize("E,H", [(3, 16), (5, 48), (1, 32)])
def test_march_frame_partial_last_workgroup(device, E, H):
    """The fused-frame march kernel when the wave count is not a multiple of 4 (the last workgroup's excess waves exit
    at once and join the XROW barrier): grid, ages, counts and frame equal the tiled kernel's, day and night."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    W = 256
    case = make_case(E, H, W, 70 + E, p_tree=0.0, dousing_p=0.2, fire_p=0.06)
    p = params(H, 0.0, seed=4)
    es, _ = slopes(device, altitude(E, H, W, 70 + E))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    op = make_obs_params(0, 1, 2, False, False, 8)
    col = torch.zeros((12, 4), dtype=torch.float32, device=device)
    call("gca_obs_color_table", op, dev.ptr(col), dev.stream_ptr())
    night = torch.as_tensor(np.arange(E, dtype=np.int32) % 2, device=device)
    rs = np.full(E, 5, np.uint32)
    ref = _run(device, "gca_alex_step_packed_rgb", p, case, coal, rs, vd, bits, rgb=(col, night))
    got = _run(device, "gca_alex_step_march_rgb", p, case, es, rs, vd, bits, rgb=(col, night))
    for k in (0, 1, 2, 4):
        assert np.array_equal(got[k], ref[k]), k


def test_march_matches_oracle(device):
    """The marching step against the C oracle (Philox mode) on the unpacked state, directly."""
    E, H, W = 2, 64, 256
    case = make_case(E, H, W, 61, p_tree=0.01, dousing_p=0.2, fire_p=0.05)
    p = params(H, 0.01, seed=77)
    es, ps = slopes(device, altitude(E, H, W, 61))
    vd, bits = _layers(device, case)
    rs = np.full(E, 11, np.uint32)
    g1, a1, c1, _, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
    go, ao, co, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"],
                                     case["dous"], ps.cpu().numpy(), case["widx"], rng_step=rs)
    assert np.array_equal(g1, go), np.argwhere(g1 != go)[:5]
    assert np.array_equal(a1, ao)
    assert np.array_equal(c1, co)


def test_march_rejects_bad_shapes(device):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import GCAError, call

    p = params(16)
    for W in (384, 768, 2048):  # widths the kernel does not take (256, 512, 1024 only)
        g = torch.zeros((1, 16, W), dtype=torch.uint8, device=device)
        with pytest.raises(GCAError):
            call("gca_alex_step_march", p, 1, 16, W, dev.ptr(g), dev.ptr(g.clone()), dev.ptr(g), dev.ptr(g),
                 dev.ptr(g), dev.ptr(g), dev.ptr(g), dev.ptr(g), None, None, None, None, dev.stream_ptr())
    # the tile activity map is read at W = 256 only
    g = torch.zeros((1, 16, 512), dtype=torch.uint8, device=device)
    act = torch.ones((2, 2), dtype=torch.uint8, device=device)
    with pytest.raises(GCAError):
        call("gca_alex_step_march", p, 1, 16, 512, dev.ptr(g), dev.ptr(g.clone()), dev.ptr(g), dev.ptr(g), dev.ptr(g),
             dev.ptr(g), dev.ptr(g), dev.ptr(g), None, None, dev.ptr(act[0]), dev.ptr(act[1]), dev.stream_ptr())


def test_march_other_cell_codes(device):
    """Arbitrary cell codes (FIRE = 0, EMPTY = 7, TREE = 3, plus cells of a fourth code the rule leaves alone): the
    marching step equals the tiled one, including the EMPTY padding outside the grid (a FIRE code of 0 must not make
    the border burn)."""
    from alex_cases import winds
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params

    E, H, W = 2, 48, 256
    case = make_case(E, H, W, 71, p_tree=0.01, dousing_p=0.2, fire_p=0.05)
    codes = np.array([7, 3, 0], np.uint8)
    g = codes[case["grid"]]
    g[:, 5, 10:20] = 9  # a code outside {empty, tree, fire}
    case["grid"] = g
    p, _ = make_alex_params(H, 7, 3, 0, winds(), 0.01, 99)
    es, _ = slopes(device, altitude(E, H, W, 71))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    rs = np.full(E, 5, np.uint32)
    g0, a0, c0, t0, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
    g1, a1, c1, t1, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
    assert np.array_equal(g1, g0), np.argwhere(g1 != g0)[:5]
    assert np.array_equal(a1, a0) and np.array_equal(c1, c0) and np.array_equal(t1, t0)
    assert (g1[:, 5, 10:20] == 9).all()


def test_march_quiet_tiles_from_the_grid(device):
    """Without an activity map (act_in = NULL) at p_tree = 0 the step copies tiles with no FIRE in their rows or the
    row on either side, found from the grid itself: fires placed on tile-boundary rows (the last row of a tile, the
    first row of the next, the grid's first and last rows) and a fire-free env; grid, ages (not in place), counts and
    the activity map equal the tiled kernel's over four steps."""
    E, H, W = 3, 96, 256
    case = make_case(E, H, W, 61, p_tree=0.0, dousing_p=0.2, fire_p=0.0)
    case["grid"][0, 15, 100] = 2    # last row of tile 0: tiles 0 and 1 are not quiet
    case["grid"][0, 48, 3:250:31] = 2  # first row of tile 3: tiles 2 and 3
    case["grid"][2, 0, 0] = 2       # the grid's first row
    case["grid"][2, 95, 255] = 2    # the grid's last row
    case["age"][case["grid"] == 2] = 4
    p = params(H, 0.0, seed=13)
    es, _ = slopes(device, altitude(E, H, W, 61))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    for s in range(4):
        rs = np.full(E, 11 * s + 1, np.uint32)
        g0, a0, c0, t0, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        g1, a1, c1, t1, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        assert np.array_equal(g1, g0), f"step {s}: {np.argwhere(g1 != g0)[:5]}"
        assert np.array_equal(a1, a0) and np.array_equal(c1, c0) and np.array_equal(t1, t0), f"step {s}"
        case["grid"], case["age"] = g1, a1
    assert (case["grid"][1] != 2).all()


@pytest.mark.parametrize("W", [512, 1024])
def test_march_segment_boundaries(device, W):
    """Fires, dousing and steep slopes placed on and next to the segment boundaries (columns 255 | 256, 511 | 512, ...)
    and the grid's side borders, growth on: the marching step at W = 512 / 1024 equals the tiled step and the C oracle
    (grid, ages, counts, map) over three steps, and its fused frame equals the tiled kernel's (night and day)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    E, H = 2, 48
    case = make_case(E, H, W, 81 + W, p_tree=0.02, dousing_p=0.0, fire_p=0.0)
    for b in range(0, W + 1, 256):  # every segment edge and the two borders
        for c in (b - 2, b - 1, b, b + 1):
            if 0 <= c < W:
                case["grid"][0, 3:45:3, c] = 2
                case["grid"][1, 20:24, c] = 2
                case["dous"][0, 10:40:4, c] = 1
    case["age"][case["grid"] == 2] = 5
    p = _with_radius(params(H, 0.02, seed=13), 8 if W == 1024 else 7)
    es, ps = slopes(device, altitude(E, H, W, 17) * 3.0)  # steep: large slope factors either way
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    for s in range(3):
        rs = np.full(E, 5 + s, np.uint32)
        g0, a0, c0, t0, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        g1, a1, c1, t1, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        go, ao, co, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"],
                                         ps.cpu().numpy(), case["widx"], rng_step=rs)
        assert np.array_equal(g1, g0), f"step {s}: {np.argwhere(g1 != g0)[:5]}"
        assert np.array_equal(g1, go) and np.array_equal(a1, ao) and np.array_equal(c1, co)
        assert np.array_equal(a1, a0) and np.array_equal(c1, c0) and np.array_equal(t1, t0)
        case["grid"], case["age"] = g1, a1
    op = make_obs_params(0, 1, 2, False, False, 8)
    col = torch.zeros((12, 4), dtype=torch.float32, device=device)
    call("gca_obs_color_table", op, dev.ptr(col), dev.stream_ptr())
    night = torch.as_tensor(np.array([0, 1], np.int32), device=device)
    rs = np.full(E, 9, np.uint32)
    ref = _run(device, "gca_alex_step_packed_rgb", p, case, coal, rs, vd, bits, rgb=(col, night))
    got = _run(device, "gca_alex_step_march_rgb", p, case, es, rs, vd, bits, rgb=(col, night))
    for k in range(5):
        assert np.array_equal(got[k], ref[k]), k


def test_march_wide_quiet_strips(device):
    """W = 512 without a map: a strip is copied only when no segment of it holds a FIRE near it (one consensus per
    workgroup); a FIRE in the right segment's first column next to a TREE in the left segment's last column must
    still burn across the boundary. Equal to the tiled kernel over three steps."""
    E, H, W = 2, 64, 512
    case = make_case(E, H, W, 91, p_tree=0.0, dousing_p=0.1, fire_p=0.0)
    case["grid"][0, 20, 256] = 2  # right segment only; the left segment's column 255 trees sit next to it
    case["grid"][0, 20, 255] = 1
    case["grid"][1, 47, 511] = 2  # last column, last row of a strip
    case["age"][case["grid"] == 2] = 9
    p = params(H, 0.0, seed=3)
    es, _ = slopes(device, altitude(E, H, W, 91))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    for s in range(3):
        rs = np.full(E, s, np.uint32)
        g0, a0, c0, t0, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        g1, a1, c1, t1, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        assert np.array_equal(g1, g0) and np.array_equal(a1, a0) and np.array_equal(c1, c0)
        assert np.array_equal(t1, t0)
        case["grid"], case["age"] = g1, a1


@pytest.mark.parametrize("N,pinecones", [(512, False), (512, True), (1024, False)])
def test_env_march_equals_tiled_at_wide_grids(device, N, pinecones):
    """The Advanced env at 512^2 / 1024^2 (R = 7 / 8, the reference's grid sizes above the headline) runs the marching
    step (segment waves per strip); the same env on the tiled step (step_kernel="tiled") reproduces its trajectory
    bit for bit: grids, ages, rewards, done, positions, over steps with shooting, pinecone spotting and a conditional
    reset (advanced_bulldozer.py:332-518)."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E = 2
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=31, num_envs=E, use_hidden=True, device=device,
                                           hidden_rng="philox", observation="grid", pinecones=pinecones,
                                           step_kernel=sk) for sk in ("auto", "tiled")]
    assert envs[0].march and not envs[1].march
    assert envs[0].alex_params.R == (7 if N == 512 else 8)
    case = make_case(E, N, N, 33, fire_p=0.03, hidden=False)
    for env in envs:
        env.reset()
        env.set_state(grid=case["grid"], fire_age=case["age"], wind_index=case["widx"])
    rng = np.random.default_rng(5)
    for t in range(6):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        outs = [env.step(act) for env in envs]
        a, b = envs
        assert np.array_equal(a.grid[a.cur].cpu().numpy(), b.grid[b.cur].cpu().numpy()), t
        assert np.array_equal(a.age[a.cur].cpu().numpy(), b.age[b.cur].cpu().numpy()), t
        assert np.array_equal(outs[0][1].cpu().numpy(), outs[1][1].cpu().numpy())
        assert np.array_equal(outs[0][2].cpu().numpy(), outs[1][2].cpu().numpy())
        assert np.array_equal(a.pos.cpu().numpy(), b.pos.cpu().numpy())
        if t == 3:
            for env in envs:
                env.done[0] = 1
                env.conditional_reset()


@pytest.mark.parametrize("uniform", [False, True])
@pytest.mark.parametrize("R,W,p_tree,seed", [(6, 256, 0.0, 81), (1, 256, 0.01, 82), (8, 256, 0.0, 83), (7, 512, 0.0, 84),
                                             (3, 512, 0.01, 85), (6, 1024, 0.0, 86)])
def test_flat_terrain_step_equals_unit_planes(device, R, W, p_tree, seed, uniform):
    """edge_slope = NULL (the flat-terrain instance: no slope planes read, every row through the factor-free pass) equals
    the general step on all-ones edge planes, bit for bit: grid, ages, counts and tile map over three chained steps,
    the fused frame at W = 256 (day and night), with and without the tile activity map. `uniform`: every cell's
    vegetation / density the same (use_hidden=False's layers) and vd = NULL as well (p.vd_uniform)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    E, H = 3, 48
    case = make_case(E, H, W, seed, p_tree=p_tree, dousing_p=0.2, fire_p=0.05)
    p = _with_radius(params(H, p_tree, seed=seed * 3), R)
    if uniform:
        case["veg"][...] = 4
        case["den"][...] = 2
        p.vd_uniform = 4 | 2 << 4
    ones = torch.ones((E, 4, H, W), dtype=torch.float32, device=device)
    vd, bits = _layers(device, case)
    if uniform:
        assert bool((vd == p.vd_uniform).all())
    rgb = None
    if W == 256:
        col = torch.zeros((12, 4), dtype=torch.float32, device=device)
        call("gca_obs_color_table", make_obs_params(0, 1, 2, False, False, 8), dev.ptr(col), dev.stream_ptr())
        rgb = (col, torch.as_tensor(np.arange(E, dtype=np.int32) % 2, device=device))
    for s in range(3):
        rs = np.full(E, 11 * s + 1, np.uint32)
        for fn, extra in (("gca_alex_step_march", {}),) + ((("gca_alex_step_march_rgb", {"rgb": rgb}),) if rgb else ()):
            act = np.ones((E, H // 16), np.uint8) if (W == 256 and p_tree == 0.0) else None
            ref = _run(device, fn, p, case, ones, rs, vd, bits, act_in=act, **extra)
            got = _run(device, fn, p, case, None, rs, None if uniform else vd, bits, act_in=act, **extra)
            for k in range(5):
                if ref[k] is not None:
                    assert np.array_equal(got[k], ref[k]), (fn, s, k)
        case["grid"], case["age"] = ref[0], ref[1]
        assert (ref[0] == 2).any()


@pytest.mark.parametrize("extensions", [False, True])
def test_env_flat_terrain_equals_general(device, extensions):
    """use_hidden=False gives flat terrain: the env's step takes edge_slope = NULL (env.flat_terrain) and equals, bit for
    bit, the same env forced through the general step (slope planes read): grid, ages, counts, reward and the fused
    RGB frame (plain, or the extension pipeline with the three choices mixed), over steps with a conditional reset;
    a non-flat slope buffer written in place is picked up by refresh_terrain()."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 6, 256
    envs = [AdvancedForestFireBulldozerEnv(N, N, key=5, num_envs=E, use_hidden=False, device=device, observation="rgb",
                                           enable_extensions=extensions) for _ in range(2)]
    assert all(env.flat_terrain and env.uniform_layers for env in envs)
    envs[1].flat_terrain = False
    for env in envs:
        env.reset()
        env.pos[:, 0], env.pos[:, 1] = 190, 60
    rng = np.random.default_rng(3)
    for s in range(6):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), rng.integers(0, 3, E)], axis=1).astype(np.int32)
        outs = [env.step(torch.as_tensor(act, device=device)) for env in envs]
        a, b = envs
        assert torch.equal(a.grid[a.cur], b.grid[b.cur]) and torch.equal(a.age[a.cur], b.age[b.cur]), s
        assert torch.equal(a.counts, b.counts) and torch.equal(outs[0][1], outs[1][1]), s
        assert torch.equal(a.rgb, b.rgb), s
        if s == 3:
            for env in envs:
                env.done[1] = 1
                env.conditional_reset()
    assert int(envs[0].counts[:, 2].sum()) > 0
    env = envs[0]
    env.set_state(vegetation=torch.full((E, N, N), 2, dtype=torch.uint8, device=device))
    assert env.flat_terrain and env.uniform_layers and env.alex_params.vd_uniform == (2 | 3 << 4)
    env.vegetation[0, 3, 3] = 5
    env.set_state(vegetation=env.vegetation.clone())
    assert env.flat_terrain and not env.uniform_layers
    env.slope_data[:, 0, 5, 5] = 1.5
    env.refresh_terrain()
    assert not env.flat_terrain and not env.uniform_layers


@pytest.mark.parametrize("W,R", [(256, 6), (512, 7), (1024, 8)])
def test_march_sparse_dousing_equals_packed(device, W, R):
    """Sparse dousing (most wave-rows see none in their 5 x 5 windows and skip the dousing term): the marching step,
    general and flat terrain, equals the tiled packed step bit for bit; doused cells placed on the 256-column segment
    edges (the HALO exchange carries their window sums across) and in the grid's first / last rows."""
    case = make_case(3, 48, W, 90 + R, p_tree=0.0, dousing_p=0.0, fire_p=0.08)
    d = case["dous"]
    d[0, 10, 255] = d[0, 30, 256 % W] = d[1, 0, 5] = d[1, 47, W - 1] = d[2, 20, 128] = 1
    if W > 256:
        d[2, 5, 511] = d[2, 6, 512 % W] = d[0, 40, 254] = 1
    p = _with_radius(params(48, 0.0, seed=R), R)
    es, _ = slopes(device, altitude(3, 48, W, 90 + R))
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    import torch

    ones = torch.ones_like(es)
    ones_coal = _coalesced(device, ones)
    for s in range(3):
        rs = np.full(3, 4 * s + 1, np.uint32)
        g0, a0, c0, _, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        g1, a1, c1, _, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        assert np.array_equal(g1, g0) and np.array_equal(a1, a0) and np.array_equal(c1, c0), s
        f0 = _run(device, "gca_alex_step_packed", p, case, ones_coal, rs, vd, bits)
        f1 = _run(device, "gca_alex_step_march", p, case, None, rs, vd, bits)
        for k in range(3):
            assert np.array_equal(f1[k], f0[k]), (s, k)
        case["grid"], case["age"] = g1, a1
