"""GPU parity of the observation builders (gca_adv_observation) with the literal numpy restatement of
the reference (oracle/observation.py): step observations over extension choices, day/night, dousing,
blur/visibility and the row/channel quirk; the reset observation; the env's RGB observation."""
import numpy as np
import pytest

from oracle import observation as ob

pytestmark = pytest.mark.gpu


def _t(x, dtype, device):
    import torch

    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


def run(device, params, mode, grid, dous, pos, night, time_step=None, action=None, channels=False):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = grid.shape
    g, d = _t(grid, torch.uint8, device), _t(dous, torch.uint8, device)
    p_, n_ = _t(pos, torch.int32, device), _t(night, torch.int32, device)
    ts = None if time_step is None else _t(time_step, torch.int32, device)
    a = None if action is None else _t(action, torch.int32, device)
    rgb = torch.full((E, H, W, 3), -1.0, dtype=torch.float32, device=device)
    ch = torch.full((E, H, W, 5), 255, dtype=torch.uint8, device=device) if channels else None
    call("gca_adv_observation", params, mode, E, H, W, dev.ptr(g), dev.ptr(d), dev.ptr(p_), dev.ptr(n_), dev.ptr(ts),
         dev.ptr(a), 0 if a is None else int(a.shape[-1]), dev.ptr(rgb), dev.ptr(ch), None, dev.stream_ptr())
    return rgb.cpu().numpy(), None if ch is None else ch.cpu().numpy()


def make(E, H, W, seed, p3=0.0):
    rng = np.random.default_rng(seed)
    p = [0.3, 0.5, 0.2 - p3, p3]
    grid = rng.choice([0, 1, 2, 3], size=(E, H, W), p=p).astype(np.uint8)
    for e in range(0, E, 3):  # some envs with empty leading rows (channel-index quirk)
        grid[e, :rng.integers(0, min(H, 4))] = 0
    dous = rng.choice([0, 1, 2], size=(E, H, W), p=[0.8, 0.15, 0.05]).astype(np.uint8)
    pos = np.stack([rng.integers(0, H, E), rng.integers(0, W, E)], axis=1)
    return rng, grid, dous, pos


@pytest.mark.parametrize("enable", [False, True])
@pytest.mark.parametrize("E,H,W,seed", [(6, 8, 8, 0), (6, 16, 24, 1), (4, 64, 64, 2), (3, 37, 53, 3), (2, 256, 256, 4),
                                        (5, 16, 48, 5), (7, 32, 8, 6)])
def test_step_observation_matches_reference(device, enable, E, H, W, seed):
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP, make_obs_params

    rng, grid, dous, pos = make(E, H, W, seed, p3=0.05)
    night_pre = rng.integers(0, 2, E)
    day_length = 400
    time_step = rng.choice([399, 400, 401, 800], size=E)          # post-step time_step
    night_post = np.where(time_step % day_length == 0, 1 - night_pre, night_pre)
    action = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), np.arange(E) % 3], axis=1)
    params = make_obs_params(0, 1, 2, enable, enable, day_length)
    rgb, ch = run(device, params, 0, grid, dous, pos, night_post, time_step, action, channels=True)
    for e in range(E):
        flags = EXTENSION_LOOKUP[action[e, 2]]
        want, want_ch = ob.step_observation(grid[e].astype(np.int32), tuple(pos[e]), flags, int(night_pre[e]),
                                            dous[e].astype(np.int32), enable, enable)
        assert np.array_equal(rgb[e], want), e
        assert np.array_equal(ch[e], want_ch.astype(np.uint8)), e


@pytest.mark.parametrize("E,N,seed", [(4, 5, 0), (4, 8, 1), (3, 64, 2), (2, 256, 3)])
def test_reset_observation_matches_reference(device, E, N, seed):
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    rng, grid, dous, pos = make(E, N, N, seed)
    night = rng.integers(0, 2, E)
    rgb, _ = run(device, make_obs_params(0, 1, 2, True, True, 400), 1, grid, dous, pos, night)
    for e in range(E):
        want = ob.reset_observation(grid[e].astype(np.int32), tuple(pos[e]), int(night[e]), dous[e].astype(np.int32))
        assert np.array_equal(rgb[e], want), e


def test_env_rgb_observation(device):
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP

    E, N = 4, 32
    env = AdvancedForestFireBulldozerEnv(N, N, key=3, num_envs=E, use_hidden=False, device=device,
                                         observation="rgb", enable_extensions=True)
    obs, _ = env.reset()
    g0 = env.grid[env.cur].cpu().numpy()
    want = [ob.reset_observation(g0[e].astype(np.int32), tuple(env.pos[e].tolist()), 0, np.zeros((N, N), np.int32))
            for e in range(E)]
    assert np.array_equal(obs[0].cpu().numpy(), np.stack(want))
    rng = np.random.default_rng(0)
    for s in range(6):
        night_pre = env.is_night.cpu().numpy().copy()
        dous_pre = env.dousing.cpu().numpy().astype(np.int32)
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), rng.integers(0, 3, E)], axis=1)
        (rgb, _), _, _, _, _ = env.step(torch.as_tensor(act, device=device))
        g = env.grid[env.cur].cpu().numpy()
        pos = env.pos.cpu().numpy()
        for e in range(E):
            want, _ = ob.step_observation(g[e].astype(np.int32), tuple(pos[e]), EXTENSION_LOOKUP[act[e, 2]],
                                          int(night_pre[e]), dous_pre[e], True, True)
            assert np.array_equal(rgb[e].cpu().numpy(), want), (s, e)


@pytest.mark.parametrize("W", [768, 512, 256])
@pytest.mark.parametrize("tile_skip", [False, True])
def test_fused_step_observation_matches_reference(device, tile_skip, W):
    """The plain observation (enable_extensions=False, the reference's default) written by the CA step's own
    epilogue on the packed layout (W = 768: gca_alex_step_packed_rgb, the tiled step, three tiles per row; W = 256 /
    512: the marching gca_alex_step_march_rgb, one / two segment waves per strip) + the bulldozer's pixel (gca_obs_position) equals the literal restatement of
    grid_to_rgb (advanced_bulldozer.py:1035-1101) of the post-step grid and position with the PRE-step dousing and
    day / night: over steps with shooting, a day / night toggle, the tile-skip path and a conditional reset."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, H = 3, 256
    env = AdvancedForestFireBulldozerEnv(H, W, key=8, num_envs=E, use_hidden=True, device=device, observation="grid",
                                         hidden_rng="philox", tile_skip=tile_skip)
    assert env.march == (W != 768)
    env.reset()
    # observation="rgb" needs a square grid for the reset frame; the step frame does not: give this env an RGB buffer
    env.rgb = torch.zeros((E, H, W, 3), dtype=torch.float32, device=device)
    assert env.fused_observation
    env.pos[:, 0], env.pos[:, 1] = 190, 60  # near the initial fire: shots land on burning / tree cells
    env.time_step.fill_(398)
    rng = np.random.default_rng(4)
    for s in range(8):
        night_pre = env.is_night.cpu().numpy().copy()
        dous_pre = env.dousing.cpu().numpy().astype(np.int32)
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        env.step(act)
        g = env.grid[env.cur].cpu().numpy()
        pos = env.pos.cpu().numpy()
        rgb = env.rgb.cpu().numpy()
        for e in range(E):
            want, _ = ob.step_observation(g[e].astype(np.int32), tuple(pos[e]), (0, 0), int(night_pre[e]),
                                          dous_pre[e], False, False)
            assert np.array_equal(rgb[e], want), (s, e)
        if s == 4:
            env.done[1] = 1
            env.conditional_reset()
    assert int(env.dousing.sum()) > 0 and env.is_night.cpu().numpy().any()


@pytest.mark.parametrize("tile_skip", [False, True])
def test_fused_extension_frame_matches_reference(device, tile_skip):
    """the extension pipeline's frame (enable_extensions=True, should_transform with it) from the
    marching step's epilogue (gca_alex_step_march_rgb_ext, W = 256) + the bulldozer's pixel + the refit pass of
    gca_adv_observation for the envs whose display the epilogue cannot give (no extension chosen: the blurred grid;
    row 0 of the chosen channel empty: the reference's row-vs-channel display scan) equals the literal restatement of
    build_observation_on_extensions / grid_to_rgb_with_extensions (advanced_bulldozer.py:988-1101,
    extension_utils.py:89-134) for every extension choice, on envs whose first rows are burnt out (speculation fails),
    an all-empty env, and through a day / night toggle and a conditional reset."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP

    E, N = 9, 256
    env = AdvancedForestFireBulldozerEnv(N, N, key=12, num_envs=E, use_hidden=True, device=device, observation="rgb",
                                         hidden_rng="philox", enable_extensions=True, tile_skip=tile_skip)
    assert env.march and env._ext_frame and env.fused_observation
    env.reset()
    g = env.grid[env.cur].clone()
    g[3, :2] = 0   # row 0 empty (and row 1): the unblur channel's row 0 is empty -> refit
    g[4, :1] = 0   # row 0 empty only
    g[5] = 0       # no TREE / FIRE at all -> the base channel
    g[6, :1, :] = 1  # a full TREE row 0: the blur of row 0 is positive
    rng = np.random.default_rng(5)
    g[7] = torch.as_tensor(rng.choice([0, 1, 2], size=(N, N), p=[0.3, 0.5, 0.2]).astype(np.uint8), device=device)
    env.set_state(grid=g)
    env.pos[:, 0], env.pos[:, 1] = 190, 60
    env.time_step.fill_(397)
    refit_seen = set()
    for s in range(7):
        night_pre = env.is_night.cpu().numpy().copy()
        dous_pre = env.dousing.cpu().numpy().astype(np.int32)
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), (np.arange(E) + s) % 3], axis=1)
        (rgb, _), _, _, _, _ = env.step(torch.as_tensor(act, device=device))
        refit_seen |= {int(x) for x in env._refit.cpu().numpy()}
        gn = env.grid[env.cur].cpu().numpy()
        pos = env.pos.cpu().numpy()
        rgb = rgb.cpu().numpy()
        for e in range(E):
            want, _ = ob.step_observation(gn[e].astype(np.int32), tuple(pos[e]), EXTENSION_LOOKUP[act[e, 2]],
                                          int(night_pre[e]), dous_pre[e], True, True)
            assert np.array_equal(rgb[e], want), (s, e, int(act[e, 2]), int(env._refit[e]))
        if s == 3:
            env.done[2] = 1
            env.conditional_reset()
    assert refit_seen == {0, 1}
    assert env.is_night.cpu().numpy().any()


@pytest.mark.parametrize("enable", [False, True])
def test_fused_frames_equal_the_observation_pass_at_config3(device, enable):
    """BASELINE config 3's full batch (4096 x 256^2, the bench's mid-episode state): the frame the marching step writes
    in its epilogue (plain: gca_alex_step_march_rgb; extension pipeline: gca_alex_step_march_rgb_ext with the three
    extension choices spread over the envs, some envs' first rows burnt out, + the refit pass) equals, on every env,
    the frame gca_adv_observation renders from the same post-step state (the pass the oracle tests pin)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 4096, 256
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device, observation="rgb",
                                         enable_extensions=enable)
    assert env.fused_observation
    env.reset()
    gen = torch.Generator(device=device).manual_seed(77)
    u = torch.rand((E, N, N), device=device, generator=gen)
    g = torch.where(u < 0.1, 0, torch.where(u < 0.9, 1, 2)).to(torch.uint8)
    g[::97, :2] = 0  # rows 0-1 burnt out in some envs (the extension frame's row-0 speculation fails there)
    age = torch.where(g == 2, torch.randint(1, 673, (E, N, N), device=device, generator=gen, dtype=torch.int16),
                      torch.zeros((), dtype=torch.int16, device=device))
    env.set_state(grid=g, fire_age=age, wind_index=torch.randint(0, 8, (E,), device=device, generator=gen,
                                                                  dtype=torch.int32))
    del u, g, age
    action = torch.stack([torch.randint(0, 9, (E,), device=device, generator=gen),
                          torch.randint(0, 2, (E,), device=device, generator=gen),
                          torch.arange(E, device=device) % 3], 1).to(torch.int32).contiguous()
    want = torch.empty_like(env.rgb)
    for s in range(2):
        env.step(action)
        call("gca_adv_observation", env.obs_params, 0, E, N, N, dev.ptr(env.grid[env.cur]), dev.ptr(env.dousing),
             dev.ptr(env.pos), dev.ptr(env.is_night), dev.ptr(env.time_step), dev.ptr(action), 3, dev.ptr(want), None,
             None, dev.stream_ptr(device))
        diff = (env.rgb != want).reshape(E, -1).any(-1)
        assert not bool(diff.any()), (s, torch.nonzero(diff)[:5].flatten().tolist())
    if enable:
        assert 0 < int(env._refit.sum()) < E  # both the epilogue's frames and refits


def test_observation_kernel_reproduces_reference_run(device, golden):
    """gca_adv_observation against the reference's own observation builders executed
    (tests/golden/observation.npz, see tests/test_observation_golden.py): every case whose extension flags the
    env's action space can express (EXTENSION_LOOKUP: choose = 1), the step frame and channels bit for bit, and the
    reset frame on square grids."""
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP, make_obs_params

    d = golden("observation")
    lookup = [tuple(int(b) for b in row) for row in EXTENSION_LOOKUP]
    checked = 0
    for i in range(int(d["n"])):
        p = f"c{i}_"
        a = d[p + "actions"]
        if tuple(int(v) for v in a[2:]) not in lookup:
            continue
        enable, transform = (bool(v) for v in d[p + "flags"])
        grid, dous = d[p + "grid"][None], d[p + "dous"][None]
        pos, night = d[p + "pos"][None], np.array([int(d[p + "night"])])
        action = np.array([[a[0], a[1], lookup.index(tuple(int(v) for v in a[2:]))]])
        params = make_obs_params(0, 1, 2, enable, transform, 400)
        rgb, ch = run(device, params, 0, grid, dous, pos, night, np.array([1]), action, channels=True)
        assert np.array_equal(rgb[0], d[p + "rgb"]), i
        assert np.array_equal(ch[0], d[p + "channels"].astype(np.uint8)), i
        if d[p + "reset"].size:
            rgb0, _ = run(device, params, 1, grid, dous, pos, night)
            assert np.array_equal(rgb0[0], d[p + "reset"]), i
        checked += 1
    assert checked >= 20
