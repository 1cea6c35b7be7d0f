"""GPU: device init of the Advanced env's context layers against the reference's own output
(tests/golden/init_utils.npz): altitude arithmetic (gca_alex_altitude_apply), get_slope
(gca_alex_slope_from_altitude) and the env's layers built from a seeded legacy stream."""
import numpy as np
import pytest

from gymca_amd.forest_fire.bulldozer import init_utils as iu
from oracle import alex_c

pytestmark = pytest.mark.gpu


def _slope_f32_close(got, ref64):
    """f32 slope vs the reference's float64 slope cast to f32 (jnp.array): equal, or one f32 ulp
    apart where device cos/atan and numpy differ in the last float64 ulp."""
    ref = ref64.astype(np.float32)
    ulp = np.spacing(np.abs(ref).astype(np.float32))
    return np.all(np.abs(got - ref) <= ulp), float(np.mean(got == ref))


def test_device_altitude_matches_reference(device, golden):
    g = golden("init_utils")
    for k in range(int(g["n"])):
        H, W, E = (int(x) for x in g[f"shape_{k}"])
        rs = np.random.RandomState(1000 + k)
        iu.init_vegetation(H, W, E, rs)
        iu.init_density(H, W, E, rs)
        plan = iu.altitude_plan(H, W, E, rs)
        alt = iu.device_altitude(plan, device).cpu().numpy()
        ref = g[f"alt_{k}"]
        assert np.max(np.abs(alt - ref) / np.maximum(np.abs(ref), 1.0)) < 1e-14, k
        assert np.array_equal(rs.randint(0, 2**31 - 1, size=4), g[f"next_{k}"])


def test_device_slope_matches_reference(device, golden):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    g = golden("init_utils")
    for k in range(int(g["n"])):
        H, W, E = (int(x) for x in g[f"shape_{k}"])
        alt = torch.as_tensor(g[f"alt_{k}"], dtype=torch.float64, device=device)
        p_slope = torch.empty((E, 8, H, W), dtype=torch.float32, device=device)
        slope = torch.empty((E, H, W, 3, 3), dtype=torch.float32, device=device)
        call("gca_alex_slope_from_altitude", dev.ptr(alt), dev.ptr(p_slope), dev.ptr(slope), E, H, W,
             dev.stream_ptr(device))
        got = slope.cpu().numpy()
        ok, frac_equal = _slope_f32_close(got, g[f"slope_{k}"])
        assert ok and frac_equal > 0.999, (k, frac_equal)
        # p_slope = exp_f32(0.078 * slope) of the device's f32 slope, bit-exact with the oracle
        assert np.array_equal(p_slope.cpu().numpy(), alex_c.prepare_slope(got.reshape(E, H, W, 9)))


def test_env_layers_from_seeded_legacy_stream(device, golden):
    """AdvancedForestFireBulldozerEnv(use_hidden=True) draws density, vegetation, altitude in the
    reference constructor's order (advanced_bulldozer.py:182-197). The fixture drew vegetation first,
    then density, with the same patch recipe, so env.density is the fixture's first layer."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    g = golden("init_utils")
    H, W, E = (int(x) for x in g["shape_0"])
    env = AdvancedForestFireBulldozerEnv(H, W, num_envs=E, use_hidden=True, device=device, observation="grid",
                                         hidden_rng=np.random.RandomState(1000))
    assert np.array_equal(env.density.cpu().numpy(), g["veg_0"])
    assert np.array_equal(env.vegetation.cpu().numpy(), g["den_0"])
    alt = env.altitude.cpu().numpy()
    assert np.max(np.abs(alt - g["alt_0"]) / np.maximum(np.abs(g["alt_0"]), 1.0)) < 1e-14
    env.reset()
    assert np.array_equal(env.density.cpu().numpy(), g["veg_0"])  # layers persist across resets


def test_device_altitude_large_batch_matches_host(device):
    """E = 64 at 256 x 256: device arithmetic vs the host restatement of the same plan."""
    plan = iu.altitude_plan(256, 256, 64, np.random.RandomState(7))
    host = iu.apply_altitude_plan(plan)
    dev_alt = iu.device_altitude(plan, device).cpu().numpy()
    assert np.max(np.abs(dev_alt - host) / np.maximum(np.abs(host), 1.0)) < 1e-14


def _hidden_restated(seed, gid, R, C):
    """gca_hidden_init for one env, restated with the numpy Philox (include/gca.h recipe)."""
    from oracle.philox import philox4x32_10, seed_key, u01_f64

    key = seed_key(seed)
    TAG, TAGC = 0x48494444, 0x48494443

    def draw(slot):
        return [int(v) for v in philox4x32_10(np.array([[slot, gid, 0, TAG]], np.uint64), key)[0]]

    def ri(x, lo, hi):
        return lo if hi <= lo else lo + ((x * (hi - lo)) >> 32)

    layers = []
    for layer in range(2):
        base = 64 * layer
        n = ri(draw(base)[0], 4, 8)
        m = np.zeros((R, C), np.int64)
        for p in range(n):
            a, b = draw(base + 8 + 2 * p), draw(base + 9 + 2 * p)
            cr, cc, ph, pw = ri(a[0], 0, R), ri(a[1], 0, C), ri(a[2], 3, max(4, R // 2)), ri(a[3], 3, max(4, C // 2))
            m[max(0, cr - ph // 2):min(R, cr + ph // 2), max(0, cc - pw // 2):min(C, cc + pw // 2)] = ri(b[0], 1, 6)
        layers.append(m)
    lin = np.arange(R * C, dtype=np.uint64)
    ctr = np.stack([lin, np.full_like(lin, gid), np.zeros_like(lin), np.full_like(lin, TAGC)], axis=1)
    x = philox4x32_10(ctr, key).astype(np.uint64)
    fill = lambda w: (1 + ((w * np.uint64(3)) >> np.uint64(32))).astype(np.int64).reshape(R, C)
    veg = np.where(layers[0] > 0, layers[0], fill(x[:, 0]))
    den = np.where(layers[1] > 0, layers[1], fill(x[:, 1]))
    noise = 5.0 * u01_f64(x[:, 2], x[:, 3]).reshape(R, C)
    cnt = draw(127)
    nh, ns = ri(cnt[0], 6, 10), ri(cnt[1], 4, 8)
    hills = np.zeros((10, 4))
    for h in range(nh):
        a = draw(128 + h)
        u = draw(144 + h)
        hills[h] = (ri(a[0], 0, R), ri(a[1], 0, C), ri(a[2], 2, max(3, min(R, C) // 4)), 2.0 + 4.0 * u01_f64(u[0], u[1]))
    slopes = np.zeros((8, 5))
    for k in range(ns):
        a = draw(160 + k)
        u = draw(176 + k)
        slopes[k] = (ri(a[0], 0, max(1, R - 4)), ri(a[1], 0, max(1, C - 4)), ri(a[2], 3, max(4, C // 4)),
                     ri(a[3], 3, max(4, R // 4)), 1.0 + 3.0 * u01_f64(u[0], u[1]))
    return veg, den, noise, nh, hills, ns, slopes


def _hidden_device(device, seed, offset, E, R, C):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    kw = dict(device=device)
    veg = torch.zeros((E, R, C), dtype=torch.uint8, **kw)
    den = torch.zeros_like(veg)
    alt = torch.zeros((E, R, C), dtype=torch.float64, **kw)
    nh, ns = torch.zeros(E, dtype=torch.int32, **kw), torch.zeros(E, dtype=torch.int32, **kw)
    hills, slopes = torch.zeros((E, 10, 4), dtype=torch.float64, **kw), torch.zeros((E, 8, 5), dtype=torch.float64, **kw)
    call("gca_hidden_init", seed, offset, E, R, C, dev.ptr(veg), dev.ptr(den), dev.ptr(alt), dev.ptr(nh),
         dev.ptr(hills), dev.ptr(ns), dev.ptr(slopes), dev.stream_ptr(device))
    return [t.cpu().numpy() for t in (veg, den, alt, nh, hills, ns, slopes)]


def test_device_hidden_layers_match_restatement(device):
    """gca_hidden_init (hidden_rng="philox") = its numpy restatement draw for draw, and a shard of envs
    (env_offset 5) draws exactly the layers the unsharded launch draws for those envs."""
    seed, R, C = 0x1234ABCD5678, 40, 56
    full = _hidden_device(device, seed, 0, 8, R, C)
    part = _hidden_device(device, seed, 5, 3, R, C)
    for a, b in zip(full, part):
        assert np.array_equal(a[5:8], b)
    for e in (0, 6):
        want = _hidden_restated(seed, e, R, C)
        got = [full[0][e], full[1][e], full[2][e], full[3][e], full[4][e], full[5][e], full[6][e]]
        for g, w in zip(got, want):
            assert np.array_equal(np.asarray(g), np.asarray(w))
    veg, den = full[0], full[1]
    assert veg.min() >= 1 and veg.max() <= 5 and den.min() >= 1 and den.max() <= 5
    assert np.all((full[3] >= 6) & (full[3] < 10)) and np.all((full[5] >= 4) & (full[5] < 8))


def test_env_philox_hidden_layers(device):
    """AdvancedForestFireBulldozerEnv(hidden_rng="philox"): layers from gca_hidden_init, altitude finished by
    gca_alex_altitude_apply (= the host arithmetic on the same plan), slopes from that altitude."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from gymca_amd.forest_fire.bulldozer.init_utils import apply_altitude_plan

    E, N = 3, 48
    env = AdvancedForestFireBulldozerEnv(N, N, key=77, num_envs=E, use_hidden=True, device=device, env_offset=2,
                                         hidden_rng="philox")
    veg, den, noise, nh, hills, ns, slopes = _hidden_device(device, 77, 2, E, N, N)
    assert np.array_equal(env.vegetation.cpu().numpy(), veg) and np.array_equal(env.density.cpu().numpy(), den)
    want = apply_altitude_plan(dict(noise=noise, hills=hills, n_hills=nh, slopes=slopes, n_slopes=ns))
    alt = env.altitude.cpu().numpy()
    assert np.max(np.abs(alt - want) / np.maximum(np.abs(want), 1.0)) < 1e-14
