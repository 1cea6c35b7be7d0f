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
    env = AdvancedForestFireBulldozerEnv(H, W, num_envs=E, use_hidden=True, device=device,
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
