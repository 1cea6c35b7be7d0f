"""CPU: the antisymmetric edge-slope layout (oracle/edge_slope.py) reproduces get_slope exactly
(numpy float64 arctan, f32 cast) on random and reference-shaped altitude fields."""
import numpy as np
import pytest

from gymca_amd.forest_fire.bulldozer.init_utils import get_slope
from oracle import edge_slope


@pytest.mark.parametrize("E,H,W,seed", [(2, 3, 3, 0), (2, 5, 7, 1), (3, 16, 16, 2), (2, 37, 53, 3), (1, 64, 256, 4)])
def test_edge_layout_reproduces_get_slope(E, H, W, seed):
    rng = np.random.default_rng(seed)
    alt = rng.uniform(0, 5, (E, H, W)) + rng.normal(0, 30, (E, H, W)) * (rng.random((E, H, W)) < 0.3)
    want = get_slope(alt, H, W, E).astype(np.float32)
    got = edge_slope.slope9_from_edge(edge_slope.edge_from_altitude(alt))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_edge_layout_flat_and_golden(golden):
    g = golden("init_utils")
    for k in range(int(g["n"])):
        H, W, E = (int(x) for x in g[f"shape_{k}"])
        alt = g[f"alt_{k}"]
        got = edge_slope.slope9_from_edge(edge_slope.edge_from_altitude(alt))
        # the reference's own slope output for this altitude (tests/golden/make_golden.py)
        assert np.array_equal(got, np.asarray(g[f"slope_{k}"], np.float32).reshape(got.shape)), k
    flat = edge_slope.edge_from_altitude(np.zeros((1, 9, 9)))
    assert not flat.any()
