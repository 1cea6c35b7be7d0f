"""CPU: the observation oracle (oracle/observation.py, a literal numpy restatement of the reference's
observation code) and the integer forms the device kernel relies on."""
import numpy as np
import pytest

from oracle import observation as ob


@pytest.mark.parametrize("seed", range(5))
def test_f32_blur_is_the_integer_rounding(seed):
    rng = np.random.default_rng(seed)
    for _ in range(40):
        H, W = rng.integers(1, 12, 2)
        g = rng.integers(0, 4, (H, W))
        p = np.pad(g, ((1, 1), (1, 1)), mode="edge")
        S = sum(p[i:i + H, j:j + W] for i in range(3) for j in range(3))
        assert np.array_equal(ob.apply_blur(g), (2 * S + 9) // 18)


def test_extension_lookup_matches_itertools_order():
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP, up_to_k_mappings

    assert EXTENSION_LOOKUP.tolist() == [[0, 0], [1, 0], [0, 1]]
    assert up_to_k_mappings(3, 2).tolist() == [[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0], [1, 0, 1],
                                               [0, 1, 1]]


def test_channel_index_quirk():
    """has_extension runs over rows: with the unblur flag on and row 0 empty the display is the (zero)
    second extension channel, i.e. every cell renders as EMPTY."""
    g = np.ones((6, 6), np.int32)
    g[0] = 0
    rgb, ch = ob.step_observation(g, (5, 5), (1, 0), 0, np.zeros((6, 6), np.int32), True, True)
    assert np.all(rgb[:5, :5] == np.array(ob.DAY["empty"], np.float32))
    g[0, 2] = 1
    rgb, _ = ob.step_observation(g, (5, 5), (1, 0), 0, np.zeros((6, 6), np.int32), True, True)
    assert np.all(rgb[1:5, :5] == np.array(ob.DAY["tree"], np.float32))


def test_reset_observation_broadcast():
    """The reference's reset observation colours cell (r, c) by grid[c][k] (k = 3 + first row with a
    positive value in columns 3..), blends dousing of (r, c), then sets the position."""
    rng = np.random.default_rng(3)
    g = rng.choice([0, 1, 2], size=(7, 7))
    d = (rng.random((7, 7)) < 0.3).astype(np.int32)
    rgb = ob.reset_observation(g, (1, 2), 1, d)
    has = (g[:, 3:] > 0).any(axis=1)
    k = 3 + min(int(np.argmax(has)), 3) if has.any() else 0
    col = lambda v: np.array(ob.NIGHT["tree" if v == 1 else "fire" if v == 2 else "empty"], np.float32)
    for r in range(7):
        for c in range(7):
            want = col(g[c, k])
            if d[r, c] == 1:
                want = want * np.float32(0.25) + np.array(ob.TINT_NIGHT, np.float32) * np.float32(0.75)
            if (r, c) == (1, 2):
                want = np.zeros(3, np.float32)
            assert np.array_equal(rgb[r, c], want)
