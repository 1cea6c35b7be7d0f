"""Shared synthetic Alexandridis inputs for the CPU and GPU parity tests."""
import numpy as np

from oracle import alexandridis_ref as ref


def winds():
    from gymca_amd.forest_fire.bulldozer.init_utils import get_winds

    return np.asarray(get_winds(True), dtype=np.float32)  # (8, 2, 3, 3)


def make_case(E, H, W, seed, fire_p=0.1, dousing_p=0.05, hidden=True, p_tree=0.0):
    """Mid-episode state: grid iid {0:.1, 1:.8, 2:.1}-ish, ages 1..672, veg/den 1..5, slopes."""
    rng = np.random.default_rng(seed)
    grid = rng.choice([0, 1, 2], size=(E, H, W), p=[0.1, 1 - 0.1 - fire_p, fire_p]).astype(np.uint8)
    age = np.where(grid == 2, rng.integers(-2, 673, size=(E, H, W)), rng.integers(-3, 4, size=(E, H, W)))
    veg = rng.integers(0, 7, size=(E, H, W)).astype(np.uint8) if hidden else np.full((E, H, W), 3, np.uint8)
    den = rng.integers(0, 7, size=(E, H, W)).astype(np.uint8) if hidden else np.full((E, H, W), 3, np.uint8)
    dous = (rng.random((E, H, W)) < dousing_p).astype(np.uint8)
    slope = (rng.normal(0, 20, size=(E, H, W, 3, 3)).clip(-89, 89) if hidden else np.zeros((E, H, W, 3, 3)))
    slope[..., 1, 1] = 0
    slope = slope.astype(np.float32)
    widx = rng.integers(0, 8, size=E).astype(np.int32)
    C = ref.constants(H)
    draws = (rng.random((E, H, W, 3, 3)).astype(np.float32), rng.random((E, H, W)).astype(np.float32),
             rng.integers(C["age_lo"], max(C["age_hi"], C["age_lo"] + 1), size=(E, H, W)).astype(np.int32))
    return dict(grid=grid, age=age.astype(np.int16), veg=veg, den=den, dous=dous, slope=slope, widx=widx,
                draws=draws, p_tree=p_tree, C=C)
