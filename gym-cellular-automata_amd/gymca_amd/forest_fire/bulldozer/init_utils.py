"""Context inputs of the Advanced env (reference bulldozer/utils/init_utils.py:10-245).

Winds follow the reference exactly. The hidden layers (vegetation / density patches,
altitude hills) are restated with numpy broadcasting over a seeded Generator instead
of the reference's per-pixel Python loops over the global np.random state (same
distributions; the reference's draws are unseeded, so no stream can be matched).
They run once per reset, not on the step path; get_slope runs on the device
(gca_alex_slope_from_altitude).
"""
import numpy as np

# init_utils.py:203-220
WIND_THETAS = [
    [[45, 0, 45], [90, 0, 90], [135, 180, 135]],
    [[90, 45, 0], [135, 0, 45], [180, 135, 90]],
    [[135, 90, 45], [180, 0, 0], [135, 90, 45]],
    [[180, 135, 90], [135, 0, 45], [90, 45, 0]],
    [[135, 180, 135], [90, 0, 90], [45, 0, 45]],
    [[90, 135, 180], [45, 0, 135], [0, 45, 90]],
    [[45, 90, 135], [0, 0, 180], [45, 90, 135]],
    [[0, 45, 90], [45, 0, 135], [90, 135, 180]],
]


def calc_pw(theta):
    """init_utils.py:225-230."""
    c_1, c_2 = 0.045, 0.131
    V = 10
    t = np.radians(theta)
    ft = np.exp(V * c_2 * (np.cos(t) - 1))
    return np.exp(c_1 * V) * ft, ft


def get_winds(use_hidden):
    """init_utils.py:233-245 — note the reference iterates wind_thetas whatever use_hidden is (:239)."""
    winds = []
    for thetas in WIND_THETAS:
        wind_matrix, ft = calc_pw(np.array(thetas))
        wind_matrix[1, 1] = 0
        winds.append((wind_matrix, ft))
    return winds


def _patches(row_count, column_count, num_envs, rng):
    """Shared patch recipe of init_vegetation / init_density (:10-73)."""
    out = np.zeros((num_envs, row_count, column_count), dtype=np.int64)
    for env in range(num_envs):
        m = out[env]
        for _ in range(rng.integers(4, 8)):
            center_row = rng.integers(0, row_count)
            center_col = rng.integers(0, column_count)
            patch_height = rng.integers(3, max(4, row_count // 2))
            patch_width = rng.integers(3, max(4, column_count // 2))
            value = rng.integers(1, 6)
            r0, r1 = max(0, center_row - patch_height // 2), min(row_count, center_row + patch_height // 2)
            c0, c1 = max(0, center_col - patch_width // 2), min(column_count, center_col + patch_width // 2)
            m[r0:r1, c0:c1] = value
        zero = m == 0
        m[zero] = rng.integers(1, 4, size=int(zero.sum()))
    return out


def init_vegetation(row_count, column_count, num_envs, rng=None):
    return _patches(row_count, column_count, num_envs, rng or np.random.default_rng())


def init_density(row_count, column_count, num_envs, rng=None):
    return _patches(row_count, column_count, num_envs, rng or np.random.default_rng())


def init_altitude(row_count, column_count, num_envs, rng=None):
    """Noise + cosine hills + linear slopes, / 10 (:76-116), vectorised per hill."""
    rng = rng or np.random.default_rng()
    altitude = np.zeros((num_envs, row_count, column_count))
    ii, jj = np.meshgrid(np.arange(row_count), np.arange(column_count), indexing="ij")
    for env in range(num_envs):
        a = altitude[env]
        a[:] = rng.uniform(0, 5, (row_count, column_count))
        for _ in range(rng.integers(6, 10)):
            center_row = rng.integers(0, row_count)
            center_col = rng.integers(0, column_count)
            radius = rng.integers(2, max(3, min(row_count, column_count) // 4))
            height = rng.uniform(2, 6)
            distance = np.sqrt((ii - center_row) ** 2 + (jj - center_col) ** 2)
            inside = distance < radius
            a[inside] += height * np.cos(distance[inside] / radius * np.pi / 2)
        for _ in range(rng.integers(4, 8)):
            start_row = rng.integers(0, max(1, row_count - 4))
            start_col = rng.integers(0, max(1, column_count - 4))
            width = rng.integers(3, max(4, column_count // 4))
            height = rng.integers(3, max(4, row_count // 4))
            height_diff = rng.uniform(1, 4)
            r1, c1 = min(start_row + height, row_count), min(start_col + width, column_count)
            progress = (np.arange(start_row, r1) - start_row) / height
            a[start_row:r1, start_col:c1] += (height_diff * progress)[:, None]
    return altitude / 10


def init_density_same(row_count, column_count, num_envs):
    return np.full((num_envs, row_count, column_count), 3, dtype=int)


def init_vegetation_same(row_count, column_count, num_envs):
    return np.full((num_envs, row_count, column_count), 3, dtype=int)


def init_altitude_same(row_count, column_count, num_envs):
    return np.zeros((num_envs, row_count, column_count), dtype=int)
