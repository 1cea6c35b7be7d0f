"""Context inputs of the Advanced env (reference bulldozer/utils/init_utils.py:10-245).

Winds follow the reference exactly. The hidden layers (vegetation / density patches, altitude
hills and slopes) consume random numbers in exactly the reference's order, so with the same
legacy stream they are identical to the reference's output:
  * rng=None            -> the global np.random state, like the reference itself
                           (np.random.seed(s) before reset reproduces the reference's layers);
  * np.random.RandomState -> the same draws from a private legacy stream;
  * np.random.Generator  -> the same recipe on Generator draws (not stream-compatible).
Pinned by tests/golden/init_utils.npz (the reference functions after np.random.seed(k)).
The per-pixel loops of the reference are vectorised per patch / hill / slope with the same
float64 operations in the same order. They run once per reset, not on the step path;
get_slope runs on the device (gca_alex_slope_from_altitude).
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


class _Draws:
    """randint / uniform with the legacy RandomState signature over any numpy random source."""

    def __init__(self, rng):
        self.rng = np.random if rng is None else rng
        self.legacy = not isinstance(self.rng, np.random.Generator)

    def randint(self, lo, hi, size=None):
        if self.legacy:
            return self.rng.randint(lo, hi, size=size)
        return self.rng.integers(lo, hi, size=size)

    def uniform(self, lo, hi, size=None):
        return self.rng.uniform(lo, hi, size)


def _patches(row_count, column_count, num_envs, rng):
    """Shared patch recipe of init_vegetation / init_density (:10-73), draw for draw."""
    d = _Draws(rng)
    out = np.zeros((num_envs, row_count, column_count), dtype=int)
    for env in range(num_envs):
        m = out[env]
        for _ in range(d.randint(4, 8)):
            center_row = d.randint(0, row_count)
            center_col = d.randint(0, column_count)
            patch_height = d.randint(3, max(4, row_count // 2))  # max(): the reference needs N >= 8
            patch_width = d.randint(3, max(4, column_count // 2))
            value = d.randint(1, 6)
            r0, r1 = max(0, center_row - patch_height // 2), min(row_count, center_row + patch_height // 2)
            c0, c1 = max(0, center_col - patch_width // 2), min(column_count, center_col + patch_width // 2)
            m[r0:r1, c0:c1] = value
        zero = m == 0
        m[zero] = d.randint(1, 4, size=int(zero.sum()))  # row-major order, like veg_matrix[env][zero_mask]
    return out


def init_vegetation(row_count, column_count, num_envs, rng=None):
    """init_utils.py:10-40."""
    return _patches(row_count, column_count, num_envs, rng)


def init_density(row_count, column_count, num_envs, rng=None):
    """init_utils.py:43-73."""
    return _patches(row_count, column_count, num_envs, rng)


MAX_HILLS, MAX_SLOPES = 10, 8  # randint(6, 10) hills, randint(4, 8) slopes (:83, :101)


def altitude_plan(row_count, column_count, num_envs, rng=None):
    """Every random draw of init_altitude (:76-116) in the reference's order, without the arithmetic:
    noise (E, H, W) f64, hills (E, MAX_HILLS, 4) = (centre row, centre col, radius, height) with
    n_hills (E,), slopes (E, MAX_SLOPES, 5) = (start row, start col, width, height, height_diff) with
    n_slopes (E,). apply_altitude_plan (host) or gca_alex_altitude_apply (device) does the rest."""
    d = _Draws(rng)
    E, R, C = num_envs, row_count, column_count
    noise = np.empty((E, R, C))
    hills = np.zeros((E, MAX_HILLS, 4))
    slopes = np.zeros((E, MAX_SLOPES, 5))
    n_hills = np.zeros(E, dtype=np.int32)
    n_slopes = np.zeros(E, dtype=np.int32)
    for env in range(E):
        noise[env] = d.uniform(0, 5, (R, C))
        n_hills[env] = d.randint(6, 10)
        for h in range(n_hills[env]):
            center_row = d.randint(0, R)
            center_col = d.randint(0, C)
            radius = d.randint(2, max(3, min(R, C) // 4))  # max(): the reference needs N >= 12
            height = d.uniform(2, 6)
            hills[env, h] = (center_row, center_col, radius, height)
        n_slopes[env] = d.randint(4, 8)
        for k in range(n_slopes[env]):
            start_row = d.randint(0, max(1, R - 4))
            start_col = d.randint(0, max(1, C - 4))
            width = d.randint(3, max(4, C // 4))
            height = d.randint(3, max(4, R // 4))
            height_diff = d.uniform(1, 4)
            slopes[env, k] = (start_row, start_col, width, height, height_diff)
    return dict(noise=noise, hills=hills, n_hills=n_hills, slopes=slopes, n_slopes=n_slopes)


def apply_altitude_plan(plan):
    """The reference's arithmetic (:89-116) on the host: one vectorised update per hill / slope with
    the per-pixel float64 expression, in the reference's order; then / 10."""
    altitude = plan["noise"].copy()
    E, R, C = altitude.shape
    ii, jj = np.meshgrid(np.arange(R), np.arange(C), indexing="ij")
    for env in range(E):
        a = altitude[env]
        for h in range(plan["n_hills"][env]):
            center_row, center_col, radius, height = plan["hills"][env, h]
            center_row, center_col, radius = int(center_row), int(center_col), int(radius)
            distance = np.sqrt((ii - center_row) ** 2 + (jj - center_col) ** 2)
            inside = distance < radius
            a[inside] += height * np.cos(distance[inside] / radius * np.pi / 2)
        for k in range(plan["n_slopes"][env]):
            start_row, start_col, width, height, height_diff = plan["slopes"][env, k]
            start_row, start_col, width, height = int(start_row), int(start_col), int(width), int(height)
            r1, c1 = min(start_row + height, R), min(start_col + width, C)
            progress = (np.arange(start_row, r1) - start_row) / height
            a[start_row:r1, start_col:c1] += (height_diff * progress)[:, None]
    return altitude / 10


def init_altitude(row_count, column_count, num_envs, rng=None):
    """Noise + cosine hills + linear slopes, / 10 (:76-116), draw for draw."""
    return apply_altitude_plan(altitude_plan(row_count, column_count, num_envs, rng))


def get_slope(altitude, row_count, column_count, num_envs):
    """Host float64 get_slope (:166-200) without the histogram print; the device path is
    gca_alex_slope_from_altitude."""
    alt = np.asarray(altitude, dtype=np.float64).reshape(num_envs, row_count, column_count)
    slope = np.zeros((num_envs, row_count, column_count, 3, 3))
    if row_count < 3 or column_count < 3:
        return slope
    cur = alt[:, 1:-1, 1:-1]
    for i in range(3):
        for j in range(3):
            if (i, j) == (1, 1):
                continue
            diffs = cur - alt[:, i:i + row_count - 2, j:j + column_count - 2]
            if i != 1 and j != 1:
                diffs = diffs / 1.414
            slope[:, 1:-1, 1:-1, i, j] = np.degrees(np.arctan(diffs))
    return slope


def init_density_same(row_count, column_count, num_envs):
    return np.full((num_envs, row_count, column_count), 3, dtype=int)


def init_vegetation_same(row_count, column_count, num_envs):
    return np.full((num_envs, row_count, column_count), 3, dtype=int)


def init_altitude_same(row_count, column_count, num_envs):
    return np.zeros((num_envs, row_count, column_count), dtype=int)


def device_altitude(plan, device):
    """init_altitude's arithmetic on the device (gca_alex_altitude_apply) for a host plan; returns the
    (E, H, W) float64 altitude tensor. Same float64 expression as the reference per cell; only cos may
    differ from numpy's in the last ulp (tests/test_gpu_init.py)."""
    import torch

    from ... import _device as dev
    from ..._lib import call

    alt = torch.as_tensor(np.ascontiguousarray(plan["noise"]), dtype=torch.float64, device=device)
    E, H, W = alt.shape
    T = lambda a, t: torch.as_tensor(np.ascontiguousarray(a), dtype=t, device=device)
    nh, hills = T(plan["n_hills"], torch.int32), T(plan["hills"], torch.float64)
    ns, slopes = T(plan["n_slopes"], torch.int32), T(plan["slopes"], torch.float64)
    call("gca_alex_altitude_apply", dev.ptr(alt), E, H, W, dev.ptr(nh), dev.ptr(hills), dev.ptr(ns), dev.ptr(slopes),
         dev.stream_ptr(device))
    return alt
