"""Pinecone spotting — host tables and parameters for gca_alex_pinecones and gca_alex_pinecones_classic
(gca_pine.hip).

Reference: PartiallyObservableForestFireJax._handle_pinecone_spread (ca_alexandridis_jax.py:229-319),
_compute_pinecone_burn_probability (:208-227) and the scatter in _update_grid (:400-420), which the
reference keeps commented out; `pinecones=True` on the env / operator enables it here.

The kernel draws the integer thrust s = round(N(0, 1) * f) of a pinecone directly: landing rows and
columns are round(r + dx * t) with dx in {-1, 0, 1}, which is r + dx * round(t) for continuous t. Its
law P(s = k) = Phi((k + 1/2) / f) - Phi((k - 1/2) / f) is tabulated here in float64 as 32-bit inverse-CDF
thresholds, one table per (wind, direction) with f = ft[ft_lookup[direction]] of that wind; the kernel and
the C oracle only compare integers against them. The tail beyond |s| = K = ceil(6.5 f + 1/2) has
probability below 2^-32 (|Z| > 6.5) and folds into s = +-K.

The classic operator (PartiallyObservableForestFire, ca_alexandridis.py:35-69, 113-133, 184-210) uses the
same construction with thrust 3 N(0, 1) ft[lookup[d]] (:189-190, f = 3 ft up to 3), an uncapped Poisson(1)
count (tail folded at 16 pinecones, P(N > 15) < 2^-32), no clipping of landings and its own burn tables;
its burn test `p_burn > uniform` (:127) becomes the integer compare u24 < ceil(p_burn 2^24) with p_burn
evaluated in float64 exactly as the reference writes it.
"""
import math

import functools

import numpy as np

from ..._lib import GCA_PINE_CDF, GCA_PINE_MAX, GCA_PINEC_CDF, GCA_PINEC_NMAX, PineClassicParams, PineParams

DX = [1, 1, 0, -1, -1, -1, 0, 1]  # E, NE, N, NW, W, SW, S, SE (:259)
DY = [0, 1, 1, 1, 0, -1, -1, -1]  # (:260)
FT_LOOKUP = [(0, 0), (0, 1), (0, 2), (1, 0), (1, 2), (2, 0), (2, 1), (2, 2)]  # (:261-272)
PINE_VEG = [-999, -0.1, 0.2, 0.5, 0.8, 1.2]  # (:211-213)
PINE_DEN = [-999, -0.2, 0.2, 0.5, 0.8, 1.2]  # (:214)
PINE_SCALE = 0.48  # (:227)
MAX_PINECONES = 5  # (:230)
PINE_AGE = (4, 11)  # random.randint(key, shape, 4, 11) (:409)


def _phi(x):
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def _u32(p):
    return min(int(round(p * 2.0 ** 32)), 2 ** 32 - 1)


def poisson_thresholds(lam=1.0, n=GCA_PINE_MAX):
    """n = #{j : x >= T_j} for a uniform u32 x is Poisson(lam) (capped at n); T_j = P(N <= j) 2^32."""
    out, acc, term = [], 0.0, math.exp(-lam)
    for j in range(n):
        acc += term
        term *= lam / (j + 1)
        out.append(_u32(acc))
    return np.array(out, dtype=np.uint32)


def thrust_table(f, size=GCA_PINE_CDF, fmax=1.0):
    """[2K, T_0 .. T_{2K-1}] padded to `size`: s = -K + #{j : x >= T_j}, T_j = P(round(Z f) <= -K + j) 2^32."""
    f = float(f)
    if not 0.0 < f <= fmax:
        raise ValueError(f"thrust scale must be in (0, {fmax}] (ft of calc_pw), got {f}")
    K = max(1, math.ceil(6.5 * f + 0.5))
    t = [2 * K] + [_u32(_phi((-K + j + 0.5) / f)) for j in range(2 * K)]
    assert len(t) <= size
    return np.array(t + [0xFFFFFFFF] * (size - len(t)), dtype=np.uint32)


def thrust_law(f, K=None):
    """Exact P(s = k) of s = round(Z f), k = -K..K (the tails folded into +-K) — for tests."""
    K = K or max(1, math.ceil(6.5 * f + 0.5))
    ks = np.arange(-K, K + 1)
    hi = np.array([_phi((k + 0.5) / f) if k < K else 1.0 for k in ks])
    lo = np.array([_phi((k - 0.5) / f) if k > -K else 0.0 for k in ks])
    return ks, hi - lo


def _host_winds(winds):
    if hasattr(winds, "is_cuda") and winds.is_cuda:
        winds = winds.cpu().numpy()
    w = np.ascontiguousarray(np.asarray(winds, dtype=np.float32))
    if w.ndim != 4 or w.shape[1] != 2:
        raise ValueError("winds must be (n, 2, 3, 3) (wind_matrix, ft) pairs")
    return w


def s_cdf_tables(winds):
    """(n_winds, 8, GCA_PINE_CDF) u32 from shared_context["winds"] (n, 2, 3, 3): the ft matrix of each wind
    at ft_lookup[direction]. Memoised on the table's contents (the operators call it per step)."""
    w = _host_winds(winds)
    return _s_cdf_tables(w.tobytes(), w.shape).copy()


@functools.lru_cache(maxsize=16)
def _s_cdf_tables(raw, shape):
    w = np.frombuffer(raw, dtype=np.float32).reshape(shape)
    return np.stack([np.stack([thrust_table(w[i, 1][a, b]) for (a, b) in FT_LOOKUP]) for i in range(len(w))])


def make_pine_params(seed, empty, tree, fire, env_offset=0, max_pinecones=MAX_PINECONES):
    p = PineParams()
    for j, t in enumerate(poisson_thresholds()):
        p.n_cdf[j] = int(t)
    p.max_pinecones = int(max_pinecones)
    for d in range(8):
        p.dx[d], p.dy[d] = DX[d], DY[d]
    p.scale = float(np.float32(PINE_SCALE))
    veg1p = (np.float32(1) + np.array(PINE_VEG, dtype=np.float32)).astype(np.float32)
    den1p = (np.float32(1) + np.array(PINE_DEN, dtype=np.float32)).astype(np.float32)
    for i in range(6):
        p.veg1p[i], p.den1p[i] = float(veg1p[i]), float(den1p[i])
    p.age_lo, p.age_hi = PINE_AGE
    p.seed = int(seed) & (2 ** 64 - 1)
    p.env_offset = int(env_offset)
    p.empty, p.tree, p.fire = int(empty), int(tree), int(fire)
    return p


# ---------------------------------------------------------------------------- classic operator
CLASSIC_THRUST = 3.0  # pinecone_thrust = 3 * standard_normal (:189)
CLASSIC_PINE_VEG = {1: 0.0, 2: 0.8, 3: 1.6, 4: 2.0, 5: 2.5}  # :122
CLASSIC_PINE_DEN = {1: 0.0, 2: 0.6, 3: 1.2, 4: 1.5, 5: 2.0}  # :123
CLASSIC_PINE_P_H = 0.58  # :124
CLASSIC_PINE_AGE = (4, 11)  # integers(4, 11) (:131)


def classic_burn_probability(veg, den):
    """p_burn of _set_fire_pinecone (:122-126) in Python float64, the reference's expression order."""
    return CLASSIC_PINE_P_H * (1 + CLASSIC_PINE_VEG[veg]) * (1 + CLASSIC_PINE_DEN[den])


def classic_burn_thresholds():
    """[veg][den] u24 thresholds: u = k / 2^24 < p  <=>  k < ceil(p 2^24) (p 2^24 is exact in f64)."""
    thr = np.zeros((6, 6), dtype=np.uint32)
    for v in range(6):
        for d in range(6):
            p = classic_burn_probability(max(1, v), max(1, d))
            thr[v, d] = min(max(math.ceil(p * 2.0 ** 24), 0), 2 ** 24)
    return thr


def classic_thrust_tables(winds):
    """(n_winds, 8, GCA_PINEC_CDF) u32: thrust tables of f = 3 ft[lookup[d]] per (wind, direction). Memoised on
    the table's contents."""
    w = _host_winds(winds)
    return _classic_thrust_tables(w.tobytes(), w.shape).copy()


@functools.lru_cache(maxsize=16)
def _classic_thrust_tables(raw, shape):
    w = np.frombuffer(raw, dtype=np.float32).reshape(shape)
    return np.stack([np.stack([thrust_table(CLASSIC_THRUST * float(w[i, 1][a, b]), GCA_PINEC_CDF, CLASSIC_THRUST)
                               for (a, b) in FT_LOOKUP]) for i in range(len(w))])


def make_classic_pine_params(seed, empty, tree, fire, env_offset=0):
    p = PineClassicParams()
    for j, t in enumerate(poisson_thresholds(1.0, GCA_PINEC_NMAX)):
        p.n_cdf[j] = int(t)
    for d in range(8):
        p.dx[d], p.dy[d] = DX[d], DY[d]
    thr = classic_burn_thresholds()
    for v in range(6):
        for d in range(6):
            p.burn_thr[v][d] = int(thr[v, d])
    p.age_lo, p.age_hi = CLASSIC_PINE_AGE
    p.seed = int(seed) & (2 ** 64 - 1)
    p.env_offset = int(env_offset)
    p.empty, p.tree, p.fire = int(empty), int(tree), int(fire)
    return p
