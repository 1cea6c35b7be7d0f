"""ctypes wrapper of oracle/build/libgca_oracle.so (gca_oracle.c). Test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libgca_oracle.so")


class OracleAlexParams(ctypes.Structure):
    _fields_ = [("R", ctypes.c_int32), ("heat_dw", ctypes.c_float * 9), ("dous_inner", ctypes.c_float),
                ("dous_border", ctypes.c_float), ("veg1p", ctypes.c_float * 6), ("den1p", ctypes.c_float * 6),
                ("p_tree", ctypes.c_float), ("age_lo", ctypes.c_int32), ("age_hi", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("env_offset", ctypes.c_int32), ("empty", ctypes.c_int32),
                ("tree", ctypes.c_int32), ("fire", ctypes.c_int32), ("n_winds", ctypes.c_int32),
                ("winds", (ctypes.c_float * 9) * 16), ("heat0", ctypes.c_float),
                ("burnout_eq1", ctypes.c_int32), ("vd_uniform", ctypes.c_int32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_exp_f32.restype = ctypes.c_float
        _lib.oracle_exp_f32.argtypes = [ctypes.c_float]
        _lib.oracle_slope_factor.restype = ctypes.c_float
        _lib.oracle_slope_factor.argtypes = [ctypes.c_float]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def params_from(p):
    """Copy a field-compatible ctypes struct (e.g. the product's AlexParams) into the oracle's."""
    o = OracleAlexParams()
    ctypes.memmove(ctypes.addressof(o), ctypes.addressof(p), ctypes.sizeof(o))
    return o


def philox(ctr, k0, k1):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.empty_like(ctr)
    lib().oracle_philox(_p(ctr), ctypes.c_uint32(k0), ctypes.c_uint32(k1), _p(out), ctypes.c_long(len(ctr)))
    return out


def exp_f32(x):
    f = lib().oracle_exp_f32
    return np.array([f(float(v)) for v in np.asarray(x, dtype=np.float32).ravel()], dtype=np.float32).reshape(
        np.shape(x))


def slope_factor(a):
    f = lib().oracle_slope_factor
    return np.array([f(float(v)) for v in np.asarray(a, dtype=np.float32).ravel()], dtype=np.float32).reshape(
        np.shape(a))


def signed_factors(slope):
    """Edge-layout values V = +-exp_f32(|0.078 * slope|) (sign of the slope) for an f32 slope array."""
    slope = np.ascontiguousarray(slope, dtype=np.float32)
    out = np.empty_like(slope)
    lib().oracle_signed_factors(_p(slope), _p(out), ctypes.c_long(slope.size))
    return out


def factor_pairs(v):
    """(own, neighbour) slope factors the edge-slope kernel derives from V."""
    v = np.ascontiguousarray(v, dtype=np.float32)
    own, nbr = np.empty_like(v), np.empty_like(v)
    lib().oracle_factor_pairs(_p(v), _p(own), _p(nbr), ctypes.c_long(v.size))
    return own, nbr


def prepare_slope(slope):
    slope = np.ascontiguousarray(slope, dtype=np.float32)
    E, H, W = slope.shape[:3]
    out = np.empty((E, 8, H, W), dtype=np.float32)
    lib().oracle_alex_prepare_slope(_p(slope), _p(out), E, H, W)
    return out


def alex_step(params, grid, age, veg, den, dous, p_slope, wind_index, rng_step=None, inj=None, want_probs=False):
    E, H, W = grid.shape
    c = lambda a, t: np.ascontiguousarray(a, dtype=t)
    grid, age, veg, den, dous = c(grid, np.uint8), c(age, np.int16), c(veg, np.uint8), c(den, np.uint8), c(dous, np.uint8)
    p_slope, wind_index = c(p_slope, np.float32), c(wind_index, np.int32)
    rs = None if rng_step is None else c(rng_step, np.uint32)
    go, ao = np.empty_like(grid), np.empty_like(age)
    counts = np.zeros((E, 3), dtype=np.int32)
    ib = ig = ia = None
    if inj is not None:
        ib, ig, ia = c(inj[0], np.float32), c(inj[1], np.float32), c(inj[2], np.int32)
    probs = np.empty((E, H, W, 8), dtype=np.float32) if want_probs else None
    lib().oracle_alex_step(ctypes.byref(params_from(params)), E, H, W, _p(grid), _p(go), _p(age), _p(ao), _p(veg),
                           _p(den), _p(dous), _p(p_slope), _p(wind_index), _p(rs), _p(ib), _p(ig), _p(ia),
                           _p(probs), _p(counts))
    return go, ao, counts, probs


def wind_change(p_change, n_winds, seed, env_offset, rng_step, wind_index):
    wi = np.ascontiguousarray(wind_index, dtype=np.int32).copy()
    rs = np.ascontiguousarray(rng_step, dtype=np.uint32)
    lib().oracle_alex_wind_change(ctypes.c_float(p_change), n_winds, ctypes.c_uint64(seed), env_offset, _p(rs),
                                  _p(wi), len(wi))
    return wi


class OraclePineParams(ctypes.Structure):
    _fields_ = [("n_cdf", ctypes.c_uint32 * 8), ("max_pinecones", ctypes.c_int32), ("dx", ctypes.c_int32 * 8),
                ("dy", ctypes.c_int32 * 8), ("scale", ctypes.c_float), ("veg1p", ctypes.c_float * 6),
                ("den1p", ctypes.c_float * 6), ("age_lo", ctypes.c_int32), ("age_hi", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("env_offset", ctypes.c_int32), ("empty", ctypes.c_int32),
                ("tree", ctypes.c_int32), ("fire", ctypes.c_int32)]


def pinecones(params, grid_in, grid_out, age_out, veg, den, wind_index, s_cdf, rng_step=None, counts=None):
    """oracle_alex_pinecones on copies of grid_out / age_out / counts; params: a field-compatible struct
    (the product's PineParams). Returns (grid_out, age_out, counts)."""
    o = OraclePineParams()
    ctypes.memmove(ctypes.addressof(o), ctypes.addressof(params), ctypes.sizeof(o))
    E, H, W = grid_in.shape
    c = lambda a, t: np.ascontiguousarray(a, dtype=t)
    gi, go, ao = c(grid_in, np.uint8), c(grid_out, np.uint8).copy(), c(age_out, np.int16).copy()
    veg, den, wi, sc = c(veg, np.uint8), c(den, np.uint8), c(wind_index, np.int32), c(s_cdf, np.uint32)
    rs = None if rng_step is None else c(rng_step, np.uint32)
    cn = None if counts is None else c(counts, np.int32).copy()
    lib().oracle_alex_pinecones(ctypes.byref(o), E, H, W, _p(gi), _p(go), _p(ao), _p(veg), _p(den), _p(wi), _p(sc),
                                _p(rs), _p(cn))
    return go, ao, cn


class OraclePineClassicParams(ctypes.Structure):
    _fields_ = [("n_cdf", ctypes.c_uint32 * 16), ("dx", ctypes.c_int32 * 8), ("dy", ctypes.c_int32 * 8),
                ("burn_thr", (ctypes.c_uint32 * 6) * 6), ("age_lo", ctypes.c_int32), ("age_hi", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("env_offset", ctypes.c_int32), ("empty", ctypes.c_int32),
                ("tree", ctypes.c_int32), ("fire", ctypes.c_int32)]


def pinecones_classic(params, grid_in, grid_out, age_out, veg, den, wind_index, s_cdf, rng_step=None, counts=None):
    """oracle_alex_pinecones_classic (the literal sequential skip-list order) on copies; params: a
    field-compatible struct (the product's PineClassicParams). Returns (grid_out, age_out, counts,
    skipped_sources[E])."""
    o = OraclePineClassicParams()
    ctypes.memmove(ctypes.addressof(o), ctypes.addressof(params), ctypes.sizeof(o))
    E, H, W = grid_in.shape
    c = lambda a, t: np.ascontiguousarray(a, dtype=t)
    gi, go, ao = c(grid_in, np.uint8), c(grid_out, np.uint8).copy(), c(age_out, np.int16).copy()
    veg, den, wi, sc = c(veg, np.uint8), c(den, np.uint8), c(wind_index, np.int32), c(s_cdf, np.uint32)
    rs = None if rng_step is None else c(rng_step, np.uint32)
    cn = None if counts is None else c(counts, np.int32).copy()
    skipped = np.zeros(E, dtype=np.int32)
    lib().oracle_alex_pinecones_classic(ctypes.byref(o), E, H, W, _p(gi), _p(go), _p(ao), _p(veg), _p(den), _p(wi),
                                        _p(sc), _p(rs), _p(cn), _p(skipped))
    return go, ao, cn, skipped
