"""ctypes binding of libgca_hip.so — the C-ABI declared in include/gca.h.

This module is the ONLY bridge between Python and the gfx950 kernels. It fails
loudly (GCAError at import of a product op) when the shared library is missing:
there is no CPU fallback anywhere in the product path.
"""
import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int16, c_int32, c_int64, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# GCA_LIB_PATH: an alternative build of the same library (A/B kernel experiments, scripts/build_variant.sh)
LIB_PATH = os.environ.get("GCA_LIB_PATH") or os.path.join(_HERE, "_lib", "libgca_hip.so")
# the host backend of the same C-ABI (csrc/gca_cpu.cpp): host pointers, `stream` ignored
CPU_LIB_PATH = os.path.join(_HERE, "_lib", "libgca_cpu.so")

GCA_OK = 0
GCA_MAX_RADIUS = 8

TAG_WINDY_ROLL = 0x574E4459
TAG_ALEX_CELL = 0x414C5843
TAG_ALEX_AGE = 0x414C5841
TAG_ALEX_WIND = 0x414C5857
TAG_ACTION = 0x41435449
TAG_INIT = 0x494E4954
TAG_DS_CELL = 0x44534345
TAG_PINE = 0x50494E45
TAG_PINE_AGE = 0x50494E41
TAG_HIDDEN = 0x48494444
TAG_HIDDEN_CELL = 0x48494443
GCA_PINE_MAX = 8
GCA_PINE_CDF = 17
TAG_PINEC = 0x50434C00
TAG_PINEC_AGE = 0x50434C41
GCA_PINEC_NMAX = 16
GCA_PINEC_CDF = 48
GCA_PINEC_LDS_MAX_HW = 262144


class GCAError(RuntimeError):
    """Raised when the HIP library is missing or a C-ABI call returns non-zero."""


class BulldozerParams(ctypes.Structure):
    """gca_bulldozer_params (include/gca.h)."""

    _fields_ = [
        ("t_move", c_double * 9),
        ("t_shoot", c_double * 2),
        ("t_any", c_double),
        ("seed", c_uint64),
        ("env_offset", c_int32),
        ("empty", c_int32),
        ("tree", c_int32),
        ("fire", c_int32),
        ("up_mask", c_int32),
        ("down_mask", c_int32),
        ("left_mask", c_int32),
        ("right_mask", c_int32),
        ("effect", c_int16 * 256),
    ]


class AlexParams(ctypes.Structure):
    """gca_alex_params (include/gca.h)."""

    _fields_ = [
        ("R", c_int32),
        ("heat_dw", c_float * (GCA_MAX_RADIUS + 1)),
        ("dous_inner", c_float),
        ("dous_border", c_float),
        ("veg1p", c_float * 6),
        ("den1p", c_float * 6),
        ("p_tree", c_float),
        ("age_lo", c_int32),
        ("age_hi", c_int32),
        ("seed", c_uint64),
        ("env_offset", c_int32),
        ("empty", c_int32),
        ("tree", c_int32),
        ("fire", c_int32),
        ("n_winds", c_int32),
        ("winds", (c_float * 9) * 16),
        ("heat0", c_float),
        ("burnout_eq1", c_int32),
        ("vd_uniform", c_int32),
    ]


class PineParams(ctypes.Structure):
    """gca_pine_params (include/gca.h)."""

    _fields_ = [
        ("n_cdf", c_uint32 * GCA_PINE_MAX),
        ("max_pinecones", c_int32),
        ("dx", c_int32 * 8),
        ("dy", c_int32 * 8),
        ("scale", c_float),
        ("veg1p", c_float * 6),
        ("den1p", c_float * 6),
        ("age_lo", c_int32),
        ("age_hi", c_int32),
        ("seed", c_uint64),
        ("env_offset", c_int32),
        ("empty", c_int32),
        ("tree", c_int32),
        ("fire", c_int32),
    ]


class PineClassicParams(ctypes.Structure):
    """gca_pine_classic_params (include/gca.h)."""

    _fields_ = [
        ("n_cdf", c_uint32 * GCA_PINEC_NMAX),
        ("dx", c_int32 * 8),
        ("dy", c_int32 * 8),
        ("burn_thr", (c_uint32 * 6) * 6),
        ("age_lo", c_int32),
        ("age_hi", c_int32),
        ("seed", c_uint64),
        ("env_offset", c_int32),
        ("empty", c_int32),
        ("tree", c_int32),
        ("fire", c_int32),
    ]


class AdvEnvParams(ctypes.Structure):
    """gca_advenv_params (include/gca.h)."""

    _fields_ = [
        ("t_move", c_float * 9),
        ("t_shoot", c_float * 2),
        ("t_any", c_float),
        ("p_wind_change", c_float),
        ("day_length", c_int32),
        ("seed", c_uint64),
        ("env_offset", c_int32),
        ("n_winds", c_int32),
        ("up_mask", c_int32),
        ("down_mask", c_int32),
        ("left_mask", c_int32),
        ("right_mask", c_int32),
    ]


GCA_OBS_MAX_EXT = 4


class ObsParams(ctypes.Structure):
    """gca_obs_params (include/gca.h)."""

    _fields_ = [
        ("empty", c_int32),
        ("tree", c_int32),
        ("fire", c_int32),
        ("n_ext", c_int32),
        ("ext_skip_visibility", c_int32 * GCA_OBS_MAX_EXT),
        ("ext_skip_blur", c_int32 * GCA_OBS_MAX_EXT),
        ("enable_extensions", c_int32),
        ("should_transform", c_int32),
        ("day_length", c_int32),
        ("color_day", (c_float * 3) * 4),
        ("color_night", (c_float * 3) * 4),
        ("tint_day", c_float * 3),
        ("tint_night", c_float * 3),
        ("n_choices", c_int32),
        ("ext_lookup", (c_int32 * GCA_OBS_MAX_EXT) * 8),
    ]


P = c_void_p  # device pointers travel as plain addresses
_SIGNATURES = {
    "gca_last_error": ([], ctypes.c_char_p),
    "gca_version": ([], c_int),
    "gca_philox": ([P, c_uint32, c_uint32, P, c_int64, P], c_int),
    "gca_count_cells": ([P, c_int, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
    "gca_windy_dirmask": ([P, c_int64, P, c_uint64, P, P, c_int, c_int, P, c_int, P], c_int),
    "gca_windy_step": ([P, P, P, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
    "gca_bulldozer_pre": ([POINTER(BulldozerParams), P, P, P, P, P, c_int64, P, P, P, c_int, P], c_int),
    "gca_bulldozer_interpass": ([POINTER(BulldozerParams), c_int, P, P, P, c_int64, P, P, P, c_int, P], c_int),
    "gca_bulldozer_post": ([POINTER(BulldozerParams), c_int, P, P, P, P, P, c_int, c_int, P, P, P, P, P, P, c_int, P],
                           c_int),
    "gca_bulldozer_step_fused": ([POINTER(BulldozerParams), P, P, P, P, P, c_int64, P, P, P, P, c_int, c_int, P, P, P,
                                  P, P, P, c_int, P], c_int),
    "gca_bulldozer_step_fused_random": ([POINTER(BulldozerParams), c_uint64, P, P, P, P, P, c_int64, P, P, P, P, c_int,
                                         c_int, P, P, P, P, P, P, c_int, P], c_int),
    "gca_bulldozer_rollout_random": ([POINTER(BulldozerParams), c_uint64, c_int, P, P, P, P, P, P, P, c_int64, P, P, P,
                                      P, c_int, c_int, P, P, P, P, P, c_int, P], c_int),
    "gca_move_modify": ([POINTER(BulldozerParams), P, P, P, c_int, c_int, P, c_int, P], c_int),
    "gca_alex_prepare_slope": ([P, P, c_int, c_int, c_int, P], c_int),
    "gca_alex_step": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
                      c_int),
    "gca_alex_wind_change": ([c_float, c_int, c_uint64, c_int, P, P, P, P, c_int, P], c_int),
    "gca_alex_slope_from_altitude": ([P, P, P, c_int, c_int, c_int, P], c_int),
    "gca_alex_step_es": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
                         c_int),
    "gca_alex_edge_slope_from_altitude": ([P, P, c_int, c_int, c_int, P], c_int),
    "gca_alex_pinecones": ([POINTER(PineParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P], c_int),
    "gca_alex_pinecones_classic": ([POINTER(PineClassicParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P,
                                    P], c_int),
    "gca_alex_step_packed": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P], c_int),
    "gca_alex_step_packed_rgb": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, P,
                                  P, P], c_int),
    "gca_alex_step_march": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P], c_int),
    "gca_alex_step_march_rgb": ([POINTER(AlexParams), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, P,
                                 P, P], c_int),
    "gca_alex_step_march_rgb_ext": ([POINTER(AlexParams), POINTER(ObsParams), c_int, c_int, c_int, P, P, P, P, P, P, P,
                                     P, P, P, P, P, P, P, P, P, c_int, P, P], c_int),
    "gca_obs_color_table": ([POINTER(ObsParams), P, P], c_int),
    "gca_obs_position": ([POINTER(ObsParams), c_int, c_int, c_int, P, P, P, P, P], c_int),
    "gca_alex_pack_layers": ([P, P, P, P, P, c_int, c_int, c_int, P], c_int),
    "gca_alex_edge_slope_coalesce": ([P, P, c_int, c_int, c_int, P], c_int),
    "gca_alex_edge_factors": ([P, P, P, c_int64, P], c_int),
    "gca_adv_observation": ([POINTER(ObsParams), c_int, c_int, c_int, c_int, P, P, P, P, P, P, c_int, P, P, P, P],
                            c_int),
    "gca_alex_altitude_apply": ([P, c_int, c_int, c_int, P, P, P, P, P], c_int),
    "gca_advenv_post": ([POINTER(AdvEnvParams), P, P, P, P, P, P, P, P, c_int, c_int, P, P, P, P, P, P, c_int, P],
                        c_int),
    "gca_reset_where": ([P, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P], c_int),
    "gca_fill_categorical": ([P, c_int64, c_int, c_int, c_uint64, P, P, c_int, P], c_int),
    "gca_random_actions": ([P, c_int, c_int, c_uint64, P, P], c_int),
    "gca_hidden_init": ([c_uint64, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P], c_int),
    "gca_ds_count_draws": ([P, c_int, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
    "gca_ds_step": ([P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_uint64, P, c_int, P, P], c_int),
    "gca_bench_copy": ([P, P, c_int64, c_int, P], c_int),
    "gca_bench_march_pattern": ([c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P], c_int),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)
# the subset libgca_cpu.so exports (tiny grids and the O(1)-per-env operators on host arrays)
CPU_SYMBOLS = ("gca_last_error", "gca_version", "gca_philox", "gca_count_cells", "gca_move_modify",
               "gca_ds_count_draws", "gca_ds_step")

_lib = None
_lib_cpu = None


def load():
    """Load libgca_hip.so once; raise GCAError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GCAError(
            f"{LIB_PATH} not found: build it with `make -C gym-cellular-automata_amd/csrc` "
            "(or __graft_entry__.build()). There is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    for name, (argtypes, restype) in _SIGNATURES.items():
        if os.environ.get("GCA_LIB_PATH") and not hasattr(lib, name):
            continue  # an A/B build of an older tree may predate an entry point
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def load_cpu():
    """Load libgca_cpu.so once; raise GCAError if it is not built."""
    global _lib_cpu
    if _lib_cpu is not None:
        return _lib_cpu
    if not os.path.exists(CPU_LIB_PATH):
        raise GCAError(f"{CPU_LIB_PATH} not found: build it with `make -C gym-cellular-automata_amd/csrc`")
    lib = ctypes.CDLL(CPU_LIB_PATH, mode=ctypes.RTLD_LOCAL)
    for name in CPU_SYMBOLS:
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = _SIGNATURES[name]
    _lib_cpu = lib
    return lib


_cpu_fns = {}


def call_cpu(name, *args):
    """Call a gca_* entry point of the host backend (host pointers) and raise GCAError on a non-zero status."""
    fn = _cpu_fns.get(name)
    if fn is None:
        fn = _cpu_fns[name] = getattr(load_cpu(), name)
    status = fn(*args)
    if status != GCA_OK:
        msg = _lib_cpu.gca_last_error().decode(errors="replace")
        raise GCAError(f"{name} (host backend) failed (status {status}): {msg}")
    return status


def call(name, *args):
    """Call a gca_* entry point and raise GCAError on a non-zero status."""
    lib = load()
    status = getattr(lib, name)(*args)
    if status != GCA_OK:
        msg = lib.gca_last_error().decode(errors="replace")
        raise GCAError(f"{name} failed (status {status}): {msg}")
    return status


SLOT = object()  # a BoundCall argument supplied per call


_lib_raw = None


class BoundCall:
    """A gca_* entry point with its argument list converted to ctypes objects once.

    A batched env's step passes the same persistent device buffers on every call; only a few arguments (the action
    pointer, the stream) change. `BoundCall(name, *args)` converts every argument to its declared ctypes type up
    front (structs by reference, so later edits of the struct are seen), marks the `SLOT` positions, and each call
    only rebinds the slots' `.value` and calls the function pointer with the prepared tuple -- no per-call argtypes
    conversion, no dev.ptr() per buffer (a 21-argument call rebuilt from tensors cost ~11 us of
    host time per 1024-env step). `keep=` holds references to the objects (tensors) whose addresses were bound, so a
    bound address can never outlive its allocation: a caller that replaces a buffer and forgets to rebind gets stale
    state, never a write into memory the caching allocator has handed to someone else (the batched envs rebind on
    assignment: BatchedForestFireBulldozerEnv.__setattr__). Not thread-safe (one object per env, like the env)."""

    __slots__ = ("name", "_fn", "_args", "_slots", "_keep")

    def __init__(self, name, *args, keep=()):
        global _lib_raw
        load()  # the checked load (raises GCAError when the library is missing)
        if _lib_raw is None:
            # a second handle on the same library: its function objects carry no argtypes, so a call passes the
            # prepared ctypes objects as they are
            _lib_raw = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        argtypes, restype = _SIGNATURES[name]
        if len(args) != len(argtypes):
            raise TypeError(f"{name}: {len(argtypes)} arguments declared, {len(args)} bound")
        fn = _lib_raw[name]
        fn.restype = restype
        prepared, slots = [], []
        for t, a in zip(argtypes, args):
            if hasattr(t, "_type_") and isinstance(t._type_, type) and issubclass(t._type_, ctypes.Structure):
                if a is SLOT or not isinstance(a, t._type_):
                    raise TypeError(f"{name}: struct arguments are bound once, as {t._type_.__name__}")
                prepared.append(ctypes.byref(a))
                continue
            obj = t() if a is SLOT else t(a)
            if a is SLOT:
                slots.append(obj)
            prepared.append(obj)
        self.name, self._fn, self._args, self._slots = name, fn, tuple(prepared), tuple(slots)
        self._keep = tuple(keep)

    def __call__(self, *values):
        if len(values) != len(self._slots):
            raise TypeError(f"{self.name}: {len(self._slots)} per-call values expected, got {len(values)}")
        for obj, v in zip(self._slots, values):
            obj.value = v
        status = self._fn(*self._args)
        if status != GCA_OK:
            msg = _lib.gca_last_error().decode(errors="replace")
            raise GCAError(f"{self.name} failed (status {status}): {msg}")
        return status
